#!/usr/bin/env python3
"""C5 full loop, sequential vs pipelined.  Sequential (bench.py's full_loop_c5): halfspace launch
over the resident [256, 50, 10000] batch, then the clustered DR-CVaR QP over its 12 800 rows, one
stream.  Pipelined: the halfspaces of step i + 1 (double-buffered records, their own stream) run
while the QP of step i runs (high-priority stream) — the halfspaces depend only on the samples and
x_ref (main.py:95-100), never on a QP's answer.  Per-step wall time over K steps, and the QP
answers of both loops compared bitwise."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import engine, sharding, synthetic  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.engine import RiskParams  # noqa: E402


_HIP = None
_RAW_STREAMS = []  # (HIP handle, raw stream) created here, destroyed by destroy_streams()


def _hip():
    global _HIP
    if _HIP is None:
        import ctypes
        _HIP = ctypes.CDLL("libamdhip64.so")
    return _HIP


def _masked_stream(dev, words, what):
    """A raw HIP stream with the CU mask `words`, wrapped for torch.  The raw stream is recorded so
    that destroy_streams() can synchronise and destroy it through the same HIP handle before the
    process exits: left alive, its queue was torn down by the runtime's static destructors after the
    profiler had finalised, and the process died in __cxa_finalize (pipe_prof.log)."""
    import ctypes
    hip = _hip()
    mask = (ctypes.c_uint32 * len(words))(*words)
    h = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(len(words)), mask)
    assert rc == 0, f"hipExtStreamCreateWithCUMask: {rc}"
    _RAW_STREAMS.append(h)
    print(f"CU-masked halfspace stream: {what}", flush=True)
    return torch.cuda.ExternalStream(h.value, device=dev)


def destroy_streams():
    hip = _hip() if _RAW_STREAMS else None
    while _RAW_STREAMS:
        h = _RAW_STREAMS.pop()
        assert hip.hipStreamSynchronize(h) == 0
        assert hip.hipStreamDestroy(h) == 0


def cu_masked_stream(dev, reserve):
    """A HIP stream whose kernels may use every CU but `reserve` of them (every (n/reserve)-th bit of
    the CU mask cleared, so the reserved CUs spread over the XCDs whatever the bit order)."""
    n = torch.cuda.get_device_properties(dev).multi_processor_count
    words = [0xFFFFFFFF] * ((n + 31) // 32)
    if n % 32:
        words[-1] = (1 << (n % 32)) - 1
    step = n // reserve
    for k in range(reserve):
        b = k * step
        words[b // 32] &= ~(1 << (b % 32))
    return _masked_stream(dev, words, f"{n} CUs, {reserve} reserved")


def cu_allowed_stream(dev, allow):
    """A HIP stream whose kernels may use only `allow` CUs (every (n/allow)-th bit of the mask)."""
    n = torch.cuda.get_device_properties(dev).multi_processor_count
    words = [0] * ((n + 31) // 32)
    step = n // allow
    for k in range(allow):
        b = k * step
        words[b // 32] |= 1 << (b % 32)
    return _masked_stream(dev, words, f"{allow} of {n} CUs")


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    O, T, N, _ = bench.WORKLOADS["c5"]
    params = RiskParams()
    sb = sharding.ShardedBatch(synthetic.nominal_paths(O, T, dev, seed=7), synthetic.straight_line_ego(T, dev),
                               N, params, seed=7)
    samples, ego = sb.samples.view(O, T, N, 2), sb.ego_units[:T]
    dt = 0.2
    A = np.block([[np.eye(2), dt * np.eye(2)], [np.zeros((2, 2)), np.eye(2)]])
    Bm = np.block([[0.5 * dt ** 2 * np.eye(2)], [dt * np.eye(2)]])
    C = np.block([np.eye(2), np.zeros((2, 2))])
    model = mf.MPCModel(A, Bm, C, 2 * np.eye(4), np.eye(2), T, (np.full(2, -5.0), np.full(2, 5.0)),
                        (np.full(2, -10.0), np.full(2, 10.0)), device=dev)
    x0, xr, uf, _ = bench._mpc_problem_inputs(ego, T, 1, dev)
    ws = torch.empty(model.workspace_doubles(1, O), dtype=torch.float64, device=dev)
    main_s = torch.cuda.current_stream(dev)
    reserve = int(os.environ.get("RESERVE_CUS", "16"))
    allow = int(os.environ.get("ALLOW_CUS", "0"))
    hs_s = (cu_allowed_stream(dev, allow) if allow else
            torch.cuda.Stream(dev) if reserve == 0 else cu_masked_stream(dev, reserve))
    qp_s = torch.cuda.Stream(dev, priority=-1)
    recs = [torch.empty((O, T, 8), dtype=torch.float64, device=dev) for _ in range(2)]
    seq_launch = engine.prepare_safe_halfspaces(samples, ego, params, out=recs[0], stream=main_s)[0]
    pipe_launch = [engine.prepare_safe_halfspaces(samples, ego, params, out=recs[b], stream=hs_s)[0] for b in range(2)]
    views = [mf.record_views(recs[b], "dr_cvar") for b in range(2)]
    res = {}

    def sequential(k):
        for _ in range(k):
            seq_launch()
            res["seq"] = mf.filter_batch(model, *views[0], x0, xr, uf, workspace=ws, stream=main_s)

    ev_hs = [torch.cuda.Event() for _ in range(2)]
    ev_qp = [torch.cuda.Event() for _ in range(2)]

    def pipelined(k):
        hs_s.wait_stream(main_s)
        qp_s.wait_stream(main_s)
        pipe_launch[0]()
        ev_hs[0].record(hs_s)
        for i in range(k):
            b, nb = i % 2, 1 - i % 2
            qp_s.wait_event(ev_hs[b])
            with torch.cuda.stream(qp_s):
                res["pipe"] = mf.filter_batch(model, *views[b], x0, xr, uf, workspace=ws, stream=qp_s)
            ev_qp[b].record(qp_s)
            if i + 1 < k:
                if i >= 1:
                    hs_s.wait_event(ev_qp[nb])   # records nb were read by the QP of step i - 1
                pipe_launch[nb]()
                ev_hs[nb].record(hs_s)
        main_s.wait_stream(qp_s)
        main_s.wait_stream(hs_s)

    def region(fn, k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(k)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e3

    sequential(2)
    pipelined(2)
    out = {}
    for k in (5, 20):
        for rep in range(5):
            out.setdefault(f"sequential K={k}", []).append(region(sequential, k))
            out.setdefault(f"pipelined K={k}", []).append(region(pipelined, k))
    torch.cuda.synchronize()
    for key, v in out.items():
        print(f"{key:20s} ms/step median {sorted(v)[len(v) // 2]:.4f}  all {[round(x, 4) for x in v]}")
    u_seq, u_pipe = res["seq"][1].cpu().numpy(), res["pipe"][1].cpu().numpy()
    i_seq, i_pipe = res["seq"][2].cpu().numpy(), res["pipe"][2].cpu().numpy()
    print("QP status seq/pipe", mf.STATUS_NAMES.get(int(i_seq[0, 0])), mf.STATUS_NAMES.get(int(i_pipe[0, 0])),
          "iterations", int(i_seq[0, 1]), int(i_pipe[0, 1]),
          "u bitwise equal", bool(np.array_equal(u_seq, u_pipe)), "max|du|", float(np.abs(u_seq - u_pipe).max()))
    del hs_s, pipe_launch, res
    destroy_streams()
    print("streams destroyed", flush=True)


if __name__ == "__main__":
    main()

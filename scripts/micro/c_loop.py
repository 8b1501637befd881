#!/usr/bin/env python3
"""K = 20 and K = 2000 timed regions of the C3 batch issued three ways: one hipGraph of K nodes
(bench.py today, replays of <= 50), K eager ctypes calls from Python, and K ABI calls from a native
loop (scripts/micro/c_loop.so).  Wall and HIP-event time per step, medians of 9 regions, each after
the bench's 5 warm-up steps."""
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import engine, synthetic  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.engine import RiskParams  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    s, e = synthetic.obstacle_batch(10, 20, 1000, dev, seed=1)
    p = RiskParams()
    launch, out = engine.prepare_safe_halfspaces(s, e, p, stream=stream)
    lib = ctypes.CDLL(os.path.join(REPO, "scripts", "micro", "c_loop.so"))
    lib.c_loop.restype = ctypes.c_int
    i64, dbl, vp = ctypes.c_int64, ctypes.c_double, ctypes.c_void_p
    cargs = (vp(s.data_ptr()), i64(10), i64(20), i64(1000), i64(s.stride(0)), i64(s.stride(1)),
             i64(s.stride(2)), vp(e.data_ptr()), i64(e.stride(0)), dbl(p.robot_radius),
             dbl(p.obstacle_radius), dbl(p.alpha), dbl(p.delta), dbl(p.epsilon), vp(out.data_ptr()),
             vp(stream.cuda_stream))
    graphs = {}
    for n in (5, 20, 50):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=torch.cuda.Stream(dev)):
            lg, _ = engine.prepare_safe_halfspaces(s, e, p, out=out, stream=torch.cuda.current_stream(dev))
            for _ in range(n):
                lg()
        g.replay()
        graphs[n] = (g, lg)
    torch.cuda.synchronize()
    ref = out.clone()

    def issue(mode, k):
        if mode == "graph":
            for _ in range(k // 50):
                graphs[50][0].replay()
            if k % 50:
                graphs[k % 50][0].replay()
        elif mode == "eager":
            for _ in range(k):
                launch()
        else:
            assert lib.c_loop(ctypes.c_int(k), *cargs) == 0

    def region(mode, k, warm):
        issue(warm, 5)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e1.record(stream)
        e0.record(stream)
        t0 = time.perf_counter()
        issue(mode, k)
        e1.record(stream)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e6, e0.elapsed_time(e1) * 1e3 / k

    res = {}
    for k in (20, 2000):
        for rep in range(9):
            for mode in ("graph", "eager", "cloop"):
                for warm in ("graph", "same"):
                    key = f"K={k} {mode} warm={warm}"
                    res.setdefault(key, []).append(region(mode, k, mode if warm == "same" else "graph"))
    assert torch.equal(out, ref)
    summary = {k: {"wall_us": round(sorted(r[0] for r in v)[4], 3),
                   "event_us": round(sorted(r[1] for r in v)[4], 3)} for k, v in res.items()}
    for k, v in summary.items():
        print(f"{k:34s} wall {v['wall_us']:7.3f} us/step   events {v['event_us']:7.3f}")
    print(json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()

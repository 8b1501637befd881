#!/usr/bin/env python3
"""Benchmark: halfspace-constraints/sec of the DR-CVaR safe-halfspace engine (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2|c4|c5]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step = one evaluation of the hot path over one batch: every (obstacle, horizon-step) unit of a
synthetic [O, T, N, 2] fp64 sample tensor -> mean / CVaR / DR-CVaR halfspaces, i.e. ONE launch
of the fused kernel through the C ABI.  Default workload c3 = BASELINE.json's metric config
(10 obstacles, T = 20, N = 1000).  Inputs are generated on the device and resident in HBM before
timing starts.  A c3 launch is ~6 us, so by default the K steps are issued as replays of a
hipGraph that holds `--graph-batch` consecutive launches (every replayed launch recomputes the
whole batch; `--launch eager` issues one ctypes call per step instead).

Multi-GPU: one process per GPU; every rank evaluates its own batch (weak scaling, no data-path
collective); with --gather each step also all-gathers the [U, 8] records over RCCL (the QP
hand-off exchange).

Prints ONE JSON line on rank 0: value = units of all ranks / max rank time, plus
  roofline        the kernel on this workload: algorithmic bytes per launch / (HIP-event time over
                  the timed region / K) — includes the ~1 us inter-launch gap, so a lower bound
  roofline_large  the same kernel on a 2 GB resident batch (256 x 50 x 10 000), event-timed
  cpu_baseline    oracle/drcvar_oracle.c (1 thread) on whole batches of the same workload
  max_abs_err     max |offset - oracle| over the benchmarked batch (the metric's second half)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import engine, synthetic  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.engine import RiskParams  # noqa: E402

WORKLOADS = {
    # name: (obstacles, steps, samples, description)
    "c2": (4, 20, 1000, "multi_obstacle-like synthetic, 4 obstacles, T=20, N=1000 (BASELINE config 2)"),
    "c3": (10, 20, 1000, "multi_obstacle-like synthetic, 10 obstacles, T=20, N=1000 (BASELINE config 3, the metric's config)"),
    "c4": (64, 30, 5000, "synthetic 64 obstacles, T=30, N=5000 (BASELINE config 4, per GPU)"),
    "c5": (256, 50, 10000, "synthetic 256 obstacles, T=50, N=10000 (BASELINE config 5, per GPU)"),
}
LARGE = (256, 50, 10000)
HBM_PEAK = 8.0e12  # B/s, MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
OUT_BYTES = 64     # 8 fp64 per unit


def algorithmic_bytes(O, T, N):
    """Bytes one launch must move: every sample once (16 B), the 64-B record, ego per step."""
    return O * T * (16 * N + OUT_BYTES) + T * 16


def load_traffic(workload):
    """HBM bytes per launch from the committed PMC profile (profiles/pmc_traffic.json), if any."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(workload, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def roofline(abytes, kernel_s, traffic):
    achieved = abytes / kernel_s
    return {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": achieved / HBM_PEAK, "traffic": traffic, "kernel_ms": kernel_s * 1e3,
            "algorithmic_bytes_per_launch": abytes}


def cpu_baseline(samples, ego, params, budget_s):
    """C oracle (1 thread) on whole batches of the same workload until ~budget_s of CPU work."""
    from oracle import c_oracle
    s = samples.cpu().numpy()
    e = ego.cpu().numpy()
    args = (params.robot_radius, params.obstacle_radius, params.alpha, params.delta, params.epsilon)
    ref = c_oracle.safe_halfspaces(s, e, *args, nthreads=1)  # warm + parity reference
    units = s.shape[0] * s.shape[1]
    reps, t0 = 0, time.perf_counter()
    while True:
        c_oracle.safe_halfspaces(s, e, *args, nthreads=1)
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    base = {"value": reps * units / el, "unit": "halfspace-constraints/s", "cores": 1, "kind": "port",
            "sample": f"{reps} full batches x {units} units of the same workload "
                      f"({el:.1f} s, oracle/drcvar_oracle.c quickselect, 1 thread)"}
    # the same port on every core of this process's CPU share (the GPU box shows
    # the whole machine in os.cpu_count(); one GPU's share is 16 threads)
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    reps, t0 = 0, time.perf_counter()
    while True:
        c_oracle.safe_halfspaces(s, e, *args, nthreads=threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s / 3:
            break
    base["all_cores"] = {"value": reps * units / el, "cores": threads,
                         "sample": f"{reps} full batches ({el:.1f} s), units split over {threads} threads"}
    # §8d(ii): the reference's algorithm class -- the two LPs per unit (core/risk_metrics.py
    # :87-125, :182-213) through scipy's HiGHS (oracle/lp_highs.py), one core, a few units
    from oracle import lp_highs
    flat_s, flat_h = s.reshape(units, s.shape[2], 2), ref.reshape(units, -1)[:, 3:5]
    done, t0 = 0, time.perf_counter()
    while done < units:
        lp_highs.solve_cvar_lp(flat_s[done], flat_h[done], params.alpha, params.delta,
                               params.robot_radius, params.obstacle_radius)
        lp_highs.solve_dr_cvar_lp(flat_s[done], flat_h[done], params.alpha, params.delta,
                                  params.epsilon, params.robot_radius, params.obstacle_radius)
        done += 1
        el = time.perf_counter() - t0
        if el >= budget_s / 3:
            break
    base["lp_highs"] = {"value": done / el, "cores": 1,
                        "sample": f"{done} units x 2 LPs ({el:.1f} s, scipy HiGHS, oracle/lp_highs.py)"}
    return ref, base


class Stepper:
    """Issues steps: eager ctypes launches, or replays of a hipGraph holding G launches."""

    def __init__(self, samples, ego, params, mode, graph_batch, dev):
        self.mode = mode
        self.G = graph_batch if mode == "graph" else 1
        self.launch, self.out = engine.prepare_safe_halfspaces(samples, ego, params)
        if mode == "graph":
            self.launch()  # warm the code object before capture
            torch.cuda.synchronize(dev)
            self.graph = torch.cuda.CUDAGraph()
            cap_stream = torch.cuda.Stream(dev)
            with torch.cuda.graph(self.graph, stream=cap_stream):
                # the frozen call must target the capturing stream
                cap, _ = engine.prepare_safe_halfspaces(samples, ego, params, out=self.out,
                                                        stream=torch.cuda.current_stream(dev))
                for _ in range(self.G):
                    cap()
            self._keep = cap

    def run(self, steps):
        """Issue `steps` steps (rounded up to whole graph replays); returns steps issued."""
        if self.mode == "graph":
            reps = -(-steps // self.G)
            for _ in range(reps):
                self.graph.replay()
            return reps * self.G
        for _ in range(steps):
            self.launch()
        return steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--launch", default="graph", choices=["graph", "eager"])
    ap.add_argument("--graph-batch", type=int, default=50)
    ap.add_argument("--gather", action="store_true", help="all-gather records each step (RCCL)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-large", action="store_true", help="skip the 2 GB roofline measurement")
    ap.add_argument("--no-mpc", action="store_true", help="skip the MPC hand-off measurement")
    ap.add_argument("--full-loop", action="store_true",
                    help="BASELINE config 5's full MPC loop: the GLOBAL batch sharded over ranks, "
                         "records all-gathered, the DR-CVaR QP solved on every rank (strong scaling)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse the N>1 path (several ranks may share one GPU)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    ndev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and local_rank >= ndev:
        raise SystemExit(f"LOCAL_RANK {local_rank} but only {ndev} GPUs visible")
    dev = torch.device("cuda", local_rank % ndev)
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    if args.full_loop:
        return full_loop(args, world, rank, dev)
    O, T, N, desc = WORKLOADS[args.workload]
    params = RiskParams()  # config/parameters.py: alpha 0.2, delta 0.1, eps 0.15, radii 0.3/0.3
    samples, ego = synthetic.obstacle_batch(O, T, N, dev, seed=42 + rank)
    U = O * T
    mode = "eager" if (args.gather and world > 1) else args.launch  # collectives stay eager
    stepper = Stepper(samples, ego, params, mode, args.graph_batch, dev)
    out = stepper.out
    gathered = None
    if args.gather and world > 1:
        gdev = dev if args.dist_backend == "nccl" else torch.device("cpu")
        gathered = torch.empty((U * world, engine.OUT_WIDTH), dtype=torch.float64, device=gdev)

    def steps(k):
        if gathered is None:
            return stepper.run(k)
        for _ in range(k):
            stepper.launch()
            rec = out.view(U, engine.OUT_WIDTH)
            dist.all_gather_into_tensor(gathered, rec if gathered.is_cuda else rec.cpu())
        return k

    steps(args.warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    K = steps(args.steps)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kernel_s = ev0.elapsed_time(ev1) * 1e-3 / K

    red_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    t_max = torch.tensor([elapsed, kernel_s], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    elapsed, kernel_s = float(t_max[0].item()), float(t_max[1].item())

    large = mpc = sampling = None
    if rank == 0 and not args.no_large:
        Ol, Tl, Nl = LARGE
        s_l, e_l = synthetic.obstacle_batch(Ol, Tl, Nl, dev, seed=7)
        launch_l, _ = engine.prepare_safe_halfspaces(s_l, e_l, params)
        for _ in range(3):
            launch_l()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        a.record(stream)
        for _ in range(reps):
            launch_l()
        b.record(stream)
        torch.cuda.synchronize()
        large = roofline(algorithmic_bytes(Ol, Tl, Nl), a.elapsed_time(b) * 1e-3 / reps,
                         load_traffic("c5"))
        large["workload"] = f"{Ol} obstacles x {Tl} steps x {Nl} samples (2.05 GB resident)"
        large["halfspaces_per_s"] = Ol * Tl / (large["kernel_ms"] * 1e-3)
        sampling = sampler_roofline(s_l, stream)
        if not args.no_mpc:
            mpc = mpc_handoff(dev, s_l, e_l, params, with_cpu=world == 1 and not args.no_cpu_baseline)
        del s_l, e_l
        torch.cuda.empty_cache()

    result = None
    if rank == 0:
        value = U * world * K / elapsed
        result = {
            "metric": "halfspace-constraints/sec (N=1000, 10 obs, T=20) + max |offset - ref|",
            "value": value,
            "unit": "halfspace-constraints/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (device-generated obstacle samples, SURVEY.md §8d distributions)",
            "config": {"workload": f"{args.workload}: {desc}", "obstacles": O, "steps": T,
                       "samples": N, "units_per_gpu": U, "global_units_per_step": U * world,
                       "parallelism": f"dp{world}" + ("+allgather" if gathered is not None else ""),
                       "launch": (f"hipGraph replays of {stepper.G} launches" if mode == "graph"
                                  else "eager ctypes launch per step"),
                       "alpha": params.alpha, "delta": params.delta, "epsilon": params.epsilon},
            "roofline": roofline(algorithmic_bytes(O, T, N), kernel_s, load_traffic(args.workload)),
            "roofline_large": large,
            "mpc_handoff": mpc,
            "sampling": sampling,
        }
        if world == 1 and not args.no_cpu_baseline:
            import numpy as np
            ref, base = cpu_baseline(samples, ego, params, args.cpu_seconds)
            got = out.cpu().numpy()
            result["max_abs_err"] = float(np.max(np.abs(got[..., [2, 5, 6, 7]] - ref[..., [2, 5, 6, 7]])))
            result["max_abs_err_h"] = float(np.max(np.abs(got[..., [0, 1, 3, 4]] - ref[..., [0, 1, 3, 4]])))
            base["host_cpu"] = _cpu_model()
            base["host_threads_visible"] = os.cpu_count()
            result["cpu_baseline"] = base
        else:
            result["cpu_baseline"] = None
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


def full_loop(args, world, rank, dev):
    """One step = this rank's contiguous block of the global (obstacle x step) units through the
    halfspace kernel -> all_gather_into_tensor of the 64-B records (RCCL) -> the DR-CVaR safety
    filter QP over all O*T halfspaces (H = T) on every rank.  value = global units / max rank time.
    """
    import numpy as np
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import sharding
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf
    O, T, N, desc = WORKLOADS[args.workload]
    params = RiskParams()
    samples, ego = synthetic.obstacle_batch(O, T, N, dev, seed=42)       # same global batch on all ranks
    U = O * T
    s_u, e_u, start, stop = sharding.shard_units(samples, ego, world, rank)
    local = torch.empty((max(stop - start, 0), engine.OUT_WIDTH), dtype=torch.float64, device=dev)
    launch = None
    if stop > start:
        launch, local = engine.prepare_safe_halfspaces(s_u.unsqueeze(0), e_u, params,
                                                       out=local.view(1, stop - start, engine.OUT_WIDTH))
        local = local.view(stop - start, engine.OUT_WIDTH)
    per = -(-U // world)
    padded = torch.zeros((per, engine.OUT_WIDTH), dtype=torch.float64, device=dev)
    gdev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    full = torch.empty((per * world, engine.OUT_WIDTH), dtype=torch.float64, device=gdev)
    dt = 0.2
    A = np.block([[np.eye(2), dt * np.eye(2)], [np.zeros((2, 2)), np.eye(2)]])
    Bm = np.block([[0.5 * dt ** 2 * np.eye(2)], [dt * np.eye(2)]])
    C = np.block([np.eye(2), np.zeros((2, 2))])
    model = mf.MPCModel(A, Bm, C, 2 * np.eye(4), np.eye(2), T, (np.full(2, -5.0), np.full(2, 5.0)),
                        (np.full(2, -10.0), np.full(2, 10.0)), device=dev)
    x0, xr, uf, _ = _mpc_problem_inputs(ego, T, 1, dev)
    ws = torch.empty(model.workspace_doubles(1, O), dtype=torch.float64, device=dev)
    rec_dev = torch.empty((U, engine.OUT_WIDTH), dtype=torch.float64, device=dev)
    res = {}

    def step():
        if launch is not None:
            launch()
        if world > 1:
            padded[: stop - start] = local
            dist.all_gather_into_tensor(full, padded if full.is_cuda else padded.cpu())
            rec_dev.copy_(full[:U], non_blocking=True)
            rec = rec_dev
        else:
            rec = local
        h, g = mf.record_views(rec.view(O, T, engine.OUT_WIDTH), "dr_cvar")
        res["u"], res["info"] = mf.filter_batch(model, h, g, x0, xr, uf, workspace=ws)[1:]

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    red_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    t_max = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    elapsed = float(t_max[0].item())
    result = None
    if rank == 0:
        info = res["info"][0].cpu().numpy()
        result = {
            "metric": "full MPC loop halfspace-constraints/sec (BASELINE config 5: halfspaces + "
                      "all-gather + QP hand-off)",
            "value": U * args.steps / elapsed, "unit": "halfspace-constraints/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (device-sampled obstacle batch, identical on every rank)",
            "config": {"workload": f"{args.workload}: {desc}", "units": U,
                       "parallelism": f"units sharded dp{world} + allgather + replicated QP",
                       "qp": f"dr_cvar safety filter, H={T}, {U} halfspace rows"},
            "qp_status": int(info[0]), "qp_iterations": int(info[1]),
            "roofline": None, "cpu_baseline": None,
        }
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


def sampler_roofline(out, stream, reps=10):
    """Device sample generator (drcvar_sample_trajectories_f64) refilling a resident batch: bytes
    written (16 per sample) per launch / event time -- an HBM-write-bound kernel."""
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.simulation import obstacles
    O, T, N, _ = out.shape
    nominal = out[:, :, 0, :].clone()                    # any [O, T, 2] nominal path
    launch = lambda: obstacles.sample_trajectories_device(nominal, N, seed=11, out=out)
    launch()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(reps):
        launch()
    b.record(stream)
    torch.cuda.synchronize()
    sec = a.elapsed_time(b) * 1e-3 / reps
    written = O * T * N * 16
    return {"workload": f"{O}x{T}x{N} samples (Philox4x32-10 + Box-Muller, fp64)", "kernel_ms": sec * 1e3,
            "samples_per_s": O * T * N / sec, "bound": "hbm", "achieved": written / sec / 1e9,
            "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": written / sec / HBM_PEAK}


def _mpc_problem_inputs(ego, H, B, dev):
    """x0 / x_ref / fallback inputs of B problems following the ego straight line (main.py:74-89)."""
    import numpy as np
    e = ego.cpu().numpy()
    xr = np.zeros((H + 1, 4))
    xr[:min(H, len(e)), :2] = e[:H]
    xr[min(H, len(e)):, :2] = e[min(H, len(e)) - 1]
    xr[:-1, 2:] = (xr[1:, :2] - xr[:-1, :2]) / 0.2
    T = lambda a: torch.as_tensor(np.ascontiguousarray(a)).to(dev)
    return (T(np.repeat(xr[None, 0], B, 0)), T(np.repeat(xr[None], B, 0)),
            T(np.zeros((B, H, 2))), xr)


def mpc_handoff(dev, samples, ego, params, with_cpu):
    """The QP hand-off (core/mpc_filter.py:40-178) measured two ways.

    full_loop_c5: BASELINE config 5's "full MPC loop with QP handoff" on one GPU — the halfspace
      kernel over the resident [256, 50, 10000] batch, then the DR-CVaR safety-filter QP over its
      12 800 halfspaces (H = 50), both on the device, timed together with HIP events.
    batched_reference: main.py's QP (multi_obstacle: 3 obstacles, H = 30, input bounds +-5,
      position bounds +-10) for 1024 independent problems in one launch -> QPs/s; CPU baseline =
      oracle/mpc_qp.py (sparse IPM + polish, 1 thread) on the same problem.
    """
    import numpy as np
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import _native
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf
    dt = 0.2
    A = np.block([[np.eye(2), dt * np.eye(2)], [np.zeros((2, 2)), np.eye(2)]])
    Bm = np.block([[0.5 * dt ** 2 * np.eye(2)], [dt * np.eye(2)]])
    C = np.block([np.eye(2), np.zeros((2, 2))])
    Q, R = 2 * np.eye(4), np.eye(2)
    ub = (np.full(2, -5.0), np.full(2, 5.0))
    pb = (np.full(2, -10.0), np.full(2, 10.0))
    stream = torch.cuda.current_stream(dev)

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(reps):
            fn()
        b.record(stream)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    out = {}
    # ---- C5 full loop ----
    O, T = samples.shape[0], samples.shape[1]
    H = T
    model = mf.MPCModel(A, Bm, C, Q, R, H, ub, pb, device=dev)
    x0, xr, uf, xr_host = _mpc_problem_inputs(ego, H, 1, dev)
    launch, rec = engine.prepare_safe_halfspaces(samples, ego, params)
    h, g = mf.record_views(rec, "dr_cvar")
    ws = torch.empty(model.workspace_doubles(1, O), dtype=torch.float64, device=dev)
    res = {}

    def qp():
        res["x"], res["u"], res["info"] = mf.filter_batch(model, h, g, x0, xr, uf, workspace=ws)

    def full():
        launch()
        qp()

    full_ms = timed(full, 5)
    qp_ms = timed(qp, 5)
    info = res["info"][0].cpu().numpy()
    c5 = {"workload": f"{O} obstacles x {T} steps x {samples.shape[2]} samples -> dr_cvar QP "
                      f"(H={H}, {O * T} halfspace rows), 1 problem",
          "full_step_ms": full_ms, "qp_ms": qp_ms, "halfspace_ms": full_ms - qp_ms,
          "halfspace_constraints_per_s_full_loop": O * T / (full_ms * 1e-3),
          "qp_status": mf.STATUS_NAMES.get(int(info[_native.MPC_INFO_STATUS])),
          "qp_iterations": int(info[_native.MPC_INFO_ITERATIONS]),
          "polished": bool(info[_native.MPC_INFO_POLISHED])}
    if with_cpu:
        from oracle import mpc_qp
        r = rec.cpu().numpy()
        hs = np.concatenate([r[..., 3:5], r[..., 7:8]], -1)
        t0 = time.perf_counter()
        xo, uo, io = mpc_qp.filter_trajectory(A, Bm, C, Q, R, H, xr_host[0], xr_host, None,
                                              [hs[:, t] for t in range(T)], ub, pb)
        c5["cpu_oracle_qp_s"] = time.perf_counter() - t0
        c5["max_abs_err_u_vs_oracle"] = float(np.abs(res["u"][0].cpu().numpy() - uo).max())
    out["full_loop_c5"] = c5
    del ws, rec
    # ---- batched reference configuration ----
    Hr, Or, Bn = 30, 3, 1024
    model_r = mf.MPCModel(A, Bm, C, Q, R, Hr, ub, pb, device=dev)
    s_r, e_r = synthetic.obstacle_batch(Or, Hr, 20, dev, seed=3)       # NUM_SAMPLES = 20
    rec_r = engine.safe_halfspaces(s_r, e_r, params)
    hb = rec_r[None, :, :, 3:5].expand(Bn, Or, Hr, 2)
    gb = rec_r[None, :, :, 7].expand(Bn, Or, Hr)
    x0r, xrr, ufr, xr_host_r = _mpc_problem_inputs(e_r, Hr, Bn, dev)
    wsr = torch.empty(model_r.workspace_doubles(Bn, Or), dtype=torch.float64, device=dev)

    def qp_batch():
        res["u"], res["info"] = mf.filter_batch(model_r, hb, gb, x0r, xrr, ufr, workspace=wsr)[1:]

    ms = timed(qp_batch, 5)
    inf = res["info"].cpu().numpy()
    br = {"workload": f"main.py QP (H={Hr}, {Or} obstacles, bounds), {Bn} problems per launch",
          "launch_ms": ms, "qps_per_s": Bn / (ms * 1e-3),
          "optimal_frac": float((inf[:, _native.MPC_INFO_STATUS] == 0).mean()),
          "mean_iterations": float(inf[:, _native.MPC_INFO_ITERATIONS].mean())}
    if with_cpu:
        from oracle import mpc_qp
        r = rec_r.cpu().numpy()
        hs = np.concatenate([r[..., 3:5], r[..., 7:8]], -1)
        reps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 3.0:
            xo, uo, io = mpc_qp.filter_trajectory(A, Bm, C, Q, R, Hr, xr_host_r[0], xr_host_r, None,
                                                  [hs[:, t] for t in range(Hr)], ub, pb)
            reps += 1
        el = time.perf_counter() - t0
        br["cpu_baseline"] = {"value": reps / el, "unit": "QPs/s", "cores": 1, "kind": "port",
                              "sample": f"{reps} solves of problem 0 by oracle/mpc_qp.py ({el:.1f} s)"}
        br["max_abs_err_u_vs_oracle"] = float(np.abs(res["u"][0].cpu().numpy() - uo).max())
    out["batched_reference"] = br
    out["bound"] = ("latency: one workgroup per problem runs the whole interior-point solve "
                    "(Riccati factorisation + solves on one wave, and at C5 the row passes over "
                    "12 800 halfspaces, dominate; see DESIGN.md)")
    return out


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


if __name__ == "__main__":
    main()

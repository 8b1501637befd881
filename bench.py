#!/usr/bin/env python3
"""Benchmark: halfspace-constraints/sec of the DR-CVaR safe-halfspace engine (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2|c4|c5]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step = one evaluation of the hot path over one batch: every (obstacle, horizon-step) unit of a
synthetic [O, T, N, 2] fp64 sample tensor -> mean / CVaR / DR-CVaR halfspaces (one fused kernel
launch).  Default workload c3 = BASELINE.json's metric config (10 obstacles, T = 20, N = 1000).
Inputs are generated on the device and resident in HBM before timing starts.  Multi-GPU: one
process per GPU, every rank evaluates its own batch (weak scaling, no data-path collective); with
--gather each step also all-gathers the [U, 8] records over RCCL (the QP hand-off exchange).

Prints ONE JSON line on rank 0 (contract in the task statement): value = units of all ranks / max
rank time, plus `roofline` (dominant kernel, HIP events on its stream), `cpu_baseline` (the C
oracle, 1 thread, on a bounded sample of the same batch) and `max_abs_err` vs that oracle.
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
HBM_PEAK = 8.0e12  # B/s, MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
OUT_BYTES = 64     # 8 fp64 per unit


def algorithmic_bytes(O, T, N):
    """Bytes one launch must move: samples once (16 B each), the 64-B record, ego per step."""
    return O * T * (16 * N + OUT_BYTES) + T * 16


def load_traffic(workload):
    """HBM bytes per launch from the committed PMC profile (profiles/pmc_traffic.json), if any."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(workload, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


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
    return ref, {"value": reps * units / el, "unit": "halfspace-constraints/s", "cores": 1,
                 "kind": "port",
                 "sample": f"{reps} full batches x {units} units of the same workload "
                           f"({el:.1f} s, oracle/drcvar_oracle.c quickselect, 1 thread)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--gather", action="store_true", help="all-gather records each step (RCCL)")
    ap.add_argument("--no-events", action="store_true", help="skip per-step HIP events")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    O, T, N, desc = WORKLOADS[args.workload]
    params = RiskParams()  # config/parameters.py: alpha 0.2, delta 0.1, eps 0.15, radii 0.3/0.3
    samples, ego = synthetic.obstacle_batch(O, T, N, dev, seed=42 + rank)
    stream = torch.cuda.current_stream(dev)
    launch, out = engine.prepare_safe_halfspaces(samples, ego, params, stream=stream)
    U = O * T
    gathered = None
    if args.gather and world > 1:
        gathered = torch.empty((U * world, engine.OUT_WIDTH), dtype=torch.float64, device=dev)

    def step():
        launch()
        if gathered is not None:
            dist.all_gather_into_tensor(gathered, out.view(U, engine.OUT_WIDTH))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    K = args.steps
    use_events = not args.no_events
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(K)] if use_events else []
    t0 = time.perf_counter()
    if use_events:
        for k in range(K):
            ev[k][0].record(stream)
            launch()
            ev[k][1].record(stream)
            if gathered is not None:
                dist.all_gather_into_tensor(gathered, out.view(U, engine.OUT_WIDTH))
    else:
        for _ in range(K):
            step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    kernel_ms = None
    if use_events:
        durs = [a.elapsed_time(b) for a, b in ev]
        kernel_ms = sum(durs) / len(durs)
    t_max = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    k_max = torch.tensor([kernel_ms or 0.0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        dist.all_reduce(k_max, op=dist.ReduceOp.MAX)
    elapsed = float(t_max.item())

    result = None
    if rank == 0:
        value = U * world * K / elapsed
        abytes = algorithmic_bytes(O, T, N)
        roofline = None
        if use_events:
            kms = float(k_max.item())
            achieved = abytes / (kms * 1e-3)
            traffic = load_traffic(args.workload)
            roofline = {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9,
                        "unit": "GB/s", "frac": achieved / HBM_PEAK, "traffic": traffic,
                        "kernel_ms": kms, "algorithmic_bytes_per_launch": abytes}
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
                       "alpha": params.alpha, "delta": params.delta, "epsilon": params.epsilon},
            "roofline": roofline,
        }
        if world == 1 and not args.no_cpu_baseline:
            ref, base = cpu_baseline(samples, ego, params, args.cpu_seconds)
            import numpy as np
            got = out.cpu().numpy()
            cols = [2, 5, 6, 7]
            result["max_abs_err"] = float(np.max(np.abs(got[..., cols] - ref[..., cols])))
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

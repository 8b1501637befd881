#!/usr/bin/env python3
"""Benchmark: halfspace-constraints/sec of the DR-CVaR safe-halfspace engine (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2|c4|c5]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step = one evaluation of the hot path over one batch: every (obstacle, horizon-step) unit of a
synthetic [O, T, N, 2] fp64 sample tensor -> mean / CVaR / DR-CVaR halfspaces, i.e. ONE launch
of the fused kernel through the C ABI.  Default workload c3 = BASELINE.json's metric config
(10 obstacles, T = 20, N = 1000).  Inputs are drawn on the device and resident in HBM before
timing starts.  Exactly K steps are timed: by default as replays of a hipGraph of
G = min(--graph-batch, K) steps plus one graph of the remainder (`--launch eager`: one ctypes
call per step).

Multi-GPU (one process per GPU): the metric line keeps BASELINE's C3 config per GPU — the global
batch has O*N_gpus obstacles, rank r draws only its own C3-sized block (units [r*O*T,
(r+1)*O*T)) with the device sampler and a step is its launch; units are independent
(core/halfspaces.py:225-246), so there is no collective in the step: WEAK scaling, identical
per-GPU work at every N, labelled so in `scaling` / `metric_form`.  The north-star form is the
`strong_scaling` key, at every N, one leg per BASELINE config with a sharded batch: c4 (64 x 30 x
5 000, 154 MB) and c5 (256 x 50 x 10 000, 2.05 GB) — ONE global batch sharded over the ranks, a
step = the shard's launch + an RCCL all_gather_into_tensor of the 64-B records to every rank (the
exchange the QP hand-off needs, core/mpc_filter.py:116-151).  Each leg also reports its phases
alone, max over ranks (`phases_rank_max`: kernel_ms, allgather_ms), so a scaling curve can be
read; c5 adds the full loop with the QP.

Prints ONE JSON line on rank 0: value = units of all ranks / max rank time, plus
  roofline        the kernel on this workload: algorithmic bytes per launch / average launch time
                  (N=1: HIP events over the timed region / K, launch gaps included)
  strong_scaling  {c4, c5}: global batch sharded over N ranks (+ all-gather), phase splits
  roofline_large  (N=1) the kernel on the resident 2 GB C5 batch, graph-replayed, event-timed
  roofline_c3_replicated  (N=1) the C3 launch plan over C3 replicated to a 2 GB working set
                  (BASELINE.md §3's roofline convention for the cache-resident configs)
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

from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import engine, sharding, synthetic  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.engine import RiskParams  # noqa: E402

# chunk counts of the pipelined RCCL step per strong-scaling workload (--chunks auto): C4's
# all-gather is latency-bound (~123 KB), two chunks at most; C5's shard kernel is long enough
# (~40 us at 8 ranks) to hide a chunk's gather behind the next chunk's kernel
CHUNKS = {"c2": [2], "c3": [2], "c4": [2], "c5": [2, 4]}
# bound of one peer-exchange wait in the strong legs: a step waits at most for a slower rank's
# kernel (~0.3 ms at C5 on one GPU); a wait that gives up sets the error word and the form is dropped
PEER_SPIN_US = 200_000
WORKLOADS = {
    # name: (obstacles, steps, samples, description)
    "c2": (4, 20, 1000, "multi_obstacle-like synthetic, 4 obstacles, T=20, N=1000 (BASELINE config 2)"),
    "c3": (10, 20, 1000, "multi_obstacle-like synthetic, 10 obstacles, T=20, N=1000 (BASELINE config 3, the metric's config)"),
    "c4": (64, 30, 5000, "synthetic 64 obstacles, T=30, N=5000 (BASELINE config 4, per GPU)"),
    "c5": (256, 50, 10000, "synthetic 256 obstacles, T=50, N=10000 (BASELINE config 5, per GPU)"),
}
HBM_PEAK = 8.0e12  # B/s, MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
OUT_BYTES = 64     # 8 fp64 per unit
# what bounds the sampler (profiles/r02/sampler_pmc.json: VALU busy 1.02 of the SIMD cycles, 190 VALU
# instructions per sample): its per-sample fp64/integer work, not the 16-B store -- its "frac" is
# the HBM-write fraction it reaches all the same
SAMPLER_BOUND = "valu"


def load_traffic(workload):
    """HBM bytes per launch from the committed PMC profile (profiles/pmc_traffic.json), if any."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(workload, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def kernel_evidence(workload, abytes, command):
    """The metric kernel's time from committed profiles of bench.py's own command
    (profiles/kernel_time.json, scripts/kernel_time.py): `busy` from a GRBM counter pass (the time the
    GPU was busy in each dispatch window) and `trace` (the kernel-trace windows, which the profiler
    stretches).  Returned as (entry, None) only while the halfspace kernel's sources still match the
    profiled ones and the command is the profiled one; otherwise (None, why) — a stale profile is
    never reported as this build's timing."""
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import _native
    path = os.path.join(REPO, "profiles", "kernel_time.json")
    try:
        with open(path) as f:
            e = json.load(f).get(workload)
    except (OSError, ValueError):
        return None, "no profiles/kernel_time.json"
    if not e:
        return None, f"no profile of workload {workload}"
    if e.get("source_key") != _native.source_key():
        return None, "profiled kernel sources differ from this build (historical profile not used)"
    if e.get("command") != command:
        return None, f"profiled command {e.get('command')!r} is not this command {command!r}"
    out = {"kernel": e["kernel"], "command": e["command"]}
    for k in ("busy", "trace"):
        ns = e[k]["mean_ns"]
        out[k] = dict(e[k], kernel_ms=ns * 1e-6, achieved=abytes / (ns * 1e-9) / 1e9,
                      frac=abytes / (ns * 1e-9) / HBM_PEAK)
    return out, None


def roofline_line(abytes, kernel_s, ktiming, traffic, args, step_s):
    """The metric line's roofline block.  achieved / frac follow from the committed profile of this
    very command and kernel build when there is one (its `busy` time: a counter pass, no larger than
    the step the driver times); otherwise from the HIP events of this run.  Both, and the profiler's
    stretched trace time, are reported beside each other."""
    command = f"python3 bench.py --gpus {args.gpus} --steps {args.steps} --warmup {args.warmup}"
    if args.workload != "c3" or args.launch != "graph":
        command += f" --workload {args.workload} --launch {args.launch}"
    if args.lib:  # another library than the in-tree build: never the profiled one
        command += f" --lib {args.lib}"
    ev = roofline(abytes, kernel_s, traffic)
    evidence, why = kernel_evidence(args.workload, abytes, command)
    if evidence is not None and evidence["busy"]["kernel_ms"] * 1e-3 <= step_s:
        busy = evidence["busy"]
        out = roofline(abytes, busy["kernel_ms"] * 1e-3, traffic)
        out["timing"] = (f"the kernel's busy time per dispatch in the committed counter pass of this "
                         f"command ({busy['file']}, {busy['dispatches']} dispatches)")
    else:
        out = dict(ev)
        out["timing"] = ktiming
    out["events"] = {"kernel_ms": ev["kernel_ms"], "frac": ev["frac"], "timing": ktiming}
    out["profile"] = evidence if evidence is not None else {"not_used": why}
    return out


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
    """Issues exactly the requested number of steps of a `ShardedBatch` — the kernel (`compute`)
    and/or the exchange (`exchange`, world > 1: the RCCL all-gather or the peer-push
    publish/wait) — as eager ctypes launches, or as hipGraph replays: a graph of G =
    min(graph_batch, steps) steps replayed steps // G times plus a graph of the remainder (and one
    of the warm-up count), so the steps issued are the steps asked for.

    The ranks AGREE on graph vs eager before any graph runs: every rank captures its graphs
    (capturing executes nothing), then a MIN all-reduce of the success flags over the control
    group (gloo, so it cannot be caught in a half-enqueued RCCL capture) decides, and only then
    are the graphs uploaded by one replay each.  If any rank's capture failed, every rank drops
    its graphs and launches eagerly — never one rank replaying a captured collective while another
    issues it eagerly, which would pair collectives of different steps or hang."""

    def __init__(self, sb, mode, graph_batch, steps, dev, exchange=True, compute=True, warmup=0,
                 world=1, ctrl=None):
        self.sb, self.mode, self.dev = sb, mode, dev
        self.exchange = exchange and sb.full is not None
        self.compute = compute
        self.G = max(1, min(graph_batch, steps)) if mode == "graph" else 1
        self.graphs, self._keep, self.fallback = {}, [], None
        if mode == "graph":
            self._one()                       # warm the code objects (and the communicator)
            torch.cuda.synchronize(dev)
            why = None
            try:
                for n in sorted({self.G, steps % self.G, warmup % self.G} - {0}):
                    self.graphs[n] = self._capture(n)
            except Exception as exc:          # noqa: BLE001 - reported, then eager launches
                why = f"{type(exc).__name__}: {exc}"
                torch.cuda.synchronize(dev)
            ok = agree(world, ctrl, why is None)
            if not ok:
                self.mode, self.G, self.graphs, self._keep = "eager", 1, {}, []
                self.fallback = (f"hipGraph capture failed ({why}); eager launches" if why else
                                 "hipGraph capture failed on another rank; eager launches on every rank")
            else:
                for n in sorted(self.graphs):
                    self.graphs[n].replay()   # upload the executable graphs outside any timed region
                torch.cuda.synchronize(dev)

    def _one(self, launch=None):
        if self.compute and self.exchange:
            self.sb.step(launch)          # kernel + exchange (RCCL: pipelined by chunks when chunks > 1)
        elif self.compute:
            self.sb.compute(launch)
        elif self.exchange:
            self.sb.exchange(launch)

    def _capture(self, n):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=torch.cuda.Stream(self.dev)):
            launch = self.sb.prepare(torch.cuda.current_stream(self.dev))  # bound to the capture stream
            for _ in range(n):
                self._one(launch)
        self._keep.append(launch)
        return g

    def run(self, steps):
        """Issue exactly `steps` steps; returns the count."""
        if self.mode == "graph":
            for _ in range(steps // self.G):
                self.graphs[self.G].replay()
            r = steps % self.G
            if r and r in self.graphs:
                self.graphs[r].replay()
            else:
                for _ in range(r):
                    self._one()
            return steps
        for _ in range(steps):
            self._one()
        return steps

    def describe(self):
        backend = dist.get_backend() if dist.is_initialized() else None
        if getattr(self.sb, "peer", None) is not None and self.sb.peer.mode == "pull":
            coll = ("peer-pull exchange (records written into the own region by the kernel; "
                    "publish/wait/copy-from-every-region launch)")
        elif getattr(self.sb, "peer", None) is not None:
            coll = "peer-push exchange (records written into every rank's region by the kernel; publish/wait/copy launch)"
        else:
            coll = f"all_gather_into_tensor ({'RCCL' if backend == 'nccl' else backend})"
        parts = (["launch"] if self.compute else []) + ([coll] if self.exchange else [])
        what = " + ".join(parts)
        if self.fallback:
            return f"{self.fallback}; step = {what}"
        if self.mode == "graph":
            extra = sorted(set(self.graphs) - {self.G})
            return (f"hipGraph replays of {self.G} steps" + (f" (+ graphs of {extra})" if extra else "")
                    + f"; step = {what}")
        return f"eager; step = {what}"


def agree(world, ctrl, ok):
    """True on every rank iff `ok` on every rank (a MIN all-reduce over the gloo control group)."""
    if world == 1:
        return bool(ok)
    flag = torch.tensor([1 if ok else 0], dtype=torch.int64)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=ctrl)
    return bool(flag.item())


def timed(world, fn, dev, stream):
    """The contract's timed region: barrier + synchronize on both sides; returns (wall s, event s
    on the launching stream, fn's result), each the max over ranks."""
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # torch creates a HIP event on its first record: both are created here, ev0 recorded just
    # before the wall clock starts and ev1 re-recorded after the last step (the first region of a
    # process otherwise paid ~8 us of event creation inside it: scripts/micro/first_region.py)
    ev1.record(stream)
    ev0.record(stream)
    t0 = time.perf_counter()
    res = fn()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:  # (one rank: no barrier, so nothing can be pending for a second synchronize)
        dist.barrier()
        torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    ev_s = ev0.elapsed_time(ev1) * 1e-3
    if world > 1:
        red = torch.tensor([elapsed, ev_s], dtype=torch.float64,
                           device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(red, op=dist.ReduceOp.MAX)
        elapsed, ev_s = float(red[0]), float(red[1])
    return elapsed, ev_s, res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--launch", default="graph", choices=["graph", "eager"])
    ap.add_argument("--graph-batch", type=int, default=50)
    ap.add_argument("--strong-workloads", default="c4,c5",
                    help="global batches of the strong-scaling legs (sharded over the ranks), comma-separated")
    ap.add_argument("--strong-steps", type=int, default=20)
    ap.add_argument("--chunks", default="auto",
                    help="strong-scaling legs at N > 1: also time the RCCL step pipelined in these chunk "
                         "counts (comma-separated; auto = per workload, CHUNKS)")
    ap.add_argument("--exchange", default="auto", choices=["auto", "rccl", "peer", "peer_pull"],
                    help="strong-scaling legs at N > 1: auto = time the RCCL all-gather and the two peer "
                         "exchanges (push, pull) and report the fastest as the leg's step; "
                         "rccl / peer / peer_pull = that one only")
    ap.add_argument("--no-strong", action="store_true", help="skip the strong-scaling line")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-large", action="store_true",
                    help="skip everything on the large batch (strong scaling, roofline_large, MPC, sampler)")
    ap.add_argument("--no-mpc", action="store_true", help="skip the MPC hand-off measurement")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse the N>1 path (several ranks may share one GPU)")
    ap.add_argument("--lib", default=None,
                    help="diagnostics: time a variant build of the engine instead of the product library")
    args = ap.parse_args()
    if args.lib:
        from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import _native
        _native.use_library(args.lib)
    if args.steps < 1:
        raise SystemExit("--steps must be >= 1")

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
    ctrl = None   # the control group: host-side agreement / handle exchange, never on a GPU stream
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
            ctrl = dist.new_group(backend="gloo")
        else:
            dist.init_process_group("gloo")
    gdev = "cpu" if (world > 1 and args.dist_backend == "gloo") else None
    mode = "eager" if (world > 1 and args.dist_backend == "gloo") else args.launch
    stream = torch.cuda.current_stream(dev)
    params = RiskParams()  # config/parameters.py: alpha 0.2, delta 0.1, eps 0.15, radii 0.3/0.3

    # ---- the metric line: every rank's shard is exactly the workload (weak scaling) ----
    O, T, N, desc = WORKLOADS[args.workload]
    nominal = synthetic.nominal_paths(O * world, T, dev, seed=42)   # the global (O*world)-obstacle batch
    ego = synthetic.straight_line_ego(T, dev)
    sb = sharding.ShardedBatch(nominal, ego, N, params, world, rank, seed=42, gather_device=gdev)
    assert sb.count == O * T
    stepper = Stepper(sb, mode, args.graph_batch, args.steps, dev, exchange=False, warmup=args.warmup,
                      world=world, ctrl=ctrl)
    stepper.run(args.warmup)                   # untimed warmup (W steps, the same launch path)
    elapsed, ev_s, K = timed(world, lambda: stepper.run(args.steps), dev, stream)
    kernel_s, ktiming = ev_s / K, "HIP events over the timed region / K (launch gaps included)"

    strong = None
    if not args.no_large and not args.no_strong:
        strong = {w: strong_scaling(args, world, rank, dev, stream, params, gdev, mode, w, ctrl)
                  for w in args.strong_workloads.split(",") if w}

    result = None
    if rank == 0:
        value = sb.U * K / elapsed               # units of ALL ranks (sb.U = O * world * T)
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
            "metric_form": ("weak scaling: every rank evaluates its own C3-sized block of a global "
                            f"{O * world}-obstacle batch, no collective in the step (units are "
                            "independent); the north-star sharded form with the RCCL all-gather is "
                            "strong_scaling"),
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (device-generated obstacle samples, SURVEY.md §8d distributions)",
            "config": {"workload": f"{args.workload}: {desc}", "obstacles": O, "steps": T,
                       "samples": N, "units_per_gpu": sb.count, "global_units_per_step": sb.U,
                       "global_batch": f"{O * world} obstacles x {T} steps x {N} samples, obstacles "
                                       f"[{O}r, {O}r + {O}) on rank r",
                       "parallelism": f"dp{world}",
                       "launch": stepper.describe(),
                       "alpha": params.alpha, "delta": params.delta, "epsilon": params.epsilon},
            "roofline": roofline_line(sb.algorithmic_bytes, kernel_s, ktiming, load_traffic(args.workload),
                                      args, elapsed / K),
            "strong_scaling": strong,
        }
    large = mpc = sampling = replicated = None
    c5leg = (strong or {}).get("c5")
    if rank == 0 and world == 1 and not args.no_large and c5leg is not None:
        big = c5leg.pop("_batch")
        large = c5leg.pop("_roofline")
        sampling = sampler_roofline(big, stream)
        if not args.no_mpc:
            mpc = mpc_handoff(dev, big.samples.view(big.O, big.T, big.N, 2), big.ego_units[:big.T],
                              params, with_cpu=not args.no_cpu_baseline)
        del big
        torch.cuda.empty_cache()
        replicated = c3_replicated(dev, stream, params)
    for leg in (strong or {}).values():
        leg.pop("_batch", None)
        leg.pop("_roofline", None)
    if rank == 0:
        result["roofline_large"] = large
        result["roofline_c3_replicated"] = replicated
        result["mpc_handoff"] = mpc
        result["sampling"] = sampling
        if world == 1 and not args.no_cpu_baseline:
            import numpy as np
            samples4 = sb.samples.view(O, T, N, 2)
            ref, base = cpu_baseline(samples4, ego, params, args.cpu_seconds)
            got = sb.records().cpu().numpy()
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


def strong_scaling(args, world, rank, dev, stream, params, gdev, mode, workload, ctrl=None):
    """The north-star multi-GPU form (BASELINE configs 4 and 5): ONE global batch sharded over
    the ranks — each rank draws only its contiguous unit block on its device and the records are
    reassembled on every rank inside the timed region.  Identical global work at every N (strong
    scaling); at N = 1 the exchange is the identity and is skipped.

    At N > 1 every exchange form is timed on the same draw (`exchanges`): the RCCL
    all_gather_into_tensor of the records, the same pipelined behind the kernel in the chunk
    counts of CHUNKS[workload], and the peer-push exchange (sharding.PeerExchange: the kernel
    writes every record into every rank's region over xGMI; one launch publishes, waits and
    copies), each checked to give records bitwise equal to the plain RCCL step's.  The leg's
    `value` / `ms_per_step` are the fastest equal form's (named in `exchange`).  Each phase is
    also timed alone, as its maximum over the ranks: `kernel_ms` (the shard's launch),
    `allgather_ms` (the RCCL collective alone) and `peer_exchange_ms` (the publish/wait/copy
    launch alone).  For C5 also the full MPC loop (shard kernel -> exchange -> the DR-CVaR QP
    over all O*T halfspaces, replicated per rank) and main.py's three filters."""
    O, T, N, desc = WORKLOADS[workload]
    seed = 7 if workload == "c5" else 11
    nominal = synthetic.nominal_paths(O, T, dev, seed=seed)
    ego = synthetic.straight_line_ego(T, dev)
    sb = sharding.ShardedBatch(nominal, ego, N, params, world, rank, seed=seed, gather_device=gdev)
    K = args.strong_steps

    def run_form(sbx, warm_check=None):
        st = Stepper(sbx, mode, 10, K, dev, world=world, ctrl=ctrl)
        st.run(min(K, 10))
        if warm_check is not None:   # (rank-agreed) a form that failed its warm-up is not timed
            torch.cuda.synchronize(dev)
            why = warm_check()
            if not agree(world, ctrl, why is None):
                return None, why or "failed its warm-up on another rank"
        el, _, _ = timed(world, lambda: st.run(K), dev, stream)
        return el, st.describe()

    elapsed, launch = run_form(sb)
    # phases alone, rank-max (HIP events on the launching stream, K steps each)
    kst = Stepper(sb, mode, 10, K, dev, exchange=False, world=world, ctrl=ctrl)
    kst.run(min(K, 10))
    _, kernel_s, _ = timed(world, lambda: kst.run(K), dev, stream)
    del kst
    gather_ms = None
    if world > 1:
        gst = Stepper(sb, mode, 10, K, dev, compute=False, world=world, ctrl=ctrl)
        gst.run(min(K, 10))
        _, gather_s, _ = timed(world, lambda: gst.run(K), dev, stream)
        gather_ms = gather_s / K * 1e3
        del gst
    kernel_s /= K
    exchanges = {"rccl": {"ms_per_step": elapsed / K * 1e3, "launch": launch,
                          "what": "all_gather_into_tensor of the 64-B records after the kernel"}}
    best, best_el, best_sb = "rccl", elapsed, sb
    peer_ms = pull_ms = None
    if world > 1:
        ref = sb.records()
        chunk_list = CHUNKS[workload] if args.chunks == "auto" else [int(c) for c in args.chunks.split(",") if c]
        if args.exchange in ("auto", "rccl"):
            for c in chunk_list:
                if c < 2:
                    continue
                # the pipelined step (sharding.chunked_all_gather): the rank's block in `chunks`
                # launches, chunk j's all-gather issued behind chunk j + 1's kernel
                sbc = sharding.ShardedBatch(nominal, ego, N, params, world, rank, seed=seed,
                                            gather_device=gdev, chunks=c)
                el_c, launch_c = run_form(sbc)
                same = agree(world, ctrl, bool(torch.equal(sbc.records().to(ref.device), ref)))
                step_c = el_c / K * 1e3
                exchanges[f"rccl_chunks{c}"] = {
                    "chunks": c, "ms_per_step": step_c, "records_equal_rccl": same, "launch": launch_c,
                    "overlap_ms": kernel_s * 1e3 + gather_ms - step_c}
                if same and el_c < best_el:
                    best, best_el, best_sb = f"rccl_chunks{c}", el_c, sbc
                else:
                    del sbc
        # the peer forms (gloo rehearsal too: ranks sharing one GPU map each other): push — the
        # kernel writes every record into every rank's region; pull — into its own region only,
        # the small launch reads every rank's rows from that rank's region
        what = {"peer": "the kernel writes every record into every rank's region (IPC-mapped, xGMI); "
                        "one launch publishes the step, waits for every peer's and copies",
                "peer_pull": "the kernel writes its records into its own region; one launch publishes "
                             "the step, waits for every peer's and copies every rank's rows from that "
                             "rank's region (IPC-mapped, xGMI)"}
        for form in ("peer", "peer_pull"):
            if args.exchange not in ("auto", form):
                continue
            try:
                sbp = sharding.ShardedBatch(nominal, ego, N, params, world, rank, seed=seed,
                                            exchange=form, ctrl=ctrl, samples=sb.samples,
                                            peer_spin_us=PEER_SPIN_US)
            except sharding.PeerExchangeUnavailable as exc:
                exchanges[form] = {"unavailable": str(exc)}
                continue
            el_p, launch_p = run_form(sbp, lambda: (None if sbp.peer.error() == 0 else
                                                    f"a wait gave up (error word {sbp.peer.error():#x})"))
            if el_p is None:
                exchanges[form] = {"unavailable": launch_p}
                sbp.close()
                continue
            err = sbp.peer.error()
            same = err == 0 and bool(torch.equal(sbp.records().to(ref.device), ref))
            same = agree(world, ctrl, same)
            pst = Stepper(sbp, mode, 10, K, dev, compute=False, world=world, ctrl=ctrl)
            pst.run(min(K, 10))
            _, peer_s, _ = timed(world, lambda: pst.run(K), dev, stream)
            del pst
            if form == "peer":
                peer_ms = peer_s / K * 1e3
            else:
                pull_ms = peer_s / K * 1e3
            exchanges[form] = {
                "ms_per_step": el_p / K * 1e3, "records_equal_rccl": same, "error_word": err,
                "launch": launch_p, "exchange_alone_ms": peer_s / K * 1e3, "what": what[form]}
            if same and el_p < best_el:   # (el_p, best_el: rank maxima; same: agreed)
                if best in what:
                    best_sb.close()       # collective, on every rank alike
                best, best_el, best_sb = form, el_p, sbp
            else:
                sbp.close()
                del sbp
    out = {"workload": f"{workload}: {desc}, global batch sharded over {world} rank(s)",
           "value": sb.U * K / best_el, "unit": "halfspace-constraints/s", "n_gpus": world,
           "steps": K, "ms_per_step": best_el / K * 1e3, "scaling": "strong",
           "exchange": best if world > 1 else None,
           "units_global": sb.U, "units_per_rank": sb.per,
           "bytes_per_rank": sb.algorithmic_bytes,
           "record_bytes_gathered": sb.per * world * 64 if world > 1 else 0,
           "parallelism": f"dp{world}" + (f"+{best} ({'RCCL' if gdev is None else 'gloo'} control)"
                                           if world > 1 else ""),
           "launch": exchanges[best]["launch"],
           "phases_rank_max": {"kernel_ms": kernel_s * 1e3, "allgather_ms": gather_ms,
                               "peer_exchange_ms": peer_ms, "peer_pull_exchange_ms": pull_ms,
                               "timing": f"HIP events over {K} steps of the phase alone, max over ranks"},
           "kernel_roofline_frac": sb.algorithmic_bytes / kernel_s / HBM_PEAK,
           # one rank: HBM bytes per launch of the whole batch from the committed PMC passes
           # (profiles/pmc_traffic.json), against bytes_per_rank (the algorithmic bytes)
           "traffic": load_traffic(workload) if world == 1 else None}
    if world > 1:
        out["exchanges"] = exchanges
    if best_sb is not sb:
        sb = best_sb          # the loops below run on the leg's fastest exchange
    # full loop: + the QP hand-off on every rank (core/mpc_filter.py:116-151 takes all halfspaces)
    if workload == "c5" and not args.no_mpc:
        import numpy as np
        from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf
        dt = 0.2
        A = np.block([[np.eye(2), dt * np.eye(2)], [np.zeros((2, 2)), np.eye(2)]])
        Bm = np.block([[0.5 * dt ** 2 * np.eye(2)], [dt * np.eye(2)]])
        C = np.block([np.eye(2), np.zeros((2, 2))])
        model = mf.MPCModel(A, Bm, C, 2 * np.eye(4), np.eye(2), T, (np.full(2, -5.0), np.full(2, 5.0)),
                            (np.full(2, -10.0), np.full(2, 10.0)), device=dev)
        x0, xr, uf, _ = _mpc_problem_inputs(ego, T, 1, dev)
        ws = torch.empty(model.workspace_doubles(1, O), dtype=torch.float64, device=dev)
        rec = sb.records()
        if rec.device != dev:
            rec = torch.empty(rec.shape, dtype=torch.float64, device=dev)
        h, g = mf.record_views(rec, "dr_cvar")
        res = {}

        def loop(k):
            for _ in range(k):
                sb.step()
                if sb.full is not None and sb.full.device != dev:
                    rec.copy_(sb.records())
                res["info"] = mf.filter_batch(model, h, g, x0, xr, uf, workspace=ws)[2]
            return k

        Kf = 5
        loop(2)
        el, _, _ = timed(world, lambda: loop(Kf), dev, stream)
        info = res["info"][0].cpu().numpy()
        out["full_loop"] = {"steps": Kf, "ms_per_step": el / Kf * 1e3,
                            "halfspace_constraints_per_s": sb.U * Kf / el,
                            "qp": f"dr_cvar safety filter, H={T}, {sb.U} halfspace rows, one problem, "
                                  f"replicated on every rank",
                            "qp_status": mf.STATUS_NAMES.get(int(info[0])), "qp_iterations": int(info[1])}
        # main.py's whole flow per step (main.py:95-112): the halfspaces, then its THREE safety
        # filters (mean, CVaR, DR-CVaR) — independent QPs over the same records, distributed over
        # the ranks (rank r solves metrics[r::world]; one rank: all three in one launch), then one
        # all-gather of the filtered inputs so every rank holds every filter's answer
        metrics = ("mean", "cvar", "dr_cvar")
        mine = metrics[rank::world]
        nb = len(mine)
        slots = -(-len(metrics) // world)
        ws3 = h3 = g3 = None
        if nb:
            cols_h = torch.tensor([c for m in mine for c in (mf.METRIC_COLUMNS[m][0], mf.METRIC_COLUMNS[m][0] + 1)],
                                  device=dev)
            cols_g = torch.tensor([mf.METRIC_COLUMNS[m][1] for m in mine], device=dev)
            x0m, xrm, ufm = (x0.expand(nb, -1).contiguous(), xr.expand(nb, -1, -1).contiguous(),
                             uf.expand(nb, -1, -1).contiguous())
            ws3 = torch.empty(model.workspace_doubles(nb, O), dtype=torch.float64, device=dev)
        usend = torch.zeros((slots, T, 2), dtype=torch.float64, device=dev)
        ufull = (torch.empty((slots * world, T, 2), dtype=torch.float64, device=gdev or dev)
                 if world > 1 else None)

        def flow(k):
            for _ in range(k):
                sb.step()
                if sb.full is not None and sb.full.device != dev:
                    rec.copy_(sb.records())
                if nb:
                    hm = rec.index_select(2, cols_h).view(O, T, nb, 2).permute(2, 0, 1, 3)
                    gm = rec.index_select(2, cols_g).permute(2, 0, 1)
                    u, info3 = mf.filter_batch(model, hm, gm, x0m, xrm, ufm, workspace=ws3)[1:]
                    usend[:nb].copy_(u)
                    res["info3"] = info3
                if ufull is not None:
                    sharding._all_gather(ufull, usend)
            return k

        flow(2)
        el3, _, _ = timed(world, lambda: flow(Kf), dev, stream)
        inf3 = res["info3"].cpu().numpy() if nb else np.zeros((0, 10))
        out["main_flow"] = {"steps": Kf, "ms_per_step": el3 / Kf * 1e3,
                            "what": "main.py's three safety filters (mean, CVaR, DR-CVaR) per step over "
                                    f"the sharded halfspaces; rank r solves {list(metrics)}[r::{world}], then "
                                    "an all-gather of the filtered inputs",
                            "rank0_filters": list(mine),
                            "rank0_qp_iterations": [int(v) for v in inf3[:, 1]],
                            "rank0_qp_status": [mf.STATUS_NAMES.get(int(v)) for v in inf3[:, 0]]}
    if rank == 0 and world == 1 and workload == "c5":
        out["_batch"] = sb
        large = roofline(sb.algorithmic_bytes, kernel_s, load_traffic("c5"))
        large["workload"] = f"{O} obstacles x {T} steps x {N} samples (2.05 GB resident)"
        large["halfspaces_per_s"] = sb.U / kernel_s
        large["timing"] = f"HIP events over {K} graph-replayed launches (replays of 10)"
        out["_roofline"] = large
    sb.close()   # collective for the peer exchange (every rank chose the same form); else a no-op
    return out


def c3_replicated(dev, stream, params, copies=640, reps=20, check_obstacles=100):
    """BASELINE.md §3's second roofline convention: the metric's C3 batch (10 obstacles x T=20 x
    N=1000, the 256x4 launch plan) replicated to a >= 2 GB working set — `copies` C3 scenes sharing
    the ego path, one launch over all of them (6 400 obstacles, 128 000 units, 2.06 GB resident) —
    graph-replayed, HIP events.  The metric line's C3 step is one 3.2 MB launch (latency- and
    dispatch-bound); this is the same kernel plan where bandwidth, not the dispatch, bounds it.
    Offsets of the first `check_obstacles` obstacles are checked against the C oracle after timing."""
    import numpy as np
    O, T, N, _ = WORKLOADS["c3"]
    O *= copies
    nominal = synthetic.nominal_paths(O, T, dev, seed=5)
    ego = synthetic.straight_line_ego(T, dev)
    sb = sharding.ShardedBatch(nominal, ego, N, params, 1, 0, seed=5)
    st = Stepper(sb, "graph", 10, reps, dev, exchange=False)
    st.run(10)
    _, ks, _ = timed(1, lambda: st.run(reps), dev, stream)
    ks /= reps
    out = roofline(sb.algorithmic_bytes, ks, None)
    out.update({"workload": f"{copies} x C3 (10 obstacles x {T} steps x {N} samples) = {O} obstacles, "
                            f"{sb.U} units, {sb.algorithmic_bytes / 1e9:.2f} GB resident, one launch",
                "halfspaces_per_s": sb.U / ks,
                "timing": f"HIP events over {reps} graph-replayed launches (replays of 10)"})
    from oracle import c_oracle
    s = sb.samples.view(O, T, N, 2)[:check_obstacles].cpu().numpy()
    ref = c_oracle.safe_halfspaces(s, ego.cpu().numpy(), params.robot_radius, params.obstacle_radius,
                                   params.alpha, params.delta, params.epsilon,
                                   nthreads=max(1, min(16, len(os.sched_getaffinity(0)))))
    got = sb.records().view(O, T, -1)[:check_obstacles].cpu().numpy()
    out["max_abs_err"] = float(np.max(np.abs(got[..., [2, 5, 6, 7]] - ref[..., [2, 5, 6, 7]])))
    out["checked"] = f"obstacles [0, {check_obstacles}) x {T} steps against oracle/drcvar_oracle.c"
    del st
    sb.close()
    return out


def sampler_roofline(sb, stream, reps=10):
    """Device sample generator (drcvar_sample_units_f64) refilling the resident large batch with
    the same draws: bytes written (16 per sample) per launch / event time."""
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.simulation import obstacles
    launch = lambda: obstacles.sample_units_device(sb.nominal, sb.N, sb.start, sb.count, seed=sb.seed,
                                                   out=sb.samples)
    launch()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(reps):
        launch()
    b.record(stream)
    torch.cuda.synchronize()
    sec = a.elapsed_time(b) * 1e-3 / reps
    n = sb.count * sb.N
    written = n * 16
    out = {"workload": f"{sb.count} units x {sb.N} samples (Philox4x32-10 + Box-Muller, fp64)",
           "kernel_ms": sec * 1e3, "samples_per_s": n / sec, "bound": SAMPLER_BOUND,
           "achieved": written / sec / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
           "frac": written / sec / HBM_PEAK}
    return out


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
    groups = model.launch_groups(1, O)
    # the same QP on one workgroup (options.cluster_size = 1), for comparison with the clustered launch
    one_wg = mf.make_options(cluster_size=1)
    qp1_ms = timed(lambda: mf.filter_batch(model, h, g, x0, xr, uf, workspace=ws, options=one_wg), 3)
    qp()  # leaves the clustered answer in res
    c5 = {"workload": f"{O} obstacles x {T} steps x {samples.shape[2]} samples -> dr_cvar QP "
                      f"(H={H}, {O * T} halfspace rows), 1 problem",
          "full_step_ms": full_ms, "qp_ms": qp_ms, "halfspace_ms": full_ms - qp_ms,
          "qp_workgroups": groups, "qp_one_workgroup_ms": qp1_ms,
          "halfspace_constraints_per_s_full_loop": O * T / (full_ms * 1e-3),
          "qp_status": mf.STATUS_NAMES.get(int(info[_native.MPC_INFO_STATUS])),
          "qp_iterations": int(info[_native.MPC_INFO_ITERATIONS]),
          "polished": bool(info[_native.MPC_INFO_POLISHED]),
          "polish_attempts": int(info[_native.MPC_INFO_POLISH_ATTEMPTS])}
    if os.environ.get("DRCVAR_BENCH_DUMP_QP"):  # diagnostics: the C5 QP's inputs (scripts/micro/ipm_lab.py)
        np.savez_compressed(os.environ["DRCVAR_BENCH_DUMP_QP"], **{
            f"H{H}_O{O}_B1_bench_h": h.cpu().numpy(), f"H{H}_O{O}_B1_bench_g": g.cpu().numpy(),
            f"H{H}_O{O}_B1_bench_x0": x0.cpu().numpy(), f"H{H}_O{O}_B1_bench_xr": xr.cpu().numpy(),
            f"H{H}_O{O}_B1_bench_u": res["u"].cpu().numpy(), f"H{H}_O{O}_B1_bench_info": res["info"].cpu().numpy()})
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
    # ---- main.py's whole flow at C5 size: the halfspaces, then the three safety filters over
    # them (mean, CVaR, DR-CVaR: main.py:95-112), the three QPs as one launch ----
    metrics = ("mean", "cvar", "dr_cvar")
    cols_h = torch.tensor([c for m in metrics for c in (mf.METRIC_COLUMNS[m][0], mf.METRIC_COLUMNS[m][0] + 1)],
                          device=dev)
    cols_g = torch.tensor([mf.METRIC_COLUMNS[m][1] for m in metrics], device=dev)
    x03, xr3, uf3 = x0.expand(3, -1).contiguous(), xr.expand(3, -1, -1).contiguous(), uf.expand(3, -1, -1).contiguous()
    ws3 = torch.empty(model.workspace_doubles(3, O), dtype=torch.float64, device=dev)

    def three():
        launch()
        h3 = rec.index_select(2, cols_h).view(O, T, 3, 2).permute(2, 0, 1, 3)   # [3, O, T, 2]
        g3 = rec.index_select(2, cols_g).permute(2, 0, 1)                       # [3, O, T]
        res["info3"] = mf.filter_batch(model, h3, g3, x03, xr3, uf3, workspace=ws3)[2]

    three_ms = timed(three, 5)
    inf3 = res["info3"].cpu().numpy()
    out["main_flow_c5"] = {
        "workload": f"main.py's flow at C5 size: {O} obstacles x {T} steps x {samples.shape[2]} samples -> "
                    f"halfspaces -> the mean, CVaR and DR-CVaR safety filters (H={H}, {O * T} rows each) "
                    "as one 3-problem QP launch",
        "step_ms": three_ms, "qp_workgroups": model.launch_groups(3, O),
        "qp_status": [mf.STATUS_NAMES.get(int(v)) for v in inf3[:, _native.MPC_INFO_STATUS]],
        "qp_iterations": [int(v) for v in inf3[:, _native.MPC_INFO_ITERATIONS]]}
    del ws, ws3, rec
    # ---- batched reference configuration: main.py's QP, 1024 DISTINCT problems per launch ----
    # (each problem its own three obstacles: one sampled batch of 3 x 1024 obstacles, the records
    # viewed as [1024, 3, H, 8]; the ego / x_ref of main.py's straight line is shared)
    Hr, Or, Bn = 30, 3, 1024
    model_r = mf.MPCModel(A, Bm, C, Q, R, Hr, ub, pb, device=dev)
    s_r, e_r = synthetic.obstacle_batch(Or * Bn, Hr, 20, dev, seed=3)  # NUM_SAMPLES = 20
    rec_r = engine.safe_halfspaces(s_r, e_r, params).view(Bn, Or, Hr, engine.OUT_WIDTH)
    del s_r
    hb, gb = rec_r[..., 3:5], rec_r[..., 7]
    x0r, xrr, ufr, xr_host_r = _mpc_problem_inputs(e_r, Hr, Bn, dev)
    wsr = torch.empty(model_r.workspace_doubles(Bn, Or), dtype=torch.float64, device=dev)

    def qp_batch():
        res["u"], res["info"] = mf.filter_batch(model_r, hb, gb, x0r, xrr, ufr, workspace=wsr)[1:]

    ms = timed(qp_batch, 5)
    inf = res["info"].cpu().numpy()
    its = inf[:, _native.MPC_INFO_ITERATIONS].astype(int)
    br = {"workload": f"main.py QP (H={Hr}, {Or} obstacles, bounds), {Bn} distinct problems per launch "
                      f"(each its own {Or} sampled obstacles)",
          "launch_ms": ms, "qps_per_s": Bn / (ms * 1e-3),
          "optimal_frac": float((inf[:, _native.MPC_INFO_STATUS] == 0).mean()),
          "polished_frac": float(inf[:, _native.MPC_INFO_POLISHED].mean()),
          "mean_iterations": float(its.mean()), "max_iterations": int(its.max()),
          "iteration_histogram": np.bincount(its).tolist(),
          "max_polish_attempts": int(inf[:, _native.MPC_INFO_POLISH_ATTEMPTS].max())}
    if with_cpu:
        from oracle import mpc_qp
        r = rec_r.cpu().numpy()
        hs = np.concatenate([r[..., 3:5], r[..., 7:8]], -1)          # [Bn, Or, Hr, 3]
        solve = lambda b: mpc_qp.filter_trajectory(A, Bm, C, Q, R, Hr, xr_host_r[0], xr_host_r, None,
                                                   [hs[b][:, t] for t in range(Hr)], ub, pb)
        reps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 3.0:
            solve(reps % Bn)
            reps += 1
        el = time.perf_counter() - t0
        br["cpu_baseline"] = {"value": reps / el, "unit": "QPs/s", "cores": 1, "kind": "port",
                              "sample": f"{reps} solves of problems 0..{reps - 1} by oracle/mpc_qp.py ({el:.1f} s)"}
        # |u - oracle| on a sample: the first problems, the slowest one, a spread of the rest
        sample = sorted(set([0, 1, 2, int(its.argmax())] + list(range(0, Bn, Bn // 12))))
        u_gpu = res["u"].cpu().numpy()
        br["max_abs_err_u_vs_oracle"] = float(max(np.abs(u_gpu[b] - solve(b)[1]).max() for b in sample))
        br["oracle_sample"] = f"{len(sample)} problems: {sample}"
    out["batched_reference"] = br
    out["bound"] = ("latency: every interior-point iteration is a chain of Riccati factorisation "
                    "and solves on one wave; batches run one workgroup per problem, a large problem "
                    "(C5: 12 800 halfspace rows) a cluster of workgroups that split the row sweeps "
                    "and exchange row sums in the launch (see DESIGN.md)")
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

"""Per-rank shard kernel time of the strong-scaling legs at W = 1, 2, 4, 8 ranks, measured on ONE
GPU: rank r's block of the C4 / C5 global batch (sharding.ShardedBatch(world=W, rank=r): its own
draw, its own launch) timed alone with HIP events over hipGraph replays — what each rank of a
W-GPU node runs before the exchange (the ranks' kernels do not share a GPU there).  Also the
peer-push exchange's publish/wait/copy launch with one rank (the exchange with itself: the launch
and copy cost, no xGMI flight) and the peer-form kernel (the records written through the
exchange).  Prints one JSON line; feeds DESIGN.md §6's prediction table.

    python scripts/micro/shard_kernel_times.py [--steps 50]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

import bench  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import sharding, synthetic  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.engine import RiskParams  # noqa: E402


def graph_time(fn, dev, steps, per_graph=10):
    s = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    fn(None)
    torch.cuda.synchronize(dev)
    with torch.cuda.graph(g, stream=s):
        for _ in range(per_graph):
            fn(torch.cuda.current_stream(dev))
    g.replay()
    torch.cuda.synchronize(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cur = torch.cuda.current_stream(dev)
    a.record(cur)
    for _ in range(steps // per_graph):
        g.replay()
    b.record(cur)
    torch.cuda.synchronize(dev)
    return a.elapsed_time(b) / (steps // per_graph * per_graph) * 1e3  # us per step


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = {}
    for w in ("c4", "c5"):
        O, T, N, _ = bench.WORKLOADS[w]
        seed = 7 if w == "c5" else 11
        nominal = synthetic.nominal_paths(O, T, dev, seed=seed)
        ego = synthetic.straight_line_ego(T, dev)
        for W in (1, 2, 4, 8):
            row = {}
            for r in sorted({0, W - 1}):
                sb = sharding.ShardedBatch(nominal, ego, N, RiskParams(), W, r, seed=seed)
                launch = {}

                def step(stream, sb=sb, launch=launch):
                    key = id(stream)
                    if key not in launch:
                        launch[key] = sb.prepare(stream)
                    sb.compute(launch[key])
                us = graph_time(step, dev, args.steps)
                row[f"rank{r}"] = {"units": sb.count, "kernel_us": us,
                                   "frac": sb.algorithmic_bytes / (us * 1e-6) / bench.HBM_PEAK}
                del sb, launch
                torch.cuda.empty_cache()
            out[f"{w}_W{W}"] = row
        # the peer form at one rank: the kernel writing through the exchange, and the
        # publish / wait / copy launch alone
        sbp = sharding.ShardedBatch(nominal, ego, N, RiskParams(), 1, 0, seed=seed, exchange="peer",
                                    force_exchange=True)
        launch = {}

        def pstep(stream, launch=launch):
            key = id(stream)
            if key not in launch:
                launch[key] = sbp.prepare(stream)
            sbp.compute(launch[key])

        def pex(stream, launch=launch):
            key = id(stream)
            if key not in launch:
                launch[key] = sbp.prepare(stream)
            sbp.exchange(launch[key])

        def pfull(stream, launch=launch):
            key = id(stream)
            if key not in launch:
                launch[key] = sbp.prepare(stream)
            sbp.step(launch[key])
        out[f"{w}_peer_W1"] = {"kernel_us": graph_time(pstep, dev, args.steps),
                               "exchange_alone_us": graph_time(pex, dev, args.steps),
                               "step_us": graph_time(pfull, dev, args.steps),
                               "error_word": sbp.peer.error()}
        sbp.close()
        del sbp
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()

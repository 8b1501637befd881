#!/usr/bin/env python3
"""Where the fixed cost of a short timed region goes (bench.py's contract at --steps 20).

For the C3 batch: per-step wall time and HIP-event time of K graph-replayed steps (K = 20, 200,
2000), the host time of the replay call itself, and the wall time of an empty timed region (two
barriers + synchronize, no work).  With DRCVAR_SCHED=spin|yield|blocking the HIP device
scheduling flag is set before torch creates its context (hipSetDeviceFlags), to see how much of
the fixed cost is the synchronize's wake-up.
"""
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

sched = os.environ.get("DRCVAR_SCHED")
if sched:
    flag = {"spin": 1, "yield": 2, "blocking": 4}[sched]
    hip = ctypes.CDLL("libamdhip64.so")
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(flag))
    print(f"hipSetDeviceFlags({sched}) rc={rc}", flush=True)

import torch  # noqa: E402

from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import sharding, synthetic  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.engine import RiskParams  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    nominal = synthetic.nominal_paths(10, 20, dev, seed=42)
    ego = synthetic.straight_line_ego(20, dev)
    sb = sharding.ShardedBatch(nominal, ego, 1000, RiskParams(), seed=42)
    out = {"sched": sched or "default"}
    graphs = {}
    for K in (20, 200, 2000):
        G = min(K, 50)
        if G not in graphs:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=torch.cuda.Stream(dev)):
                launch = sb.prepare(torch.cuda.current_stream(dev))
                for _ in range(G):
                    sb.compute(launch)  # prepare() returns one frozen launch per chunk
            g.replay()
            torch.cuda.synchronize()
            graphs[G] = (g, launch)
        g = graphs[G][0]
        rows = []
        for rep in range(7):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(stream)
            th0 = time.perf_counter()
            for _ in range(K // G):
                g.replay()
            th1 = time.perf_counter()
            e1.record(stream)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            rows.append({"wall_us_per_step": (t1 - t0) / K * 1e6,
                         "event_us_per_step": e0.elapsed_time(e1) * 1e3 / K,
                         "replay_host_us": (th1 - th0) * 1e6 / (K // G),
                         "sync_tail_us": (t1 - th1) * 1e6})
        rows.sort(key=lambda r: r["wall_us_per_step"])
        out[f"K{K}"] = {"median": rows[len(rows) // 2], "best": rows[0]}
    # empty region: what bench.py's bracketing alone costs
    empties = []
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        empties.append((time.perf_counter() - t0) * 1e6)
    out["empty_sync_us_median"] = sorted(empties)[len(empties) // 2]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""What a short timed region (bench.py --steps 20 --warmup 5, the driver's form) measures after
an idle gap: the C3 graph of 20 steps timed (wall + HIP events) after

  idle    50 ms of host-side idling, then 5 eager warm-up launches (bench.py's round-2 flow)
  graphw  50 ms idle, then the 5 warm-up steps as a replay of a captured 5-step graph
  busy    the same as graphw, but right after ~20 ms of other device work (a C5-sized sampler
          refill + halfspace launches, as the bench's large legs would leave the device)
  steady  back-to-back timed regions (no idle gap)

Each protocol is repeated 7 times; the median and the spread are printed as one JSON line.
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import sharding, synthetic  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.engine import RiskParams  # noqa: E402


def graph_of(sb, n, dev):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=torch.cuda.Stream(dev)):
        launch = sb.prepare(torch.cuda.current_stream(dev))
        for _ in range(n):
            sb.compute(launch)  # prepare() returns one frozen launch per chunk
    g.replay()
    torch.cuda.synchronize()
    return g, launch


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    sb = sharding.ShardedBatch(synthetic.nominal_paths(10, 20, dev, seed=42),
                               synthetic.straight_line_ego(20, dev), 1000, RiskParams(), seed=42)
    big = sharding.ShardedBatch(synthetic.nominal_paths(64, 30, dev, seed=7),
                                synthetic.straight_line_ego(30, dev), 5000, RiskParams(), seed=7)
    g20, _ = graph_of(sb, 20, dev)
    g5, _ = graph_of(sb, 5, dev)

    def region():
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        g20.replay()
        e1.record(stream)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / 20 * 1e6, e0.elapsed_time(e1) * 1e3 / 20

    out = {}
    for proto in ("idle", "graphw", "busy", "steady"):
        rows = []
        for _ in range(7):
            if proto != "steady":
                time.sleep(0.05)
            if proto == "busy":
                for _ in range(4):
                    big.compute()
                torch.cuda.synchronize()
            if proto == "idle":
                for _ in range(5):
                    sb.compute()
            elif proto in ("graphw", "busy"):
                g5.replay()
            rows.append(region())
        rows.sort()
        out[proto] = {"wall_us_median": rows[3][0], "event_us_median": rows[3][1],
                      "wall_us_min": rows[0][0], "wall_us_max": rows[-1][0]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

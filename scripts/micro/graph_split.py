#!/usr/bin/env python3
"""How the K = 20 timed region (bench.py --steps 20, the driver's form) depends on how its 20
steps are split into graph replays.  A hipGraph launch of G kernel nodes costs the host ~10-16 us
before it returns; if the device only starts once the launch has been submitted, a region issued
as one 20-node graph idles the device for that long.  A short leading graph (or one eager launch)
starts the device sooner while the host submits the rest.

Splits timed (C3 batch, exactly 20 steps each, wall and HIP events, medians of 9 regions after
back-to-back warm-up and after a 50 ms idle gap):
  [20]        one 20-node graph (bench.py today)
  [1e, 19]    one eager launch, then a 19-node graph
  [2, 18], [4, 16], [5, 15], [2, 4, 14]
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

SPLITS = [[20], ["e", 19], [2, 18], [4, 16], [5, 15], [2, 4, 14]]


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    sb = sharding.ShardedBatch(synthetic.nominal_paths(10, 20, dev, seed=42),
                               synthetic.straight_line_ego(20, dev), 1000, RiskParams(), seed=42)
    graphs = {}
    for n in sorted({x for s in SPLITS for x in s if x != "e"}):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=torch.cuda.Stream(dev)):
            launch = sb.prepare(torch.cuda.current_stream(dev))
            for _ in range(n):
                sb.compute(launch)  # prepare() returns one frozen launch per chunk
        g.replay()
        graphs[n] = (g, launch)
    torch.cuda.synchronize()
    warm = graphs[5][0]

    def region(split):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for part in split:
            if part == "e":
                sb.compute()
            else:
                graphs[part][0].replay()
        e1.record(stream)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / 20 * 1e6, e0.elapsed_time(e1) * 1e3 / 20

    out = {}
    for mode in ("back_to_back", "after_idle"):
        res = {}
        for rep in range(9):
            for split in SPLITS:
                if mode == "after_idle":
                    time.sleep(0.05)
                warm.replay()  # the bench's 5 warm-up steps
                res.setdefault(str(split), []).append(region(split))
        out[mode] = {k: {"wall_us_median": sorted(r[0] for r in v)[4],
                         "event_us_median": sorted(r[1] for r in v)[4]} for k, v in res.items()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

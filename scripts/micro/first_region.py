#!/usr/bin/env python3
"""Is the first K = 20 timed region after setup slower than later ones?  Mirrors bench.py's flow
(Stepper: capture the 20- and 5-step graphs with one upload replay each, replay the 5-step graph as
warm-up, then the timed region) and times regions 1..6 individually (wall and HIP events), in a
fresh process each time the script runs."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import sharding, synthetic  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.engine import RiskParams  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    sb = sharding.ShardedBatch(synthetic.nominal_paths(10, 20, dev, seed=42),
                               synthetic.straight_line_ego(20, dev), 1000, RiskParams(), seed=42)
    st = bench.Stepper(sb, "graph", 50, 20, dev, exchange=False, warmup=5)
    rows = []
    for r in range(6):
        st.run(5)
        wall, ev, _ = bench.timed(1, lambda: st.run(20), dev, stream)
        rows.append((wall / 20 * 1e6, ev / 20 * 1e6))
    print(json.dumps({"regions_wall_us_per_step": [round(a, 3) for a, _ in rows],
                      "regions_event_us_per_step": [round(b, 3) for _, b in rows]}), flush=True)


if __name__ == "__main__":
    main()

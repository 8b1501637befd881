#!/usr/bin/env python3
"""Two processes sharing one GPU (as the gloo rehearsal's ranks do), each running the C5 full loop
(halfspace launch + clustered QP) for TWO_PROC_SECONDS of wall time (so that the two overlap): per-step time and QP status of every solve, so a cluster
exchange that outlasts the spin bound (CLUSTER_TIMEOUT) shows up by name."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import _native, engine, sharding, synthetic  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.engine import RiskParams  # noqa: E402


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "p"
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
    launch, rec = engine.prepare_safe_halfspaces(samples, ego, params)
    h, g = mf.record_views(rec, "dr_cvar")
    rows = []
    t_end = time.perf_counter() + float(os.environ.get("TWO_PROC_SECONDS", "4"))
    while time.perf_counter() < t_end:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        launch()
        info = mf.filter_batch(model, h, g, x0, xr, uf, workspace=ws)[2]
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        st = mf.STATUS_NAMES.get(int(info[0, _native.MPC_INFO_STATUS].item()))
        rows.append((ms, st))
    ms = sorted(r[0] for r in rows[1:])
    print(tag, f"{len(rows)} steps, ms median {ms[len(ms) // 2]:.2f} p99 {ms[int(len(ms) * 0.99)]:.2f} max {ms[-1]:.2f}", flush=True)
    print(tag, "statuses:", sorted(set(r[1] for r in rows)), {s: sum(1 for r in rows if r[1] == s) for s in set(r[1] for r in rows)}, flush=True)


if __name__ == "__main__":
    main()

"""Dump bench.py's main_flow_c5 problems (C5 batch, seed 7: the halfspaces, then main.py's three
safety filters mean / CVaR / DR-CVaR over them, core/mpc_filter.py:116-151 per metric) with the
kernel's answers and info rows, to gpurun_out/main_flow_c5.npz — for the CPU lab
(scripts/micro/ipm_lab.py) and the golden fixture tests/golden/qp_c5_mean.npz
(tests/golden/make_golden_qp_c5_mean.py)."""
import os
import sys

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import sharding, synthetic  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.engine import RiskParams  # noqa: E402

dev = torch.device("cuda", 0)
dt = 0.2
A = np.block([[np.eye(2), dt * np.eye(2)], [np.zeros((2, 2)), np.eye(2)]])
Bm = np.block([[0.5 * dt ** 2 * np.eye(2)], [dt * np.eye(2)]])
C = np.block([np.eye(2), np.zeros((2, 2))])
O, T, N, seed = 256, 50, 10000, 7
model = mf.MPCModel(A, Bm, C, 2 * np.eye(4), np.eye(2), T, (np.full(2, -5.0), np.full(2, 5.0)),
                    (np.full(2, -10.0), np.full(2, 10.0)), device=dev)
nominal = synthetic.nominal_paths(O, T, dev, seed=seed)
ego = synthetic.straight_line_ego(T, dev)
sb = sharding.ShardedBatch(nominal, ego, N, RiskParams(), 1, 0, seed=seed)
sb.step()
rec = sb.records()
x0, xr, uf, _ = bench._mpc_problem_inputs(ego, T, 1, dev)
out = {"records": rec.cpu().numpy(), "x0": x0.cpu().numpy()[0], "x_ref": xr.cpu().numpy()[0]}
for m in ("mean", "cvar", "dr_cvar"):
    h, g = mf.record_views(rec, m)
    x, u, info = mf.filter_batch(model, h, g, x0, xr, uf)
    out[f"{m}_u"] = u.cpu().numpy()[0]
    out[f"{m}_info"] = info.cpu().numpy()[0]
    print(m, "status", int(info[0, 0]), "iterations", int(info[0, 1]), "polish attempts", int(info[0, 9]))
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed("gpurun_out/main_flow_c5.npz", **out)
print("saved gpurun_out/main_flow_c5.npz")

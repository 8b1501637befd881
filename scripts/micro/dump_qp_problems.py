"""Dump scripts/mpc_bench.py's QP problems (halfspace rows from the engine on the device) and the
kernel's answers to gpurun_out/qp_problems.npz, for CPU experiments with the interior-point method
(scripts/micro/ipm_lab.py)."""
import os
import sys

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "scripts"))
sys.path.insert(0, os.path.join(os.getcwd(), "scripts", "micro"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import _native  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf  # noqa: E402
from mpc_bench import problem_batch  # noqa: E402

dev = torch.device("cuda", 0)
out = {}
SHAPES = ["50,256,1,0", "50,256,1,1", "50,256,1,2", "50,256,3,5", "30,3,4,0", "20,10,3,0",
          "20,100,1,0", "30,64,2,0"]
if len(sys.argv) > 1 and sys.argv[1] == "wide":  # a wider set for validation: more seeds per shape
    SHAPES = ([f"50,256,2,{s}" for s in range(10, 20, 2)] + [f"30,3,8,{s}" for s in (20, 30)] +
              [f"20,100,2,{s}" for s in (40, 42, 44)] + [f"30,64,2,{s}" for s in (50, 52, 54)] +
              [f"40,128,2,{s}" for s in (60, 62)] + [f"20,10,4,{s}" for s in (70, 71)])
OUT = "gpurun_out/qp_problems_wide.npz" if SHAPES[0] != "50,256,1,0" else "gpurun_out/qp_problems.npz"
if len(sys.argv) > 1 and sys.argv[1] == "benchbatch":  # bench.py's batched_reference: 1024 distinct problems
    import bench  # noqa: E402
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import engine, synthetic  # noqa: E402
    Hr, Or, Bn = 30, 3, 1024
    s_r, e_r = synthetic.obstacle_batch(Or * Bn, Hr, 20, dev, seed=3)
    rec = engine.safe_halfspaces(s_r, e_r, engine.RiskParams()).view(Bn, Or, Hr, 8)
    x0, xr, uf, _ = bench._mpc_problem_inputs(e_r, Hr, Bn, dev)
    model, _, _, _, _ = __import__("mpc_bench").problem_batch(Hr, 1, 1, dev)
    h, g = rec[..., 3:5], rec[..., 7]
    x, u, info = mf.filter_batch(model, h, g, x0, xr, uf)
    torch.cuda.synchronize()
    key = f"H{Hr}_O{Or}_B{Bn}_bench"
    for nm, t in (("h", h), ("g", g), ("x0", x0), ("xr", xr), ("u", u), ("info", info)):
        out[f"{key}_{nm}"] = t.cpu().numpy()
    its = info[:, _native.MPC_INFO_ITERATIONS].cpu().numpy()
    print(key, "iterations: mean", its.mean(), "max", its.max(), "argmax", its.argmax(), flush=True)
    SHAPES, OUT = [], "gpurun_out/qp_problems_benchbatch.npz"
for shape in SHAPES:
    H, O, B, seed = (int(v) for v in shape.split(","))
    model, rec, x0, xr, uf = problem_batch(H, O, B, dev, seed=seed)
    h, g = rec[..., 3:5], rec[..., 7]
    x, u, info = mf.filter_batch(model, h, g, x0, xr, uf)
    torch.cuda.synchronize()
    key = f"H{H}_O{O}_B{B}_s{seed}"
    out[key + "_h"] = h.cpu().numpy()
    out[key + "_g"] = g.cpu().numpy()
    out[key + "_x0"] = x0.cpu().numpy()
    out[key + "_xr"] = xr.cpu().numpy()
    out[key + "_u"] = u.cpu().numpy()
    out[key + "_info"] = info.cpu().numpy()
    print(key, "iters", info[:, _native.MPC_INFO_ITERATIONS].cpu().numpy(), flush=True)
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed(OUT, **out)

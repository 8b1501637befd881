"""Robustness census of the MPC kernel on the batches of tests/test_mpc.py::
test_gpu_many_problems_every_form: per shape, the problems that end non-OPTIMAL in the
many-problem form (one launch of 150) and the few-problem form (launches of <= 128), their info
records, and the oracle distance of the first few.  GPU only; honours DRCVAR_DIAG_LIB."""
import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import diaglib  # noqa: E402
diaglib.apply()  # DRCVAR_DIAG_LIB: a variant build (diagnostics)
import numpy as np, torch
import test_mpc as tm
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import _native
dev = torch.device("cuda", 0)
for dyn, H, O in [("double", 30, 3), ("double", 32, 6), ("double", 40, 4), ("single", 20, 5), ("generic1", 32, 4), ("generic3", 24, 3), ("generic4", 30, 4), ("generic8", 16, 3)]:
    rng = np.random.default_rng(H * 100 + O)
    Bn = 150
    base = tm._random_problem(rng, O, H, H, dyn)
    probs = []
    for _ in range(Bn):
        pr = dict(base)
        other = tm._random_problem(rng, O, H, H, "double" if dyn == "double" else "single")
        pr["x0"] = np.zeros_like(base["x0"]); pr["x0"][:2] = other["x0"][:2]
        pr["x_ref"] = np.zeros_like(base["x_ref"]); pr["x_ref"][:, :2] = other["x_ref"][:, :2]
        pr["hs"] = other["hs"]
        probs.append(pr)
    model = mf.MPCModel(base["A"], base["B"], base["C"], base["Q"], base["R"], H, base["ub"], base["pb"], device=dev)
    T_ = lambda a: torch.as_tensor(np.ascontiguousarray(a)).to(dev)
    hs = T_(np.stack([p["hs"] for p in probs]))
    args = lambda sl: (model, hs[sl, ..., 0:2], hs[sl, ..., 2], T_(np.stack([p["x0"] for p in probs[sl]])),
                       T_(np.stack([p["x_ref"] for p in probs[sl]])), T_(np.stack([p["u_ref"] for p in probs[sl]])))
    x, u, info = mf.filter_batch(*args(slice(0, Bn)))
    x1, u1, i1 = mf.filter_batch(*args(slice(0, 100)))
    x2, u2, i2 = mf.filter_batch(*args(slice(100, Bn)))
    info = info.cpu().numpy(); few = np.concatenate([i1.cpu().numpy(), i2.cpu().numpy()])
    u = u.cpu().numpy(); uf = np.concatenate([u1.cpu().numpy(), u2.cpu().numpy()])
    bad = np.nonzero(info[:, 0] != 0)[0]
    badf = np.nonzero(few[:, 0] != 0)[0]
    print(dyn, H, O, "counts", len(bad), len(badf), "many-form non-optimal:", bad, info[bad][:, :6] if len(bad) else "", "few-form non-optimal:", badf, "max|du|", np.abs(u - uf).max())
    for b in list(bad[:3]):
        xo, uo, io = tm._oracle(probs[b])
        print("  oracle", b, io["status"], "max|u-uo| many", np.abs(u[b] - uo).max(), "few", np.abs(uf[b] - uo).max())

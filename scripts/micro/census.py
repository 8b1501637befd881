"""Polish / status census of tests/test_mpc.py::test_gpu_many_problems_every_form's problem sets
(150 random problems per shape, both kernel forms) on the GPU: prints the polished fraction."""
import os
import sys

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import _native  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf  # noqa: E402
from test_mpc import _random_problem  # noqa: E402

dev = torch.device("cuda", 0)
SHAPES = [("double", 30, 3), ("double", 32, 6), ("double", 40, 4), ("single", 20, 5),
          ("generic1", 32, 4), ("generic3", 24, 3), ("generic4", 30, 4), ("generic8", 16, 3)]
if os.environ.get("CENSUS_MANY"):  # problems with >= 64 obstacles (the many-rows start and polish threshold)
    SHAPES = [("double", 30, 64), ("double", 40, 96), ("double", 20, 128), ("single", 30, 64)]
for dyn, H, O in SHAPES:
    rng = np.random.default_rng(H * 100 + O)
    Bn = 150
    base = _random_problem(rng, O, H, H, dyn)
    probs = []
    for _ in range(Bn):
        pr = dict(base)
        other = _random_problem(rng, O, H, H, "double" if dyn == "double" else "single")
        pr["x0"] = np.zeros_like(base["x0"])
        pr["x0"][:2] = other["x0"][:2]
        pr["x_ref"] = np.zeros_like(base["x_ref"])
        pr["x_ref"][:, :2] = other["x_ref"][:, :2]
        pr["hs"] = other["hs"]
        probs.append(pr)
    model = mf.MPCModel(base["A"], base["B"], base["C"], base["Q"], base["R"], H, base["ub"],
                        base["pb"], device=dev)
    T_ = lambda a: torch.as_tensor(np.ascontiguousarray(a)).to(dev)
    hs = T_(np.stack([p["hs"] for p in probs]))
    args = lambda sl: (model, hs[sl, ..., 0:2], hs[sl, ..., 2], T_(np.stack([p["x0"] for p in probs[sl]])),
                       T_(np.stack([p["x_ref"] for p in probs[sl]])), T_(np.stack([p["u_ref"] for p in probs[sl]])))
    many = mf.filter_batch(*args(slice(0, Bn)))[2].cpu().numpy()
    few = np.concatenate([mf.filter_batch(*args(sl))[2].cpu().numpy() for sl in (slice(0, 100), slice(100, Bn))])
    for name, info in (("many", many), ("few", few)):
        st = info[:, _native.MPC_INFO_STATUS]
        print(f"{dyn:9s} H={H} O={O} {name}: polished {np.mean(info[:, _native.MPC_INFO_POLISHED] == 1):.3f} "
              f"optimal {np.mean(st == 0):.3f} inaccurate {np.mean(st == 3):.3f} "
              f"iters {info[:, _native.MPC_INFO_ITERATIONS].mean():.1f}", flush=True)

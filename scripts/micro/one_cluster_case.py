"""One case of tests/test_mpc_cluster.py against DRCVAR_DIAG_LIB (a printf build traces it):
python scripts/micro/one_cluster_case.py dyn H O B tight"""
import os
import sys

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import diaglib  # noqa: E402
diaglib.apply()  # DRCVAR_DIAG_LIB: a variant build (diagnostics)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_mpc_cluster as t  # noqa: E402

dyn, H, O, B, tight = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5] == "1"
dev = torch.device("cuda", 0)
probs = t._batch(dyn, H, O, B, tight, seed=H * 1000 + O + B)
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf  # noqa: E402
for c in (0, 1):
    x, u, info, groups = t._solve(probs, dev, mf.make_options(cluster_size=c))
    torch.cuda.synchronize()
    for b, pr in enumerate(probs):
        xo, uo, io = t._oracle(pr)
        print(f"groups {groups} problem {b}: info {np.round(info[b], 10)} |u - oracle| {np.abs(u[b] - uo).max():.2e}",
              flush=True)

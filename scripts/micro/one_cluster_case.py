"""One case of tests/test_mpc_cluster.py against DRCVAR_DIAG_LIB (a printf build traces it):
python scripts/micro/one_cluster_case.py dyn H O B tight"""
import os
import sys

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_mpc_cluster as t  # noqa: E402

dyn, H, O, B, tight = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5] == "1"
dev = torch.device("cuda", 0)
probs = t._batch(dyn, H, O, B, tight, seed=H * 1000 + O + B)
for c in (None, "1"):
    if c is None:
        os.environ.pop("DRCVAR_MPC_CLUSTER", None)
    else:
        os.environ["DRCVAR_MPC_CLUSTER"] = c
    x, u, info, groups = t._solve(probs, dev)
    torch.cuda.synchronize()
    for b, pr in enumerate(probs):
        xo, uo, io = t._oracle(pr)
        print(f"groups {groups} problem {b}: info {np.round(info[b], 10)} |u - oracle| {np.abs(u[b] - uo).max():.2e}",
              flush=True)

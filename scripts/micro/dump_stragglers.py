"""Dump the slowest problems of scripts/mpc_bench.py's batch (H, O, B; problem b uses seed b) with
the kernel's answers and iteration counts: gpurun_out/stragglers.npz, for the CPU restatement
(scripts/micro/ipm_lab.py) and the oracle (oracle/mpc_qp.py).

    python scripts/micro/dump_stragglers.py [H,O,B] [min_iterations]
"""
import os
import sys

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "scripts"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import _native  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf  # noqa: E402
from mpc_bench import problem_batch  # noqa: E402

H, O, B = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "30,3,1024").split(","))
lim = int(sys.argv[2]) if len(sys.argv) > 2 else 11
dev = torch.device("cuda", 0)
model, rec, x0, xr, uf = problem_batch(H, O, B, dev)
h, g = rec[..., 3:5], rec[..., 7]
x, u, info = mf.filter_batch(model, h, g, x0, xr, uf)
torch.cuda.synchronize()
it = info[:, _native.MPC_INFO_ITERATIONS].cpu().numpy()
pa = info[:, _native.MPC_INFO_POLISH_ATTEMPTS].cpu().numpy()
sel = np.nonzero(it >= lim)[0]
print("iterations: mean", it.mean(), "max", it.max(), "selected", sel.tolist(), it[sel].tolist(),
      "polish attempts", pa[sel].tolist(), flush=True)
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed("gpurun_out/stragglers.npz", index=sel, h=h[sel].cpu().numpy(), g=g[sel].cpu().numpy(),
                    x0=x0[sel].cpu().numpy(), xr=xr[sel].cpu().numpy(), u=u[sel].cpu().numpy(),
                    info=info[sel].cpu().numpy(), iterations=it, polish_attempts=pa)

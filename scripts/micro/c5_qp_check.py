"""Re-solve a dumped QP hand-off problem (bench.py with DRCVAR_BENCH_DUMP_QP=<npz>) on the device
with several cluster sizes and both kernel forms, and print each answer's status, iterations,
polish attempts and max |u - u_bench|; saves the answers to <npz>.resolved.npz for the CPU
oracle / KKT check (scripts/micro/c5_qp_kkt.py)."""
import os
import sys

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import _native  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf  # noqa: E402

path = sys.argv[1]
z = np.load(path)
key = sorted(k[:-2] for k in z.files if k.endswith("_h"))[0]
dev = torch.device("cuda", 0)
dt = 0.2
A = np.block([[np.eye(2), dt * np.eye(2)], [np.zeros((2, 2)), np.eye(2)]])
Bm = np.block([[0.5 * dt ** 2 * np.eye(2)], [dt * np.eye(2)]])
C = np.block([np.eye(2), np.zeros((2, 2))])
h = torch.as_tensor(z[key + "_h"]).to(dev)
g = torch.as_tensor(z[key + "_g"]).to(dev)
x0 = torch.as_tensor(z[key + "_x0"]).to(dev)
xr = torch.as_tensor(z[key + "_xr"]).to(dev)
H = xr.shape[1] - 1
O = h.shape[0]
model = mf.MPCModel(A, Bm, C, 2 * np.eye(4), np.eye(2), H, (np.full(2, -5.0), np.full(2, 5.0)),
                    (np.full(2, -10.0), np.full(2, 10.0)), device=dev)
uf = torch.zeros((1, H, 2), dtype=torch.float64, device=dev)
u_bench = z[key + "_u"][0]
out = {}
for cs in (0, 1, 2, 4, 8, 16):
    opts = mf.make_options(cluster_size=cs) if cs else None
    x, u, info = mf.filter_batch(model, h, g, x0, xr, uf, options=opts)
    torch.cuda.synchronize()
    i = info[0].cpu().numpy()
    un = u[0].cpu().numpy()
    out[f"u_cs{cs}"] = un
    out[f"info_cs{cs}"] = i
    print(f"cluster {cs or 'auto'}: status {mf.STATUS_NAMES.get(int(i[_native.MPC_INFO_STATUS]))} "
          f"iterations {int(i[_native.MPC_INFO_ITERATIONS])} polished {int(i[_native.MPC_INFO_POLISHED])} "
          f"attempts {int(i[_native.MPC_INFO_POLISH_ATTEMPTS])} max|u - u_bench| {np.abs(un - u_bench).max():.3e}",
          flush=True)
np.savez_compressed(path + ".resolved.npz", **out)

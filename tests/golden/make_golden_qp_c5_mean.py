"""Writes tests/golden/qp_c5_mean.npz: the MEAN-metric safety filter of bench.py's main_flow_c5
(main.py:104-112's first filter at C5 size: 256 obstacles x 50 steps of device-computed halfspaces,
columns 0..2 of the record = MeanSafeHalfspace, core/halfspaces.py:70-106; H = 50, the
straight-line ego reference, input bounds +-5, position bounds +-10), dumped on the GPU box by
scripts/micro/dump_main_flow_qps.py, with the oracle's KKT-certified answer.  The slowest of the
three filters (15 interior-point iterations at the end of round 5 against 10 for CVaR / DR-CVaR),
kept as a fixture for the start / polish work on it.  Run once; output committed.

    python tests/golden/make_golden_qp_c5_mean.py gpurun_out/main_flow_c5.npz
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from oracle import mpc_qp  # noqa: E402


def main(src):
    z = np.load(src)
    rec = z["records"]                                  # [256, 50, 8]
    h, g = rec[..., 0:2], rec[..., 2]                   # the mean halfspace (DRCVAR_COL_MEAN_*)
    x0, xr = z["x0"], z["x_ref"]
    dt = 0.2
    A = np.block([[np.eye(2), dt * np.eye(2)], [np.zeros((2, 2)), np.eye(2)]])
    B = np.block([[0.5 * dt ** 2 * np.eye(2)], [dt * np.eye(2)]])
    C = np.block([np.eye(2), np.zeros((2, 2))])
    H = xr.shape[0] - 1
    ub, pb = (np.full(2, -5.0), np.full(2, 5.0)), (np.full(2, -10.0), np.full(2, 10.0))
    rows = [np.concatenate([h[:, t], g[:, t, None]], -1) for t in range(H)]
    x, u, info = mpc_qp.filter_trajectory(A, B, C, 2 * np.eye(4), np.eye(2), H, x0, xr, None, rows, ub, pb)
    assert info["status"] == "optimal" and max(info["kkt"].values()) < 1e-10, info
    kernel = z["mean_info"]
    out = os.path.join(REPO, "tests", "golden", "qp_c5_mean.npz")
    np.savez_compressed(out, h=np.ascontiguousarray(h), g=np.ascontiguousarray(g), x0=x0, x_ref=xr,
                        u_bounds=np.stack(ub), p_bounds=np.stack(pb), u_expected=u, x_expected=x,
                        objective=np.float64(info["objective"]),
                        kernel_iterations_r05=np.float64(kernel[1]))
    print(out, "oracle iterations", info["iterations"], info["kkt"], "kernel", kernel[:3],
          "|u_kernel - u_oracle|", float(np.abs(z["mean_u"] - u).max()))


if __name__ == "__main__":
    main(sys.argv[1])

"""Writes tests/golden/qp_h30_straggler.npz: problem 13 of scripts/mpc_bench.py's 30,3,1024 batch
(3 obstacles x 30 steps of device-computed DR-CVaR halfspaces, problem b drawn with seed b; the
straight-line ego reference, input bounds +-5, position bounds +-10), the slowest problem of that
batch (20 interior-point iterations against a mean of 5.3: weakly active halfspace rows of obstacle
0 at steps 14-16, w_hs and lambda_hs both heading to zero, make the Mehrotra steps alternate long and
short), dumped on the GPU box by ``python scripts/micro/dump_stragglers.py 30,3,1024 11``, with the
oracle's KKT-certified answer.  Run once; output committed.

    python tests/golden/make_golden_qp_straggler.py gpurun_out/stragglers.npz
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from oracle import mpc_qp  # noqa: E402

PROBLEM = 13


def main(src):
    z = np.load(src)
    b = list(z["index"]).index(PROBLEM)
    h, g, x0, xr = z["h"][b], z["g"][b], z["x0"][b], z["xr"][b]
    dt = 0.2
    A = np.block([[np.eye(2), dt * np.eye(2)], [np.zeros((2, 2)), np.eye(2)]])
    B = np.block([[0.5 * dt ** 2 * np.eye(2)], [dt * np.eye(2)]])
    C = np.block([np.eye(2), np.zeros((2, 2))])
    H = xr.shape[0] - 1
    ub, pb = (np.full(2, -5.0), np.full(2, 5.0)), (np.full(2, -10.0), np.full(2, 10.0))
    rows = [np.concatenate([h[:, t], g[:, t, None]], -1) for t in range(H)]
    x, u, info = mpc_qp.filter_trajectory(A, B, C, 2 * np.eye(4), np.eye(2), H, x0, xr, None, rows, ub, pb)
    assert info["status"] == "optimal" and max(info["kkt"].values()) < 1e-9, info
    out = os.path.join(REPO, "tests", "golden", "qp_h30_straggler.npz")
    np.savez_compressed(out, h=h, g=g, x0=x0, x_ref=xr, u_bounds=np.stack(ub), p_bounds=np.stack(pb),
                        u_expected=u, x_expected=x, objective=np.float64(info["objective"]),
                        kernel_iterations=np.float64(z["info"][b, 1]))
    print(out, info["iterations"], info["polished"], info["kkt"], "kernel u error",
          np.abs(z["u"][b] - u).max())


if __name__ == "__main__":
    main(sys.argv[1])

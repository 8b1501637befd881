"""Writes tests/golden/qp_c5_degenerate.npz: bench.py's C5 QP hand-off problem (256 obstacles x
50 steps of device-computed DR-CVaR halfspaces from the round-3 device sampler, H = 50, the
straight-line ego reference, input bounds +-5, position bounds +-10), dumped on the GPU box by
``DRCVAR_BENCH_DUMP_QP=gpurun_out/c5qp.npz python bench.py`` (scripts/micro/gpu_c5qp.sh), with the
oracle's answer.  On this instance the oracle's interior-point method stalls at merit ~4e-10 and
its three guessed active sets all fail; the answer comes from its one-row-per-step active-set
refinement (oracle/mpc_qp.py:_polish_steps), KKT-certified to ~1e-13.  Run once; output committed.

    python tests/golden/make_golden_qp_c5.py gpurun_out/c5qp.npz
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from oracle import mpc_qp  # noqa: E402


def main(src):
    z = np.load(src)
    key = sorted(k[:-2] for k in z.files if k.endswith("_h"))[0]
    h, g = z[key + "_h"][0], z[key + "_g"][0]
    x0, xr = z[key + "_x0"][0], z[key + "_xr"][0]
    dt = 0.2
    A = np.block([[np.eye(2), dt * np.eye(2)], [np.zeros((2, 2)), np.eye(2)]])
    B = np.block([[0.5 * dt ** 2 * np.eye(2)], [dt * np.eye(2)]])
    C = np.block([np.eye(2), np.zeros((2, 2))])
    H = xr.shape[0] - 1
    ub, pb = (np.full(2, -5.0), np.full(2, 5.0)), (np.full(2, -10.0), np.full(2, 10.0))
    rows = [np.concatenate([h[:, t], g[:, t, None]], -1) for t in range(H)]
    x, u, info = mpc_qp.filter_trajectory(A, B, C, 2 * np.eye(4), np.eye(2), H, x0, xr, None, rows, ub, pb)
    assert info["status"] == "optimal" and info["polished"] and max(info["kkt"].values()) < 1e-10, info
    out = os.path.join(REPO, "tests", "golden", "qp_c5_degenerate.npz")
    np.savez_compressed(out, h=h, g=g, x0=x0, x_ref=xr, u_bounds=np.stack(ub), p_bounds=np.stack(pb),
                        u_expected=u, x_expected=x, objective=np.float64(info["objective"]))
    print(out, info["iterations"], info["kkt"])


if __name__ == "__main__":
    main(sys.argv[1])

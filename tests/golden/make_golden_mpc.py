"""Generate the MPC hand-off golden vectors tests/golden/mpc_*.npz (build container only).

    python tests/golden/make_golden_mpc.py [--reference /root/reference]

The safety-filter QP of ``core/mpc_filter.py:40-178`` is set up exactly as ``main.py:43-115`` does:
dynamics from the reference's own ``core/dynamics.py:7-33`` ``create_double_integrator_matrices``
(imported read-only, bytecode writing disabled), ``Q = 2 I``, ``R = I`` (``config/parameters.py:20-21``),
input bounds +-5 and position bounds ``state_bounds[:2]`` (+-10, truncated to C's rows as
``mpc_filter.py:103-110`` does), ``HORIZON = 30``; ``x_ref`` / ``u_ref`` restate
``simulation/planner.py:120-197`` (that module imports cvxpy, absent here); the halfspaces are the
``expected`` records of the existing halfspace fixtures (mean / cvar / dr_cvar columns, the objects
``get_constraint_params`` returns, ``core/halfspaces.py:56-64``).

The reference solves with CVXPY's default QP solver (OSQP, not installed); the expected (x, u) are
the unique optimum computed by ``oracle/mpc_qp.py`` (full-space IPM + active-set polish) and every
case is written only with its KKT certificate below 1e-8.  Each file holds A, B, C, Q, R, horizon,
x0, x_ref, u_ref, u_bounds [2, nu], p_bounds [2, 2], hs [3 metrics, O, T, 3] (h0, h1, g),
x_expected / u_expected [3, ...], objective [3] and meta (JSON).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import mpc_qp  # noqa: E402

METRICS = (("mean", (0, 1, 2)), ("cvar", (3, 4, 5)), ("dr_cvar", (3, 4, 7)))


def straight_line(A, B, start, goal, horizon, dt, velocity=1.5):
    """x_ref / u_ref of ``ReferenceTrajectoryPlanner.straight_line_trajectory`` (planner.py:120-197)."""
    nx = A.shape[0]
    direction = goal - start
    distance = np.linalg.norm(direction)
    direction = direction / distance
    n_steps = int((distance / velocity) / dt)
    x_ref = np.zeros((horizon + 1, nx))
    x_ref[0, :2] = start
    for t in range(1, horizon + 1):
        if t <= n_steps:
            x_ref[t, :2] = start + (t / n_steps) * (goal - start)
            x_ref[t, 2:] = velocity * direction
        else:
            x_ref[t, :2] = goal
    u_ref = np.array([np.linalg.pinv(B) @ (x_ref[t + 1] - A @ x_ref[t]) for t in range(horizon)])
    return x_ref, u_ref


def make_case(name, halfspace_fixture, start, goal, dynamics, horizon=30, dt=0.2):
    A, B, C = dynamics.create_double_integrator_matrices(dt)
    Q, R = 2.0 * np.eye(4), np.eye(2)
    ub = np.array([[-5.0, -5.0], [5.0, 5.0]])
    pb = np.array([[-10.0, -10.0], [10.0, 10.0]])
    rec = np.load(os.path.join(HERE, halfspace_fixture), allow_pickle=False)["expected"]
    x0 = np.zeros(4)
    x0[:2] = start
    x_ref, u_ref = straight_line(A, B, np.asarray(start, float), np.asarray(goal, float), horizon, dt)
    hs = np.stack([rec[..., list(cols)] for _, cols in METRICS])          # [3, O, T, 3]
    xs, us, objs, kkts = [], [], [], []
    for m, (metric, _) in enumerate(METRICS):
        rows = [hs[m][:, t] for t in range(hs.shape[2])]
        x, u, info = mpc_qp.filter_trajectory(A, B, C, Q, R, horizon, x0, x_ref, u_ref, rows,
                                              (ub[0], ub[1]), (pb[0], pb[1]))
        assert info["status"] == "optimal", (name, metric, info["status"])
        worst = max(info["kkt"].values())
        assert worst < 1e-8, (name, metric, info["kkt"])
        xs.append(x)
        us.append(u)
        objs.append(info["objective"])
        kkts.append(worst)
    meta = {"source": "reference dynamics + main.py setup; oracle/mpc_qp.py (polished IPM)",
            "halfspaces": halfspace_fixture, "horizon": horizon, "metrics": [m for m, _ in METRICS],
            "kkt_max": kkts}
    np.savez(os.path.join(HERE, f"{name}.npz"), A=A, B=B, C=C, Q=Q, R=R,
             horizon=np.int64(horizon), x0=x0, x_ref=x_ref, u_ref=u_ref, u_bounds=ub, p_bounds=pb,
             hs=hs, x_expected=np.stack(xs), u_expected=np.stack(us), objective=np.array(objs),
             meta=json.dumps(meta))
    print(name, "objectives", objs, "kkt", kkts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    sys.dont_write_bytecode = True
    sys.path.insert(0, args.reference)
    from core import dynamics  # reference core/dynamics.py (numpy only)
    make_case("mpc_multi_obstacle_h30", "multi_obstacle_n20_h30.npz", [-2.0, -1.0], [4.0, 0.0],
              dynamics)
    make_case("mpc_head_on_h30", "head_on_n100_t20.npz", [-4.0, 0.0], [4.0, 0.0], dynamics)


if __name__ == "__main__":
    main()

"""Generate the golden vectors under tests/golden/ (run in the build container only).

    python tests/golden/make_golden.py [--reference /root/reference]

What is taken from the reference, and how:

* Inputs come from the reference's OWN generators, imported read-only from ``/root/reference``
  (bytecode writing disabled): ``simulation/obstacles.py:115-197`` ``generate_obstacle_scenarios``
  seeded with ``np.random.seed(42)`` exactly as ``main.py:191``, scenarios from
  ``config/scenarios.py:11-68``, constants from ``config/parameters.py:11-33``.
* ``simulation/planner.py`` imports cvxpy at module level (absent here), so its straight-line
  ego reference (``simulation/planner.py:120-197``) is restated below; the timing-analysis sampler
  (``evaluation/timing_analysis.py:56-70``, also behind a cvxpy import) likewise.
* Expected separating vectors come from the reference's ``core/geometry.py:35-53``
  ``compute_separating_vector`` (imported).  Expected CVaR / DR-CVaR offsets are the optimum of the
  reference's LP rows (``core/risk_metrics.py:87-125,182-213``, written out in
  ``oracle/lp_highs.py``) solved by HiGHS in place of ECOS; the mean-halfspace offset restates
  ``core/halfspaces.py:94``.  Every expected value is cross-checked against the closed form
  (``oracle/closed_form.py``) to 1e-9 before it is written.

Each ``.npz`` holds: ``samples`` [O,T,N,2], ``ego`` [T,2], ``params`` [robot_radius,
obstacle_radius, alpha, delta, epsilon], ``expected`` [O,T,8] (columns of
``oracle.closed_form.COLS``) and ``meta`` (a JSON string).  Nothing here travels to the GPU box
except the ``.npz`` data.
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

from oracle import closed_form as cf  # noqa: E402
from oracle import lp_highs  # noqa: E402


def straight_line_ego(start, goal, horizon, dt, velocity=1.5):
    """Positions of ``ReferenceTrajectoryPlanner.straight_line_trajectory`` (planner.py:120-197),
    i.e. ``C @ x_ref[t]`` for t = 0..horizon."""
    start = np.asarray(start, dtype=np.float64)
    goal = np.asarray(goal, dtype=np.float64)
    direction = goal - start
    distance = np.linalg.norm(direction)
    pos = np.zeros((horizon + 1, 2))
    if distance < 1e-10:
        pos[:] = start
        return pos
    n_steps = int((distance / velocity) / dt)
    pos[0] = start
    for t in range(1, horizon + 1):
        if t <= n_steps:
            pos[t] = start + (t / n_steps) * (goal - start)
        else:
            pos[t] = goal
    return pos


def expected_outputs(samples, ego, rr, ro, alpha, delta, eps, geometry):
    O, T, N, _ = samples.shape
    out = np.empty((O, T, 8))
    rc = rr + ro
    for o in range(O):
        for t in range(T):
            s = samples[o, t]
            mu = np.mean(s, axis=0)
            hm = geometry.compute_separating_vector(np.zeros(2), mu)
            out[o, t, 0:2] = hm
            out[o, t, 2] = -(np.dot(hm, mu) - rc * np.linalg.norm(hm))
            h = geometry.compute_separating_vector(ego[t], mu)
            out[o, t, 3:5] = h
            out[o, t, 5] = lp_highs.solve_cvar_lp(s, h, alpha, delta, rr, ro)
            out[o, t, 6:8] = lp_highs.solve_dr_cvar_lp(s, h, alpha, delta, eps, rr, ro)
    closed = cf.safe_halfspaces(samples, ego, rr, ro, alpha, delta, eps)
    err = np.nanmax(np.abs(closed - out))
    assert err < 1e-9, f"closed form disagrees with the LP restatement: {err}"
    return out, float(err)


def save(name, samples, ego, params, expected, meta):
    path = os.path.join(HERE, name + ".npz")
    np.savez(path, samples=samples, ego=ego, params=np.asarray(params, dtype=np.float64),
             expected=expected, meta=np.asarray(json.dumps(meta)))
    print(f"wrote {path}: samples {samples.shape}, max|closed-LP| {meta['closed_vs_lp']:.2e}")


def scenario_case(name, scenario, n_samples, horizon, keep_steps, ref):
    from config import parameters as P
    from config.scenarios import get_scenario_config
    from core import geometry
    from simulation.obstacles import generate_obstacle_scenarios

    np.random.seed(42)                                               # main.py:191
    cfg = get_scenario_config(scenario)
    data = generate_obstacle_scenarios(cfg, P.SIM_TIME, P.DT, n_samples)   # main.py:61
    ego_all = straight_line_ego(cfg["ego_start"], cfg["ego_goal"], horizon, P.DT)  # main.py:83
    n_steps = min(len(ego_all), horizon)                             # environment.py:72
    T = min(n_steps, keep_steps)
    # environment.py:88 slices traj_i[:, t, :]; pack to [O, T, N, 2]
    samples = np.stack([np.transpose(tr[:, :T, :], (1, 0, 2)) for tr in data["sample_trajectories"]])
    samples = np.ascontiguousarray(samples)
    ego = np.ascontiguousarray(ego_all[:T])
    params = (P.ROBOT_RADIUS, P.OBSTACLE_RADIUS, P.ALPHA, P.DELTA, P.EPSILON)
    expected, err = expected_outputs(samples, ego, *params, geometry)
    meta = dict(source="reference generators (seed 42) + HiGHS on reference LP rows",
                scenario=scenario, n_samples=n_samples, horizon=horizon, steps_kept=T,
                closed_vs_lp=err)
    save(name, samples, ego, params, expected, meta)


def timing_analysis_case(ref):
    """evaluation/timing_analysis.py:51-104: per-element normal draws, ego (0,0), seed 42."""
    from config import parameters as P
    from core import geometry

    np.random.seed(42)
    units = []
    sizes = [10, 50, 100]
    for n in sizes:
        for _run in range(3):
            s = np.zeros((n, 2))
            for i in range(n):                                       # timing_analysis.py:65-68
                s[i, 0] = np.random.normal(0.5, 0.1)
                s[i, 1] = np.random.normal(0.0, 0.1)
            units.append(s)
    params = (P.ROBOT_RADIUS, P.OBSTACLE_RADIUS, P.ALPHA, P.DELTA, P.EPSILON)
    for n in sizes:
        batch = np.stack([u for u in units if u.shape[0] == n])[:, None]     # [runs, 1, n, 2]
        ego = np.zeros((1, 2))
        expected, err = expected_outputs(batch, ego, *params, geometry)
        meta = dict(source="timing_analysis sampler restated (seed 42) + HiGHS on reference LP rows",
                    n_samples=n, runs=batch.shape[0], closed_vs_lp=err)
        save(f"timing_analysis_n{n}", batch, ego, params, expected, meta)


def edge_cases(ref):
    """Small hand-built units for the branches the reference's LPs take on unusual data."""
    from core import geometry

    rng = np.random.RandomState(7)
    rr, ro = 0.3, 0.3
    cases = {}
    # fractional k = alpha*N (N=37 -> 7.4), ties, zero variance, degenerate directions, N=1..3
    base = rng.normal(size=(37, 2)) * 0.2 + np.array([1.0, -0.5])
    cases["fractional_k"] = (base[None, None], np.array([[0.0, 0.0]]), 0.2)
    ties = np.round(rng.normal(size=(64, 2)), 1)
    cases["ties"] = (ties[None, None], np.array([[0.3, -0.2]]), 0.25)
    zero_var = np.tile(np.array([[2.0, 1.0]]), (50, 1))
    cases["zero_variance"] = (zero_var[None, None], np.array([[0.0, 0.0]]), 0.2)
    mean_at_ego = rng.normal(size=(40, 2)) * 0.1
    mean_at_ego -= mean_at_ego.mean(axis=0)
    mean_at_ego += np.array([1.0, 2.0])
    ego_eq = np.array([[mean_at_ego[:, 0].mean(), mean_at_ego[:, 1].mean()]])
    cases["degenerate_h"] = (mean_at_ego[None, None], ego_eq, 0.2)
    at_origin = rng.normal(size=(30, 2)) * 0.1
    at_origin -= at_origin.mean(axis=0)
    cases["mean_at_origin"] = (at_origin[None, None], np.array([[1.0, 1.0]]), 0.2)
    for n in (1, 2, 3):
        cases[f"n{n}"] = (rng.normal(size=(1, 1, n, 2)), np.array([[-1.0, 0.5]]), 0.2)
    cases["alpha_one"] = (rng.normal(size=(1, 1, 25, 2)), np.array([[0.0, 0.0]]), 1.0)
    cases["alpha_small"] = (rng.normal(size=(1, 1, 25, 2)), np.array([[0.0, 0.0]]), 0.01)
    cases["alpha_gt_one"] = (rng.normal(size=(1, 1, 25, 2)), np.array([[0.0, 0.0]]), 1.5)
    for name, (s, ego, alpha) in cases.items():
        params = (rr, ro, alpha, 0.1, 0.15)
        expected, err = expected_outputs(np.ascontiguousarray(s), ego, *params, geometry)
        meta = dict(source="hand-built edge case + HiGHS on reference LP rows", case=name,
                    closed_vs_lp=err)
        save(f"edge_{name}", np.ascontiguousarray(s), ego, params, expected, meta)
    # epsilon < 0: DR LP unbounded -> sentinel; CVaR unaffected
    s = rng.normal(size=(1, 1, 30, 2))
    ego = np.array([[0.0, 0.0]])
    params = (rr, ro, 0.2, 0.1, -0.05)
    expected, err = expected_outputs(s, ego, *params, geometry)
    save("edge_negative_epsilon", s, ego, params, expected,
         dict(source="hand-built edge case + HiGHS on reference LP rows", case="negative_epsilon",
              closed_vs_lp=err))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    sys.dont_write_bytecode = True
    sys.path.insert(0, args.reference)
    scenario_case("head_on_n100_t20", "head_on", 100, 20, 20, args.reference)
    scenario_case("multi_obstacle_n1000_t8", "multi_obstacle", 1000, 20, 8, args.reference)
    scenario_case("multi_obstacle_n20_h30", "multi_obstacle", 20, 30, 30, args.reference)
    timing_analysis_case(args.reference)
    edge_cases(args.reference)


if __name__ == "__main__":
    main()

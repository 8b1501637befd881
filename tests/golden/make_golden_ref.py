"""Golden vectors produced by the REFERENCE's OWN orchestration code (run in the build container only).

    python tests/golden/make_golden_ref.py [--reference /root/reference]

SURVEY.md §8(c)(3) / VERDICT r1 "What's missing" #1.  The reference's hot-path modules are pure
Python but import ``cvxpy`` at module level, which this image lacks (an ordinary
``ModuleNotFoundError``, not a denial).  So:

* ``sys.modules['cvxpy']`` is a ``MagicMock`` stub — the reference only touches ``cp.*`` inside the
  two optimiser classes (``core/risk_metrics.py:84-265``), the CVXPY planner
  (``simulation/planner.py:36-118``, never called here) and the MPC filter (not imported);
* ``core.risk_metrics.DRCVaROptimizer`` / ``CVaROptimizer`` are replaced by HiGHS-backed classes
  with the same constructor (``alpha, [epsilon,] delta, max_samples``) and the same
  ``solve(h, samples, combined_radius) -> (solved, g, info)`` contract.  They solve exactly the
  reference's LP rows on exactly the parameters the reference sets (``h_xi = h @ samples.T`` and
  ``r = combined_radius`` (DR, :145-146) or ``combined_radius * |h|`` (CVaR, :233-234)) and call
  the reference's own ``save_timing_info`` (:16-33).  The LP solve is the ONLY restated piece.

Everything else runs as the reference's code: the wrappers ``dr_cvar_halfspace`` /
``cvar_halfspace`` (:267-338, singletons keyed on N, radius conventions, sentinels),
``MeanSafeHalfspace`` / ``CVaRSafeHalfspace`` / ``DRCVaRSafeHalfspace.create`` and
``compute_safe_halfspaces`` (``core/halfspaces.py:70-248``), ``compute_separating_vector``
(``core/geometry.py:35-53``), ``SafetyFilteringEnvironment.compute_safe_halfspaces_for_trajectory``
(``simulation/environment.py:60-106``), ``ReferenceTrajectoryPlanner.straight_line_trajectory``
(``simulation/planner.py:120-197``), ``generate_obstacle_scenarios`` (``simulation/obstacles.py``),
and for the timing-analysis vectors ``analyze_dr_cvar_computation_time``
(``evaluation/timing_analysis.py:13-132``) itself, whose ``create()`` calls are recorded.

Column 6 (``g_dr_star``, which ``SafeHalfspace`` does not keep) is the first return value of the
reference's ``dr_cvar_halfspace`` from the very call ``DRCVaRSafeHalfspace.create`` makes
(recorded by wrapping it).  Every vector is cross-checked against the closed form
(``oracle/closed_form.py``) and against the previous restated fixture before it is written; the
meta records both differences.  ``singleton_session.npz`` records a call sequence that exercises
the N-keyed singletons (``core/risk_metrics.py:289,325``).  Only the ``.npz`` data travels.
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import os
import sys
import tempfile
import time
from unittest import mock

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import closed_form as cf  # noqa: E402
from oracle import lp_highs  # noqa: E402

SOURCE = ("reference orchestration imported from /root/reference (cvxpy stubbed); LP rows of "
          "core/risk_metrics.py solved by HiGHS in place of ECOS")


def load_reference(path):
    """Import the reference's modules with cvxpy stubbed and the two LP optimisers swapped."""
    sys.dont_write_bytecode = True
    sys.modules.setdefault("cvxpy", mock.MagicMock(name="cvxpy-stub"))
    sys.path.insert(0, path)
    import matplotlib
    matplotlib.use("Agg")
    import core.risk_metrics as rm

    class HighsDRCVaROptimizer:
        """``DRCVaROptimizer`` (:84-177) with the LP handed to HiGHS."""

        def __init__(self, alpha, epsilon, delta, max_samples):
            self.alpha, self.epsilon, self.delta, self.n_samples = alpha, epsilon, delta, max_samples

        def solve(self, h, samples, combined_radius):
            t0 = time.time()
            h_xi = h @ samples.T                                      # :145
            r = float(np.asarray([combined_radius]).reshape(-1)[0])   # :146
            t1 = time.time()
            ok, g = lp_highs.dr_cvar_lp(h_xi, r, self.alpha, self.delta, self.epsilon)
            t2 = time.time()
            info = {"setup_time": t1 - t0, "solve_time": t2 - t1, "solve_call_time": t2 - t0}
            rm.save_timing_info("drcvar", t1 - t0, t2 - t1)
            return (True, g, info) if ok else (False, 100.0, info)

    class HighsCVaROptimizer:
        """``CVaROptimizer`` (:179-265) with the LP handed to HiGHS."""

        def __init__(self, alpha, delta, max_samples):
            self.alpha, self.delta, self.n_samples = alpha, delta, max_samples

        def solve(self, h, samples, combined_radius):
            t0 = time.time()
            h_xi = h @ samples.T                                      # :233
            r = combined_radius * np.linalg.norm(h)                   # :234
            t1 = time.time()
            ok, g = lp_highs.cvar_lp(h_xi, r, self.alpha, self.delta)
            t2 = time.time()
            info = {"setup_time": t1 - t0, "solve_time": t2 - t1, "solve_call_time": t2 - t0}
            rm.save_timing_info("cvar", t1 - t0, t2 - t1)
            return (True, g, info) if ok else (False, 100.0, info)

    rm.DRCVaROptimizer = HighsDRCVaROptimizer
    rm.CVaROptimizer = HighsCVaROptimizer
    import core.halfspaces as hs
    recorded = []
    inner = hs.dr_cvar_halfspace

    def recording_dr(*a, **k):                 # keep g* of the call create() makes (:178)
        res = inner(*a, **k)
        recorded.append(res)
        return res
    hs.dr_cvar_halfspace = recording_dr
    return rm, hs, recorded


def reset_singletons(rm):
    rm.drcvar_optimizer = None
    rm.cvar_optimizer = None


def record_of(mean, cvar, dr, g_star):
    """The build's 8-column record from the reference's three SafeHalfspace objects."""
    return np.array([mean.h[0], mean.h[1], mean.g_tilde, dr.h[0], dr.h[1], cvar.g_tilde, g_star,
                     dr.g_tilde], dtype=np.float64), (np.asarray(cvar.h) - np.asarray(dr.h))


def check_and_save(name, samples, ego, params, expected, meta):
    closed = cf.safe_halfspaces(samples, ego, *params)
    d_closed = float(np.nanmax(np.abs(closed - expected)))
    assert d_closed < 1e-9, f"{name}: closed form vs reference orchestration {d_closed}"
    meta = dict(meta, source=SOURCE, closed_vs_ref=d_closed)
    path = os.path.join(HERE, name + ".npz")
    if os.path.exists(path):
        old = np.load(path, allow_pickle=False)
        if old["samples"].shape == samples.shape and np.array_equal(old["samples"], samples):
            meta["previous_restated_fixture_vs_ref"] = float(np.nanmax(np.abs(old["expected"] - expected)))
    np.savez(path, samples=samples, ego=ego, params=np.asarray(params, dtype=np.float64),
             expected=expected, meta=np.asarray(json.dumps(meta)))
    print(f"wrote {path}: {samples.shape} |closed-ref| {d_closed:.1e} "
          f"|old-ref| {meta.get('previous_restated_fixture_vs_ref', float('nan')):.1e}")


def environment_case(name, scenario, n_samples, planner_horizon, env_horizon, rm, recorded):
    """main.py:38-97 up to the halfspaces, with the reference's classes."""
    from config import parameters as P
    from config.scenarios import get_scenario_config
    from core.dynamics import create_double_integrator_matrices
    from simulation.environment import SafetyFilteringEnvironment
    from simulation.obstacles import generate_obstacle_scenarios
    from simulation.planner import ReferenceTrajectoryPlanner

    reset_singletons(rm)
    np.random.seed(42)                                                    # main.py:191
    cfg = get_scenario_config(scenario)
    env = SafetyFilteringEnvironment(ROBOT_RADIUS=P.ROBOT_RADIUS, OBSTACLE_RADIUS=P.OBSTACLE_RADIUS,
                                     HORIZON=env_horizon, DT=P.DT, ALPHA=P.ALPHA, DELTA=P.DELTA,
                                     EPSILON=P.EPSILON)
    A, B, C = create_double_integrator_matrices(P.DT)
    data = generate_obstacle_scenarios(cfg, P.SIM_TIME, P.DT, n_samples)   # main.py:61
    planner = ReferenceTrajectoryPlanner(A, B, C, P.Q_WEIGHT * np.eye(4), P.R_WEIGHT * np.eye(2),
                                         planner_horizon, P.DT)
    x_ref, _, _ = planner.straight_line_trajectory(cfg["ego_start"], cfg["ego_goal"])
    recorded.clear()
    with contextlib.redirect_stdout(io.StringIO()):
        out = env.compute_safe_halfspaces_for_trajectory(data["sample_trajectories"], x_ref)
    T = len(out["dr_cvar"])
    O = len(data["sample_trajectories"])
    expected = np.empty((O, T, 8))
    k = 0
    for t in range(T):                       # call order: t outer, obstacle inner (:82, :225)
        for o in range(O):
            expected[o, t], dh = record_of(out["mean"][t][o], out["cvar"][t][o], out["dr_cvar"][t][o],
                                           recorded[k][0])
            assert not np.any(dh)
            k += 1
    samples = np.ascontiguousarray(np.stack([np.transpose(tr[:, :T, :], (1, 0, 2))
                                             for tr in data["sample_trajectories"]]))
    ego = np.ascontiguousarray((C @ x_ref[:T].T).T)                      # environment.py:92
    params = (P.ROBOT_RADIUS, P.OBSTACLE_RADIUS, P.ALPHA, P.DELTA, P.EPSILON)
    check_and_save(name, samples, ego, params, expected,
                   dict(scenario=scenario, n_samples=n_samples, horizon=env_horizon,
                        planner_horizon=planner_horizon, steps_kept=T,
                        route="SafetyFilteringEnvironment.compute_safe_halfspaces_for_trajectory"))


def timing_analysis_cases(rm, hs):
    """evaluation/timing_analysis.py:13-132 run as-is (sizes 10/50/100, 3 runs, seed 42); every
    create() call's samples and result recorded."""
    import evaluation.timing_analysis as ta
    from config import parameters as P

    calls = {"dr": [], "cvar": []}
    dr_create, cvar_create = hs.DRCVaRSafeHalfspace.create, hs.CVaRSafeHalfspace.create

    def rec_dr(samples, ego, *a, **k):
        r = dr_create(samples, ego, *a, **k)
        calls["dr"].append((np.array(samples), np.array(ego), r))
        return r

    def rec_cvar(samples, ego, *a, **k):
        r = cvar_create(samples, ego, *a, **k)
        calls["cvar"].append((np.array(samples), r))
        return r
    reset_singletons(rm)
    np.random.seed(42)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp, \
            mock.patch.object(hs.DRCVaRSafeHalfspace, "create", staticmethod(rec_dr)), \
            mock.patch.object(hs.CVaRSafeHalfspace, "create", staticmethod(rec_cvar)), \
            mock.patch.object(ta, "plot_timing_results", lambda *a, **k: None), \
            contextlib.redirect_stdout(io.StringIO()):
        os.chdir(tmp)
        try:
            ta.analyze_dr_cvar_computation_time(sample_sizes=[10, 50, 100], n_runs=3, save_dir=tmp)
        finally:
            os.chdir(cwd)
    params = (P.ROBOT_RADIUS, P.OBSTACLE_RADIUS, P.ALPHA, P.DELTA, P.EPSILON)
    rc = P.ROBOT_RADIUS + P.OBSTACLE_RADIUS
    for n in (10, 50, 100):
        sel = [i for i, (s, _, _) in enumerate(calls["dr"]) if s.shape[0] == n]
        batch = np.stack([calls["dr"][i][0] for i in sel])[:, None]       # [runs, 1, n, 2]
        ego = calls["dr"][sel[0]][1].reshape(1, 2)
        expected = np.empty((len(sel), 1, 8))
        for j, i in enumerate(sel):
            s, _, dr = calls["dr"][i]
            cs, cv = calls["cvar"][i]
            assert np.array_equal(cs, s)
            mean = hs.MeanSafeHalfspace.create(s, P.ROBOT_RADIUS, P.OBSTACLE_RADIUS)
            g_star = dr.g_tilde + rc * np.linalg.norm(dr.h)   # not kept by create(): g~ + R_c|h| (:299)
            expected[j, 0], _ = record_of(mean, cv, dr, g_star)
        check_and_save(f"timing_analysis_n{n}", np.ascontiguousarray(batch), ego, params, expected,
                       dict(n_samples=n, runs=len(sel),
                            route="evaluation.timing_analysis.analyze_dr_cvar_computation_time "
                                  "(create() calls recorded); col 6 = g~ + R_c|h|"))


def edge_cases(rm, hs):
    """The hand-built edge units (same data as make_golden.py) through the reference's
    compute_safe_halfspaces, singletons reset before each case (alpha differs between cases)."""
    path_cases = sorted(f for f in os.listdir(HERE) if f.startswith("edge_") and f.endswith(".npz"))
    for f in path_cases:
        z = np.load(os.path.join(HERE, f), allow_pickle=False)
        s, ego, p = z["samples"], z["ego"], z["params"]
        rr, ro, alpha, delta, eps = (float(v) for v in p)
        reset_singletons(rm)
        rec = []
        hs.dr_cvar_halfspace, inner = (lambda *a, **k: rec.append(inner(*a, **k)) or rec[-1]), hs.dr_cvar_halfspace
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                out = hs.compute_safe_halfspaces([s[0, 0]], ego[0], rr, ro, alpha, delta, eps)
        finally:
            hs.dr_cvar_halfspace = inner
        expected = np.empty((1, 1, 8))
        expected[0, 0], dh = record_of(out["mean"][0], out["cvar"][0], out["dr_cvar"][0], rec[0][0])
        assert not np.any(dh)
        meta = json.loads(str(z["meta"]))
        check_and_save(f[:-4], s, ego, tuple(p), expected,
                       dict(case=meta.get("case"), route="core.halfspaces.compute_safe_halfspaces"))


def singleton_session(rm, hs):
    """A call sequence through the reference's compute_safe_halfspaces whose later calls hit the
    N-keyed optimiser singletons (core/risk_metrics.py:289,325): the alpha/delta/epsilon of the
    FIRST call for a given N stay in force, CVaR and DR independently."""
    rng = np.random.RandomState(11)
    rr, ro = 0.3, 0.3
    ego = np.array([0.2, -0.1])
    calls = [  # (N, alpha, delta, epsilon, via)
        (50, 0.2, 0.1, 0.15, "compute"),     # creates both singletons for N=50
        (50, 0.1, 0.05, 0.3, "compute"),     # same N: the reference keeps 0.2 / 0.1 / 0.15
        (60, 0.1, 0.05, 0.3, "compute"),     # new N: new singletons with these parameters
        (60, 0.3, 0.2, 0.05, "cvar_only"),   # cvar_halfspace alone: CVaR singleton kept (N=60)
        (50, 0.3, 0.2, 0.05, "compute"),     # N=50 again: both re-created with 0.3 / 0.2 / 0.05
    ]
    reset_singletons(rm)
    samples, params, expected, via = [], [], [], []
    for n, alpha, delta, eps, how in calls:
        s = rng.normal(size=(n, 2)) * 0.15 + np.array([1.2, 0.4])
        rec = []
        inner = hs.dr_cvar_halfspace
        hs.dr_cvar_halfspace = lambda *a, **k: rec.append(inner(*a, **k)) or rec[-1]
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                if how == "compute":
                    out = hs.compute_safe_halfspaces([s], ego, rr, ro, alpha, delta, eps)
                    row, _ = record_of(out["mean"][0], out["cvar"][0], out["dr_cvar"][0], rec[0][0])
                else:
                    from core.geometry import compute_separating_vector
                    h = compute_separating_vector(ego, np.mean(s, axis=0))
                    g = rm.cvar_halfspace(s, h, alpha, delta, rr, ro)
                    row = np.full(8, np.nan)
                    row[3:6] = h[0], h[1], g
        finally:
            hs.dr_cvar_halfspace = inner
        samples.append(s)
        params.append((rr, ro, alpha, delta, eps))
        expected.append(row)
        via.append(how)
    # what the singletons held is checkable from the data: record the parameters in force
    eff = [(0.2, 0.1, 0.15), (0.2, 0.1, 0.15), (0.1, 0.05, 0.3), (0.1, 0.05, None), (0.3, 0.2, 0.05)]
    for (n, *_), row, s, e in zip(calls, expected, samples, eff):
        a, d, eps = e
        cvar_direct = cf.safe_halfspaces(s[None, None], ego[None], rr, ro, a, d, eps if eps is not None else 0.15)
        assert abs(cvar_direct[0, 0, 5] - row[5]) < 1e-9
    path = os.path.join(HERE, "singleton_session.npz")
    np.savez(path, ego=ego, n=np.array([c[0] for c in calls]), params=np.array(params),
             samples=np.concatenate(samples), expected=np.array(expected),
             via=np.array(via), effective=np.array([[x if x is not None else np.nan for x in e] for e in eff]),
             meta=np.asarray(json.dumps(dict(source=SOURCE, route="core.halfspaces.compute_safe_halfspaces"
                                             " / core.risk_metrics.cvar_halfspace in sequence"))))
    print(f"wrote {path}")


def singleton_environment(rm, hs):
    """SafetyFilteringEnvironment.compute_safe_halfspaces_for_trajectory after a prior
    compute_safe_halfspaces call left singletons with other parameters: (a) every obstacle with
    the prior call's N (all units keep the prior parameters), (b) ragged N (the prior parameters
    hold only until another N rebuilds the singleton — per step and obstacle in the reference's
    loop order)."""
    from simulation.environment import SafetyFilteringEnvironment
    rng = np.random.RandomState(23)
    T = 6
    x_ref = np.zeros((T + 1, 4))
    x_ref[:, 0] = np.linspace(-1.0, 1.0, T + 1)
    x_ref[:, 1] = 0.1
    prior = (0.3, 0.3, 0.35, 0.05, 0.4)
    out = {}
    for case, ns in (("uniform", (20, 20)), ("ragged", (20, 30))):
        trajs = [rng.normal(size=(n, T + 3, 2)) * 0.12 + np.array([0.8 + o, 0.9 - 0.5 * o])
                 for o, n in enumerate(ns)]
        prior_s = rng.normal(size=(20, 2)) * 0.1 + np.array([1.0, 1.0])
        reset_singletons(rm)
        env = SafetyFilteringEnvironment(ROBOT_RADIUS=0.3, OBSTACLE_RADIUS=0.3, HORIZON=T, DT=0.2,
                                         ALPHA=0.2, DELTA=0.1, EPSILON=0.15)
        rec = []
        inner = hs.dr_cvar_halfspace
        hs.dr_cvar_halfspace = lambda *a, **k: rec.append(inner(*a, **k)) or rec[-1]
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                hs.compute_safe_halfspaces([prior_s], np.zeros(2), *prior)
                rec.clear()
                res = env.compute_safe_halfspaces_for_trajectory(trajs, x_ref)
        finally:
            hs.dr_cvar_halfspace = inner
        O = len(trajs)
        expected = np.empty((O, T, 8))
        k = 0
        for t in range(T):
            for o in range(O):
                expected[o, t], _ = record_of(res["mean"][t][o], res["cvar"][t][o],
                                              res["dr_cvar"][t][o], rec[k][0])
                k += 1
        out[f"{case}_expected"] = expected
        out[f"{case}_prior_samples"] = prior_s
        for o, tr in enumerate(trajs):
            out[f"{case}_traj{o}"] = tr
    path = os.path.join(HERE, "singleton_environment.npz")
    np.savez(path, x_ref=x_ref, prior_params=np.array(prior), horizon=np.array(T), **out,
             meta=np.asarray(json.dumps(dict(source=SOURCE, route="core.halfspaces.compute_safe_"
                                             "halfspaces (prior call) then SafetyFilteringEnvironment."
                                             "compute_safe_halfspaces_for_trajectory"))))
    print(f"wrote {path}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    rm, hs, recorded = load_reference(args.reference)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:       # the reference writes tmp/timing_info_*.json
        os.chdir(tmp)
        try:
            environment_case("head_on_n100_t20", "head_on", 100, 20, 20, rm, recorded)
            environment_case("multi_obstacle_n1000_t8", "multi_obstacle", 1000, 20, 8, rm, recorded)
            environment_case("multi_obstacle_n20_h30", "multi_obstacle", 20, 30, 30, rm, recorded)
        finally:
            os.chdir(cwd)
    timing_analysis_cases(rm, hs)
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        try:
            edge_cases(rm, hs)
            singleton_session(rm, hs)
            singleton_environment(rm, hs)
        finally:
            os.chdir(cwd)


if __name__ == "__main__":
    main()

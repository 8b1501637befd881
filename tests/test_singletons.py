"""The reference's optimiser singletons keyed on N (core/risk_metrics.py:12-13, :289, :325) on the
batched paths (VERDICT r1 "What's missing" #2).

Fixtures `tests/golden/singleton_*.npz` come from the REFERENCE's own code
(tests/golden/make_golden_ref.py): a sequence of `compute_safe_halfspaces` / `cvar_halfspace`
calls, and `SafetyFilteringEnvironment.compute_safe_halfspaces_for_trajectory` after a prior call
with other parameters (uniform and ragged N).  CPU: the closed form with the parameters the
fixture says were in force, and `risk_metrics.singleton_params` replaying the call order.  GPU:
the build's `compute_safe_halfspaces`, `cvar_halfspace` and `SafetyFilteringEnvironment`
replaying the same calls.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN_DIR, OFFSET_TOL
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import risk_metrics

SESSION = os.path.join(GOLDEN_DIR, "singleton_session.npz")
ENVIRON = os.path.join(GOLDEN_DIR, "singleton_environment.npz")


def _session():
    z = np.load(SESSION, allow_pickle=False)
    n = z["n"]
    offs = np.concatenate([[0], np.cumsum(n)])
    samples = [z["samples"][offs[i]:offs[i + 1]] for i in range(len(n))]
    return z, samples


def test_session_fixture_against_closed_form():
    from oracle import closed_form as cf
    z, samples = _session()
    for i, s in enumerate(samples):
        a, d, e = z["effective"][i]
        rr, ro = z["params"][i][:2]
        ref = cf.safe_halfspaces(s[None, None], z["ego"][None], rr, ro, a, d,
                                 0.15 if np.isnan(e) else e)[0, 0]
        exp = z["expected"][i]
        cols = [3, 4, 5] if str(z["via"][i]) == "cvar_only" else list(range(8))
        assert np.max(np.abs(ref[cols] - exp[cols])) < 1e-12, i


def test_singleton_params_replays_the_reference_order(monkeypatch):
    """Host logic only (no device): the parameters each call of the session is solved with."""
    z, samples = _session()
    risk_metrics.reset_optimizers()
    try:
        for i, s in enumerate(samples):
            rr, ro, a, d, e = z["params"][i]
            (ac, dc), (ad, dd, ed) = risk_metrics.singleton_params([s.shape[0]], a, d, e)[0]
            ea, ed_, ee = z["effective"][i]
            assert (ac, dc) == (ea, ed_)
            if str(z["via"][i]) != "cvar_only":
                assert (ad, dd, ed) == (ea, ed_, ee)
    finally:
        risk_metrics.reset_optimizers()


def test_environment_order_ragged_singletons():
    """Steps outer, obstacles inner: with a prior N=20 singleton, obstacle 0 (N=20) keeps the prior
    parameters only at t = 0 when obstacle 1 (N=30) rebuilds the singleton every step."""
    risk_metrics.reset_optimizers()
    try:
        risk_metrics.singleton_params([20], 0.35, 0.05, 0.4)
        keys = risk_metrics.singleton_params([20, 30] * 3, 0.2, 0.1, 0.15)
        assert keys[0] == ((0.35, 0.05), (0.35, 0.05, 0.4))
        assert all(k == ((0.2, 0.1), (0.2, 0.1, 0.15)) for k in keys[1:])
    finally:
        risk_metrics.reset_optimizers()


@pytest.fixture()
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    risk_metrics.reset_optimizers()
    yield torch.device("cuda", 0)
    risk_metrics.reset_optimizers()


@pytest.mark.gpu
def test_gpu_session_matches_reference(dev, tmp_path, monkeypatch):
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import halfspaces
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core.geometry import (
        compute_separating_vector)
    monkeypatch.chdir(tmp_path)
    z, samples = _session()
    for i, s in enumerate(samples):
        rr, ro, a, d, e = z["params"][i]
        exp = z["expected"][i]
        if str(z["via"][i]) == "compute":
            out = halfspaces.compute_safe_halfspaces([s], z["ego"], rr, ro, a, d, e)
            got = np.array([*out["mean"][0].h, out["mean"][0].g_tilde, *out["dr_cvar"][0].h,
                            out["cvar"][0].g_tilde, np.nan, out["dr_cvar"][0].g_tilde])
            cols = [0, 1, 2, 3, 4, 5, 7]
        else:
            h = compute_separating_vector(z["ego"], np.mean(s, axis=0))
            got = np.full(8, np.nan)
            got[3:5] = h
            got[5] = risk_metrics.cvar_halfspace(s, h, a, d, rr, ro)
            cols = [3, 4, 5]
        assert np.max(np.abs(got[cols] - exp[cols])) < OFFSET_TOL, (i, got, exp)
        assert np.max(np.abs(got[cols] - exp[cols])) < 1e-12, i


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["uniform", "ragged"])
def test_gpu_environment_after_prior_call_matches_reference(dev, tmp_path, monkeypatch, case):
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import halfspaces
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.simulation.environment import (
        SafetyFilteringEnvironment)
    monkeypatch.chdir(tmp_path)
    z = np.load(ENVIRON, allow_pickle=False)
    T = int(z["horizon"])
    trajs = [z[f"{case}_traj{o}"] for o in range(2)]
    halfspaces.compute_safe_halfspaces([z[f"{case}_prior_samples"]], np.zeros(2), *z["prior_params"])
    env = SafetyFilteringEnvironment(ROBOT_RADIUS=0.3, OBSTACLE_RADIUS=0.3, HORIZON=T, DT=0.2,
                                     ALPHA=0.2, DELTA=0.1, EPSILON=0.15)
    rec = env.compute_halfspace_batch(trajs, z["x_ref"]).record.cpu().numpy()
    exp = z[f"{case}_expected"]
    assert rec.shape == exp.shape
    assert np.max(np.abs(rec - exp)) < 1e-12
    # and the dict-of-lists surface agrees with the record
    lists = env.compute_safe_halfspaces_for_trajectory(trajs, z["x_ref"])
    assert len(lists["dr_cvar"]) == T

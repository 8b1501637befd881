"""CPU: the oracle itself, pinned before anything is compared against it.

* golden vectors (reference generators + reference LP rows solved by HiGHS) vs the NumPy closed
  form and vs the C restatement;
* HiGHS restatement vs closed form on random units incl. ties, fractional alpha*N, tiny N,
  alpha = 1 and the unbounded-LP sentinels (alpha > 1, epsilon < 0);
* hypothesis property tests of the closed form (lower-tail mean bounds, translation equivariance,
  permutation invariance).
"""
import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from conftest import OFFSET_TOL
from oracle import c_oracle
from oracle import closed_form as cf
from oracle import lp_highs


def _params(g):
    rr, ro, alpha, delta, eps = (float(v) for v in g["params"])
    return rr, ro, alpha, delta, eps


def test_golden_closed_form(golden):
    rr, ro, alpha, delta, eps = _params(golden)
    out = cf.safe_halfspaces(golden["samples"], golden["ego"], rr, ro, alpha, delta, eps)
    np.testing.assert_allclose(out, golden["expected"], rtol=0, atol=1e-12, equal_nan=True)


def test_golden_c_oracle(golden):
    rr, ro, alpha, delta, eps = _params(golden)
    out = c_oracle.safe_halfspaces(golden["samples"], golden["ego"], rr, ro, alpha, delta, eps)
    np.testing.assert_allclose(out, golden["expected"], rtol=0, atol=1e-12, equal_nan=True)


def test_golden_known_answers():
    """Values quoted in SURVEY.md §8c (seed 42 probe) are reproduced by the committed vectors."""
    from conftest import GOLDEN_DIR, load_golden
    import os
    g = load_golden(os.path.join(GOLDEN_DIR, "head_on_n100_t20.npz"))["expected"]
    np.testing.assert_allclose(g[0, 0, [0, 1, 2, 5, 7]], [1, 0, -3.4, -3.5, -3.35], atol=1e-12)
    np.testing.assert_allclose(g[0, 1, [3, 4, 7, 5]],
                               [0.999999896579, 0.000454798184, -3.019209801469, -3.169209801469],
                               atol=1e-11)
    np.testing.assert_allclose(g[0, 1, [0, 1, 2]], [0.999999596748, 0.000898055100, -3.188445102218],
                               atol=1e-11)
    np.testing.assert_allclose(g[0, 19, [3, 4, 7]], [-0.999997200068, -0.002366401620, 0.984980979791],
                               atol=1e-11)
    m = load_golden(os.path.join(GOLDEN_DIR, "multi_obstacle_n1000_t8.npz"))["expected"]
    np.testing.assert_allclose(m[0, 0, [3, 4, 7]], [0.554700196225, 0.832050294338, -1.014100588676],
                               atol=1e-11)


def _random_unit(rng, n, ties=False):
    s = rng.normal(size=(n, 2)) * rng.uniform(0.01, 2.0) + rng.normal(size=2) * 3
    if ties:
        s = np.round(s, 1)
    h = rng.normal(size=2)
    return s, h / np.linalg.norm(h)


@pytest.mark.parametrize("seed", range(12))
def test_highs_matches_closed_form(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 90))
    s, h = _random_unit(rng, n, ties=seed % 3 == 0)
    alpha = float(rng.choice([0.05, 0.2, 0.37, 0.5, 1.0]))
    delta, eps = float(rng.uniform(-0.2, 0.3)), float(rng.uniform(0, 0.4))
    if seed % 4 == 1:
        h = h * 1.7  # non-unit h: the reference scales the radius by |h| (risk_metrics.py:293,234)
    g_cvar = lp_highs.solve_cvar_lp(s, h, alpha, delta, 0.3, 0.3)
    g_star, g_tilde = lp_highs.solve_dr_cvar_lp(s, h, alpha, delta, eps, 0.3, 0.3)
    c, gs, gt = cf.offsets_given_h(s, h, alpha, delta, eps, 0.3, 0.3)
    assert abs(g_cvar - c) < 1e-9
    assert abs(g_star - gs) < 1e-9
    assert abs(g_tilde - gt) < 1e-9


def test_unbounded_lps_give_sentinels():
    rng = np.random.default_rng(3)
    s, h = _random_unit(rng, 40)
    r = 0.6 * np.linalg.norm(h)
    assert lp_highs.solve_cvar_lp(s, h, 1.5, 0.1, 0.3, 0.3) == 100.0
    g_star, g_tilde = lp_highs.solve_dr_cvar_lp(s, h, 0.2, 0.1, -0.1, 0.3, 0.3)
    assert g_star == 100.0 and abs(g_tilde - (100.0 - r)) < 1e-12
    c, gs, gt = cf.offsets_given_h(s, h, 1.5, 0.1, 0.15, 0.3, 0.3)
    assert c == 100.0 and gs == 100.0
    c, gs, gt = cf.offsets_given_h(s, h, 0.2, 0.1, -0.1, 0.3, 0.3)
    assert gs == 100.0 and c != 100.0


def test_c_oracle_matches_numpy_random():
    rng = np.random.default_rng(11)
    for n in (1, 2, 7, 37, 128, 1000, 4097):
        s = rng.normal(size=(2, 3, n, 2))
        if n > 100:
            s[0, 0] = np.round(s[0, 0], 1)
        ego = rng.normal(size=(3, 2))
        a = c_oracle.safe_halfspaces(s, ego, 0.3, 0.3, 0.2, 0.1, 0.15, nthreads=2)
        b = cf.safe_halfspaces(s, ego, 0.3, 0.3, 0.2, 0.1, 0.15)
        np.testing.assert_allclose(a, b, rtol=0, atol=1e-12)


def test_c_oracle_strided_layout():
    rng = np.random.default_rng(5)
    traj = rng.normal(size=(3, 50, 31, 2))          # [O, N, S+1, 2] reference layout
    view = traj.transpose(0, 2, 1, 3)[:, :20]      # [O, T, N, 2] strided
    ego = rng.normal(size=(20, 2))
    a = c_oracle.safe_halfspaces(view, ego, 0.3, 0.3, 0.2, 0.1, 0.15)
    b = cf.safe_halfspaces(np.ascontiguousarray(view), ego, 0.3, 0.3, 0.2, 0.1, 0.15)
    np.testing.assert_allclose(a, b, rtol=0, atol=1e-12)


def test_non_finite_samples_sentinel():
    rng = np.random.default_rng(9)
    s = rng.normal(size=(1, 2, 30, 2))
    s[0, 1, 4, 1] = np.nan
    out = cf.safe_halfspaces(s, np.zeros((2, 2)), 0.3, 0.3, 0.2, 0.1, 0.15)
    assert out[0, 1, 5] == 100.0 and out[0, 1, 6] == 100.0 and np.isnan(out[0, 1, 7])
    assert np.isfinite(out[0, 0]).all()
    c = c_oracle.safe_halfspaces(s, np.zeros((2, 2)), 0.3, 0.3, 0.2, 0.1, 0.15)
    np.testing.assert_array_equal(np.isnan(c), np.isnan(out))
    np.testing.assert_allclose(c, out, atol=1e-12, equal_nan=True)


_unit = st.integers(min_value=1, max_value=60).flatmap(
    lambda n: st.lists(st.tuples(st.floats(-50, 50), st.floats(-50, 50)), min_size=n, max_size=n))


@settings(max_examples=150, deadline=None)
@given(pts=_unit, alpha=st.floats(0.01, 1.0), shift=st.tuples(st.floats(-10, 10), st.floats(-10, 10)))
def test_lower_tail_mean_properties(pts, alpha, shift):
    s = np.asarray(pts, dtype=np.float64)
    d = s[:, 0] * 0.6 + s[:, 1] * 0.8
    L = cf.lower_tail_mean(d[None], alpha)[0]
    srt = np.sort(d)
    # L lies between the minimum and the mean, and is monotone in alpha
    assert srt[0] - 1e-9 <= L <= d.mean() + 1e-9
    assert cf.lower_tail_mean(d[None], 1.0)[0] == pytest.approx(d.mean(), abs=1e-9)
    # permutation invariance and translation equivariance
    perm = np.random.default_rng(0).permutation(len(d))
    assert cf.lower_tail_mean(d[perm][None], alpha)[0] == pytest.approx(L, abs=1e-9)
    c = 0.6 * shift[0] + 0.8 * shift[1]
    assert cf.lower_tail_mean((d + c)[None], alpha)[0] == pytest.approx(L + c, abs=1e-8)


@settings(max_examples=40, deadline=None)
@given(pts=_unit, alpha=st.sampled_from([0.1, 0.2, 0.25, 0.5, 1.0]))
def test_closed_form_vs_highs_hypothesis(pts, alpha):
    s = np.asarray(pts, dtype=np.float64)
    h = np.array([0.6, -0.8])
    g = lp_highs.solve_cvar_lp(s, h, alpha, 0.1, 0.3, 0.3)
    c, _, _ = cf.offsets_given_h(s, h, alpha, 0.1, 0.15, 0.3, 0.3)
    assert abs(g - float(c)) <= OFFSET_TOL

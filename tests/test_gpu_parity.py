"""GPU parity: the HIP engine (through the C ABI) against the oracle and the golden vectors.

Tolerance: offsets within 1e-6 absolute (north star); directions to 1e-12.  Observed differences
are ~1e-15 — only summation order differs.  Sentinel and NaN positions must match exactly.
"""
import numpy as np
import pytest
import torch

from conftest import OFFSET_TOL
from oracle import c_oracle
from oracle import closed_form as cf

pytestmark = pytest.mark.gpu

from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import engine  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.engine import RiskParams  # noqa: E402

DEV = torch.device("cuda", 0)
H_TOL = 1e-12


def _run(samples, ego, params):
    s = torch.as_tensor(samples).to(DEV)
    e = torch.as_tensor(np.ascontiguousarray(ego)).to(DEV)
    return engine.safe_halfspaces(s, e, params).cpu().numpy()


def _assert_match(got, want):
    assert got.shape == want.shape
    np.testing.assert_array_equal(np.isnan(got), np.isnan(want))
    g, w = np.nan_to_num(got, nan=0.0), np.nan_to_num(want, nan=0.0)
    np.testing.assert_allclose(g[..., [0, 1, 3, 4]], w[..., [0, 1, 3, 4]], rtol=0, atol=H_TOL)
    np.testing.assert_allclose(g[..., [2, 5, 6, 7]], w[..., [2, 5, 6, 7]], rtol=0, atol=OFFSET_TOL)
    # sentinels exactly where the oracle has them
    np.testing.assert_array_equal(got[..., 5] == 100.0, want[..., 5] == 100.0)
    np.testing.assert_array_equal(got[..., 6] == 100.0, want[..., 6] == 100.0)


def _params(g):
    return RiskParams(*(float(v) for v in g["params"]))


def test_golden_vectors(golden):
    got = _run(golden["samples"], golden["ego"], _params(golden))
    _assert_match(got, golden["expected"])
    assert np.nanmax(np.abs(got - golden["expected"])) < 1e-12


@pytest.mark.parametrize("n", [1, 2, 3, 5, 63, 64, 65, 100, 128, 129, 300, 512, 513, 1000, 1024,
                               1025, 2048, 3000, 4096, 4097, 5000, 5120, 5121, 8192, 8193, 10000,
                               10240, 10241, 12288, 16384])
def test_every_launch_plan_random(n):
    rng = np.random.default_rng(n)
    O, T = 2, 3
    samples = rng.normal(size=(O, T, n, 2)) * 0.1 + rng.uniform(-3, 3, size=(O, T, 1, 2))
    ego = rng.uniform(-3, 3, size=(T, 2))
    p = RiskParams()
    _assert_match(_run(samples, ego, p), c_oracle.safe_halfspaces(samples, ego, 0.3, 0.3, 0.2, 0.1, 0.15))


@pytest.mark.parametrize("alpha", [0.001, 0.01, 0.2, 0.37, 0.5, 0.999, 1.0, 1.5])
def test_alpha_range(alpha):
    rng = np.random.default_rng(int(alpha * 1000))
    samples = rng.normal(size=(3, 4, 777, 2))
    ego = rng.normal(size=(4, 2))
    p = RiskParams(0.3, 0.3, alpha, 0.1, 0.15)
    _assert_match(_run(samples, ego, p), cf.safe_halfspaces(samples, ego, 0.3, 0.3, alpha, 0.1, 0.15))


@pytest.mark.parametrize("kind", ["ties_coarse", "ties_heavy", "all_equal", "two_values",
                                  "outliers", "tiny_spread", "huge_offset", "denormal_spread",
                                  "straddle_zero", "geometric"])
def test_adversarial_distributions(kind):
    rng = np.random.default_rng(sum(kind.encode()))
    n = 3000
    if kind == "ties_coarse":
        s = np.round(rng.normal(size=(n, 2)), 1)
    elif kind == "ties_heavy":
        s = rng.integers(0, 3, size=(n, 2)).astype(np.float64)
    elif kind == "all_equal":
        s = np.tile([[1.25, -0.5]], (n, 1))
    elif kind == "two_values":
        s = np.where(rng.random((n, 1)) < 0.5, [[0.0, 0.0]], [[1.0, 1.0]])
    elif kind == "outliers":
        s = rng.normal(size=(n, 2))
        s[:5] = 1e6
    elif kind == "tiny_spread":
        s = 3.0 + rng.normal(size=(n, 2)) * 1e-12
    elif kind == "huge_offset":
        s = 1e6 + rng.normal(size=(n, 2))
    elif kind == "denormal_spread":
        s = rng.normal(size=(n, 2)) * 1e-310
    elif kind == "straddle_zero":
        s = rng.normal(size=(n, 2)) * 1e-3
    else:  # geometric: one candidate eliminated per value-linear pass -> exercises key mode
        s = np.stack([2.0 ** -np.arange(n, dtype=np.float64) * 0 + 2.0 ** -(np.arange(n) % 900),
                      np.zeros(n)], axis=1)
    samples = np.ascontiguousarray(s[None, None])
    ego = np.array([[-1.0, 0.3]])
    _assert_match(_run(samples, ego, RiskParams()),
                  cf.safe_halfspaces(samples, ego, 0.3, 0.3, 0.2, 0.1, 0.15))


@pytest.mark.parametrize("n", [100, 1000, 2049, 3000, 4096, 4097, 5000, 5120, 8192, 10000, 16384])
def test_all_equal_units_every_plan(n):
    """Units whose samples are all one point (every obstacle's noise-free step 0,
    simulation/obstacles.py:63) on every register plan — the 256-thread large plans settle them
    from the moments' differ flag, the others from the register min/max or the exact fallback —
    beside units where ONE sample differs (the first, i.e. the pivot; the last; one in the middle),
    which must take the ordinary path: all against the closed form."""
    T = 4
    pts = np.array([[1.25, -0.5], [-3.0, 2.0], [0.1, 0.1], [7.5, -2.25]])
    samples = np.repeat(pts[None, :, None, :], 4, axis=0).repeat(n, axis=2)   # [4, T, n, 2]
    samples[1, :, 0, 0] += 0.5          # the pivot differs
    samples[2, :, n - 1, 1] -= 0.25     # the last sample differs
    samples[3, :, n // 2, 0] += 1e-9    # one sample in the middle, barely
    ego = np.array([[-1.0, 0.3], [2.0, 2.0], [0.0, -4.0], [5.0, 5.0]])
    got = _run(samples, ego, RiskParams())
    want = cf.safe_halfspaces(samples, ego, 0.3, 0.3, 0.2, 0.1, 0.15)
    _assert_match(got, want)
    assert np.max(np.abs(got - want)) < 1e-12


def test_non_finite_and_unbounded_sentinels():
    rng = np.random.default_rng(1)
    samples = rng.normal(size=(2, 3, 200, 2))
    samples[0, 1, 17, 0] = np.nan
    samples[1, 2, 3, 1] = np.inf
    ego = rng.normal(size=(3, 2))
    want = cf.safe_halfspaces(samples, ego, 0.3, 0.3, 0.2, 0.1, 0.15)
    got = _run(samples, ego, RiskParams())
    _assert_match(got, want)
    assert got[0, 1, 5] == 100.0 and got[1, 2, 6] == 100.0
    got = _run(samples[:, :1], ego[:1], RiskParams(epsilon=-0.1))
    assert (got[..., 6] == 100.0).all() and (got[..., 5] != 100.0).all()


def test_strided_reference_layout():
    """[O, N, S+1, 2] per-obstacle trajectories consumed with their own strides (no transpose)."""
    rng = np.random.default_rng(8)
    traj = torch.as_tensor(rng.normal(size=(4, 1000, 151, 2))).to(DEV)
    view = traj.permute(0, 2, 1, 3)[:, :20]
    ego = rng.normal(size=(20, 2))
    got = engine.safe_halfspaces(view, torch.as_tensor(ego).to(DEV), RiskParams()).cpu().numpy()
    want = cf.safe_halfspaces(view.cpu().numpy(), ego, 0.3, 0.3, 0.2, 0.1, 0.15)
    _assert_match(got, want)


def test_unaligned_scalar_load_path():
    rng = np.random.default_rng(4)
    buf = torch.as_tensor(rng.normal(size=(2 * 3 * 500 * 2 + 1))).to(DEV)
    s = buf[1:].reshape(2, 3, 500, 2)          # base pointer 8 B past 16-B alignment
    ego = rng.normal(size=(3, 2))
    got = engine.safe_halfspaces(s, torch.as_tensor(ego).to(DEV), RiskParams()).cpu().numpy()
    _assert_match(got, cf.safe_halfspaces(s.cpu().numpy(), ego, 0.3, 0.3, 0.2, 0.1, 0.15))


def test_given_h_entry_point():
    rng = np.random.default_rng(6)
    U, N = 50, 999
    s = rng.normal(size=(U, N, 2))
    h = rng.normal(size=(U, 2)) * rng.uniform(0.5, 2.0, size=(U, 1))   # non-unit directions too
    got = engine.offsets_given_h(torch.as_tensor(s).to(DEV), torch.as_tensor(h).to(DEV),
                                 RiskParams()).cpu().numpy()
    gc, gs, gt = cf.offsets_given_h(s, h, 0.2, 0.1, 0.15, 0.3, 0.3)
    np.testing.assert_allclose(got[:, 3:5], h, atol=0)
    np.testing.assert_allclose(got[:, 5], gc, atol=OFFSET_TOL)
    np.testing.assert_allclose(got[:, 6], gs, atol=OFFSET_TOL)
    np.testing.assert_allclose(got[:, 7], gt, atol=OFFSET_TOL)


def test_bitwise_deterministic():
    rng = np.random.default_rng(12)
    s = torch.as_tensor(rng.normal(size=(8, 10, 5000, 2))).to(DEV)
    e = torch.as_tensor(rng.normal(size=(10, 2))).to(DEV)
    a = engine.safe_halfspaces(s, e, RiskParams())
    b = engine.safe_halfspaces(s, e, RiskParams())
    assert torch.equal(a, b)


@pytest.mark.parametrize("O,T", [(65535, 2), (65536, 1), (140_001, 2)])
def test_obstacle_counts_beyond_one_grid(O, T):
    """More obstacles than the grid's y dimension holds: the launch is split into obstacle
    chunks on the host; every unit still lands in its own record."""
    rng = np.random.default_rng(O + T)
    N = 24
    s = rng.normal(size=(O, T, N, 2)) * rng.uniform(0.05, 2.0, size=(O, T, 1, 1))
    s += rng.uniform(-4, 4, size=(O, 1, 1, 2))
    e = rng.uniform(-4, 4, size=(T, 2))
    got = _run(s, e, RiskParams())
    want = c_oracle.safe_halfspaces(s, e, 0.3, 0.3, 0.2, 0.1, 0.15, nthreads=8)
    _assert_match(got, want)


def test_given_h_many_units():
    """offsets_given_h puts its units on the grid's x dimension: far beyond 65535 of them."""
    rng = np.random.default_rng(9)
    U, N = 200_000, 16
    s = rng.normal(size=(U, N, 2))
    h = rng.normal(size=(U, 2))
    got = engine.offsets_given_h(torch.as_tensor(s).to(DEV), torch.as_tensor(h).to(DEV),
                                 RiskParams()).cpu().numpy()
    gc, gs, gt = cf.offsets_given_h(s, h, 0.2, 0.1, 0.15, 0.3, 0.3)
    np.testing.assert_allclose(got[:, 5], gc, atol=OFFSET_TOL)
    np.testing.assert_allclose(got[:, 7], gt, atol=OFFSET_TOL)


@pytest.mark.parametrize("O,T,N", [(10, 20, 1000), (64, 30, 5000)])
def test_baseline_configs_vs_c_oracle(O, T, N):
    """BASELINE configs 3 and 4 at full size, every unit checked against the C oracle."""
    g = torch.Generator(device=DEV).manual_seed(42)
    s = torch.randn((O, T, N, 2), dtype=torch.float64, device=DEV, generator=g) * 0.1
    s += torch.rand((O, T, 1, 2), dtype=torch.float64, device=DEV, generator=g) * 8 - 4
    e = torch.rand((T, 2), dtype=torch.float64, device=DEV, generator=g) * 8 - 4
    got = engine.safe_halfspaces(s, e, RiskParams()).cpu().numpy()
    want = c_oracle.safe_halfspaces(s.cpu().numpy(), e.cpu().numpy(), 0.3, 0.3, 0.2, 0.1, 0.15,
                                    nthreads=8)
    _assert_match(got, want)


def test_config5_full_size_properties():
    """BASELINE config 5 size (256 x 50 x 10000, 2 GB): exact vs the C oracle on a strided subset
    of units, plus size-independent properties on all units (g_dr - g_cvar = eps/alpha, sentinels
    absent, |h| = 1, determinism)."""
    O, T, N = 256, 50, 10000
    g = torch.Generator(device=DEV).manual_seed(7)
    s = torch.randn((O, T, N, 2), dtype=torch.float64, device=DEV, generator=g) * 0.1
    s += torch.rand((O, T, 1, 2), dtype=torch.float64, device=DEV, generator=g) * 8 - 4
    e = torch.rand((T, 2), dtype=torch.float64, device=DEV, generator=g) * 8 - 4
    rec = engine.safe_halfspaces(s, e, RiskParams())
    rec2 = engine.safe_halfspaces(s, e, RiskParams())
    assert torch.equal(rec, rec2)
    r = rec.cpu().numpy()
    assert np.isfinite(r).all()
    np.testing.assert_allclose(np.hypot(r[..., 3], r[..., 4]), 1.0, atol=1e-14)
    # g_cvar = r - delta - L and g* = r - delta + eps/alpha - L  =>  g* - g_cvar = eps/alpha
    np.testing.assert_allclose(r[..., 6] - r[..., 5], 0.15 / 0.2, atol=1e-12)
    np.testing.assert_allclose(r[..., 6] - r[..., 7], 0.6, atol=1e-12)
    sub = s[::37, ::7].cpu().numpy()
    want = c_oracle.safe_halfspaces(sub, e[::7].cpu().numpy(), 0.3, 0.3, 0.2, 0.1, 0.15, nthreads=8)
    _assert_match(r[::37, ::7], want)
    del s, rec, rec2
    torch.cuda.empty_cache()


GEOMETRIES = [(64, 2), (128, 4), (256, 4), (256, 8), (256, 16), (512, 16), (512, 20), (1024, 12),
              (1024, 16), (64, 16), (128, 8), (512, 2), (1024, 10), (256, 20)]


@pytest.mark.parametrize("n", [100, 1000, 5000, 10000])
def test_every_geometry_agrees(n):
    """All compiled launch geometries (drcvar_safe_halfspaces_f64_ex) give the oracle's answer."""
    rng = np.random.default_rng(n + 1)
    samples = rng.normal(size=(2, 3, n, 2)) * 0.2 + rng.uniform(-3, 3, size=(2, 3, 1, 2))
    samples[0, 0] = np.round(samples[0, 0], 1)   # heavy ties -> refinement path
    samples[1, 0] = 1.5                          # zero variance -> degenerate path
    ego = rng.uniform(-3, 3, size=(3, 2))
    want = c_oracle.safe_halfspaces(samples, ego, 0.3, 0.3, 0.2, 0.1, 0.15)
    s = torch.as_tensor(samples).to(DEV)
    e = torch.as_tensor(ego).to(DEV)
    for g in GEOMETRIES:
        if g[0] * g[1] < n:
            continue
        launch, out = engine.prepare_safe_halfspaces(s, e, RiskParams(), geometry=g)
        launch()
        _assert_match(out.cpu().numpy(), want)


@pytest.mark.parametrize("n", [16385, 20000, 65536, 250_000])
def test_streaming_kernel_beyond_register_plans(n):
    """N > DRCVAR_MAX_SAMPLES runs the streaming kernel (samples re-read, nothing on chip)."""
    rng = np.random.default_rng(n)
    O, T = 2, 2
    samples = rng.normal(size=(O, T, n, 2)) * 0.1 + rng.uniform(-3, 3, size=(O, T, 1, 2))
    ego = rng.uniform(-3, 3, size=(T, 2))
    _assert_match(_run(samples, ego, RiskParams()),
                  c_oracle.safe_halfspaces(samples, ego, 0.3, 0.3, 0.2, 0.1, 0.15))


@pytest.mark.parametrize("alpha", [0.001, 0.2, 0.999, 1.5])
def test_streaming_kernel_alpha_ties_and_sentinels(alpha):
    rng = np.random.default_rng(7)
    n = 40_000
    samples = rng.normal(size=(3, 1, n, 2))
    samples[1] = np.round(samples[1] * 2.0) / 2.0           # heavy ties
    samples[2, 0, :, :] = 0.25                               # all equal
    ego = np.array([[-2.0, 0.5]])
    p = RiskParams(alpha=alpha)
    _assert_match(_run(samples, ego, p),
                  cf.safe_halfspaces(samples, ego, 0.3, 0.3, alpha, 0.1, 0.15))
    bad = samples.copy()
    bad[0, 0, 12345, 1] = np.nan
    got = _run(bad, ego, p)
    assert got[0, 0, 5] == 100.0


def test_streaming_kernel_strided_layout():
    rng = np.random.default_rng(3)
    n, S = 17000, 4
    traj = rng.normal(size=(2, n, S, 2)) * 0.2                # reference [O, N, S+1, 2] order
    import torch
    dev = torch.device("cuda", 0)
    t = torch.as_tensor(traj).to(dev).permute(0, 2, 1, 3)    # [O, S, N, 2] view, strided
    ego = rng.normal(size=(S, 2))
    got = engine.safe_halfspaces(t, torch.as_tensor(ego).to(dev), RiskParams()).cpu().numpy()
    want = c_oracle.safe_halfspaces(np.ascontiguousarray(np.transpose(traj, (0, 2, 1, 3))), ego,
                                    0.3, 0.3, 0.2, 0.1, 0.15)
    _assert_match(got, want)

"""Obstacle sample generation: simulation/obstacles.py, host and device.

CPU: the host mirror reproduces the reference's RNG stream bit for bit (the golden vectors were
drawn by the reference's own generate_obstacle_scenarios with seed 42) and the layout packer is
a pure transpose; the device generator's NumPy mirror (oracle/philox_sampler.py) reproduces the
published Philox4x32-10 known-answer vectors and its log / cos / sin series agree with extended-
precision references.  GPU: the kernel against that mirror value for value, the sampler's
distribution (moments, correlation, normality), determinism and stream separation, the noise-free
first step, strided outputs, and the sampler -> halfspace kernel pipeline against the C oracle on
the same samples.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN_DIR, OFFSET_TOL, REPO, load_golden
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.config.scenarios import get_scenario_config
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.simulation import obstacles as ob


@pytest.mark.parametrize("name,scenario,n,keep", [("head_on_n100_t20", "head_on", 100, 20),
                                                  ("multi_obstacle_n1000_t8", "multi_obstacle", 1000, 8),
                                                  ("multi_obstacle_n20_h30", "multi_obstacle", 20, 30)])
def test_host_generator_reproduces_reference_stream(name, scenario, n, keep):
    gold = load_golden(os.path.join(GOLDEN_DIR, f"{name}.npz"))
    np.random.seed(42)                                            # main.py:191
    data = ob.generate_obstacle_scenarios(get_scenario_config(scenario), 30.0, 0.2, n)
    got = np.stack([np.transpose(tr[:, :keep], (1, 0, 2)) for tr in data["sample_trajectories"]])
    np.testing.assert_array_equal(got, gold["samples"])
    assert len(data["realization_trajectories"]) == got.shape[0]
    for nom, real in zip(data["nominal_trajectories"], data["realization_trajectories"]):
        assert nom.shape == (151, 2) and real.shape == (151, 2)
        np.testing.assert_array_equal(real[0], nom[0])


def test_nominal_trajectory_rules():
    p = ob.generate_nominal_trajectory(np.array([1.0, 2.0]), np.array([0.0, 0.0]), 1.0, 5, 0.2)
    np.testing.assert_array_equal(p, np.tile([1.0, 2.0], (6, 1)))        # stationary (:23-25)
    p = ob.generate_nominal_trajectory(np.array([0.0, 0.0]), np.array([3.0, 4.0]), 2.0, 3, 0.5)
    np.testing.assert_allclose(p[-1], [3 * 0.5 * 2.0 * 0.6, 3 * 0.5 * 2.0 * 0.8], atol=1e-15)


def test_pack_layout_is_a_transpose():
    import torch
    rng = np.random.default_rng(0)
    trs = [rng.normal(size=(7, 11, 2)) for _ in range(3)]
    packed = ob.pack_sample_trajectories(trs, 9, torch.device("cpu"), pin=False)
    assert tuple(packed.shape) == (3, 9, 7, 2) and packed.is_contiguous()
    np.testing.assert_array_equal(packed.numpy(), np.stack([np.transpose(t[:, :9], (1, 0, 2)) for t in trs]))


# Random123 kat_vectors, philox4x32 10 rounds: (counter, key) -> output
PHILOX_KAT = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
              ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
              ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
               (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]


@pytest.mark.parametrize("ctr,key,want", PHILOX_KAT)
def test_philox_mirror_known_answers(ctr, key, want):
    from oracle import philox_sampler as ps
    got = ps.philox4x32_10(*ctr, *key)
    assert tuple(int(x) for x in got) == want


def test_sampler_series_accuracy():
    """The kernel's table-driven log / cos / sin (restated by the mirror with the kernel's own
    tables) against extended-precision references: log uniform32(x) within 2 ulp over every
    kind of 32-bit word (u -> 1 included: the last mantissa centre is 1), cos / sin of
    2 pi w / 2^32 within 2.5e-16."""
    from oracle import philox_sampler as ps
    rng = np.random.default_rng(3)
    x = np.concatenate([rng.integers(0, 2 ** 32, size=1_000_000, dtype=np.uint64),
                        np.array([0, 1, 2, 2 ** 31 - 1, 2 ** 31, 2 ** 32 - 2, 2 ** 32 - 1,
                                  (2 ** 32 - 2 ** 24), 2 ** 25, 2 ** 24 - 1], dtype=np.uint64)])
    u = ps.uniform32(x)
    ref = np.log(u.astype(np.longdouble))
    ulp = np.spacing(np.abs(ref.astype(np.float64)))
    assert np.max(np.abs(ps.log_u32(x) - ref) / ulp) <= 2.0
    c, s = ps.cos_sin_u32(x)
    pi = np.longdouble("3.14159265358979323846264338327950288")
    th = (x.astype(np.longdouble) / np.longdouble(2.0 ** 32)) * (2 * pi)
    assert np.max(np.abs(c - np.cos(th))) < 2.5e-16 and np.max(np.abs(s - np.sin(th))) < 2.5e-16
    assert np.allclose(c * c + s * s, 1.0, atol=5e-16, rtol=0)


def test_sampler_tables_are_the_generated_ones():
    """csrc/drcvar_sampling_tables.inc holds exactly what scripts/gen_sampler_tables.py computes
    (the kernel and the mirror read the same bits)."""
    import importlib.util
    from oracle import philox_sampler as ps
    spec = importlib.util.spec_from_file_location("gen", os.path.join(REPO, "scripts", "gen_sampler_tables.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    cs, sn = gen.turn_table()
    inv, nl = gen.log_table()
    np.testing.assert_array_equal(ps.TURN, np.stack([cs, sn], 1))
    np.testing.assert_array_equal(ps.LOGT, np.stack([inv, nl], 1))
    assert ps.LOGT[-1, 0] == 1.0 and ps.LOGT[-1, 1] == 0.0


def test_uniform_open_interval_extremes():
    """no word may map to u = 0 or 1 (log -> -inf / 0: an infinite or zero Box-Muller
    radius); the 32-bit uniform is exact and stays in [2^-33, 1 - 2^-33]."""
    from oracle import philox_sampler as ps
    hi = ps.uniform32(np.array([0xFFFFFFFF], dtype=np.uint64))[0]
    lo = ps.uniform32(np.array([0], dtype=np.uint64))[0]
    assert hi == 1.0 - 2.0 ** -33 and lo == 2.0 ** -33
    for w in (0, 0xFFFFFFFF):
        r = np.sqrt(-2.0 * ps.log_u32(np.array([w], dtype=np.uint64)))[0]
        assert np.isfinite(r) and r > 0


@pytest.fixture(scope="module")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def _nominal(dev, O=2, T=3):
    import torch
    nom = torch.tensor([[[0.5 * o + 0.1 * t, -0.25 * o + 0.2 * t] for t in range(T)] for o in range(O)],
                       dtype=torch.float64)
    return nom.to(dev)


@pytest.mark.gpu
def test_device_sampler_moments_and_normality(dev):
    from scipy import stats
    nom = _nominal(dev)
    N = 400_000
    for cov in (ob.NOISE_COV, np.array([[0.04, 0.012], [0.012, 0.02]])):
        s = ob.sample_trajectories_device(nom, N, cov, seed=123).cpu().numpy()
        nh = nom.cpu().numpy()
        np.testing.assert_array_equal(s[:, 0], np.broadcast_to(nh[:, 0, None, :], s[:, 0].shape))
        L = np.linalg.cholesky(cov)
        for o in range(s.shape[0]):
            for t in range(1, s.shape[1]):
                d = s[o, t] - nh[o, t]
                se = np.sqrt(np.diag(cov) / N)
                assert np.all(np.abs(d.mean(0)) < 5 * se), (o, t, d.mean(0))
                emp = np.cov(d.T)
                assert np.all(np.abs(emp - cov) < 6 * np.sqrt(2.0 / N) * np.max(cov)), emp
                z = np.linalg.solve(L, d.T)
                for comp in z:
                    assert stats.kstest(comp, "norm").pvalue > 1e-4


@pytest.mark.gpu
def test_device_sampler_radius_tail(dev):
    """the Box-Muller radius comes from a 32-bit uniform (u >= 2^-33), so |z| is capped
    at sqrt(66 ln 2) = 6.76 sd (P(R > 6.76) = 2^-33 for the reference's 53-bit draws: 0.0075 samples
    per 128 M-sample C5 refill).  The tail below the cap must keep the Rayleigh frequencies
    P(R > r) = exp(-r^2 / 2): counts of R > 3, 4, 5 sd over 32 M samples within 5 Poisson sd."""
    import torch
    nom = torch.zeros((1, 2, 2), dtype=torch.float64, device=dev)
    N = 1 << 25
    s = ob.sample_trajectories_device(nom, N, np.eye(2), seed=2024)[0, 1]
    r2 = (s * s).sum(-1)
    assert float(r2.max()) <= 66 * np.log(2) + 1e-9
    for r in (3.0, 4.0, 5.0):
        got = int((r2 > r * r).sum())
        want = N * np.exp(-r * r / 2)
        assert abs(got - want) < 5 * np.sqrt(want) + 1, (r, got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("O,T,N,seed,stream,zero_first", [(2, 3, 5000, 123, 0, True),
                                                          (3, 5, 777, 2 ** 40 + 9, 2 ** 33 + 1, False),
                                                          (1, 2, 1, 0, 0, True)])
def test_device_sampler_matches_mirror(dev, O, T, N, seed, stream, zero_first):
    """Kernel vs oracle/philox_sampler.py on the same (seed, stream, indices): equal up to the
    FMA contraction of the series (a few ulp)."""
    import torch
    from oracle import philox_sampler as ps
    cov = np.array([[0.04, 0.012], [0.012, 0.02]])
    nom = _nominal(dev, O, T)
    got = ob.sample_trajectories_device(nom, N, cov, seed=seed, stream_offset=stream,
                                        zero_first_step=zero_first).cpu().numpy()
    L = np.linalg.cholesky(cov)
    want = ps.sample_trajectories(nom.cpu().numpy(), N, (L[0, 0], L[1, 0], L[1, 1]), seed, stream,
                                  zero_first)
    assert got.shape == want.shape
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-14)


@pytest.mark.gpu
def test_device_sampler_determinism_streams_and_strides(dev):
    import torch
    nom = _nominal(dev, 3, 4)
    a = ob.sample_trajectories_device(nom, 1000, seed=7)
    b = ob.sample_trajectories_device(nom, 1000, seed=7)
    assert torch.equal(a, b)
    c = ob.sample_trajectories_device(nom, 1000, seed=8)
    d = ob.sample_trajectories_device(nom, 1000, seed=7, stream_offset=1)
    assert not torch.equal(a[:, 1:], c[:, 1:]) and not torch.equal(a[:, 1:], d[:, 1:])
    # a strided destination (the reference's [O, N, T, 2] order) receives the same values
    big = torch.zeros((3, 1000, 4, 2), dtype=torch.float64, device=dev)
    ob.sample_trajectories_device(nom, 1000, seed=7, out=big.permute(0, 2, 1, 3))
    assert torch.equal(big.permute(0, 2, 1, 3), a)
    # the noise-free first step is optional
    e = ob.sample_trajectories_device(nom, 1000, seed=7, zero_first_step=False)
    assert torch.equal(e[:, 1:], a[:, 1:]) and not torch.equal(e[:, 0], a[:, 0])


@pytest.mark.gpu
def test_device_scenario_feeds_the_engine(dev):
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import engine, synthetic
    from oracle import c_oracle
    data = ob.generate_obstacle_scenarios_device(get_scenario_config("multi_obstacle"), 30.0, 0.2,
                                                 1000, seed=5, device=dev)
    samples = data["sample_trajectories"][:, :20]                  # [O, 20, N, 2] view
    ego = synthetic.straight_line_ego(20, dev, start=(-2.0, -1.0), goal=(4.0, 0.0))
    rec = engine.safe_halfspaces(samples, ego, engine.RiskParams()).cpu().numpy()
    ref = c_oracle.safe_halfspaces(samples.contiguous().cpu().numpy(), ego.cpu().numpy(),
                                   0.3, 0.3, 0.2, 0.1, 0.15)
    assert np.max(np.abs(rec - ref)) < OFFSET_TOL


@pytest.mark.gpu
@pytest.mark.parametrize("O,T,N,begin,count", [(4, 5, 300, 0, 20), (4, 5, 300, 3, 9), (4, 5, 300, 7, 13),
                                               (3, 7, 1000, 20, 1), (2, 3, 1, 1, 4), (5, 4, 64, 6, 0)])
def test_device_sampler_unit_range_is_a_slice_of_the_batch(dev, O, T, N, begin, count):
    """drcvar_sample_units_f64 draws exactly the whole batch's samples of units [begin, begin+count)
    (same counters, same arithmetic: bit-equal), including the noise-free step 0 of obstacles whose
    start falls inside the range — the per-rank sampling of a sharded global batch."""
    import torch
    nom = _nominal(dev, O, T)
    whole = ob.sample_trajectories_device(nom, N, seed=99, stream_offset=5)
    part = ob.sample_units_device(nom, N, begin, count, seed=99, stream_offset=5)
    assert part.shape == (count, N, 2)
    assert torch.equal(part, whole.reshape(O * T, N, 2)[begin:begin + count])
    # a strided destination (every other unit of a larger buffer)
    big = torch.full((2 * count + 1, N, 2), -7.0, dtype=torch.float64, device=dev)
    ob.sample_units_device(nom, N, begin, count, seed=99, stream_offset=5, out=big[::2][:count])
    assert torch.equal(big[::2][:count], part)
    if count:
        assert bool((big[1::2] == -7.0).all())


@pytest.mark.gpu
def test_device_sampler_large_batch_paths(dev):
    """A batch above the 256 MB MALL (12 800 units x 2 600 samples, 532 MB) takes the nontemporal
    store path and workgroup rows that loop over several units; its values equal the ordinary path's
    (small unit-range draws: packed stores, one unit per row) bit for bit, and the mirror's."""
    import torch
    from oracle import philox_sampler as ps
    O, T, N = 256, 50, 2600
    cov = np.array([[0.04, 0.012], [0.012, 0.02]])
    nom = _nominal(dev, O, T)
    whole = ob.sample_trajectories_device(nom, N, cov, seed=31, stream_offset=3)
    flat = whole.reshape(O * T, N, 2)
    for begin, count in ((0, 3), (4321, 5), (O * T - 4, 4)):
        part = ob.sample_units_device(nom, N, begin, count, cov, seed=31, stream_offset=3)
        assert torch.equal(part, flat[begin:begin + count]), (begin, count)
    L = np.linalg.cholesky(cov)
    want = ps.sample_trajectories(nom[:1].cpu().numpy(), N, (L[0, 0], L[1, 0], L[1, 1]), 31, 3, True)
    np.testing.assert_allclose(whole[:1].cpu().numpy(), want, rtol=0, atol=1e-14)
    del whole, flat


@pytest.mark.gpu
@pytest.mark.parametrize("cov", ["iso", "full"])
def test_device_sampler_full_blocks_repeatable_and_mirrored(dev, cov):
    """The full-block store path (every pair of a workgroup's range in the unit: no per-pair test)
    on a batch above the MALL (nontemporal stores), for the isotropic covariance (the scale rides in
    the log) and a full one: two refills into buffers pre-filled with different values are bitwise
    equal (a store-data hazard once corrupted a few hundred samples per refill at random,
    scripts/micro/sampler_check.py), every sample is written, and full-block units match the
    NumPy mirror and the ordinary-store unit-range draws."""
    import torch
    from oracle import philox_sampler as ps
    O, T, N = 64, 50, 10001                      # odd N: the last workgroup of a unit takes the checked loop
    c = ob.NOISE_COV if cov == "iso" else np.array([[0.04, 0.012], [0.012, 0.02]])
    nom = _nominal(dev, O, T)
    a = torch.full((O, T, N, 2), 7.0, dtype=torch.float64, device=dev)
    b = torch.full((O, T, N, 2), -7.0, dtype=torch.float64, device=dev)
    ob.sample_trajectories_device(nom, N, c, seed=17, out=a)
    ob.sample_trajectories_device(nom, N, c, seed=17, out=b)
    assert torch.equal(a, b), int((a != b).any(-1).sum())
    flat = a.view(O * T, N, 2)
    for begin in (1, 1601, O * T - 2):
        part = ob.sample_units_device(nom, N, begin, 2, c, seed=17)
        assert torch.equal(part, flat[begin:begin + 2]), begin
    L = np.linalg.cholesky(c)
    want = ps.sample_trajectories(nom[:1, :3].cpu().numpy(), N, (L[0, 0], L[1, 0], L[1, 1]), 17, 0, True)
    np.testing.assert_allclose(a[:1, :3].cpu().numpy(), want, rtol=0, atol=1e-14)
    del a, b, flat


@pytest.mark.gpu
@pytest.mark.parametrize("cov,N", [(np.diag([1e-6, 1e-6]), 4097), (np.diag([9.0, 9.0]), 4097),
                                   (np.diag([0.01, 0.04]), 4097),
                                   (np.array([[0.04, 0.01], [0.01, 0.04]]), 4097),
                                   (np.diag([0.01, 0.01]), 4096), (np.diag([0.01, 0.04]), 4096)])
def test_device_sampler_covariance_forms_match_mirror(dev, cov, N):
    """Each covariance form against the mirror, on full-block and checked workgroups (N = 4097:
    2 049 pairs, the first workgroup's 2 048 full; N = 4096: exactly one full workgroup per unit):
    isotropic at a small and a large scale (the scale carried by the log's coefficients and table),
    diagonal but not isotropic and a correlated one with equal variances (both nominal + L z)."""
    from oracle import philox_sampler as ps
    O, T = 2, 3
    nom = _nominal(dev, O, T)
    got = ob.sample_trajectories_device(nom, N, cov, seed=5, stream_offset=2).cpu().numpy()
    L = np.linalg.cholesky(cov)
    want = ps.sample_trajectories(nom.cpu().numpy(), N, (L[0, 0], L[1, 0], L[1, 1]), 5, 2, True)
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-14 * max(1.0, float(L[0, 0])))


def test_device_sampler_unit_range_validation():
    import torch
    if not torch.cuda.is_available():
        with pytest.raises(ValueError):
            ob.sample_units_device(torch.zeros((2, 3, 2), dtype=torch.float64), 10, 0, 6)
        return
    nom = torch.zeros((2, 3, 2), dtype=torch.float64, device="cuda")
    with pytest.raises(ValueError):
        ob.sample_units_device(nom, 10, 4, 3)

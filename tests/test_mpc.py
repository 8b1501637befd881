"""MPC hand-off (core/mpc_filter.py:40-219): the QP that consumes the safe halfspaces.

CPU: the oracle against its golden vectors and KKT certificates, the host-side condensation in
``drcvar_mpc_model_init`` against a NumPy restatement, argument validation, the reference's
list packing and fallback-input rules.  GPU (-m gpu): the HIP interior-point kernel against the
oracle — golden scenarios, every metric, random problems with active slacks / input bounds /
position bounds, several dynamics and input widths, batches, strided record views, the fallback
path and the C5 hand-off shape.  Tolerance: the optimum is unique (strictly convex objective),
both solvers return it to ~1e-9, so inputs and states must agree within MPC_TOL.
"""
import ctypes
import glob
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN_DIR
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import _native
from oracle import mpc_qp

MPC_TOL = 1e-6      # |u - u_oracle|, |x - x_oracle| (the halfspace offsets themselves are 1e-6)
OBJ_RTOL = 1e-7

MPC_GOLDEN = sorted(glob.glob(os.path.join(GOLDEN_DIR, "mpc_*.npz")))


def load(path):
    z = np.load(path, allow_pickle=False)
    return {k: z[k] for k in z.files}


def double_integrator(dt=0.2):
    A = np.block([[np.eye(2), dt * np.eye(2)], [np.zeros((2, 2)), np.eye(2)]])
    B = np.block([[0.5 * dt ** 2 * np.eye(2)], [dt * np.eye(2)]])
    C = np.block([np.eye(2), np.zeros((2, 2))])
    return A, B, C


def condense(A, B, C, Q, R, H):
    """NumPy restatement of the condensation drcvar_mpc_model_init performs."""
    nx, nu = A.shape[0], B.shape[1]
    n = nu * H
    Ap = [np.eye(nx)]
    for _ in range(H):
        Ap.append(A @ Ap[-1])
    Gx = np.zeros((H * nx, n))
    Phi = np.zeros((H * nx, nx))
    for k in range(H):
        Phi[k * nx:(k + 1) * nx] = Ap[k + 1]
        for j in range(k + 1):
            Gx[k * nx:(k + 1) * nx, j * nu:(j + 1) * nu] = Ap[k - j] @ B
    Qb = np.kron(np.eye(H), Q)
    return {"H0": 2 * (Gx.T @ Qb @ Gx + np.kron(np.eye(H), R)), "F1": 2 * Gx.T @ Qb @ Phi,
            "F2": 2 * Gx.T @ Qb, "Mp": np.array([C @ Ap[i] @ B for i in range(H)]),
            "CA": np.array([C @ Ap[k + 1] for k in range(H)])}


def model_init(A, B, C, Q, R, H, ub=None, pb=None, blob=True):
    lib = _native.lib()
    arrs = [np.ascontiguousarray(m, dtype=np.float64) for m in (A, B, C, Q, R)]
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p) if a is not None else None
    ubs = [np.ascontiguousarray(b, dtype=np.float64) for b in ub] if ub is not None else [None, None]
    pbs = [np.ascontiguousarray(b, dtype=np.float64) for b in pb] if pb is not None else [None, None]
    m = _native.MpcModel()
    args = [*(p(a) for a in arrs), arrs[0].shape[0], arrs[1].shape[1], arrs[2].shape[0], H,
            p(ubs[0]), p(ubs[1]), p(pbs[0]), p(pbs[1]), ctypes.byref(m)]
    rc = lib.drcvar_mpc_model_init(*args, None)
    if rc != 0 or not blob:
        return rc, m, None
    out = np.zeros(m.blob_doubles)
    rc = lib.drcvar_mpc_model_init(*args, p(out))
    return rc, m, out


# ------------------------------------------------------------------------------ CPU

@pytest.mark.parametrize("path", MPC_GOLDEN, ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_reproduces_golden_with_kkt_certificate(path):
    z = load(path)
    H = int(z["horizon"])
    for m in range(3):
        rows = [z["hs"][m][:, t] for t in range(z["hs"].shape[2])]
        x, u, info = mpc_qp.filter_trajectory(z["A"], z["B"], z["C"], z["Q"], z["R"], H, z["x0"],
                                              z["x_ref"], z["u_ref"], rows, tuple(z["u_bounds"]),
                                              tuple(z["p_bounds"]))
        assert info["status"] == "optimal"
        assert max(info["kkt"].values()) < 1e-8
        np.testing.assert_allclose(u, z["u_expected"][m], atol=1e-9)
        np.testing.assert_allclose(x, z["x_expected"][m], atol=1e-9)
        assert abs(info["objective"] - z["objective"][m]) <= 1e-9 * abs(z["objective"][m])


def _c5_degenerate():
    z = load(os.path.join(GOLDEN_DIR, "qp_c5_degenerate.npz"))
    rows = [np.concatenate([z["h"][:, t], z["g"][:, t, None]], -1) for t in range(z["h"].shape[1])]
    return z, rows


def test_oracle_polishes_the_degenerate_c5_handoff():
    """bench.py's C5 hand-off of round 3 (tests/golden/make_golden_qp_c5.py): the oracle's IPM
    stalls at merit ~4e-10 and its three guessed active sets fail; the one-row-per-step refinement
    (mpc_qp._polish_steps) must find the exact answer (before it, the oracle returned an
    OPTIMAL_INACCURATE iterate 2e-4 away from the device's better answer)."""
    z, rows = _c5_degenerate()
    A, B, C = double_integrator()
    H = z["x_ref"].shape[0] - 1
    x, u, info = mpc_qp.filter_trajectory(A, B, C, 2 * np.eye(4), np.eye(2), H, z["x0"], z["x_ref"],
                                          None, rows, tuple(z["u_bounds"]), tuple(z["p_bounds"]))
    assert info["status"] == "optimal" and info["polished"]
    assert max(info["kkt"].values()) < 1e-9, info["kkt"]
    np.testing.assert_allclose(u, z["u_expected"], atol=1e-9)
    assert abs(info["objective"] - float(z["objective"])) <= 1e-12 * float(z["objective"])


def _h30_straggler():
    z = load(os.path.join(GOLDEN_DIR, "qp_h30_straggler.npz"))
    rows = [np.concatenate([z["h"][:, t], z["g"][:, t, None]], -1) for t in range(z["h"].shape[1])]
    return z, rows


def test_oracle_certifies_the_h30_straggler():
    """The slowest of scripts/mpc_bench.py's 1024 distinct main.py-like QPs (tests/golden/
    make_golden_qp_straggler.py: weakly active rows, the kernel's Mehrotra steps alternate long and
    short): the oracle's answer is KKT-certified and reproduces the fixture."""
    z, rows = _h30_straggler()
    A, B, C = double_integrator()
    H = z["x_ref"].shape[0] - 1
    x, u, info = mpc_qp.filter_trajectory(A, B, C, 2 * np.eye(4), np.eye(2), H, z["x0"], z["x_ref"],
                                          None, rows, tuple(z["u_bounds"]), tuple(z["p_bounds"]))
    assert info["status"] == "optimal"
    assert max(info["kkt"].values()) < 1e-9, info["kkt"]
    np.testing.assert_allclose(u, z["u_expected"], atol=1e-9)
    assert abs(info["objective"] - float(z["objective"])) <= 1e-12 * float(z["objective"])


def _c5_mean():
    z = load(os.path.join(GOLDEN_DIR, "qp_c5_mean.npz"))
    rows = [np.concatenate([z["h"][:, t], z["g"][:, t, None]], -1) for t in range(z["g"].shape[1])]
    return z, rows


def test_oracle_certifies_the_c5_mean_filter():
    """bench.py's main_flow_c5 mean-metric filter (tests/golden/make_golden_qp_c5_mean.py: the
    MeanSafeHalfspace rows of 256 obstacles x 50 steps, core/halfspaces.py:70-106 — directions from
    the origin, so many rows are violated by the ego line and their slacks are active): the
    oracle's answer is KKT-certified and reproduces the fixture."""
    z, rows = _c5_mean()
    A, B, C = double_integrator()
    H = z["x_ref"].shape[0] - 1
    x, u, info = mpc_qp.filter_trajectory(A, B, C, 2 * np.eye(4), np.eye(2), H, z["x0"], z["x_ref"],
                                          None, rows, tuple(z["u_bounds"]), tuple(z["p_bounds"]))
    assert info["status"] == "optimal"
    assert max(info["kkt"].values()) < 1e-9, info["kkt"]
    np.testing.assert_allclose(u, z["u_expected"], atol=1e-9)
    assert abs(info["objective"] - float(z["objective"])) <= 1e-12 * float(z["objective"])


def test_oracle_without_constraints_is_the_lq_tracking_solution():
    A, B, C = double_integrator()
    H = 12
    Q, R = 2 * np.eye(4), np.eye(2)
    x0 = np.array([0.3, -0.2, 0.1, 0.0])
    x_ref = np.cumsum(np.full((H + 1, 4), 0.05), axis=0)
    x, u, info = mpc_qp.filter_trajectory(A, B, C, Q, R, H, x0, x_ref, None, [])
    cd = condense(A, B, C, Q, R, H)
    f = cd["F1"] @ x0 - cd["F2"] @ x_ref[1:].reshape(-1)
    u_star = np.linalg.solve(cd["H0"], -f).reshape(H, 2)
    np.testing.assert_allclose(u, u_star, atol=1e-10)


def test_oracle_fallback_rules_match_reference():
    """_fallback (mpc_filter.py:197-210): shifted last optimum, tail from u_ref; else u_ref."""
    H, nu = 5, 2
    u_ref = np.arange(H * nu, dtype=float).reshape(H, nu)
    np.testing.assert_array_equal(mpc_qp.fallback_inputs(H, nu, u_ref, None), u_ref)
    last = 100 + np.arange(H * nu, dtype=float).reshape(H, nu)
    got = mpc_qp.fallback_inputs(H, nu, u_ref, last)
    np.testing.assert_array_equal(got[:H - 1], last[1:])
    np.testing.assert_array_equal(got[H - 1:], u_ref[H - 1:])


@pytest.mark.parametrize("dyn", ["double", "single", "generic"])
def test_model_init_condensation(dyn):
    rng = np.random.default_rng(3)
    if dyn == "double":
        A, B, C = double_integrator()
        H = 30
    elif dyn == "single":
        A, B, C = np.eye(2), 0.2 * np.eye(2), np.eye(2)
        H = 60
    else:
        A = np.eye(3) + 0.05 * rng.normal(size=(3, 3))
        B = rng.normal(size=(3, 1))
        C = rng.normal(size=(2, 3))
        H = 64
    nx, nu = A.shape[0], B.shape[1]
    Q, R = 2 * np.eye(nx), np.eye(nu)
    rc, m, blob = model_init(A, B, C, Q, R, H)
    assert rc == 0
    assert (m.n_states, m.n_inputs, m.n_outputs, m.horizon) == (nx, nu, 2, H)
    ref = condense(A, B, C, Q, R, H)
    o = 0
    for key in ("H0", "F1", "F2", "Mp", "CA"):
        size = ref[key].size
        np.testing.assert_allclose(blob[o:o + size], ref[key].reshape(-1), rtol=1e-12, atol=1e-12,
                                   err_msg=key)
        o += size
    tail = np.concatenate([A.ravel(), B.ravel(), C.ravel(), Q.ravel(), R.ravel()])
    np.testing.assert_array_equal(blob[o:o + tail.size], tail)
    o += tail.size
    # the starting point's maps: u_free = -H0^-1 f = UF1 x0 + UF2 xr, then the flag
    uf1 = -np.linalg.solve(ref["H0"], ref["F1"])
    uf2 = np.linalg.solve(ref["H0"], ref["F2"])
    for name, want in (("UF1", uf1), ("UF2", uf2)):
        np.testing.assert_allclose(blob[o:o + want.size], want.reshape(-1), rtol=1e-9,
                                   atol=1e-8 * np.abs(want).max(), err_msg=name)
        o += want.size
    assert blob[o] == 1.0
    o += 1
    # the planar isotropic flag (the double integrator: the register-form factorisation)
    assert blob[o] == (1.0 if dyn == "double" else 0.0)
    o += 1
    assert o == m.blob_doubles


def test_model_init_bounds_and_validation():
    A, B, C = double_integrator()
    Q, R = 2 * np.eye(4), np.eye(2)
    rc, m, _ = model_init(A, B, C, Q, R, 30, ub=([-5, -4], [5, 4]), pb=([-10, -9], [10, 9]),
                          blob=False)
    assert rc == 0 and m.has_input_bounds and m.has_position_bounds
    assert list(m.u_min)[:2] == [-5, -4] and list(m.p_max) == [10, 9]
    E = _native.ERR_INVALID_ARGUMENT
    assert model_init(A, B, np.eye(4), Q, R, 30)[0] == E                  # n_outputs must be 2
    assert model_init(A, B, C, Q, R, 0)[0] == E
    assert model_init(A, B, C, Q, R, 61)[0] == _native.ERR_UNSUPPORTED    # nu*H > 120
    assert model_init(A, B, C, Q, R, 65)[0] == _native.ERR_UNSUPPORTED
    bad = A.copy()
    bad[0, 0] = np.nan
    assert model_init(bad, B, C, Q, R, 10)[0] == E
    assert model_init(A, B, C, Q, R, 10, ub=([-5, np.inf], [5, 5]))[0] == E


def test_workspace_size():
    A, B, C = double_integrator()
    _, m, _ = model_init(A, B, C, 2 * np.eye(4), np.eye(2), 30, blob=False)
    ws = _native.lib().drcvar_mpc_workspace_doubles(ctypes.byref(m), 3, 10)
    assert ws == 3 * (10 * 10 * 64 + 1152)


def test_filter_argument_validation_host_side():
    A, B, C = double_integrator()
    _, m, _ = model_init(A, B, C, 2 * np.eye(4), np.eye(2), 30, blob=False)
    lib = _native.lib()
    vp = ctypes.c_void_p

    def call(**kw):
        a = dict(blob=16, B=1, h=16, g=16, O=1, K=1, x0=16, xr=16, uf=16, it=60, tol=1e-9, out=16,
                 ws=16, wsn=10 ** 6)
        a.update(kw)
        return lib.drcvar_mpc_filter_f64(
            ctypes.byref(m), vp(a["blob"]), a["B"], vp(a["h"]), vp(a["g"]), a["O"], a["K"],
            0, 0, 0, 0, 0, 0, vp(a["x0"]), 4, vp(a["xr"]), 124, 4, vp(a["uf"]), 60, 2, a["it"],
            a["tol"], 1, vp(a["out"]), vp(a["out"]), vp(a["out"]), vp(a["ws"]), a["wsn"], None)

    assert call(B=0) == 0                                   # empty batch: nothing enqueued
    assert call(it=0) == _native.ERR_INVALID_ARGUMENT
    assert call(tol=0.0) == _native.ERR_INVALID_ARGUMENT
    assert call(h=0) == _native.ERR_INVALID_ARGUMENT
    assert call(ws=0) == _native.ERR_INVALID_ARGUMENT
    assert call(wsn=10) == _native.ERR_INVALID_ARGUMENT
    assert call(B=-1) == _native.ERR_INVALID_ARGUMENT


def test_pack_halfspace_lists_pads_ragged_steps():
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core.halfspaces import SafeHalfspace
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core.mpc_filter import (
        pack_halfspace_lists)
    lists = [[SafeHalfspace(np.array([1.0, 0.0]), -2.0)],
             [SafeHalfspace(np.array([0.0, 1.0]), -1.0), SafeHalfspace(np.array([0.6, 0.8]), 0.5)],
             [SafeHalfspace(np.array([1.0, 0.0]), 3.0)]]
    h, g = pack_halfspace_lists(lists, horizon=2)      # steps beyond the horizon are dropped
    assert h.shape == (2, 2, 2) and g.shape == (2, 2)
    np.testing.assert_array_equal(h[:, 0], [[1, 0], [0, 0]])
    np.testing.assert_array_equal(g[:, 0], [-2, -1])   # padded row: h = 0, g = -1
    np.testing.assert_array_equal(h[:, 1], [[0, 1], [0.6, 0.8]])
    np.testing.assert_array_equal(g[:, 1], [-1, 0.5])


# ------------------------------------------------------------------------------ GPU

def _random_problem(rng, O, T, H, dyn="double", bounds=True, tight=True):
    if dyn == "double":
        A, B, C = double_integrator()
    elif dyn == "single":
        A, B, C = np.eye(2), 0.2 * np.eye(2), np.eye(2)
    elif dyn == "generic1":
        A = np.eye(3) + 0.01 * rng.normal(size=(3, 3))
        B = rng.normal(size=(3, 1))
        C = np.eye(3)[:2]
    elif dyn == "generic3":
        A = np.eye(4) + 0.01 * rng.normal(size=(4, 4))
        B = 0.2 * rng.normal(size=(4, 3))
        C = np.eye(4)[:2]
    elif dyn == "generic44":  # four inputs on the 4-state template (the widest NX <= 4 kernels)
        A = np.eye(4) + 0.01 * rng.normal(size=(4, 4))
        B = 0.2 * rng.normal(size=(4, 4))
        C = np.eye(4)[:2]
    elif dyn == "generic8":  # the widest state (padded template NX = 8), a dense output map
        A = np.eye(8) + 0.01 * rng.normal(size=(8, 8))
        B = 0.2 * rng.normal(size=(8, 2))
        C = np.eye(8)[:2] + 0.2 * rng.normal(size=(2, 8))
    elif dyn == "double_full":  # the isotropic double integrator (register-form factorisation)
        A, B, C = double_integrator()  # with a full Q, a dense output map and a coupled R
        C = C + 0.2 * rng.normal(size=(2, 4))
    elif dyn == "drag":  # a true 4-state, 2-input model that is not isotropic: per-axis drag
        dt = 0.2
        A = np.array([[1, 0, dt, 0], [0, 1, 0, dt], [0, 0, 1 - 0.3 * dt, 0], [0, 0, 0, 1 - 0.7 * dt]])
        B = np.array([[0.5 * dt ** 2, 0], [0, 0.5 * dt ** 2], [dt, 0], [0, 1.2 * dt]])
        C = np.eye(4)[:2]
    else:  # generic4
        A = np.eye(5) + 0.01 * rng.normal(size=(5, 5))
        B = 0.2 * rng.normal(size=(5, 4))
        C = np.eye(5)[:2]
    nx, nu = A.shape[0], B.shape[1]
    Q, R = 2 * np.eye(nx), np.eye(nu)
    if dyn == "double_full":
        M = rng.normal(size=(4, 4))
        Q = M @ M.T / 4 + 0.5 * np.eye(4)
        R = np.array([[1.0, 0.3], [0.3, 0.8]])
    x0 = np.zeros(nx)
    x0[:2] = rng.uniform(-3, 3, 2)
    x_ref = np.zeros((H + 1, nx))
    x_ref[:, :2] = x0[:2] + np.outer(np.linspace(0, 1, H + 1), rng.uniform(-6, 6, 2))
    ang = rng.uniform(0, 2 * np.pi, (O, T))
    hs = np.stack([np.cos(ang), np.sin(ang), rng.normal(-1.0 if tight else -6.0, 2.0, (O, T))], -1)
    ub = (np.full(nu, -1.5), np.full(nu, 1.5)) if bounds else None
    pb = (np.array([-4.0, -4.0]), np.array([4.0, 4.0])) if bounds else None
    return dict(A=A, B=B, C=C, Q=Q, R=R, H=H, x0=x0, x_ref=x_ref, u_ref=np.zeros((H, nu)), hs=hs,
                ub=ub, pb=pb)


def _oracle(pr):
    rows = [pr["hs"][:, t] for t in range(pr["hs"].shape[1])]
    return mpc_qp.filter_trajectory(pr["A"], pr["B"], pr["C"], pr["Q"], pr["R"], pr["H"], pr["x0"],
                                    pr["x_ref"], pr["u_ref"], rows, pr["ub"], pr["pb"])


def _gpu(pr, dev, B=1):
    import torch
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf
    model = mf.MPCModel(pr["A"], pr["B"], pr["C"], pr["Q"], pr["R"], pr["H"], pr["ub"], pr["pb"],
                        device=dev)
    T = lambda a: torch.as_tensor(np.ascontiguousarray(a)).to(dev)
    hs = T(pr["hs"])
    x, u, info = mf.filter_batch(model, hs[None, :, :, 0:2], hs[None, :, :, 2], T(pr["x0"][None]),
                                 T(pr["x_ref"][None]), T(pr["u_ref"][None]))
    return x[0].cpu().numpy(), u[0].cpu().numpy(), info[0].cpu().numpy()


@pytest.fixture(scope="module")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


@pytest.mark.gpu
@pytest.mark.parametrize("path", MPC_GOLDEN, ids=lambda p: os.path.basename(p)[:-4])
def test_gpu_golden_scenarios_every_metric(path, dev):
    import torch
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core.halfspaces import (
        HalfspaceBatch)
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core.mpc_filter import (
        MPCSafetyFilter)
    z = load(path)
    H = int(z["horizon"])
    name = os.path.basename(path)[:-4]
    src = json.loads(str(z["meta"]))["halfspaces"]
    record = torch.as_tensor(np.load(os.path.join(GOLDEN_DIR, src))["expected"]).to(dev)
    batch = HalfspaceBatch(record)
    lists = batch.to_lists()
    for m, metric in enumerate(("mean", "cvar", "dr_cvar")):
        f = MPCSafetyFilter(z["A"], z["B"], z["C"], z["Q"], z["R"], H, 0.2)
        args = (z["x0"], z["x_ref"], z["u_ref"])
        bounds = ((z["u_bounds"][0], z["u_bounds"][1]),
                  (np.array([-10, -10, -5, -5.0]), np.array([10, 10, 5, 5.0])))  # main.py:55,111
        x1, u1, i1 = f.filter_trajectory(*args, lists[metric], *bounds)             # reference lists
        x2, u2, i2 = f.filter_trajectory(*args, batch, *bounds, metric=metric)       # device record
        for x, u, info in ((x1, u1, i1), (x2, u2, i2)):
            assert info["status"] == "optimal", (name, metric, info)
            np.testing.assert_allclose(u, z["u_expected"][m], atol=MPC_TOL, err_msg=f"{name} {metric}")
            np.testing.assert_allclose(x, z["x_expected"][m], atol=MPC_TOL, err_msg=f"{name} {metric}")
            assert abs(info["objective"] - z["objective"][m]) <= OBJ_RTOL * abs(z["objective"][m])
        np.testing.assert_array_equal(u1, u2)           # same rows, same launch -> same bits
        np.testing.assert_array_equal(f.last_optimal_u, u2)


@pytest.mark.gpu
@pytest.mark.parametrize("path", MPC_GOLDEN, ids=lambda p: os.path.basename(p)[:-4])
def test_gpu_three_metrics_one_launch(path, dev):
    """main.py:104-112's three filters (mean, CVaR, DR-CVaR) over one halfspace record as ONE
    3-problem launch (bench.py's main_flow_c5 form): each problem equals its metric's golden optimum."""
    import torch
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf
    z = load(path)
    H = int(z["horizon"])
    src = json.loads(str(z["meta"]))["halfspaces"]
    record = torch.as_tensor(np.load(os.path.join(GOLDEN_DIR, src))["expected"]).to(dev)[:, :H]
    O, T = record.shape[0], record.shape[1]
    f = mf.MPCSafetyFilter(z["A"], z["B"], z["C"], z["Q"], z["R"], H, 0.2)
    model = f.model((z["u_bounds"][0], z["u_bounds"][1]),
                    (np.array([-10, -10, -5, -5.0]), np.array([10, 10, 5, 5.0])))
    metrics = ("mean", "cvar", "dr_cvar")
    cols_h = torch.tensor([c for m in metrics for c in (mf.METRIC_COLUMNS[m][0], mf.METRIC_COLUMNS[m][0] + 1)],
                          device=dev)
    cols_g = torch.tensor([mf.METRIC_COLUMNS[m][1] for m in metrics], device=dev)
    h3 = record.index_select(2, cols_h).view(O, T, 3, 2).permute(2, 0, 1, 3)
    g3 = record.index_select(2, cols_g).permute(2, 0, 1)
    nx = z["A"].shape[0]
    x0 = torch.as_tensor(np.repeat(np.asarray(z["x0"], dtype=np.float64).reshape(1, nx), 3, 0)).to(dev)
    xr = torch.as_tensor(np.repeat(np.asarray(z["x_ref"], dtype=np.float64)[None, :H + 1], 3, 0)).to(dev)
    uf = torch.as_tensor(np.repeat(f._fallback_inputs(z["u_ref"])[None], 3, 0)).to(dev)
    x, u, info = mf.filter_batch(model, h3, g3, x0, xr, uf, f.max_iter, f.tol)
    u, info = u.cpu().numpy(), info.cpu().numpy()
    for m, metric in enumerate(metrics):
        assert int(info[m, _native.MPC_INFO_STATUS]) == _native.MPC_STATUS_OPTIMAL, (metric, info[m])
        np.testing.assert_allclose(u[m], z["u_expected"][m], atol=MPC_TOL, err_msg=metric)


@pytest.mark.gpu
@pytest.mark.parametrize("dyn,H,O,T,bounds,tight", [
    ("double", 30, 6, 30, True, True), ("double", 50, 40, 50, True, True),
    ("double", 60, 3, 60, True, False), ("double", 1, 2, 1, True, True),
    ("double", 7, 5, 12, True, True), ("double", 20, 4, 9, False, True),
    ("double", 25, 0, 0, True, True), ("single", 60, 8, 60, True, True),
    ("generic1", 64, 4, 64, True, True), ("generic3", 40, 5, 40, True, True),
    ("generic4", 30, 5, 30, True, True), ("generic44", 30, 5, 30, True, True),
    ("generic8", 24, 4, 24, False, True), ("double_full", 30, 6, 30, True, True),
    ("double_full", 50, 20, 50, True, True), ("drag", 30, 6, 30, True, True), ("drag", 50, 20, 50, True, True),
])
def test_gpu_random_problems_match_oracle(dyn, H, O, T, bounds, tight, dev):
    rng = np.random.default_rng(H * 1000 + O * 10 + T)
    for trial in range(3):
        pr = _random_problem(rng, O, T, H, dyn, bounds, tight)
        xo, uo, io = _oracle(pr)
        assert io["status"] == "optimal" and max(io["kkt"].values()) < 1e-8
        x, u, info = _gpu(pr, dev)
        assert int(info[_native.MPC_INFO_STATUS]) in (_native.MPC_STATUS_OPTIMAL,
                                                     _native.MPC_STATUS_OPTIMAL_INACCURATE), info
        assert info[_native.MPC_INFO_USED_FALLBACK] == 0
        assert info[_native.MPC_INFO_POLISHED] == 1, info
        np.testing.assert_allclose(u, uo, atol=MPC_TOL, err_msg=f"{dyn} H={H} O={O} trial {trial}")
        np.testing.assert_allclose(x, xo, atol=MPC_TOL)
        assert abs(info[_native.MPC_INFO_OBJECTIVE] - io["objective"]) <= 1e-6 * max(1.0, abs(io["objective"]))
        assert abs(info[_native.MPC_INFO_MAX_SLACK] - max(io["slacks"].max(initial=0.0), 0.0)) < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("H,O", [(30, 6), (50, 20)])
def test_gpu_isotropic_and_general_factorisations_agree(H, O, dev):
    """The register-form factorisation (chosen when A and B are blocks of multiples of I2, checked
    exactly) against the general LDS form on the SAME model: A's zero (0, 1) entry set to 1e-300
    defeats the exact check without changing the model at fp64 resolution.  A full Q, a dense C and
    a coupled R (only A and B select the form): both forms' answers agree with each other and with
    the oracle (the isotropic form was only ever checked with Q = 2I, C = [I 0])."""
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf
    rng = np.random.default_rng(7 * H + O)
    for trial in range(3):
        pr = _random_problem(rng, O, H, H, "double_full")
        iso = mf.MPCModel(pr["A"], pr["B"], pr["C"], pr["Q"], pr["R"], H, pr["ub"], pr["pb"], device=dev)
        A2 = pr["A"].copy()
        A2[0, 1] = 1e-300
        gen = mf.MPCModel(A2, pr["B"], pr["C"], pr["Q"], pr["R"], H, pr["ub"], pr["pb"], device=dev)
        assert iso.host_blob[-1] == 1.0 and gen.host_blob[-1] == 0.0   # the ISO flag of each
        _, uo, io = _oracle(pr)
        x1, u1, i1 = _gpu(pr, dev)
        x2, u2, i2 = _gpu(dict(pr, A=A2), dev)
        for u, info in ((u1, i1), (u2, i2)):
            assert int(info[_native.MPC_INFO_STATUS]) == _native.MPC_STATUS_OPTIMAL, info
            np.testing.assert_allclose(u, uo, atol=MPC_TOL, err_msg=f"H={H} O={O} trial {trial}")
        np.testing.assert_allclose(u1, u2, atol=1e-9)
        np.testing.assert_allclose(x1, x2, atol=1e-9)


@pytest.mark.gpu
def test_gpu_batch_and_strided_views_and_determinism(dev):
    import torch
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf
    rng = np.random.default_rng(11)
    H, O, T, Bn = 30, 5, 30, 6
    probs = [_random_problem(rng, O, T, H) for _ in range(Bn)]
    model = mf.MPCModel(probs[0]["A"], probs[0]["B"], probs[0]["C"], probs[0]["Q"], probs[0]["R"], H,
                        probs[0]["ub"], probs[0]["pb"], device=dev)
    # records laid out like drcvar_safe_halfspaces_f64 output: [B, O, T, 8], h at 3:5, g at 7
    rec = np.zeros((Bn, O, T, 8))
    for b, pr in enumerate(probs):
        rec[b, :, :, 3:5] = pr["hs"][..., :2]
        rec[b, :, :, 7] = pr["hs"][..., 2]
    rec_d = torch.as_tensor(rec).to(dev)
    T_ = lambda a: torch.as_tensor(np.ascontiguousarray(a)).to(dev)
    x0 = T_(np.stack([p["x0"] for p in probs]))
    xr = T_(np.stack([p["x_ref"] for p in probs]))
    uf = T_(np.stack([p["u_ref"] for p in probs]))
    x, u, info = mf.filter_batch(model, rec_d[..., 3:5], rec_d[..., 7], x0, xr, uf)
    x2, u2, _ = mf.filter_batch(model, rec_d[..., 3:5], rec_d[..., 7], x0, xr, uf)
    assert torch.equal(u, u2) and torch.equal(x, x2)
    u, x = u.cpu().numpy(), x.cpu().numpy()
    for b, pr in enumerate(probs):
        xo, uo, io = _oracle(pr)
        np.testing.assert_allclose(u[b], uo, atol=MPC_TOL, err_msg=f"problem {b}")
        np.testing.assert_allclose(x[b], xo, atol=MPC_TOL)


@pytest.mark.gpu
@pytest.mark.parametrize("dyn,H,O", [("double", 30, 3), ("double", 32, 6), ("double", 40, 4),
                                     ("single", 20, 5), ("generic1", 32, 4), ("generic3", 24, 3),
                                     ("generic4", 30, 4), ("generic44", 30, 4), ("generic8", 16, 3)])
def test_gpu_many_problems_every_form(dyn, H, O, dev):
    """More than kFewProblems (128) problems per launch: H <= 32 takes the 128-thread form (its own
    LDS plan), longer horizons the 256-thread form; the same problems launched in chunks of <= 128
    take the 512-thread form (a different summation order).  Every problem converges without the
    fallback; problems polished in both forms agree; sampled problems match the oracle.

    Random instances with several tight halfspaces binding at one step are degenerate (more active
    rows than inputs).  There the first active-set polish often fails; the kernel then resumes the
    interior-point method towards tol * 1e-3 and polishes again (csrc/drcvar_mpc.hip, ipm_round),
    which polishes >= 99 % of every set here (scripts/micro/census.py; before the resume round
    ~10-15 % of the one-input problems ended OPTIMAL_INACCURATE).  The bound below holds that."""
    import torch
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf
    rng = np.random.default_rng(H * 100 + O)
    Bn = 150
    base = _random_problem(rng, O, H, H, dyn)
    probs = []
    for _ in range(Bn):
        pr = dict(base)
        other = _random_problem(rng, O, H, H, "double" if dyn == "double" else "single")
        pr["x0"] = np.zeros_like(base["x0"])
        pr["x0"][:2] = other["x0"][:2]
        pr["x_ref"] = np.zeros_like(base["x_ref"])
        pr["x_ref"][:, :2] = other["x_ref"][:, :2]
        pr["hs"] = other["hs"]
        probs.append(pr)
    model = mf.MPCModel(base["A"], base["B"], base["C"], base["Q"], base["R"], H, base["ub"],
                        base["pb"], device=dev)
    T_ = lambda a: torch.as_tensor(np.ascontiguousarray(a)).to(dev)
    hs = T_(np.stack([p["hs"] for p in probs]))
    args = lambda sl: (model, hs[sl, ..., 0:2], hs[sl, ..., 2], T_(np.stack([p["x0"] for p in probs[sl]])),
                       T_(np.stack([p["x_ref"] for p in probs[sl]])),
                       T_(np.stack([p["u_ref"] for p in probs[sl]])))
    many = [t.cpu().numpy() for t in mf.filter_batch(*args(slice(0, Bn)))]
    parts = [[t.cpu().numpy() for t in mf.filter_batch(*args(sl))] for sl in (slice(0, 100), slice(100, Bn))]
    few = [np.concatenate([a[i] for a in parts]) for i in range(3)]
    ok_status = (_native.MPC_STATUS_OPTIMAL, _native.MPC_STATUS_OPTIMAL_INACCURATE)
    polished = []
    for x, u, info in (many, few):
        assert np.all(np.isin(info[:, _native.MPC_INFO_STATUS], ok_status)), info[:, 0]
        assert np.all(info[:, _native.MPC_INFO_USED_FALLBACK] == 0)
        pol = info[:, _native.MPC_INFO_POLISHED] == 1
        assert pol.mean() >= 0.97, pol.mean()
        polished.append(pol)
    both = polished[0] & polished[1]
    np.testing.assert_allclose(many[1][both], few[1][both], atol=MPC_TOL)
    np.testing.assert_allclose(many[0][both], few[0][both], atol=MPC_TOL)
    for b in (0, 1, Bn // 2, Bn - 1):
        xo, uo, io = _oracle(probs[b])
        tol = MPC_TOL if polished[0][b] else 1e-5
        np.testing.assert_allclose(many[1][b], uo, atol=tol, err_msg=f"{dyn} problem {b}")
        np.testing.assert_allclose(many[0][b], xo, atol=tol)


@pytest.mark.gpu
def test_gpu_horizon_longer_than_halfspace_steps_and_vice_versa(dev):
    rng = np.random.default_rng(5)
    for T, H in ((10, 30), (40, 30)):       # mpc_filter.py:119 uses safe_halfspaces[t-1] if t-1 < len
        pr = _random_problem(rng, 4, T, H)
        xo, uo, io = _oracle(pr)
        x, u, info = _gpu(pr, dev)
        np.testing.assert_allclose(u, uo, atol=MPC_TOL)


@pytest.mark.gpu
def test_gpu_fallback_when_infeasible(dev):
    """Position box unreachable from x0 with the input bounds -> not solved -> _fallback rollout."""
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core.mpc_filter import (
        MPCSafetyFilter)
    A, B, C = double_integrator()
    H = 10
    f = MPCSafetyFilter(A, B, C, 2 * np.eye(4), np.eye(2), H, 0.2)
    x0 = np.array([0.0, 0.0, 0.0, 0.0])
    x_ref = np.zeros((H + 1, 4))
    u_ref = np.full((H, 2), 0.25)
    hs = [[]] * H
    # solvable first call sets last_optimal_u
    x, u, info = f.filter_trajectory(x0, x_ref, u_ref, hs, (np.full(2, -1.0), np.full(2, 1.0)),
                                     (np.full(2, -5.0), np.full(2, 5.0)))
    assert info["status"] == "optimal"
    last = u.copy()
    # position box [8, 9] cannot be reached in 10 steps with |u| <= 1 from the origin
    x, u, info = f.filter_trajectory(x0, x_ref, u_ref, hs, (np.full(2, -1.0), np.full(2, 1.0)),
                                     (np.full(2, 8.0), np.full(2, 9.0)))
    assert info["used_fallback"] is True and info["status"] != "optimal"
    expect_u = mpc_qp.fallback_inputs(H, 2, u_ref, last)
    np.testing.assert_array_equal(u, expect_u)
    np.testing.assert_allclose(x, mpc_qp.rollout(A, B, x0, expect_u), atol=1e-12)


@pytest.mark.gpu
def test_gpu_c5_handoff_shape(dev):
    """256 obstacles x 50 steps of engine-computed DR-CVaR halfspaces -> one QP (C5 hand-off)."""
    import torch
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import engine, synthetic
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf
    O, T, N = 256, 50, 500
    s, ego = synthetic.obstacle_batch(O, T, N, dev, seed=7)
    rec = engine.safe_halfspaces(s, ego, engine.RiskParams())
    A, B, C = double_integrator()
    model = mf.MPCModel(A, B, C, 2 * np.eye(4), np.eye(2), T, (np.full(2, -5.0), np.full(2, 5.0)),
                        (np.full(2, -10.0), np.full(2, 10.0)), device=dev)
    e = ego.cpu().numpy()
    x_ref = np.zeros((T + 1, 4))
    x_ref[:T, :2] = e
    x_ref[T, :2] = e[-1]
    x0 = x_ref[0].copy()
    Tt = lambda a: torch.as_tensor(np.ascontiguousarray(a)).to(dev)
    h, g = mf.record_views(rec, "dr_cvar")
    x, u, info = mf.filter_batch(model, h, g, Tt(x0[None]), Tt(x_ref[None]), Tt(np.zeros((1, T, 2))))
    info = info[0].cpu().numpy()
    assert int(info[_native.MPC_INFO_STATUS]) in (0, 3), info
    r = rec.cpu().numpy()
    hs = np.concatenate([r[..., 3:5], r[..., 7:8]], -1)
    xo, uo, io = mpc_qp.filter_trajectory(A, B, C, 2 * np.eye(4), np.eye(2), T, x0, x_ref, None,
                                          [hs[:, t] for t in range(T)],
                                          (np.full(2, -5.0), np.full(2, 5.0)),
                                          (np.full(2, -10.0), np.full(2, 10.0)))
    assert io["status"] == "optimal"
    np.testing.assert_allclose(u[0].cpu().numpy(), uo, atol=MPC_TOL)


@pytest.mark.gpu
def test_gpu_degenerate_c5_handoff_matches_polished_oracle(dev):
    """The degenerate C5 hand-off (12 800 rows) on the clustered launch and on one workgroup: both
    polished, within MPC_TOL of the oracle's KKT-certified answer, objective to 1e-9; the clustered
    launch in at most 8 interior-point iterations and one polish attempt (round 6's early polish
    from merit 1e-2: bench.py's full_loop_c5)."""
    import torch
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf
    z, _ = _c5_degenerate()
    A, B, C = double_integrator()
    H = z["x_ref"].shape[0] - 1
    model = mf.MPCModel(A, B, C, 2 * np.eye(4), np.eye(2), H, tuple(z["u_bounds"]), tuple(z["p_bounds"]),
                        device=dev)
    Tt = lambda a: torch.as_tensor(np.ascontiguousarray(a)).to(dev)
    for opts in (None, mf.make_options(cluster_size=1)):
        x, u, info = mf.filter_batch(model, Tt(z["h"][None]), Tt(z["g"][None]), Tt(z["x0"][None]),
                                     Tt(z["x_ref"][None]), Tt(np.zeros((1, H, 2))), options=opts)
        info = info[0].cpu().numpy()
        assert int(info[_native.MPC_INFO_STATUS]) == _native.MPC_STATUS_OPTIMAL, info
        assert info[_native.MPC_INFO_POLISHED] == 1, info
        if opts is None:
            assert info[_native.MPC_INFO_ITERATIONS] <= 8, info
            assert info[_native.MPC_INFO_POLISH_ATTEMPTS] <= 1, info
        np.testing.assert_allclose(u[0].cpu().numpy(), z["u_expected"], atol=MPC_TOL)
        np.testing.assert_allclose(x[0].cpu().numpy(), z["x_expected"], atol=MPC_TOL)
        assert abs(info[_native.MPC_INFO_OBJECTIVE] - float(z["objective"])) <= 1e-9 * float(z["objective"])


@pytest.mark.gpu
def test_gpu_h30_straggler_matches_oracle(dev):
    """The batch straggler (tests/golden/qp_h30_straggler.npz) alone and inside a 64-problem batch
    of itself (the 128-thread form): polished, within MPC_TOL of the oracle's KKT-certified answer,
    objective to 1e-9, and no more interior-point iterations than the dump recorded."""
    import torch
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf
    z, _ = _h30_straggler()
    A, B, C = double_integrator()
    H = z["x_ref"].shape[0] - 1
    model = mf.MPCModel(A, B, C, 2 * np.eye(4), np.eye(2), H, tuple(z["u_bounds"]), tuple(z["p_bounds"]),
                        device=dev)
    Tt = lambda a: torch.as_tensor(np.ascontiguousarray(a)).to(dev)
    for Bn in (1, 160):  # 160 > kFewProblems: the batched (many-problem) kernel form
        rep = lambda a: Tt(np.repeat(a[None], Bn, axis=0))
        x, u, info = mf.filter_batch(model, rep(z["h"]), rep(z["g"]), rep(z["x0"]), rep(z["x_ref"]),
                                     Tt(np.zeros((Bn, H, 2))))
        info = info.cpu().numpy()
        assert (info[:, _native.MPC_INFO_STATUS] == _native.MPC_STATUS_OPTIMAL).all(), info[0]
        assert (info[:, _native.MPC_INFO_POLISHED] == 1).all(), info[0]
        assert (info[:, _native.MPC_INFO_ITERATIONS] <= float(z["kernel_iterations"])).all(), info[0]
        np.testing.assert_allclose(u.cpu().numpy(), np.repeat(z["u_expected"][None], Bn, 0), atol=MPC_TOL)
        assert np.all(np.abs(info[:, _native.MPC_INFO_OBJECTIVE] - float(z["objective"])) <= 1e-9 * float(z["objective"]))


@pytest.mark.gpu
def test_gpu_c5_mean_filter_matches_oracle(dev):
    """The C5 mean-metric filter (tests/golden/qp_c5_mean.npz) on the clustered form and on one
    workgroup: optimal, polished, within MPC_TOL of the oracle, objective to 1e-9, and no more
    interior-point iterations than the round-6 kernel takes (12: the early polish from merit
    1e-2; the round-5 kernel took 15, kernel_iterations_r05)."""
    import torch
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf
    z, _ = _c5_mean()
    A, B, C = double_integrator()
    H = z["x_ref"].shape[0] - 1
    model = mf.MPCModel(A, B, C, 2 * np.eye(4), np.eye(2), H, tuple(z["u_bounds"]), tuple(z["p_bounds"]),
                        device=dev)
    Tt = lambda a: torch.as_tensor(np.ascontiguousarray(a)).to(dev)
    for opts in (None, mf.make_options(cluster_size=1)):
        x, u, info = mf.filter_batch(model, Tt(z["h"][None]), Tt(z["g"][None]), Tt(z["x0"][None]),
                                     Tt(z["x_ref"][None]), Tt(np.zeros((1, H, 2))), options=opts)
        info = info[0].cpu().numpy()
        assert int(info[_native.MPC_INFO_STATUS]) == _native.MPC_STATUS_OPTIMAL, info
        assert info[_native.MPC_INFO_POLISHED] == 1, info
        assert info[_native.MPC_INFO_ITERATIONS] <= min(12.0, float(z["kernel_iterations_r05"])), info
        np.testing.assert_allclose(u[0].cpu().numpy(), z["u_expected"], atol=MPC_TOL)
        np.testing.assert_allclose(x[0].cpu().numpy(), z["x_expected"], atol=MPC_TOL)
        assert abs(info[_native.MPC_INFO_OBJECTIVE] - float(z["objective"])) <= 1e-9 * float(z["objective"])


@pytest.mark.gpu
def test_gpu_failed_early_polish_resumes_to_the_oracle(dev):
    """The straggler leaves its first round by the early polish (merit <= 1e-2);
    options.debug_force_resume makes that polish give up at once, so the solve resumes the
    interior-point method from the early iterate (its u, slacks and duals together) to the normal
    tolerance and polishes there: the answer must still be the oracle's, alone and in a 160-problem
    batch (the many-problem form) (the early break once left an older u beside the
    current rows)."""
    import torch
    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf
    z, _ = _h30_straggler()
    A, B, C = double_integrator()
    H = z["x_ref"].shape[0] - 1
    model = mf.MPCModel(A, B, C, 2 * np.eye(4), np.eye(2), H, tuple(z["u_bounds"]), tuple(z["p_bounds"]),
                        device=dev)
    Tt = lambda a: torch.as_tensor(np.ascontiguousarray(a)).to(dev)
    base = mf.filter_batch(model, Tt(z["h"][None]), Tt(z["g"][None]), Tt(z["x0"][None]), Tt(z["x_ref"][None]),
                           Tt(np.zeros((1, H, 2))))[2][0].cpu().numpy()
    for Bn in (1, 160):
        rep = lambda a: Tt(np.repeat(a[None], Bn, axis=0))
        x, u, info = mf.filter_batch(model, rep(z["h"]), rep(z["g"]), rep(z["x0"]), rep(z["x_ref"]),
                                     Tt(np.zeros((Bn, H, 2))), options=mf.make_options(debug_force_resume=True))
        info = info.cpu().numpy()
        assert (info[:, _native.MPC_INFO_STATUS] == _native.MPC_STATUS_OPTIMAL).all(), info[0]
        assert (info[:, _native.MPC_INFO_POLISHED] == 1).all(), info[0]
        # the resumed round really ran: more interior-point iterations than the early exit took
        assert (info[:, _native.MPC_INFO_ITERATIONS] > base[_native.MPC_INFO_ITERATIONS]).all(), (info[0], base)
        np.testing.assert_allclose(u.cpu().numpy(), np.repeat(z["u_expected"][None], Bn, 0), atol=MPC_TOL)
        np.testing.assert_allclose(x.cpu().numpy(), np.repeat(z["x_expected"][None], Bn, 0), atol=MPC_TOL)

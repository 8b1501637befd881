"""CPU check of the algebra of two round-5 changes to the MPC kernel (csrc/drcvar_mpc.hip):

* the Newton solve with a state-space source, K du = b - Gp' z (riccati_solve_dpp with z): z_k is
  the linear cost C'z_k on the state x_{k+1} of the LQ problem, so the backward pass takes it as a
  source, p_k = C'z_{k-1} + F_k p_{k+1} + Kg_k' b_k with p_H = C'z_{H-1}, instead of a Gp' z
  convolution;
* the dual residual of the inputs without the condensed H0 (dual_residual_wave):
  r_du = f + H0 u + Gp' v = f + 2 R u + B' lambda_{j+1} with the forward states x = Gx u and the
  adjoint lambda_k = 2 Q x_k + C' v_{k-1} + A' lambda_{k+1}.

NumPy restatements of exactly those recurrences against dense solves of the condensed system, on
LQ problems shaped like the interior-point method's Newton systems (double integrator, per-step
output weights S_k, input weights up to 1e8).  The reference's QP (core/mpc_filter.py:114-151) is
solved by OSQP through CVXPY; this pins only the kernel's linear algebra.
"""
import numpy as np
import pytest

DT = 0.2
A = np.block([[np.eye(2), DT * np.eye(2)], [np.zeros((2, 2)), np.eye(2)]])
B = np.block([[0.5 * DT ** 2 * np.eye(2)], [DT * np.eye(2)]])
C = np.block([np.eye(2), np.zeros((2, 2))])
Q, R = 2 * np.eye(4), np.eye(2)


def condensed(H):
    nx, nu = 4, 2
    Ap = [np.eye(nx)]
    for _ in range(H):
        Ap.append(A @ Ap[-1])
    Gx = np.zeros((H * nx, H * nu))
    for k in range(H):
        for j in range(k + 1):
            Gx[k * nx:(k + 1) * nx, j * nu:(j + 1) * nu] = Ap[k - j] @ B
    Gp = np.kron(np.eye(H), C) @ Gx
    return Gx, Gp


def factor(S, DU, H):
    """The kernel's backward recursion: Qb_{k+1} = 2Q + C'S_k C on x_{k+1}, Rb_k = 2R + diag(DU_k)."""
    qb = lambda k: 2 * Q + C.T @ S[k] @ C
    P = qb(H - 1)
    Kg, Ri = [None] * H, [None] * H
    for k in range(H - 1, -1, -1):
        Re = 2 * R + np.diag(DU[k]) + B.T @ P @ B
        Ri[k] = np.linalg.inv(Re)
        Kg[k] = Ri[k] @ (B.T @ P @ A)
        if k > 0:
            P = qb(k - 1) + A.T @ P @ A - (B.T @ P @ A).T @ Kg[k]
            P = np.tril(P) + np.tril(P, -1).T  # the kernel forms P from its lower triangle
    return Kg, Ri


def solve_sources(Kg, Ri, b, z, H):
    """riccati_solve_dpp with a state source z: K du = b - Gp' z."""
    p = C.T @ z[H - 1]
    ps = [None] * (H + 1)
    ps[H] = p
    for k in range(H - 1, 0, -1):
        F = A.T - Kg[k].T @ B.T
        p = C.T @ z[k - 1] + F @ p + Kg[k].T @ b[k]
        ps[k] = p
    x = np.zeros(4)
    du = np.zeros((H, 2))
    for k in range(H):
        kff = -Ri[k] @ (B.T @ ps[k + 1] - b[k])
        du[k] = kff - Kg[k] @ x
        x = A @ x + B @ du[k]
    return du


@pytest.mark.parametrize("H,scale", [(20, 1.0), (30, 1e4), (50, 1e8)])
def test_solve_with_state_source_matches_dense(H, scale):
    rng = np.random.default_rng(H)
    S = []
    for _ in range(H):
        M = rng.normal(size=(2, 2))
        S.append(M @ M.T * rng.uniform(0, scale))
    S = np.array(S)
    DU = rng.uniform(0, scale, size=(H, 2)) * (rng.uniform(size=(H, 2)) < 0.3)
    b = rng.normal(size=(H, 2))
    z = rng.normal(size=(H, 2)) * 10
    Gx, Gp = condensed(H)
    Sb = np.zeros((2 * H, 2 * H))
    for k in range(H):
        Sb[2 * k:2 * k + 2, 2 * k:2 * k + 2] = S[k]
    K = np.kron(np.eye(H), 2 * R) + np.diag(DU.reshape(-1)) + Gx.T @ np.kron(np.eye(H), 2 * Q) @ Gx + Gp.T @ Sb @ Gp
    want = np.linalg.solve(K, b.reshape(-1) - Gp.T @ z.reshape(-1))
    Kg, Ri = factor(S, DU, H)
    got = solve_sources(Kg, Ri, b, z, H).reshape(-1)
    # the source form is the convolution form up to rounding, and both solve the condensed system
    rhs = b.reshape(-1) - Gp.T @ z.reshape(-1)
    conv = solve_sources(Kg, Ri, rhs.reshape(H, 2), np.zeros((H, 2)), H).reshape(-1)
    assert np.abs(got - conv).max() <= 1e-12 * max(1.0, np.abs(conv).max())
    assert np.abs(K @ got - rhs).max() <= 1e-9 * np.abs(K).max() * max(1.0, np.abs(got).max())
    if scale <= 1e4:
        assert np.abs(got - want).max() <= 1e-8 * max(1.0, np.abs(want).max())


@pytest.mark.parametrize("H", [10, 30, 50])
def test_dual_residual_by_the_adjoint(H):
    rng = np.random.default_rng(100 + H)
    Gx, Gp = condensed(H)
    H0 = 2 * (Gx.T @ np.kron(np.eye(H), Q) @ Gx + np.kron(np.eye(H), R))
    u = rng.normal(size=(H, 2))
    v = rng.normal(size=(H, 2)) * 20
    f = rng.normal(size=2 * H)
    want = f + H0 @ u.reshape(-1) + Gp.T @ v.reshape(-1)
    # forward states of u from x_0 = 0, then the adjoint
    X = np.zeros((H + 1, 4))
    for k in range(H):
        X[k + 1] = A @ X[k] + B @ u[k]
    lam = np.zeros((H + 2, 4))
    for k in range(H, 0, -1):
        lam[k] = 2 * Q @ X[k] + C.T @ v[k - 1] + A.T @ lam[k + 1]
    got = np.array([f[2 * j:2 * j + 2] + 2 * R @ u[j] + B.T @ lam[j + 1] for j in range(H)]).reshape(-1)
    np.testing.assert_allclose(got, want, rtol=1e-11, atol=1e-11 * np.abs(want).max())

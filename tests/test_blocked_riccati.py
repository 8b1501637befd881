"""CPU check of the algebra behind the blocked Riccati factorisation and blocked solve chains that
round 4 measured in the MPC kernel and did not keep (the kernel code is in git
history, commit 2f6f9c7): a NumPy restatement of exactly those steps — the same 8 block bounds
(w H) // 8, the zero-terminal element recursion (J_E, A_E, C_E), the block-end map
P_s = J_E + A_E' (I + P_e C_E)^-1 P_e A_E by elimination without pivoting, each block's recursion
rerun from its true end value, and the three-pass chains through the block products Phi_b — against
the sequential Riccati recursion and a dense solve of the condensed system K du = b, on LQ problems
shaped like the interior-point method's Newton systems (double integrator, per-step output weights
S_k, input weights growing to 1e8).  Also H0 u through the dynamics (two convolutions) against the
blob's condensed H0.

The reference's QP (core/mpc_filter.py:114-151) is solved by OSQP through CVXPY; the kernel
replaces it, and this test pins only the restructured linear algebra, not the interior-point method.
"""
import numpy as np
import pytest

DT = 0.2
A = np.block([[np.eye(2), DT * np.eye(2)], [np.zeros((2, 2)), np.eye(2)]])
B = np.block([[0.5 * DT ** 2 * np.eye(2)], [DT * np.eye(2)]])
C = np.block([np.eye(2), np.zeros((2, 2))])
W = 8  # blocks (kBlkW)


def bounds(H):
    return [(w * H) // W for w in range(W + 1)]


def lq(rng, H, scale):
    """Qb[k] = Hessian on x_{k+1}... as the kernel indexes it: qb(k) = 2Q + C'S_k C is Qb_{k+1}."""
    S = []
    for _ in range(H):
        g = rng.normal(size=(2, 3))
        S.append(scale * rng.uniform(0, 1) * g @ g.T)
    DU = scale * rng.uniform(0, 1, size=2 * H) * (rng.uniform(size=2 * H) < 0.3)
    qb = [2 * np.eye(4) + C.T @ S[k] @ C for k in range(H)]  # qb[k] = Qb_{k+1}
    rb = [2 * np.eye(2) + np.diag(DU[2 * k:2 * k + 2]) for k in range(H)]
    return qb, rb


def step(J, k, qb, rb, update):
    """One step of the kernel's recursion on J = P_{k+1}: (Kg_k, Re_k^-1, P_k)."""
    Re = rb[k] + B.T @ J @ B
    Ri = np.linalg.inv(Re)
    L = B.T @ J @ A
    Kg = Ri @ L
    Jn = None
    if update:
        Jn = qb[k - 1] + A.T @ J @ A - L.T @ Kg
        Jn = 0.5 * (Jn + Jn.T)
    return Kg, Ri, Jn


def sequential(qb, rb, H):
    J = qb[H - 1].copy()
    Kg, Ri = [None] * H, [None] * H
    for k in range(H - 1, -1, -1):
        Kg[k], Ri[k], Jn = step(J, k, qb, rb, k > 0)
        if k > 0:
            J = Jn
    return Kg, Ri


def solve_nopivot(N, M):
    N, M = N.copy(), M.copy()
    for q in range(4):
        for r in range(q + 1, 4):
            f = N[r, q] / N[q, q]
            N[r, q:] -= f * N[q, q:]
            M[r] -= f * M[q]
    Y = np.zeros_like(M)
    for q in range(3, -1, -1):
        Y[q] = (M[q] - N[q, q + 1:] @ Y[q + 1:]) / N[q, q]
    return Y


def blocked(qb, rb, H):
    kb = bounds(H)
    Kg, Ri = [None] * H, [None] * H
    elem = {}
    for w in range(1, W):  # phase 1
        last = w == W - 1
        J = qb[H - 1].copy() if last else np.zeros((4, 4))
        AE, CE = np.eye(4), np.zeros((4, 4))
        for k in range(kb[w + 1] - 1, kb[w] - 1, -1):
            K, R, Jn = step(J, k, qb, rb, True)
            if last:
                Kg[k], Ri[k] = K, R
            else:
                G = AE @ B
                CE = CE + G @ R @ G.T
                AE = AE @ (A - B @ K)
            J = Jn
        elem[w] = (J, AE, CE)
    Pe = {W - 2: elem[W - 1][0]}  # phase 2
    for w in range(W - 2, 0, -1):
        JE, AE, CE = elem[w]
        P = Pe[w]
        Y = solve_nopivot(np.eye(4) + P @ CE, P @ AE)
        R = JE + AE.T @ Y
        Pe[w - 1] = 0.5 * (R + R.T)
    for w in range(W - 1):  # phase 3
        J = Pe[w].copy()
        for k in range(kb[w + 1] - 1, kb[w] - 1, -1):
            Kg[k], Ri[k], Jn = step(J, k, qb, rb, k > 0)
            J = Jn
    return Kg, Ri


def maps(Kg, H):
    return [A.T - Kg[k].T @ B.T for k in range(H)]


def solve_seq(Kg, Ri, b, H):
    """The kernel's solve: backward p, kff, forward x, du (riccati_solve_dpp)."""
    F = maps(Kg, H)
    p = np.zeros((H + 1, 4))
    for k in range(H - 1, -1, -1):
        p[k] = F[k] @ p[k + 1] + Kg[k].T @ b[k]
    kff = [-Ri[k] @ ((B.T @ p[k + 1] if k + 1 < H else 0) - b[k]) for k in range(H)]
    x = np.zeros((H + 1, 4))
    for k in range(H):
        x[k + 1] = F[k].T @ x[k] + B @ kff[k]
    return np.array([kff[k] - Kg[k] @ x[k] for k in range(H)])


def solve_blocked(Kg, Ri, b, H):
    """The same solve with chain_back_blocked / chain_fwd_blocked's three passes."""
    F = maps(Kg, H)
    kb = bounds(H)
    Phi = {}
    for w in range(1, W - 1):
        P = np.eye(4)
        for k in range(kb[w + 1] - 1, kb[w] - 1, -1):
            P = F[k] @ P
        Phi[w] = P
    src = [Kg[k].T @ b[k] for k in range(H)]
    p = np.zeros((H + 1, 4))
    for w in range(W):  # (A) from zero at each block's end
        q = np.zeros(4)
        for k in range(kb[w + 1] - 1, kb[w] - 1, -1):
            q = F[k] @ q + src[k]
            p[k] = q
    PE = {W - 2: p[kb[W - 1]].copy()}  # (B)
    cur = p[kb[W - 1]].copy()
    for w in range(W - 2, 0, -1):
        PE[w] = cur
        cur = p[kb[w]] + Phi[w] @ cur
    PE[0] = cur
    for w in range(W - 1):  # (C)
        d = PE[w].copy()
        for k in range(kb[w + 1] - 1, kb[w] - 1, -1):
            d = F[k] @ d
            p[k] = p[k] + d
    kff = [-Ri[k] @ ((B.T @ p[k + 1] if k + 1 < H else 0) - b[k]) for k in range(H)]
    g = [B @ kff[k] for k in range(H)]
    x = np.zeros((H + 1, 4))
    RE = {}
    for w in range(W):  # (A) from zero at each block's start
        r = np.zeros(4)
        for k in range(kb[w], kb[w + 1]):
            x[k] = r
            r = F[k].T @ r + g[k]
        RE[w] = r
        if w == W - 1:
            x[H] = r
    XS = {}
    cur = RE[0].copy()  # (B)
    for w in range(1, W - 1):
        XS[w] = cur
        cur = RE[w] + Phi[w].T @ cur
    XS[W - 1] = cur
    for w in range(1, W):  # (C)
        d = XS[w].copy()
        for k in range(kb[w], kb[w + 1]):
            x[k] = x[k] + d
            d = F[k].T @ d
        if w == W - 1:
            x[H] = x[H] + d
    return np.array([kff[k] - Kg[k] @ x[k] for k in range(H)])


def dense_K(qb, rb, H):
    """K = blockdiag(Rb) + Gx' blockdiag(Qb) Gx (x_0 = 0), the system the recursion factorises."""
    n = 2 * H
    Gx = np.zeros((4 * H, n))
    for k in range(H):  # x_{k+1} = sum_{j<=k} A^{k-j} B u_j
        for j in range(k + 1):
            Gx[4 * k:4 * k + 4, 2 * j:2 * j + 2] = np.linalg.matrix_power(A, k - j) @ B
    Qbar = np.zeros((4 * H, 4 * H))
    for k in range(H):
        Qbar[4 * k:4 * k + 4, 4 * k:4 * k + 4] = qb[k]
    Rbar = np.zeros((n, n))
    for k in range(H):
        Rbar[2 * k:2 * k + 2, 2 * k:2 * k + 2] = rb[k]
    return Rbar + Gx.T @ Qbar @ Gx


@pytest.mark.parametrize("H,scale,seed", [(16, 1.0, 0), (30, 10.0, 1), (50, 1e3, 2), (50, 1e8, 3), (64, 1e5, 4)])
def test_blocked_factorisation_and_solve_match_sequential(H, scale, seed):
    rng = np.random.default_rng(seed)
    qb, rb = lq(rng, H, scale)
    Ks, Rs = sequential(qb, rb, H)
    Kb, Rb_ = blocked(qb, rb, H)
    for k in range(H):
        np.testing.assert_allclose(Kb[k], Ks[k], rtol=1e-9, atol=1e-9 * np.abs(Ks[k]).max())
        np.testing.assert_allclose(Rb_[k], Rs[k], rtol=1e-9, atol=1e-12)
    b = rng.normal(size=(H, 2))
    du_seq = solve_seq(Ks, Rs, b, H)
    du_blk = solve_blocked(Kb, Rb_, b, H)
    K = dense_K(qb, rb, H)
    du_dense = np.linalg.solve(K, b.reshape(-1))
    ref = np.abs(du_dense).max()
    assert np.abs(du_seq.reshape(-1) - du_dense).max() <= 1e-8 * ref
    assert np.abs(du_blk.reshape(-1) - du_dense).max() <= 1e-8 * ref
    assert np.abs(du_blk - du_seq).max() <= 1e-9 * ref


def test_h0u_through_the_dynamics_matches_the_blob():
    """H0 u as 2 (Gx' Q (Gx u) + R u) from an A^i B table (round 4's dynamics variant) — two
    convolutions instead of the condensed n x n H0 that drcvar_mpc_model_init stores in the blob.
    Same numbers (to rounding) as the blob's H0 times u, for the reference's double integrator."""
    from tests.test_mpc import model_init
    H = 50
    Q, R = 2 * np.eye(4), np.eye(2)
    rc, m, blob = model_init(A, B, C, Q, R, H)
    assert rc == 0
    n = 2 * H
    H0 = blob[:n * n].reshape(n, n)
    u = np.random.default_rng(5).normal(size=n)
    AB = [np.linalg.matrix_power(A, i) @ B for i in range(H)]  # the kernel's s.xs table
    X = np.zeros((H, 4))  # states x_{k+1} = sum_{j<=k} A^{k-j} B u_j (Gx u)
    for k in range(H):
        for j in range(k + 1):
            X[k] += AB[k - j] @ u[2 * j:2 * j + 2]
    Z = X @ Q.T  # Q x_{k+1}
    h0u = np.zeros(n)
    for j in range(H):
        for k in range(j, H):
            h0u[2 * j:2 * j + 2] += AB[k - j].T @ Z[k]
        h0u[2 * j:2 * j + 2] += R @ u[2 * j:2 * j + 2]
    np.testing.assert_allclose(2 * h0u, H0 @ u, rtol=1e-12, atol=1e-12 * np.abs(H0 @ u).max())

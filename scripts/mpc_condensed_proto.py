"""Design prototype (NumPy) of the condensed interior-point method in csrc/drcvar_mpc.hip.

Not shipped and not an oracle: it is the algorithm written step by step in the order the kernel
executes it, used to validate the condensed formulation against oracle/mpc_qp.py on the CPU
before porting.  Run: python scripts/mpc_condensed_proto.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def model(A, B, C, Q, R, H):
    nx, nu, ny = A.shape[0], B.shape[1], C.shape[0]
    n = nu * H
    Apow = [np.eye(nx)]
    for _ in range(H):
        Apow.append(A @ Apow[-1])
    Mp = np.array([C @ Apow[i] @ B for i in range(H)])          # [H, ny, nu]
    CA = np.array([C @ Apow[k + 1] for k in range(H)])          # [H, ny, nx]
    Gx = np.zeros((H * nx, n))
    Phi = np.zeros((H * nx, nx))
    for k in range(H):                                          # x_{k+1}
        Phi[k * nx:(k + 1) * nx] = Apow[k + 1]
        for j in range(k + 1):
            Gx[k * nx:(k + 1) * nx, j * nu:(j + 1) * nu] = Apow[k - j] @ B
    Qb = np.kron(np.eye(H), Q)
    Rb = np.kron(np.eye(H), R)
    H0 = 2.0 * (Gx.T @ Qb @ Gx + Rb)
    F1 = 2.0 * Gx.T @ Qb @ Phi
    F2 = 2.0 * Gx.T @ Qb
    return dict(nx=nx, nu=nu, ny=ny, H=H, n=n, Mp=Mp, CA=CA, H0=H0, F1=F1, F2=F2)


def solve(md, x0, xref, hs, ib, pb, tol=1e-10, max_iter=60):
    """hs: [O, K, 3] rows for steps k < K (constrain p_{k+1}); ib/pb: (lo, hi) or None."""
    H, nu, n = md["H"], md["nu"], md["n"]
    Mp, CA = md["Mp"], md["CA"]
    O, K = hs.shape[0], min(hs.shape[1], H)
    h0, h1, g = hs[:, :K, 0], hs[:, :K, 1], hs[:, :K, 2]
    c = np.einsum("kij,j->ki", CA, x0)                           # [H, 2]
    f = md["F1"] @ x0 - md["F2"] @ xref[1:H + 1].reshape(-1)

    def Gp(u):                                                   # positions from inputs
        U = u.reshape(H, nu)
        return np.array([sum(Mp[k - j] @ U[j] for j in range(k + 1)) for k in range(H)])

    def GpT(z):                                                  # [H,2] -> [n]
        return np.concatenate([sum(Mp[k - j].T @ z[k] for k in range(j, H)) for j in range(H)])

    u = np.zeros(n)
    s = np.zeros((O, K))
    p = c + Gp(u)
    # slacks w = max(d - Gz, 1), duals 1 (same start as the oracle, in condensed variables)
    wA = np.maximum(s - (h0 * p[None, :K, 0] + h1 * p[None, :K, 1]) - g, 1.0)
    wB = np.maximum(s, 1.0)
    lA = np.ones_like(wA)
    lB = np.ones_like(wB)
    hasU, hasP = ib is not None, pb is not None
    if hasU:
        umin = np.tile(ib[0], H)
        umax = np.tile(ib[1], H)
        wUu = np.maximum(umax - u, 1.0); wUl = np.maximum(u - umin, 1.0)
        lUu = np.ones(n); lUl = np.ones(n)
    if hasP:
        pmin, pmax = pb
        wPu = np.maximum(pmax[None] - p, 1.0); wPl = np.maximum(p - pmin[None], 1.0)
        lPu = np.ones((H, 2)); lPl = np.ones((H, 2))
    m = 2 * O * K + (2 * n if hasU else 0) + (4 * H if hasP else 0)
    scale_d = 1.0 + max([np.abs(g).max(initial=0)] + ([np.abs(ib).max()] if hasU else [])
                        + ([np.abs(pb).max()] if hasP else []))
    scale_q = 1.0 + max(np.abs(f).max(), 50.0)
    status = "max_iter"
    best = (np.inf, None, None, None)

    def _groups():
        g_ = {"A": (wA, lA), "B": (wB, lB)}
        if hasU:
            g_["Uu"], g_["Ul"] = (wUu, lUu), (wUl, lUl)
        if hasP:
            g_["Pu"], g_["Pl"] = (wPu, lPu), (wPl, lPl)
        return g_

    for it in range(1, max_iter + 1):
        p = c + Gp(u)
        hp = h0 * p[None, :K, 0] + h1 * p[None, :K, 1]
        # residuals
        v = np.zeros((H, 2))
        v[:K, 0] = (lA * h0).sum(0)
        v[:K, 1] = (lA * h1).sum(0)
        if hasP:
            v += lPu - lPl
        r_du = md["H0"] @ u + f + GpT(v) + ((lUu - lUl) if hasU else 0)
        r_ds = 100.0 * s + 50.0 - lA - lB
        r_pA = hp + g - s + wA
        r_pB = -s + wB
        gap = (wA * lA).sum() + (wB * lB).sum()
        rp = max(np.abs(r_pA).max(initial=0), np.abs(r_pB).max(initial=0))
        if hasU:
            r_pUu = u - umax + wUu; r_pUl = umin - u + wUl
            gap += (wUu * lUu).sum() + (wUl * lUl).sum()
            rp = max(rp, np.abs(r_pUu).max(), np.abs(r_pUl).max())
        if hasP:
            r_pPu = p - pmax + wPu; r_pPl = pmin - p + wPl
            gap += (wPu * lPu).sum() + (wPl * lPl).sum()
            rp = max(rp, np.abs(r_pPu).max(), np.abs(r_pPl).max())
        mu = gap / m
        rd = max(np.abs(r_du).max(), np.abs(r_ds).max(initial=0))
        merit = max(rp / scale_d, rd / scale_q, mu)
        if merit < best[0]:
            best = (merit, u.copy(), s.copy(), {k: (v[0].copy(), v[1].copy()) for k, v in _groups().items()})
        if merit <= tol:
            status = "optimal"
            break
        DA, DB = lA / wA, lB / wB
        sig = 100.0 + DA + DB
        om = DA * (100.0 + DB) / sig
        S = np.zeros((H, 2, 2))
        S[:K, 0, 0] = (om * h0 * h0).sum(0)
        S[:K, 0, 1] = S[:K, 1, 0] = (om * h0 * h1).sum(0)
        S[:K, 1, 1] = (om * h1 * h1).sum(0)
        if hasP:
            DPu, DPl = lPu / wPu, lPl / wPl
            S[:, 0, 0] += DPu[:, 0] + DPl[:, 0]
            S[:, 1, 1] += DPu[:, 1] + DPl[:, 1]
        Kmat = md["H0"].copy()
        if hasU:
            DUu, DUl = lUu / wUu, lUl / wUl
            Kmat += np.diag(DUu + DUl)
        for j in range(H):
            for l in range(H):
                blk = np.zeros((nu, nu))
                for k in range(max(j, l), H):
                    blk += Mp[k - j].T @ S[k] @ Mp[k - l]
                Kmat[j * nu:(j + 1) * nu, l * nu:(l + 1) * nu] += blk
        try:
            L = np.linalg.cholesky(Kmat)
        except np.linalg.LinAlgError:
            status = "numerical"
            break

        def direction(rc):
            """rc: dict of complementarity targets per inequality group."""
            rhoA = DA * r_pA + rc["A"] / wA
            rhoB = DB * r_pB + rc["B"] / wB
            rhs_s = -r_ds + rhoA + rhoB
            coef = rhoA - DA * rhs_s / sig
            z = np.zeros((H, 2))
            z[:K, 0] = (coef * h0).sum(0)
            z[:K, 1] = (coef * h1).sum(0)
            rhs = -r_du
            if hasU:
                rhoUu = DUu * r_pUu + rc["Uu"] / wUu
                rhoUl = DUl * r_pUl + rc["Ul"] / wUl
                rhs = rhs - (rhoUu - rhoUl)
            if hasP:
                rhoPu = DPu * r_pPu + rc["Pu"] / wPu
                rhoPl = DPl * r_pPl + rc["Pl"] / wPl
                z += rhoPu - rhoPl
            rhs = rhs - GpT(z)
            du = np.linalg.solve(L.T, np.linalg.solve(L, rhs))
            dp = Gp(du)
            hdp = h0 * dp[None, :K, 0] + h1 * dp[None, :K, 1]
            ds = (rhs_s + DA * hdp) / sig
            d = {}
            gA = hdp - ds
            d["A"] = (-r_pA - gA, DA * gA + rhoA)
            d["B"] = (-r_pB + ds, -DB * ds + rhoB)
            if hasU:
                d["Uu"] = (-r_pUu - du, DUu * du + rhoUu)
                d["Ul"] = (-r_pUl + du, -DUl * du + rhoUl)
            if hasP:
                d["Pu"] = (-r_pPu - dp, DPu * dp + rhoPu)
                d["Pl"] = (-r_pPl + dp, -DPl * dp + rhoPl)
            return du, ds, d

        state = {"A": (wA, lA), "B": (wB, lB)}
        if hasU:
            state["Uu"] = (wUu, lUu); state["Ul"] = (wUl, lUl)
        if hasP:
            state["Pu"] = (wPu, lPu); state["Pl"] = (wPl, lPl)

        def alpha_max(d):
            a = 1.0
            for key, (dw, dl) in d.items():
                w_, l_ = state[key]
                for x, dx in ((w_, dw), (l_, dl)):
                    neg = dx < 0
                    if neg.any():
                        a = min(a, np.min(-x[neg] / dx[neg]))
            return a

        rc_aff = {k: -w_ * l_ for k, (w_, l_) in state.items()}
        du_a, ds_a, d_a = direction(rc_aff)
        a_aff = alpha_max(d_a)
        gap_aff = sum(((state[k][0] + a_aff * d_a[k][0]) * (state[k][1] + a_aff * d_a[k][1])).sum()
                      for k in state)
        sigma = (gap_aff / gap) ** 3
        rc = {k: -w_ * l_ - d_a[k][0] * d_a[k][1] + sigma * mu for k, (w_, l_) in state.items()}
        du, ds, d = direction(rc)
        a = min(1.0, 0.995 * alpha_max(d))
        u = u + a * du
        s = s + a * ds
        for key, (dw, dl) in d.items():
            state[key][0][...] += a * dw
            state[key][1][...] += a * dl
    if status != "optimal":
        _, u, s, duals = best
    else:
        duals = _groups()
    return u.reshape(H, nu), s, {"status": status, "iterations": it, "duals": duals,
                                 "merit": best[0]}


if __name__ == "__main__":
    from oracle import mpc_qp
    import time
    z = np.load("tests/golden/multi_obstacle_n20_h30.npz")
    exp = z["expected"]
    dt = 0.2
    A = np.block([[np.eye(2), dt * np.eye(2)], [np.zeros((2, 2)), np.eye(2)]])
    B = np.block([[0.5 * dt ** 2 * np.eye(2)], [dt * np.eye(2)]])
    C = np.block([np.eye(2), np.zeros((2, 2))])
    Q, R, H = 2 * np.eye(4), np.eye(2), 30
    start, goal = np.array([-2., -1.]), np.array([4., 0.])
    d = goal - start; dist = np.linalg.norm(d); dirn = d / dist; n_steps = int(dist / 1.5 / dt)
    xr = np.zeros((H + 1, 4)); xr[0, :2] = start
    for t in range(1, H + 1):
        if t <= n_steps:
            xr[t, :2] = start + t / n_steps * (goal - start); xr[t, 2:] = 1.5 * dirn
        else:
            xr[t, :2] = goal
    ur = np.array([np.linalg.pinv(B) @ (xr[t + 1] - A @ xr[t]) for t in range(H)])
    x0 = np.zeros(4); x0[:2] = start
    sb = (np.array([-10., -10.]), np.array([10., 10.]))
    ib = (np.array([-5., -5.]), np.array([5., 5.]))
    md = model(A, B, C, Q, R, H)
    for name, cols in [("mean", (0, 1, 2)), ("cvar", (3, 4, 5)), ("dr_cvar", (3, 4, 7))]:
        hs = exp[:, :, list(cols)]
        rows = [hs[:, t] for t in range(hs.shape[1])]
        xo, uo, io = mpc_qp.filter_trajectory(A, B, C, Q, R, H, x0, xr, ur, rows, ib, sb)
        t0 = time.time()
        u, s, info = solve(md, x0, xr, hs, ib, sb)
        print(name, info, "max|du| vs oracle", np.abs(u - uo).max(), "%.2fs" % (time.time() - t0))
    # a tight case: pull obstacles onto the reference line so many slacks are active
    rng = np.random.default_rng(0)
    for trial in range(5):
        O = 6
        hs = np.zeros((O, H, 3))
        ang = rng.uniform(0, 2 * np.pi, (O, H))
        hs[..., 0], hs[..., 1] = np.cos(ang), np.sin(ang)
        hs[..., 2] = rng.normal(-1.0, 2.0, (O, H))
        rows = [hs[:, t] for t in range(H)]
        xo, uo, io = mpc_qp.filter_trajectory(A, B, C, Q, R, H, x0, xr, ur, rows, ib, sb)
        u, s, info = solve(md, x0, xr, hs, ib, sb)
        print("random", trial, io["status"], io["iterations"], info, np.abs(u - uo).max(), io.get("kkt"),
              (io.get("slacks", np.zeros(1)) > 1e-8).sum())


def polish(md, x0, xref, hs, ib, pb, u, s, duals, rho=1e6, iters=12, attempts=4):
    """Active-set polish (kernel design): method of multipliers on the equality-constrained QP of
    the IPM's active set, then primal-dual active-set corrections of the rows that violate their
    sign conditions, up to `attempts` times.  Returns (u_polished, ok, diag)."""
    H, nu, n = md["H"], md["nu"], md["n"]
    Mp, CA = md["Mp"], md["CA"]
    O, K = hs.shape[0], min(hs.shape[1], H)
    h0, h1, g = hs[:, :K, 0], hs[:, :K, 1], hs[:, :K, 2]
    c = np.einsum("kij,j->ki", CA, x0)
    f = md["F1"] @ x0 - md["F2"] @ xref[1:H + 1].reshape(-1)
    Gp = lambda v: np.array([sum(Mp[k - j] @ v.reshape(H, nu)[j] for j in range(k + 1)) for k in range(H)])
    GpT = lambda z: np.concatenate([sum(Mp[k - j].T @ z[k] for k in range(j, H)) for j in range(H)])
    (wA, lA), (wB, lB) = duals["A"], duals["B"]
    eq = (lA > wA) & (lB > wB)            # h.p + g = s = 0
    pen = (lA > wA) & ~(lB > wB)          # s = h.p + g > 0: quadratic penalty
    b = h0 * c[None, :K, 0] + h1 * c[None, :K, 1] + g
    nu_hs = np.where(eq, lA, 0.0)
    hasU, hasP = ib is not None, pb is not None
    if hasU:
        umin, umax = np.tile(ib[0], H), np.tile(ib[1], H)
        aUu, aUl = duals["Uu"][1] > duals["Uu"][0], duals["Ul"][1] > duals["Ul"][0]
        nUu, nUl = np.where(aUu, duals["Uu"][1], 0.0), np.where(aUl, duals["Ul"][1], 0.0)
    if hasP:
        aPu, aPl = duals["Pu"][1] > duals["Pu"][0], duals["Pl"][1] > duals["Pl"][0]
        nPu, nPl = np.where(aPu, duals["Pu"][1], 0.0), np.where(aPl, duals["Pl"][1], 0.0)
    tolf = 1e-9 * (1 + np.abs(g).max(initial=0))
    tol_dual = 1e-7
    for attempt in range(attempts):
        S = np.zeros((H, 2, 2))
        wgt = np.where(pen, 100.0, 0.0) + np.where(eq, rho, 0.0)
        S[:K, 0, 0] = (wgt * h0 * h0).sum(0); S[:K, 0, 1] = S[:K, 1, 0] = (wgt * h0 * h1).sum(0)
        S[:K, 1, 1] = (wgt * h1 * h1).sum(0)
        Kmat = md["H0"].copy()
        if hasU:
            Kmat += np.diag(rho * (aUu.astype(float) + aUl))
        if hasP:
            S[:, 0, 0] += rho * (aPu[:, 0].astype(float) + aPl[:, 0])
            S[:, 1, 1] += rho * (aPu[:, 1].astype(float) + aPl[:, 1])
        for j in range(H):
            for l in range(H):
                Kmat[j * nu:(j + 1) * nu, l * nu:(l + 1) * nu] += sum(
                    Mp[k - j].T @ S[k] @ Mp[k - l] for k in range(max(j, l), H))
        L = np.linalg.cholesky(Kmat)
        for _ in range(iters):
            coef = np.where(pen, 50.0 + 100.0 * b, 0.0) + np.where(eq, nu_hs + rho * b, 0.0)
            z = np.zeros((H, 2))
            z[:K, 0] = (coef * h0).sum(0); z[:K, 1] = (coef * h1).sum(0)
            rhs = -f.copy()
            if hasU:
                rhs -= np.where(aUu, nUu - rho * umax, 0.0) - np.where(aUl, nUl + rho * umin, 0.0)
            if hasP:
                z += np.where(aPu, nPu - rho * (pb[1][None] - c), 0.0) - np.where(aPl, nPl - rho * (c - pb[0][None]), 0.0)
            u = np.linalg.solve(L.T, np.linalg.solve(L, rhs - GpT(z)))
            p = c + Gp(u)
            hp = h0 * p[None, :K, 0] + h1 * p[None, :K, 1] + g
            nu_hs = np.where(eq, nu_hs + rho * hp, 0.0)
            if hasU:
                nUu = np.where(aUu, nUu + rho * (u - umax), 0.0)
                nUl = np.where(aUl, nUl + rho * (umin - u), 0.0)
            if hasP:
                nPu = np.where(aPu, nPu + rho * (p - pb[1][None]), 0.0)
                nPl = np.where(aPl, nPl + rho * (pb[0][None] - p), 0.0)
        # sign conditions; violators are moved (primal-dual active-set step)
        too_big = eq & (nu_hs > 50.0 + tol_dual)       # s > 0 after all
        too_small = eq & (nu_hs < -tol_dual)           # halfspace not binding
        neg_s = pen & (hp < -tolf)                     # penalised row with s < 0
        viol_in = ~eq & ~pen & (hp > tolf)             # dropped row violated
        bad = [too_big.sum(), too_small.sum(), neg_s.sum(), viol_in.sum()]
        eq = (eq & ~too_big & ~too_small) | neg_s | viol_in
        pen = (pen & ~neg_s) | too_big
        nu_hs = np.where(eq, np.clip(nu_hs, 0.0, 50.0), 0.0)
        if hasU:
            bu = [(aUu & (nUu < -tol_dual)), (aUl & (nUl < -tol_dual)), (~aUu & (u - umax > tolf)), (~aUl & (umin - u > tolf))]
            bad += [x.sum() for x in bu]
            aUu = (aUu & ~bu[0]) | bu[2]; aUl = (aUl & ~bu[1]) | bu[3]
            nUu = np.where(aUu, np.maximum(nUu, 0), 0); nUl = np.where(aUl, np.maximum(nUl, 0), 0)
        if hasP:
            bp = [(aPu & (nPu < -tol_dual)), (aPl & (nPl < -tol_dual)), (~aPu & (p - pb[1][None] > tolf)), (~aPl & (pb[0][None] - p > tolf))]
            bad += [x.sum() for x in bp]
            aPu = (aPu & ~bp[0]) | bp[2]; aPl = (aPl & ~bp[1]) | bp[3]
            nPu = np.where(aPu, np.maximum(nPu, 0), 0); nPl = np.where(aPl, np.maximum(nPl, 0), 0)
        if sum(bad) == 0:
            return u.reshape(H, nu), True, {"attempts": attempt + 1, "n_eq": int(eq.sum()),
                                             "n_pen": int(pen.sum())}
    return u.reshape(H, nu), False, {"attempts": attempts, "bad": [int(x) for x in bad]}

"""CPU laboratory for the interior-point method of csrc/drcvar_mpc.hip (design tool, not an oracle).

Vectorised NumPy restatement of the kernel's iteration (same start, same Mehrotra predictor-
corrector, same step rule, same merit), run on the problems scripts/micro/dump_qp_problems.py
saved from the device, to count iterations of algorithmic variants before porting any of them:

    python scripts/micro/ipm_lab.py [--variant base|...] [--trace]
"""
import argparse
import sys

import numpy as np

SLACK_LIN, SLACK_HESS, STEP_FRAC = 50.0, 100.0, 0.995


def model(H, dt=0.2):
    A = np.block([[np.eye(2), dt * np.eye(2)], [np.zeros((2, 2)), np.eye(2)]])
    B = np.block([[0.5 * dt ** 2 * np.eye(2)], [dt * np.eye(2)]])
    C = np.block([np.eye(2), np.zeros((2, 2))])
    Q, R = 2 * np.eye(4), np.eye(2)
    nx, nu = 4, 2
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
    Cb = np.kron(np.eye(H), C)
    return dict(H=H, n=n, nu=nu, Gp=Cb @ Gx, CPhi=Cb @ Phi,
                H0=2.0 * (Gx.T @ Qb @ Gx + np.kron(np.eye(H), R)),
                F1=2.0 * Gx.T @ Qb @ Phi, F2=2.0 * Gx.T @ Qb,
                umin=np.full(n, -5.0), umax=np.full(n, 5.0),
                pmin=np.full(2 * H, -10.0), pmax=np.full(2 * H, 10.0))


START = dict(wA_floor=1.0, lA=1.0, wB=1.0, lB=0.5 * SLACK_LIN, box_l=1.0, lA_many=5.0, wB_many=1.5, many=64)


def solve(md, h, g, x0, xr, variant="base", tol=None, max_iter=60, trace=False, on_system=None):
    tol = START.get("tol", 1e-8) if tol is None else tol
    """h [O, H, 2], g [O, H].  Returns (u, iterations, merit history)."""
    H, n = md["H"], md["n"]
    Gp = md["Gp"]                                   # [2H, n]: p = c + Gp u
    O = h.shape[0]
    h0, h1 = h[..., 0], h[..., 1]                   # [O, H]
    c = md["CPhi"] @ x0                             # [2H]
    f = md["F1"] @ x0 - md["F2"] @ xr[1:H + 1].reshape(-1)

    def hp_of(p):                                   # h . p per row
        P = p.reshape(H, 2)
        return h0 * P[None, :, 0] + h1 * P[None, :, 1]

    def ht_of(z):                                   # sum over rows of z * h -> [2H]
        return np.stack([(z * h0).sum(0), (z * h1).sum(0)], -1).reshape(-1)

    u = np.zeros(n)
    s = np.zeros((O, H))
    wA = np.maximum(-(hp_of(c) + g), START["wA_floor"])
    many = O >= START.get("many", 1e9)  # the kernel's rule: other starting values for many rows
    lA = np.full((O, H), START["lA_many"] if many else START["lA"])
    wB = np.full((O, H), START["wB_many"] if many else START["wB"])
    lB = np.full((O, H), START["lB"])
    bl = START["box_l"]
    wUu, lUu = np.maximum(md["umax"], 1.0), np.full(n, bl)
    wUl, lUl = np.maximum(-md["umin"], 1.0), np.full(n, bl)
    wPu, lPu = np.maximum(md["pmax"] - c, 1.0), np.full(2 * H, bl)
    wPl, lPl = np.maximum(c - md["pmin"], 1.0), np.full(2 * H, bl)
    if START.get("u_free", 0.0) > 0.0:       # the tracking optimum without rows, clipped to the box
        span = md["umax"] - md["umin"]
        mg = START.get("u_margin", 0.05)
        u = np.clip(-np.linalg.solve(md["H0"], f), md["umin"] + mg * span, md["umax"] - mg * span)
        pu = c + Gp @ u
        wUu, wUl = md["umax"] - u, u - md["umin"]
        wPu, wPl = np.maximum(md["pmax"] - pu, START.get("wp_floor", 1e-2)), np.maximum(pu - md["pmin"], START.get("wp_floor", 1e-2))
    if START.get("central_mu", 0.0) > 0.0:   # every row on its own central path at u
        cmu = START["central_mu"] if O >= START.get("many", 1e9) else START.get("central_mu_few", START["central_mu"])
        r = hp_of(c + Gp @ u) + g
        lo, hi = np.maximum(r, 0.0), np.maximum(r, 0.0) + 1.0 + 2.0 * np.sqrt(cmu)
        for _ in range(200):
            mid = 0.5 * (lo + hi)
            phi = SLACK_LIN + SLACK_HESS * mid - cmu / (mid - r) - cmu / mid
            lo, hi = np.where(phi < 0, mid, lo), np.where(phi < 0, hi, mid)
        s = 0.5 * (lo + hi)
        wA, wB = s - r, s.copy()
        lA, lB = cmu / wA, cmu / wB
        if START.get("lam_cap", 0.0) > 0.0:
            lA = np.minimum(lA, START["lam_cap"])
        bmu = START.get("central_box_mu", cmu)
        lUu, lUl = bmu / wUu, bmu / wUl
        lPu, lPl = bmu / wPu, bmu / wPl
    scale_d = 1.0 + max(np.abs(g).max(), 5.0, 10.0)
    scale_q = 1.0 + max(np.abs(f).max(), SLACK_LIN)
    m = 2 * O * H + 2 * n + 4 * H
    hist = []
    for it in range(1, max_iter + 1):
        p = c + Gp @ u
        hp = hp_of(p)
        v = ht_of(lA) + (lPu - lPl)
        r_du = md["H0"] @ u + f + Gp.T @ v + (lUu - lUl)
        r_ds = SLACK_HESS * s + SLACK_LIN - lA - lB
        r_pA = hp + g - s + wA
        r_pB = wB - s
        r_Uu, r_Ul = u - md["umax"] + wUu, md["umin"] - u + wUl
        r_Pu, r_Pl = p - md["pmax"] + wPu, md["pmin"] - p + wPl
        gap = ((wA * lA).sum() + (wB * lB).sum() + wUu @ lUu + wUl @ lUl + wPu @ lPu + wPl @ lPl)
        rp = max(np.abs(r_pA).max(), np.abs(r_pB).max(), np.abs(r_Uu).max(), np.abs(r_Ul).max(),
                 np.abs(r_Pu).max(), np.abs(r_Pl).max())
        rd = max(np.abs(r_du).max(), np.abs(r_ds).max())
        mu = gap / m
        merit = max(rp / scale_d, rd / scale_q, mu)
        hist.append((merit, rp / scale_d, rd / scale_q, mu))
        if trace:
            print(f"  it {it:2d} merit {merit:.3e} rp {rp / scale_d:.2e} rd {rd / scale_q:.2e} mu {mu:.2e}")
        if merit <= tol:
            return u, it, hist
        DA, DB = lA / wA, lB / wB
        sig = SLACK_HESS + DA + DB
        om = DA * (SLACK_HESS + DB) / sig
        DUu, DUl, DPu, DPl = lUu / wUu, lUl / wUl, lPu / wPu, lPl / wPl
        S = np.zeros((H, 2, 2))
        S[:, 0, 0] = (om * h0 * h0).sum(0)
        S[:, 0, 1] = S[:, 1, 0] = (om * h0 * h1).sum(0)
        S[:, 1, 1] = (om * h1 * h1).sum(0)
        S[:, 0, 0] += DPu[0::2] + DPl[0::2]
        S[:, 1, 1] += DPu[1::2] + DPl[1::2]
        Sb = np.zeros((2 * H, 2 * H))
        for k in range(H):
            Sb[2 * k:2 * k + 2, 2 * k:2 * k + 2] = S[k]
        K = md["H0"] + np.diag(DUu + DUl) + Gp.T @ Sb @ Gp
        if on_system is not None:  # scripts/micro/riccati_scan_lab.py: the Newton system's LQ data
            on_system(it, merit, S, DUu + DUl, K)
        L = np.linalg.cholesky(K)
        state = dict(A=(wA, lA), B=(wB, lB), Uu=(wUu, lUu), Ul=(wUl, lUl), Pu=(wPu, lPu), Pl=(wPl, lPl))

        def direction(rc):
            rhoA = DA * r_pA + rc["A"] / wA
            rhoB = DB * r_pB + rc["B"] / wB
            rhs_s = -r_ds + rhoA + rhoB
            coef = rhoA - DA * rhs_s / sig
            rhoUu, rhoUl = DUu * r_Uu + rc["Uu"] / wUu, DUl * r_Ul + rc["Ul"] / wUl
            rhoPu, rhoPl = DPu * r_Pu + rc["Pu"] / wPu, DPl * r_Pl + rc["Pl"] / wPl
            z = ht_of(coef) + rhoPu - rhoPl
            rhs = -r_du - (rhoUu - rhoUl) - Gp.T @ z
            du = np.linalg.solve(L.T, np.linalg.solve(L, rhs))
            dp = Gp @ du
            hdp = hp_of(dp)
            ds = (rhs_s + DA * hdp) / sig
            gA = hdp - ds
            d = dict(A=(-r_pA - gA, DA * gA + rhoA), B=(-r_pB + ds, -DB * ds + rhoB),
                     Uu=(-r_Uu - du, DUu * du + rhoUu), Ul=(-r_Ul + du, -DUl * du + rhoUl),
                     Pu=(-r_Pu - dp, DPu * dp + rhoPu), Pl=(-r_Pl + dp, -DPl * dp + rhoPl))
            return du, ds, d

        def amax_of(d, who=None):
            a = np.inf
            for key, (dw, dl) in d.items():
                w_, l_ = state[key]
                for nm, x, dx in (("w", w_, dw), ("l", l_, dl)):
                    neg = dx < 0
                    if neg.any():
                        r = np.where(neg, -x / np.where(neg, dx, -1.0), np.inf)
                        i = np.unravel_index(np.argmin(r), r.shape)
                        if r[i] < a:
                            a = r[i]
                            if who is not None:
                                who[:] = [key + nm, i, x[i], dx[i], (w_[i], l_[i])]
            return a

        rc_aff = {k: -w_ * l_ for k, (w_, l_) in state.items()}
        du_a, ds_a, d_a = direction(rc_aff)
        who = [None] * 5
        a_aff = min(1.0, amax_of(d_a, who))
        gap_aff = sum(((state[k][0] + a_aff * d_a[k][0]) * (state[k][1] + a_aff * d_a[k][1])).sum()
                      for k in state)
        sigma_mu = (gap_aff / gap) ** START.get("sig_exp", 3.0) * mu
        if variant.startswith("nosoc"):  # no second-order correction: corrector = affine + sigma mu unit
            rc = {k: -w_ * l_ + sigma_mu for k, (w_, l_) in state.items()}
        else:
            rc = {k: -w_ * l_ - d_a[k][0] * d_a[k][1] + sigma_mu for k, (w_, l_) in state.items()}
        du, ds, d = direction(rc)
        amax = amax_of(d)
        if variant == "gondzio":
            du, ds, d, amax = gondzio(direction, amax_of, state, rc, du, ds, d, amax, sigma_mu)
        alpha = min(1.0, (1.0 - min(1.0 - START.get("frac", STEP_FRAC), mu)) * amax)
        if variant == "split":   # separate primal (u, s, w) and dual (lambda) step lengths
            ap_ = np.inf
            ad_ = np.inf
            for key, (dw, dl) in d.items():
                w_, l_ = state[key]
                for x, dx, prim in ((w_, dw, True), (l_, dl, False)):
                    neg = dx < 0
                    if neg.any():
                        r = np.min(-x[neg] / dx[neg])
                        if prim:
                            ap_ = min(ap_, r)
                        else:
                            ad_ = min(ad_, r)
            fr = 1.0 - min(1.0 - STEP_FRAC, mu)
            ap_, ad_ = min(1.0, fr * ap_), min(1.0, fr * ad_)
            u = u + ap_ * du
            s = s + ap_ * ds
            for key, (dw, dl) in d.items():
                state[key][0][...] += ap_ * dw
                state[key][1][...] += ad_ * dl
            if trace:
                print(f"      a_aff {a_aff:.3f} primal {ap_:.3f} dual {ad_:.3f}")
            continue
        if trace:
            print(f"      a_aff {a_aff:.3f} sigma {sigma_mu / mu:.2e} alpha {alpha:.3f} blocked by {who}")
        u = u + alpha * du
        s = s + alpha * ds
        for key, (dw, dl) in d.items():
            state[key][0][...] += alpha * dw
            state[key][1][...] += alpha * dl
    return u, max_iter, hist


def gondzio(direction, amax_of, state, rc, du, ds, d, amax, sigma_mu, k_max=2, beta_min=0.1,
            beta_max=10.0, delta_a=0.1, gamma=0.1):
    """Gondzio's multiple centrality correctors: aim the complementarity products of the trial
    point x + a_t d (a_t a little longer than the current step) at [beta_min, beta_max] sigma mu
    and keep a corrected direction while it lengthens the step."""
    for _ in range(k_max):
        a_t = min(1.0, 1.5 * amax + delta_a)
        rc2 = {}
        for k, (w_, l_) in state.items():
            vt = (w_ + a_t * d[k][0]) * (l_ + a_t * d[k][1])
            lo, hi = beta_min * sigma_mu, beta_max * sigma_mu
            t = np.where(vt < lo, lo - vt, np.where(vt > hi, np.maximum(hi - vt, -hi), 0.0))
            rc2[k] = rc[k] + t
        du2, ds2, d2 = direction(rc2)
        a2 = amax_of(d2)
        if a2 >= amax + gamma * delta_a:
            du, ds, d, amax, rc = du2, ds2, d2, a2, rc2
        else:
            break
    return du, ds, d, amax


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--npz", default="gpurun_out/qp_problems.npz")
    ap.add_argument("--variant", default="base")
    ap.add_argument("--only", default="")
    ap.add_argument("--trace", action="store_true")
    ap.add_argument("--start", default="", help="k=v,... overrides of START")
    ap.add_argument("--quiet", action="store_true")
    args = ap.parse_args()
    for kv in filter(None, args.start.split(",")):
        k, v = kv.split("=")
        START[k] = float(v)
    z = np.load(args.npz)
    keys = sorted({k.rsplit("_", 1)[0] for k in z.files if k.endswith("_h")})
    tot_k, tot_l, c5, its = 0, 0, 0, []
    for key in keys:
        if args.only and args.only not in key:
            continue
        H = int(key.split("_")[0][1:])
        md = model(H)
        hb, gb, x0b, xrb, ub, infb = (z[f"{key}_{s}"] for s in ("h", "g", "x0", "xr", "u", "info"))
        for b in range(hb.shape[0]):
            u, it, hist = solve(md, hb[b], gb[b], x0b[b], xrb[b], args.variant, trace=args.trace)
            kit = int(infb[b, 1])
            err = np.abs(u.reshape(-1) - ub[b].reshape(-1)).max()
            tot_k += kit
            tot_l += it
            its.append(it)
            if "O256" in key:
                c5 += it
            if not args.quiet:
                print(f"{key} b{b}: lab {it:2d} iterations (kernel {kit:2d}), |u - u_kernel| {err:.1e}",
                  flush=True)
    print(f"{args.variant} {args.start}: total iterations: lab {tot_l} (C5 {c5}), kernel {tot_k}, "
          f"max {max(its)}, histogram {np.bincount(its).tolist()}")


if __name__ == "__main__":
    sys.exit(main())

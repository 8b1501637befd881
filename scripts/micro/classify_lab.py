"""CPU laboratory (design tool): how well the polish's active-set guess at the interior-point
endpoint matches the optimum's active set, for two guesses —
  current : lambda > w for every complementary pair (the kernel's rule through round 4)
  tapia   : d lambda / lambda > d w / w with the affine (predictor) direction at the endpoint
            (Tapia's indicators: a pair whose w shrinks faster than its lambda is active)
The interior-point endpoint is scripts/micro/ipm_lab.py's restatement of the kernel (its start,
Mehrotra steps and tolerance); the optimum is oracle/mpc_qp.py's KKT-certified answer.

    python scripts/micro/classify_lab.py scripts/micro/data/qp_small.npz [...]
"""
import inspect
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", ".."))
import ipm_lab as L  # noqa: E402
from oracle import mpc_qp  # noqa: E402

_src = inspect.getsource(L.solve).replace(
    "return u, it, hist\n",
    "return u, it, hist, dict(s=s, wA=wA, lA=lA, wB=wB, lB=lB, wUu=wUu, lUu=lUu, wUl=wUl, lUl=lUl, "
    "wPu=wPu, lPu=lPu, wPl=wPl, lPl=lPl, f=f, c=c)\n", 1)
_ns = dict(L.__dict__)
exec(_src, _ns)
solve = _ns["solve"]
for kv in "central_mu=20,central_mu_few=1,u_free=1,many=64,lam_cap=25,tol=1e-7".split(","):
    k, v = kv.split("=")
    L.START[k] = float(v)


def affine(md, h, g, u, st):
    H = md["H"]
    Gp, H0, c, f = md["Gp"], md["H0"], st["c"], st["f"]
    h0, h1 = h[..., 0], h[..., 1]
    s_, wA, lA, wB, lB = (st[k] for k in ("s", "wA", "lA", "wB", "lB"))
    lUu, lUl, lPu, lPl, wUu, wUl, wPu, wPl = (st[k] for k in ("lUu", "lUl", "lPu", "lPl", "wUu", "wUl", "wPu", "wPl"))
    p = c + Gp @ u
    P = p.reshape(H, 2)
    hp = h0 * P[None, :, 0] + h1 * P[None, :, 1]
    v = np.stack([(lA * h0).sum(0), (lA * h1).sum(0)], -1).reshape(-1) + (lPu - lPl)
    r_du = H0 @ u + f + Gp.T @ v + (lUu - lUl)
    r_ds = 100 * s_ + 50 - lA - lB
    r_pA, r_pB = hp + g - s_ + wA, wB - s_
    r_Uu, r_Ul = u - md["umax"] + wUu, md["umin"] - u + wUl
    r_Pu, r_Pl = p - md["pmax"] + wPu, md["pmin"] - p + wPl
    DA, DB = lA / wA, lB / wB
    sig = 100 + DA + DB
    om = DA * (100 + DB) / sig
    DUu, DUl, DPu, DPl = lUu / wUu, lUl / wUl, lPu / wPu, lPl / wPl
    Sb = np.zeros((2 * H, 2 * H))
    for k in range(H):
        Sb[2 * k:2 * k + 2, 2 * k:2 * k + 2] = [[(om[:, k] * h0[:, k] ** 2).sum() + DPu[2 * k] + DPl[2 * k], (om[:, k] * h0[:, k] * h1[:, k]).sum()],
                                                [(om[:, k] * h0[:, k] * h1[:, k]).sum(), (om[:, k] * h1[:, k] ** 2).sum() + DPu[2 * k + 1] + DPl[2 * k + 1]]]
    K = H0 + np.diag(DUu + DUl) + Gp.T @ Sb @ Gp
    rhoA, rhoB = DA * r_pA - lA, DB * r_pB - lB
    rhs_s = -r_ds + rhoA + rhoB
    coef = rhoA - DA * rhs_s / sig
    rhoUu, rhoUl = DUu * r_Uu - lUu, DUl * r_Ul - lUl
    rhoPu, rhoPl = DPu * r_Pu - lPu, DPl * r_Pl - lPl
    zz = np.stack([(coef * h0).sum(0), (coef * h1).sum(0)], -1).reshape(-1) + rhoPu - rhoPl
    du = np.linalg.solve(K, -r_du - (rhoUu - rhoUl) - Gp.T @ zz)
    dp = Gp @ du
    dP = dp.reshape(H, 2)
    hdp = h0 * dP[None, :, 0] + h1 * dP[None, :, 1]
    ds = (rhs_s + DA * hdp) / sig
    gA = hdp - ds
    return dict(A=(-r_pA - gA, DA * gA + rhoA), B=(-r_pB + ds, -DB * ds + rhoB),
                Uu=(-r_Uu - du, DUu * du + rhoUu), Ul=(-r_Ul + du, -DUl * du + rhoUl),
                Pu=(-r_Pu - dp, DPu * dp + rhoPu), Pl=(-r_Pl + dp, -DPl * dp + rhoPl))


def main():
    tot = {"current": 0, "tapia": 0}
    probs = 0
    bad_probs = {"current": 0, "tapia": 0}
    for path in sys.argv[1:]:
        z = np.load(path)
        keys = sorted({k.rsplit("_", 1)[0] for k in z.files if k.endswith("_h")})
        for key in keys:
            H = int(key.split("_")[0][1:])
            md = L.model(H)
            h, g, x0, xr = (z[f"{key}_{s}"][0] for s in ("h", "g", "x0", "xr"))
            u, it, hist, st = solve(md, h, g, x0, xr)
            d = affine(md, h, g, u, st)
            A = np.block([[np.eye(2), 0.2 * np.eye(2)], [np.zeros((2, 2)), np.eye(2)]])
            B = np.block([[0.02 * np.eye(2)], [0.2 * np.eye(2)]])
            C = np.block([np.eye(2), np.zeros((2, 2))])
            rows = [np.concatenate([h[:, t], g[:, t, None]], 1) for t in range(H)]
            xo, uo, io = mpc_qp.filter_trajectory(A, B, C, 2 * np.eye(4), np.eye(2), H, x0, xr, None, rows,
                                                  (np.full(2, -5.0), np.full(2, 5.0)), (np.full(2, -10.0), np.full(2, 10.0)))
            us = uo.reshape(-1)
            p = st["c"] + md["Gp"] @ us
            P = p.reshape(H, 2)
            hp = h[..., 0] * P[None, :, 0] + h[..., 1] * P[None, :, 1] + g
            optA = hp > -1e-9          # halfspace row binding or violated (s = max(hp, 0))
            optB = hp < 1e-9           # slack at zero
            opt = {"A": optA, "B": optB, "Uu": us >= md["umax"] - 1e-9, "Ul": us <= md["umin"] + 1e-9,
                   "Pu": p >= md["pmax"] - 1e-9, "Pl": p <= md["pmin"] + 1e-9}
            state = {"A": ("wA", "lA"), "B": ("wB", "lB"), "Uu": ("wUu", "lUu"), "Ul": ("wUl", "lUl"),
                     "Pu": ("wPu", "lPu"), "Pl": ("wPl", "lPl")}
            mis = {}
            for rule in ("current", "tapia"):
                m = 0
                for key2, (wn, ln) in state.items():
                    w, lam = st[wn], st[ln]
                    dw, dl = d[key2]
                    act = lam > w if rule == "current" else dl * w > dw * lam
                    m += int((act != opt[key2]).sum())
                mis[rule] = m
                tot[rule] += m
                bad_probs[rule] += m > 0
            probs += 1
            print(f"{key}: {it} iterations, |u_ipm - u*| {np.abs(u - us).max():.1e}, misclassified: current {mis['current']}, tapia {mis['tapia']}", flush=True)
    print(f"{probs} problems: misclassified pairs current {tot['current']} ({bad_probs['current']} problems), "
          f"tapia {tot['tapia']} ({bad_probs['tapia']} problems)")


if __name__ == "__main__":
    main()

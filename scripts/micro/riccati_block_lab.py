"""CPU laboratory (design tool, not an oracle): the MPC Riccati factorisation split into horizon
blocks, the form a multi-wave device factorisation would run, against the sequential recursion
csrc/drcvar_mpc.hip runs on one wave.

  phase 1  every block [s, e) runs the recursion from the identity element at its end (J = 0),
           carrying beside it the block's element E^(k) = (A_E, C_E, J_E) of steps k..e-1:
             Re = Rb_k + B' J_E B,  Kg = Re^-1 B' J_E A,
             J_E <- Qb_k + A' J_E A - (B' J_E A)' Kg          (the ordinary step)
             A_E <- A_E (A - B Kg),  C_E <- C_E + (A_E B) Re^-1 (A_E B)'   (old A_E on the right)
           (the last block starts from the true terminal P_H and is exact already);
  phase 2  the true P at each block end, from the back: P_s = J_E + A_E' (I + P_e C_E)^-1 P_e A_E;
  phase 3  every step at once: P_{k+1} from its block's partial element E^(k+1) and P_e, then
           Re_k, Kg_k, Re_k^-1 — no serial chain.

Reported per captured Newton system: max relative difference of Kg and Re^-1 against the
sequential recursion, and the smallest relative pivot of I + P_e C_E without pivoting.

    python scripts/micro/riccati_block_lab.py --npz <qp set> [--blocks 4]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import ipm_lab  # noqa: E402
from riccati_scan_lab import A, B, backward_error, lq_blocks, nopivot_rel_pivot  # noqa: E402

PIV = {"min": np.inf}


def seq_factor(Qb, Rb, H):
    P = Qb[H].copy()
    Kg, Ri = [None] * H, [None] * H
    for k in range(H - 1, -1, -1):
        Re = Rb[k] + B.T @ P @ B
        L = B.T @ P @ A
        Ri[k] = np.linalg.inv(Re)
        Kg[k] = Ri[k] @ L
        if k > 0:
            P = Qb[k] + A.T @ P @ A - L.T @ Kg[k]
            P = 0.5 * (P + P.T)
    return Kg, Ri


def solve_with(Kg, Ri, b, H):
    """K du = b from the gains (the device's solve: backward p pass, forward rollout)."""
    p = np.zeros(4)
    kff = [None] * H
    for k in range(H - 1, -1, -1):
        bk = b[2 * k:2 * k + 2]
        ge = B.T @ p - bk
        kff[k] = -Ri[k] @ ge
        p = A.T @ p - Kg[k].T @ ge
    x, u = np.zeros(4), np.zeros(2 * H)
    for k in range(H):
        uk = kff[k] - Kg[k] @ x
        u[2 * k:2 * k + 2] = uk
        x = A @ x + B @ uk
    return u


def apply_element(P, AE, CE, JE):
    N = np.eye(4) + P @ CE
    PIV["min"] = min(PIV["min"], nopivot_rel_pivot(N))
    Y = np.linalg.solve(N, P @ AE)
    R = JE + AE.T @ Y
    return 0.5 * (R + R.T)


def block_factor(Qb, Rb, H, W):
    bounds = np.linspace(0, H, W + 1).round().astype(int)
    part = {}  # k -> partial element (A_E, C_E, J_E) of steps k..e-1 of k's block
    Pstart = {}
    for w in range(W):  # phase 1 (blocks independent)
        s, e = bounds[w], bounds[w + 1]
        last = w == W - 1
        AE, CE = np.eye(4), np.zeros((4, 4))
        JE = Qb[H].copy() if last else np.zeros((4, 4))
        part[e] = (AE, CE, JE)
        for k in range(e - 1, s - 1, -1):
            Re = Rb[k] + B.T @ JE @ B
            L = B.T @ JE @ A
            Rinv = np.linalg.inv(Re)
            Kg = Rinv @ L
            G = AE @ B
            CE = CE + G @ Rinv @ G.T
            CE = 0.5 * (CE + CE.T)
            AE = AE @ (A - B @ Kg)
            JE = Qb[k] + A.T @ JE @ A - L.T @ Kg
            JE = 0.5 * (JE + JE.T)
            part[k] = (AE, CE, JE)
        Pstart[w] = (AE, CE, JE)
    Pend = {W - 1: None}  # phase 2: the true P at each block's end
    P_next = Pstart[W - 1][2]  # the last block is exact: its P at s
    for w in range(W - 2, -1, -1):
        Pend[w] = P_next
        if w > 0:
            P_next = apply_element(P_next, *Pstart[w])
    Kg, Ri = [None] * H, [None] * H
    for w in range(W):  # phase 3 (every step independent)
        s, e = bounds[w], bounds[w + 1]
        for k in range(s, e):
            AE, CE, JE = part[k + 1]
            P1 = JE if w == W - 1 else (JE if k + 1 == e else apply_element(Pend[w], AE, CE, JE))
            if k + 1 == e and w < W - 1:
                P1 = Pend[w]
            Re = Rb[k] + B.T @ P1 @ B
            Ri[k] = np.linalg.inv(Re)
            Kg[k] = Ri[k] @ (B.T @ P1 @ A)
    return Kg, Ri


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--npz", default="scripts/micro/data/qp_set.npz")
    ap.add_argument("--only", default="")
    ap.add_argument("--blocks", type=int, default=4)
    ap.add_argument("--start", default="u_free=1,central_mu=20,central_mu_few=1,lam_cap=25,tol=1e-7")
    args = ap.parse_args()
    for kv in filter(None, args.start.split(",")):
        k, v = kv.split("=")
        ipm_lab.START[k] = float(v)
    z = np.load(args.npz)
    keys = sorted({k.rsplit("_", 1)[0] for k in z.files if k.endswith("_h")})
    worst = {"Kg": 0.0, "Ri": 0.0}
    for key in keys:
        if args.only and args.only not in key:
            continue
        H = int(key.split("_")[0][1:])
        md = ipm_lab.model(H)
        rows = []

        def on_system(it, merit, S, DU, K):
            Qb, Rb = lq_blocks(S, DU, H)
            Ks, Rs = seq_factor(Qb, Rb, H)
            Kb, Rbk = block_factor(Qb, Rb, H, args.blocks)
            ek = max(np.abs(Kb[k] - Ks[k]).max() / max(np.abs(Ks[k]).max(), 1e-300) for k in range(H))
            er = max(np.abs(Rbk[k] - Rs[k]).max() / np.abs(Rs[k]).max() for k in range(H))
            b = np.random.default_rng(it).standard_normal(2 * H)
            be_s = backward_error(K, solve_with(Ks, Rs, b, H), b)
            be_b = backward_error(K, solve_with(Kb, Rbk, b, H), b)
            rows.append((it, merit, ek, er, be_s, be_b))

        try:
            ipm_lab.solve(md, z[f"{key}_h"][0], z[f"{key}_g"][0], z[f"{key}_x0"][0], z[f"{key}_xr"][0],
                          on_system=on_system)
        except np.linalg.LinAlgError:
            pass
        for it, merit, ek, er, be_s, be_b in rows:
            worst["be_seq"] = max(worst.get("be_seq", 0.0), be_s)
            worst["be_block"] = max(worst.get("be_block", 0.0), be_b)
            worst["Kg"] = max(worst["Kg"], ek)
            worst["Ri"] = max(worst["Ri"], er)
        print(f"{key}: {len(rows)} systems, max rel diff Kg {max(r[2] for r in rows):.1e} "
              f"Ri {max(r[3] for r in rows):.1e}, solve backward error seq {max(r[4] for r in rows):.1e} "
              f"block {max(r[5] for r in rows):.1e}")
    print("worst:", {k: f"{v:.1e}" for k, v in worst.items()}, f"min relative pivot {PIV['min']:.1e}")


if __name__ == "__main__":
    sys.exit(main())

"""CPU laboratory (design tool, not an oracle): the MPC Newton systems solved by a parallel-in-horizon
Riccati (associative suffix scan of LQ value-function elements, Särkkä & García-Fernández 2023,
"Temporal parallelization of dynamic programming and linear quadratic control") against the
sequential Riccati recursion csrc/drcvar_mpc.hip runs on one wave, on the systems the interior-point
method actually meets (barrier weights up to 1e10-1e18 near the optimum).

The systems are taken from scripts/micro/ipm_lab.py (the kernel's iteration restated in NumPy) on
problems bench.py's C5 hand-off produces (scripts/micro/dump_bench_qps.py on the GPU box):

    python scripts/micro/riccati_scan_lab.py --npz gpurun_out/qp_bench_set.npz [--only O256]

Per captured Newton system K du = b (random b), reported for the dense Cholesky, the sequential
Riccati and the scan (Hillis-Steele order, as a kernel would run it): the normwise backward error
|K du - b| / (|K| |du| + |b|) (residual in long double), and |du_scan - du_seq| / |du_seq|.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import ipm_lab  # noqa: E402

DT = 0.2
A = np.block([[np.eye(2), DT * np.eye(2)], [np.zeros((2, 2)), np.eye(2)]])
B = np.block([[0.5 * DT ** 2 * np.eye(2)], [DT * np.eye(2)]])
C = np.block([np.eye(2), np.zeros((2, 2))])
Q, R = 2 * np.eye(4), np.eye(2)


def lq_blocks(S, DU, H):
    """State Hessians Qb[k] on x_k (k = 0..H, Qb[0] = 0) and input Hessians Rb[k] on u_k."""
    Qb = [np.zeros((4, 4))] + [2 * Q + C.T @ S[k] @ C for k in range(H)]
    Rb = [2 * R + np.diag(DU[2 * k:2 * k + 2]) for k in range(H)]
    return Qb, Rb


def seq_riccati(Qb, Rb, b, H):
    """The kernel's recursion (symmetrised P), backward p pass, forward rollout from x_0 = 0."""
    P, p = Qb[H].copy(), np.zeros(4)
    Kg, kff = [None] * H, [None] * H
    for k in range(H - 1, -1, -1):
        bk = b[2 * k:2 * k + 2]
        Re = Rb[k] + B.T @ P @ B
        L = B.T @ P @ A
        Kg[k] = np.linalg.solve(Re, L)
        kff[k] = np.linalg.solve(Re, bk + B.T @ p)
        p = (A - B @ Kg[k]).T @ p - Kg[k].T @ bk
        P = Qb[k] + A.T @ P @ A - L.T @ Kg[k]
        P = 0.5 * (P + P.T)
    x, u = np.zeros(4), np.zeros(2 * H)
    for k in range(H):
        uk = -Kg[k] @ x + kff[k]
        u[2 * k:2 * k + 2] = uk
        x = A @ x + B @ uk
    return u


PIVOTS = {"min_rel_pivot": np.inf}


def nopivot_rel_pivot(M):
    """Smallest |pivot| / max|row| of Gauss elimination WITHOUT pivoting on M (what a pivot-free
    in-register elimination on the device would meet)."""
    a = M.astype(float).copy()
    worst = np.inf
    for q in range(a.shape[0]):
        worst = min(worst, abs(a[q, q]) / max(np.abs(a[q]).max(), 1e-300))
        if a[q, q] == 0.0:
            return 0.0
        a[q + 1:] -= np.outer(a[q + 1:, q] / a[q, q], a[q])
    return worst


def combine(e1, e2):
    """e1 (i -> j) followed by e2 (j -> k): (A, b, C, eta, J) of the composed element."""
    A1, b1, C1, n1, J1 = e1
    A2, b2, C2, n2, J2 = e2
    M = np.eye(4) + C1 @ J2                    # (I + J2 C1) = M^T for symmetric C1, J2
    PIVOTS["min_rel_pivot"] = min(PIVOTS["min_rel_pivot"], nopivot_rel_pivot(M))
    MiA1 = np.linalg.solve(M, A1)
    A12 = A2 @ MiA1
    b12 = A2 @ np.linalg.solve(M, b1 + C1 @ n2) + b2
    C12 = A2 @ np.linalg.solve(M, C1) @ A2.T + C2
    C12 = 0.5 * (C12 + C12.T)
    MTi = np.linalg.solve(M.T, np.column_stack([n2 - J2 @ b1, J2 @ A1]))
    n12 = A1.T @ MTi[:, 0] + n1
    J12 = A1.T @ MTi[:, 1:] + J1
    J12 = 0.5 * (J12 + J12.T)
    return A12, b12, C12, n12, J12


def scan_riccati(Qb, Rb, b, H):
    """Suffix scan e_k (x) ... (x) e_H in Hillis-Steele order: S_k = J, v_k = eta; then the gains of
    every step at once and the forward rollout."""
    els = []
    for k in range(H):
        Rinv = np.linalg.inv(Rb[k])
        els.append((A.copy(), B @ Rinv @ b[2 * k:2 * k + 2], B @ Rinv @ B.T, np.zeros(4), Qb[k].copy()))
    els.append((np.zeros((4, 4)), np.zeros(4), np.zeros((4, 4)), np.zeros(4), Qb[H].copy()))
    n, d = H + 1, 1
    while d < n:
        els = [combine(els[i], els[i + d]) if i + d < n else els[i] for i in range(n)]
        d *= 2
    x, u = np.zeros(4), np.zeros(2 * H)
    for k in range(H):
        S1, v1 = els[k + 1][4], els[k + 1][3]
        bk = b[2 * k:2 * k + 2]
        Rinv = np.linalg.inv(Rb[k])
        c = B @ Rinv @ bk
        Re = Rb[k] + B.T @ S1 @ B
        ubar = np.linalg.solve(Re, -B.T @ S1 @ A @ x + B.T @ (v1 - S1 @ c))
        uk = ubar + Rinv @ bk
        u[2 * k:2 * k + 2] = uk
        x = A @ x + B @ uk
    return u


def backward_error(K, du, b):
    Kl, dl, bl = K.astype(np.longdouble), du.astype(np.longdouble), b.astype(np.longdouble)
    r = Kl @ dl - bl
    den = np.abs(Kl).sum(1).max() * np.abs(dl).max() + np.abs(bl).max()
    return float(np.abs(r).max() / den)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--npz", default="gpurun_out/qp_bench_set.npz")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    z = np.load(args.npz)
    keys = sorted({k.rsplit("_", 1)[0] for k in z.files if k.endswith("_h")})
    rng = np.random.default_rng(0)
    worst = {"dense": 0.0, "seq": 0.0, "scan": 0.0, "scan_vs_seq": 0.0}
    for key in keys:
        if args.only and args.only not in key:
            continue
        H = int(key.split("_")[0][1:])
        md = ipm_lab.model(H)
        rows = []

        def on_system(it, merit, S, DU, K):
            b = rng.standard_normal(2 * H)
            Qb, Rb = lq_blocks(S, DU, H)
            du_d = np.linalg.solve(K, b)
            du_s = seq_riccati(Qb, Rb, b, H)
            du_p = scan_riccati(Qb, Rb, b, H)
            rows.append((it, merit, np.abs(S).max(), DU.max(), backward_error(K, du_d, b),
                         backward_error(K, du_s, b), backward_error(K, du_p, b),
                         np.abs(du_p - du_s).max() / np.abs(du_s).max()))

        try:
            ipm_lab.solve(md, z[f"{key}_h"][0], z[f"{key}_g"][0], z[f"{key}_x0"][0], z[f"{key}_xr"][0],
                          on_system=on_system)
            print(f"{key}: {len(rows)} Newton systems")
        except np.linalg.LinAlgError as e:  # the lab's own dense Cholesky (the kernel would polish)
            print(f"{key}: {len(rows)} Newton systems, then the lab's dense Cholesky failed ({e})")
        for it, merit, smax, dumax, e_d, e_s, e_p, rel in rows:
            print(f"  it {it:2d} merit {merit:.1e} max|S| {smax:.1e} max D_u {dumax:.1e}  backward error "
                  f"dense {e_d:.1e} seq {e_s:.1e} scan {e_p:.1e}  |du_scan - du_seq|/|du_seq| {rel:.1e}")
            for name, v in (("dense", e_d), ("seq", e_s), ("scan", e_p), ("scan_vs_seq", rel)):
                worst[name] = max(worst[name], v)
    print("worst:", {k: f"{v:.1e}" for k, v in worst.items()},
          f"smallest relative pivot of M = I + C1 J2 without pivoting: {PIVOTS['min_rel_pivot']:.1e}")


if __name__ == "__main__":
    sys.exit(main())

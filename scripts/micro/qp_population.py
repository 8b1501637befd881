"""A CPU population of main.py-like QPs (scripts/mpc_bench.py's shape: H steps, O obstacles, the
double integrator and its bounds), halfspaces from the C oracle on numpy-drawn samples, solved by
the kernel's CPU restatement (scripts/micro/ipm_lab.py) under START variants: iteration histograms,
to choose interior-point rules against stragglers before porting any.  Design tool, not an oracle.

    python scripts/micro/qp_population.py [--n 512] [--shape 30,3] [--set k=v,...] ...
"""
import argparse
import math
import os
import sys
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)
import ipm_lab as L  # noqa: E402
from oracle import c_oracle  # noqa: E402

KERNEL_START = dict(central_mu=20, central_mu_few=1, u_free=1, many=64, lam_cap=25)


def problem(H, O, seed, N=200):
    rng = np.random.default_rng(seed)
    start = rng.uniform(-5, 5, (O, 2))
    heading = rng.uniform(0, 2 * math.pi, O)
    speed = rng.uniform(0.6, 1.5, O)
    vel = np.stack([np.cos(heading), np.sin(heading)], 1) * speed[:, None]
    t = np.arange(H) * 0.2
    nom = start[:, None, :] + t[None, :, None] * vel[:, None, :]
    samples = nom[:, :, None, :] + 0.1 * rng.standard_normal((O, H, N, 2))
    samples[:, 0] = nom[:, 0, None, :]
    ego = np.zeros((H, 2))
    ego[:, 0] = -4.0
    n_move = int((8.0 / 1.5) / 0.2)
    for k in range(1, H):
        ego[k, 0] = -4.0 + 8.0 * min(k / n_move, 1.0)
    rec = c_oracle.safe_halfspaces(samples, ego, 0.3, 0.3, 0.2, 0.1, 0.15)
    xr = np.zeros((H + 1, 4))
    xr[:H, :2] = ego
    xr[H, :2] = ego[-1]
    return rec[..., 3:5].copy(), rec[..., 7].copy(), xr[0].copy(), xr


def run_one(job):
    H, O, seed, start, variant = job
    L.START.update(start)
    h, g, x0, xr = problem(H, O, seed)
    u, it, hist = L.solve(L.model(H), h, g, x0, xr, variant, tol=1e-7)
    return seed, it


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--shape", default="30,3")
    ap.add_argument("--variant", default="base")
    ap.add_argument("--set", action="append", default=[""], help="START overrides k=v,... (one run each)")
    ap.add_argument("--procs", type=int, default=8)
    a = ap.parse_args()
    H, O = (int(v) for v in a.shape.split(","))
    for spec in a.set:
        start = dict(KERNEL_START)
        for kv in filter(None, spec.split(",")):
            k, v = kv.split("=")
            start[k] = float(v)
        with Pool(a.procs) as pool:
            res = pool.map(run_one, [(H, O, s, start, a.variant) for s in range(a.n)])
        its = np.array([r[1] for r in res])
        worst = sorted(res, key=lambda r: -r[1])[:5]
        print(f"{a.variant} {spec or 'kernel'}: mean {its.mean():.2f} max {its.max()} hist {np.bincount(its).tolist()} "
              f"worst {worst}", flush=True)


if __name__ == "__main__":
    main()

"""CPU generator of C5-like safety-filter QPs for scripts/micro/ipm_lab.py / start_lab.py (design
tool): synthetic nominal paths (synthetic.nominal_paths on the CPU), N(0, 0.01 I) samples drawn by
numpy, DR-CVaR halfspaces by the closed form (oracle/closed_form.py), the bench's ego line and
model.  Same distributions as bench.py's C5 hand-off, not the same draws.  Writes
scripts/micro/data/qp_set.npz in ipm_lab's key layout (u / info: zeros)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, REPO)
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import synthetic  # noqa: E402
from oracle import closed_form  # noqa: E402

SHAPES = [(50, 256, s) for s in range(6)] + [(30, 64, s) for s in range(3)] + [(20, 100, s) for s in range(3)]
if os.environ.get("QP_SET") == "metrics":  # main.py's three filters at C5 size
    SHAPES = [(50, 256, s, m) for s in range(3) for m in ("mean", "cvar")] + [(20, 10, s, m) for s in range(4) for m in ("mean", "cvar", "dr")]
if os.environ.get("QP_SET") == "batch":  # mpc_bench.py's 30,3,B shape: many seeds
    SHAPES = [(30, 3, s) for s in range(64)]
if os.environ.get("QP_SET") == "small":  # main.py-like: a few obstacles, H = 30 / 20
    SHAPES = [(30, 3, s) for s in range(8)] + [(20, 10, s) for s in range(4)] + [(40, 6, s) for s in range(4)]


METRIC_COLS = {"dr": ((3, 4), 7), "mean": ((0, 1), 2), "cvar": ((3, 4), 5)}


def one(H, O, seed, N=1000, metric="dr"):
    rng = np.random.default_rng(seed)
    nom = synthetic.nominal_paths(O, H, "cpu", seed=seed + 100).numpy()
    ego = synthetic.straight_line_ego(H, "cpu").numpy()
    smp = nom[:, :, None, :] + 0.1 * rng.standard_normal((O, H, N, 2))
    smp[:, 0] = nom[:, 0, None, :]
    rec = closed_form.safe_halfspaces(smp, ego, 0.3, 0.3, 0.2, 0.1, 0.15)
    (c0, c1), cg = METRIC_COLS[metric]
    h, g = rec[..., [c0, c1]], rec[..., cg]
    xr = np.zeros((H + 1, 4))
    xr[:H, :2] = ego[:H]
    xr[H:, :2] = ego[H - 1]
    xr[:-1, 2:] = (xr[1:, :2] - xr[:-1, :2]) / 0.2
    return h, g, xr[0].copy(), xr


def main():
    out = {}
    for shape in SHAPES:
        H, O, seed = shape[:3]
        metric = shape[3] if len(shape) > 3 else "dr"
        h, g, x0, xr = one(H, O, seed, metric=metric)
        key = f"H{H}_O{O}_B1_s{seed}{metric}"
        out.update({f"{key}_h": h[None], f"{key}_g": g[None], f"{key}_x0": x0[None], f"{key}_xr": xr[None],
                    f"{key}_u": np.zeros((1, H, 2)), f"{key}_info": np.zeros((1, 10))})
        print(key, flush=True)
    os.makedirs(os.path.join(REPO, "scripts", "micro", "data"), exist_ok=True)
    np.savez_compressed(os.path.join(REPO, "scripts", "micro", "data", {"small": "qp_small.npz", "metrics": "qp_metrics.npz", "batch": "qp_batch.npz"}.get(os.environ.get("QP_SET"), "qp_set.npz")), **out)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Diagnostic: per-phase shader-clock totals of the MPC kernel from a -DDRCVAR_MPC_STAMPS build."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import diaglib  # noqa: E402
diaglib.apply()  # DRCVAR_DIAG_LIB: a variant build (diagnostics)
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import _native  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf  # noqa: E402
from mpc_bench import problem_batch  # noqa: E402

NAMES = {0: "setup", 1: "P1 residuals+weights", 2: "affine rhs", 3: "Riccati factor (ipm)",
         4: "Riccati solves (ipm)", 5: "row passes P2-P5", 6: "loop exit", 7: "polish other",
         8: "output", 10: "polish classify+assemble", 11: "polish Riccati factor",
         12: "polish row passes", 13: "polish solves", 14: "positions (ipm)", 15: "loop top",
         16: "cluster exchanges", 17: "setup: model, c, x_ref, f", 18: "setup: u start + positions",
         19: "setup: rows' start"}
dev = torch.device("cuda", 0)
lib = _native.lib()
lib.drcvar_diag_mpc_stamps.argtypes = [ctypes.c_void_p]
def npz_problem(path, key):
    """A problem saved by scripts/micro/dump_bench_qps.py / dump_qp_problems.py (double integrator),
    or, with key "fixture", a tests/golden/qp_*.npz fixture (h [O, H, 2], g, x0, x_ref)."""
    z = np.load(path)
    if key == "fixture":
        h, g, x0, xr = (torch.as_tensor(z[s][None]).to(dev) for s in ("h", "g", "x0", "x_ref"))
        H = int(z["x_ref"].shape[0]) - 1
    else:
        h, g, x0, xr = (torch.as_tensor(z[f"{key}_{s}"]).to(dev) for s in ("h", "g", "x0", "xr"))
        H = int(key.split("_")[0][1:])
    dt = 0.2
    A = np.block([[np.eye(2), dt * np.eye(2)], [np.zeros((2, 2)), np.eye(2)]])
    Bm = np.block([[0.5 * dt ** 2 * np.eye(2)], [dt * np.eye(2)]])
    C = np.block([np.eye(2), np.zeros((2, 2))])
    model = mf.MPCModel(A, Bm, C, 2 * np.eye(4), np.eye(2), H, (np.full(2, -5.0), np.full(2, 5.0)),
                        (np.full(2, -10.0), np.full(2, 10.0)), device=dev)
    return model, h, g, x0, xr, torch.zeros((h.shape[0], H, 2), dtype=torch.float64, device=dev)


for shape in sys.argv[1:] or ["30,3,1", "50,256,1"]:
    if shape.startswith("npz:"):  # npz:<path>:<key>
        _, path, key = shape.split(":")
        model, h, g, x0, xr, uf = npz_problem(path, key)
        B, O, H = h.shape[0], h.shape[1], h.shape[2]
    else:
        H, O, B = (int(v) for v in shape.split(","))
        model, rec, x0, xr, uf = problem_batch(H, O, B, dev)
        h, g = rec[..., 3:5], rec[..., 7]
    x, u, info = mf.filter_batch(model, h, g, x0, xr, uf)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (64 * 20))()
    assert lib.drcvar_diag_mpc_stamps(ctypes.cast(buf, ctypes.c_void_p)) == 64
    st = np.frombuffer(buf, dtype=np.uint64).reshape(64, 20)[0].astype(np.int64)
    tot = sum(st[k] for k in NAMES)
    print(f"groups {model.launch_groups(B, O)}")
    print(f"H={H} O={O}: total {tot} cycles ({tot / 2.4e9 * 1e3:.3f} ms at 2.4 GHz shader clock), "
          f"iterations {st[9]}, polish attempts {info[0, _native.MPC_INFO_POLISH_ATTEMPTS].item():.0f}")
    for k, nm in NAMES.items():
        print(f"  {nm:28s} {st[k]:10d} ({st[k] / tot * 100:5.1f}%)")
    cb = (ctypes.c_ulonglong * 8)()
    lib.drcvar_diag_cluster_stamps.argtypes = [ctypes.c_void_p]
    if st[16] and lib.drcvar_diag_cluster_stamps(ctypes.cast(cb, ctypes.c_void_p)) == 8:
        cs = np.frombuffer(cb, dtype=np.uint64).astype(np.int64)  # cumulative over every launch so far
        names = ["partials+barrier", "combine+stores+drain", "barrier", "arrive+poll", "barrier", "gather"]
        print("  cluster exchange sub-phases (cumulative, workgroup 0):",
              ", ".join(f"{n} {cs[i] / max(cs[:6].sum(), 1) * 100:.0f}%" for i, n in enumerate(names)))
    try:  # which workgroup of problem 0's cluster arrives last at the exchanges, and how long each waits
        ca = lib.drcvar_diag_cluster_arrivals
        ca.argtypes = [ctypes.c_void_p]
        ab = (ctypes.c_ulonglong * 96)()
        if st[16] and ca(ctypes.cast(ab, ctypes.c_void_p)) == 96:
            a = np.frombuffer(ab, dtype=np.uint64).reshape(3, 32)
            g = int((a[2] > 0).sum())
            if g and len(set(a[2, :g].tolist())) == 1:
                n = int(a[2, 0])
                arr = a[0, :g].astype(np.float64) / n  # mean arrival clock (10 ns ticks)
                rel = a[1, :g].astype(np.float64) / n
                late = (arr - arr.min()) * 10.0
                print(f"  cluster arrivals over {n} exchanges (mean ns after the earliest workgroup): " +
                      ", ".join(f"g{i} {late[i]:.0f}" for i in range(g)))
                print("  mean wait from arrival to release (ns): " +
                      ", ".join(f"g{i} {(rel[i] - arr[i]) * 10.0:.0f}" for i in range(g)))
    except AttributeError:
        pass
    try:
        ws = lib.drcvar_diag_wave_stamps
        ws.argtypes = [ctypes.c_void_p]
        wb = (ctypes.c_ulonglong * 16)()
        if ws(ctypes.cast(wb, ctypes.c_void_p)) == 16:
            w = np.frombuffer(wb, dtype=np.uint64).astype(np.int64).reshape(8, 2)
            print("  P1 span per wave (cumulative over launches so far, cycles per entry): " +
                  ", ".join(f"w{i} {w[i, 0] / max(w[i, 1], 1):.0f}" for i in range(8) if w[i, 1]))
    except AttributeError:
        pass

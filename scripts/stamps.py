#!/usr/bin/env python3
"""Diagnostic: per-phase shader-clock shares from a -DDRCVAR_STAMPS build (DRCVAR_DIAG_LIB)."""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import diaglib  # noqa: E402
diaglib.apply()  # DRCVAR_DIAG_LIB: a variant build (diagnostics)
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import _native, engine, synthetic  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.engine import RiskParams  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="10,20,1000")
ap.add_argument("--geometry", default="")
args = ap.parse_args()
O, T, N = (int(v) for v in args.shape.split(","))
geo = tuple(int(v) for v in args.geometry.split(",")) if args.geometry else None
dev = torch.device("cuda", 0)
s, e = synthetic.obstacle_batch(O, T, N, dev)
launch, out = engine.prepare_safe_halfspaces(s, e, RiskParams(), geometry=geo)
for _ in range(30):
    launch()
torch.cuda.synchronize()
lib = _native.lib()
U = min(O * T, 16384)
KS = 16 if os.environ.get("DRCVAR_STAMPS_WAVES") else 8  # a -DDRCVAR_STAMPS_WAVES build
buf = (ctypes.c_ulonglong * (U * KS))()
lib.drcvar_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
assert lib.drcvar_diag_stamps(ctypes.cast(buf, ctypes.c_void_p), U) == U
st = np.frombuffer(buf, dtype=np.uint64).reshape(U, KS).astype(np.int64)
if KS == 16:  # per-wave: loads summed (slots 8..11), reduction done before barrier 1 (12..15)
    nw = 4
    ld = st[:, 8:8 + nw] - st[:, :1]
    rd = st[:, 12:12 + nw] - st[:, :1]
    print("  per wave, cycles from entry (median over units): loads summed",
          np.median(ld, 0).round().tolist(), " reduced", np.median(rd, 0).round().tolist(),
          " barrier 1 passed", float(np.median(st[:, 2] - st[:, 0])))
    print("  latest wave's loads summed - earliest (median)", float(np.median(ld.max(1) - ld.min(1))))
    st = st[:, :8]
names = ["entry->loads done", "moments reduce+barrier1", "h/var/histogram atomics",
         "barrier2+scan", "compaction", "barrier3", "rank+finish"]
d = np.diff(st, axis=1)
tot = st[:, 7] - st[:, 0]
print(f"shape {args.shape} geometry {geo}: median unit cycles {np.median(tot):.0f} "
      f"(min {tot.min()}, max {tot.max()})")
for k, nm in enumerate(names):
    print(f"  {nm:28s} median {np.median(d[:, k]):8.0f} cycles  ({np.median(d[:, k]) / np.median(tot) * 100:5.1f}%)")
slow = np.argsort(tot)[-3:][::-1]
for u_ in slow:  # where the slowest units (they set the kernel's end) lose their time
    print(f"  slow unit {u_} (obstacle {u_ // T}, step {u_ % T}): total {tot[u_]}, phases {d[u_].tolist()}")
if os.environ.get("DRCVAR_STAMPS_REALTIME"):  # built with -DDRCVAR_STAMPS_REALTIME: 10 ns ticks
    t0 = st[:, 0].min()
    start, end = (st[:, 0] - t0) * 10, (st[:, 7] - t0) * 10
    q = [0, 10, 50, 90, 100]
    print("  realtime (ns from the first unit's entry): entry percentiles",
          np.percentile(start, q).round(), " exit percentiles", np.percentile(end, q).round())
    # the launch's occupancy over time (units in flight per 1 us bin): the ramp, the rounds, the tail
    span = int(end.max()) + 1
    edges = np.arange(0, span + 1000, 1000)
    inflight = [int(((start < e1) & (end > e0)).sum()) for e0, e1 in zip(edges[:-1], edges[1:])]
    print("  units in flight per us:", inflight)
    peak = max(inflight)
    full = [i for i, v in enumerate(inflight) if v >= 0.9 * peak]
    print(f"  peak {peak} in flight; >= 90% of it from {full[0]} to {full[-1] + 1} us of {span / 1000:.1f} us;"
          f" last entry {start.max() / 1000:.2f} us, first exit {end.min() / 1000:.2f} us,"
          f" exits 50% {np.percentile(end, 50) / 1000:.2f}, 90% {np.percentile(end, 90) / 1000:.2f},"
          f" 99% {np.percentile(end, 99) / 1000:.2f}, 100% {end.max() / 1000:.2f} us")
else:
    print("  (phase cycles are per-XCD shader clocks; build with -DDRCVAR_STAMPS_REALTIME for the"
          " spread of entries/exits across workgroups)")

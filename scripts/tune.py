#!/usr/bin/env python3
"""Time every compiled launch geometry for a workload (run under rocprofv3 --kernel-trace --stats
for per-kernel durations; the wall numbers printed here include launch gaps)."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import diaglib  # noqa: E402
diaglib.apply()  # DRCVAR_DIAG_LIB: a variant build (diagnostics)
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import engine, synthetic  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.engine import RiskParams  # noqa: E402

GEOMS = [(64, 2), (128, 4), (256, 4), (256, 8), (256, 16), (512, 16), (512, 20), (1024, 12),
         (1024, 16), (64, 16), (128, 8), (512, 2), (1024, 10), (256, 20)]

ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="10,20,1000")
ap.add_argument("--launches", type=int, default=300)
ap.add_argument("--only-auto", action="store_true")
ap.add_argument("--graph", type=int, default=0, help="time hipGraph replays of this many launches")
ap.add_argument("--geoms", default="", help="only these geometries, e.g. 256x4,512x2")
args = ap.parse_args()
O, T, N = (int(v) for v in args.shape.split(","))
dev = torch.device("cuda", 0)
s, e = synthetic.obstacle_batch(O, T, N, dev)
ref = None
geoms = [None] + ([] if args.only_auto else [g for g in GEOMS if g[0] * g[1] >= N])
if args.geoms:
    geoms = [tuple(int(v) for v in x.split("x")) for x in args.geoms.split(",")]
for rep in range(2):  # every geometry twice, interleaved: the first timings of a process run cold
  for g in geoms:
    launch, out = engine.prepare_safe_halfspaces(s, e, RiskParams(), geometry=g)
    fire = launch
    if args.graph:
        gr = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream(dev)
        with torch.cuda.graph(gr, stream=side):
            lg, _ = engine.prepare_safe_halfspaces(s, e, RiskParams(), geometry=g, out=out,
                                                   stream=torch.cuda.current_stream(dev))
            for _ in range(args.graph):
                lg()
        fire = gr.replay
    reps = args.launches // args.graph if args.graph else args.launches
    for _ in range(max(2, reps // 10)):
        fire()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fire()
    b.record()
    torch.cuda.synchronize()
    total = reps * (args.graph or 1)
    wall = (time.perf_counter() - t0) / total * 1e6
    ev = a.elapsed_time(b) / total * 1e3
    if ref is None:
        ref = out.clone()
    same = torch.equal(out, ref)
    print(f"{'graph' if args.graph else 'eager'} rep {rep} geometry={g} O={O} T={T} N={N}: "
          f"{wall:8.2f} us/launch wall, {ev:8.2f} us/launch events, bitwise-equal-to-auto={same}",
          flush=True)

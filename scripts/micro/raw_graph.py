#!/usr/bin/env python3
"""K = 20 timed region of the C3 batch: torch.cuda.CUDAGraph.replay() against a hipGraph built and
launched through the HIP runtime directly (hipStreamBeginCapture / hipGraphInstantiate /
hipGraphLaunch by ctypes).  Host time of the launch call alone, and the region's wall and event
time per step (medians of 15 regions, each after 5 warm-up steps)."""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import engine, synthetic  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.engine import RiskParams  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s, e = synthetic.obstacle_batch(10, 20, 1000, dev, seed=1)
    p = RiskParams()
    hip = ctypes.CDLL("libamdhip64.so")
    K = 20
    # torch graph
    tg = torch.cuda.CUDAGraph()
    with torch.cuda.graph(tg, stream=torch.cuda.Stream(dev)):
        lt, out = engine.prepare_safe_halfspaces(s, e, p, stream=torch.cuda.current_stream(dev))
        for _ in range(K):
            lt()
    tg.replay()
    # raw HIP graph on a stream of our own
    st = torch.cuda.Stream(dev)
    lr, _ = engine.prepare_safe_halfspaces(s, e, p, out=out, stream=st)
    h = ctypes.c_void_p(st.cuda_stream)
    assert hip.hipStreamBeginCapture(h, 0) == 0
    for _ in range(K):
        lr()
    graph, gexec = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipStreamEndCapture(h, ctypes.byref(graph)) == 0
    assert hip.hipGraphInstantiate(ctypes.byref(gexec), graph, None, None, ctypes.c_size_t(0)) == 0
    launch = hip.hipGraphLaunch
    launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    assert launch(gexec, h) == 0
    torch.cuda.synchronize()

    def region(kind):
        warm = tg.replay if kind == "torch" else (lambda: launch(gexec, h))
        stream = torch.cuda.current_stream(dev) if kind == "torch" else st
        warm()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e1.record(stream)
        e0.record(stream)
        t0 = time.perf_counter()
        if kind == "torch":
            tg.replay()
        else:
            launch(gexec, h)
        t1 = time.perf_counter()
        e1.record(stream)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        return (t1 - t0) * 1e6, (t2 - t0) / K * 1e6, e0.elapsed_time(e1) * 1e3 / K

    res = {"torch": [], "raw": []}
    for _ in range(15):
        for kind in res:
            res[kind].append(region(kind))
    for kind, v in res.items():
        med = [sorted(x[i] for x in v)[len(v) // 2] for i in range(3)]
        print(f"{kind:6s} launch call {med[0]:6.2f} us   region wall {med[1]:6.3f} us/step   events {med[2]:6.3f} us/step")


if __name__ == "__main__":
    main()

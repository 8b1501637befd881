"""Diagnostic: a clustered QP launch (C5-shaped problem, 2 problems) eager and replayed from a
hipGraph; prints the info rows and the problems' arrival counters after each run."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))

from test_mpc_cluster import _batch  # noqa: E402
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core import mpc_filter as mf  # noqa: E402

dev = torch.device("cuda", 0)
probs = _batch("double", 50, 256, 2, True, seed=9)
p0 = probs[0]
model = mf.MPCModel(p0["A"], p0["B"], p0["C"], p0["Q"], p0["R"], p0["H"], p0["ub"], p0["pb"], device=dev)
T_ = lambda a: torch.as_tensor(np.ascontiguousarray(a)).to(dev)
hs = T_(np.stack([p["hs"] for p in probs]))
args = (model, hs[..., 0:2], hs[..., 2], T_(np.stack([p["x0"] for p in probs])),
        T_(np.stack([p["x_ref"] for p in probs])), T_(np.stack([p["u_ref"] for p in probs])))
ws = torch.empty(model.workspace_doubles(2, hs.shape[1]), dtype=torch.float64, device=dev)
print("groups", model.launch_groups(2, hs.shape[1]), "ws", ws.numel(), flush=True)
ctr = lambda: [int(v) for v in ws[:32].view(torch.int64)[[0, 16]].cpu()]
x, u, info = mf.filter_batch(*args, workspace=ws)
torch.cuda.synchronize()
print("eager info", info[:, :4].cpu().numpy().tolist(), "ctr", ctr(), flush=True)
mode = sys.argv[1] if len(sys.argv) > 1 else "plain"
g = torch.cuda.CUDAGraph()
side = torch.cuda.Stream(dev)
side.wait_stream(torch.cuda.current_stream(dev))
with torch.cuda.stream(side):
    mf.filter_batch(*args, workspace=ws)
torch.cuda.current_stream(dev).wait_stream(side)
torch.cuda.synchronize()
print("side info ctr", ctr(), flush=True)
with torch.cuda.graph(g):
    if mode == "zero":
        ws[:32].zero_()
    out = mf.filter_batch(*args, workspace=ws)
torch.cuda.synchronize()
print("after capture ctr", ctr(), flush=True)
for r in range(5):
    if mode == "eagerzero":
        ws[:32].zero_()
        torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    print("replay", r, "info", out[2][:, :4].cpu().numpy().tolist(), "ctr", ctr(),
          "same_u", bool(torch.equal(out[1], u)), flush=True)

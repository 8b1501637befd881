"""``core/halfspaces.py`` surface backed by the HIP engine.

Reference: ``SafeHalfspace`` (:11-64), ``MeanSafeHalfspace.create`` (:70-106),
``CVaRSafeHalfspace.create`` (:112-149), ``DRCVaRSafeHalfspace.create`` (:155-194),
``compute_safe_halfspaces`` (:196-248).

``compute_safe_halfspaces`` keeps its signature and its ``{'mean','cvar','dr_cvar'}`` dict of
per-obstacle ``SafeHalfspace`` lists, but all obstacles are evaluated by ONE kernel launch (one
per distinct sample count when the obstacles are ragged) instead of 2 LP solves per obstacle.
``compute_safe_halfspaces_batched`` is the device-tensor form the simulation layer uses: a whole
``[O, T, N, 2]`` horizon in one launch.
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import numpy as np
import torch

from .. import _native, engine
from ..engine import RiskParams
from . import risk_metrics
from .geometry import compute_separating_vector
from .risk_metrics import cvar_halfspace, dr_cvar_halfspace


class SafeHalfspace:
    """Halfspace ``{y | h.y + g <= 0}`` (:11-64)."""

    def __init__(self, h, g_tilde):
        self.h = h
        self.g_tilde = g_tilde
        self.info = None

    def is_point_safe(self, point):
        return np.dot(self.h, point) + self.g_tilde <= 0

    def distance_to_boundary(self, point):
        h_norm = self.h / np.linalg.norm(self.h)
        return np.dot(h_norm, point) + self.g_tilde / np.linalg.norm(self.h)

    def get_constraint_params(self):
        return self.h, self.g_tilde


_ZERO_INFO = {"setup_time": 0, "solve_time": 0, "solve_call_time": 0}


def _unit_record(samples, ego_ref_pos, params: RiskParams):
    """One unit through the batched kernel; returns the 8-column record and timing info."""
    t0 = time.time()
    dev = risk_metrics.device()
    s = torch.as_tensor(np.ascontiguousarray(samples, dtype=np.float64)).to(dev).reshape(1, 1, -1, 2)
    ego = torch.as_tensor(np.asarray(ego_ref_pos, dtype=np.float64).reshape(1, 2)).to(dev)
    t1 = time.time()
    rec = engine.safe_halfspaces(s, ego, params)[0, 0].cpu().numpy()
    t2 = time.time()
    return rec, {"setup_time": t1 - t0, "solve_time": t2 - t1, "solve_call_time": t2 - t0}


class MeanSafeHalfspace(SafeHalfspace):
    @staticmethod
    def create(samples, robot_radius, obstacle_radius):
        """Mean-position halfspace; direction from the ORIGIN (:70-106)."""
        rec, _ = _unit_record(samples, np.zeros(2), RiskParams(robot_radius, obstacle_radius))
        hs = MeanSafeHalfspace(rec[0:2].copy(), float(rec[2]))
        hs.info = dict(_ZERO_INFO)
        return hs


class CVaRSafeHalfspace(SafeHalfspace):
    @staticmethod
    def create(samples, ego_ref_pos, alpha, delta, robot_radius, obstacle_radius):
        """CVaR halfspace (:112-149): ``h`` from ego to the sample mean, ``g`` from the CVaR LP."""
        h = compute_separating_vector(ego_ref_pos, np.mean(samples, axis=0))
        g_value = cvar_halfspace(samples, h, alpha, delta, robot_radius, obstacle_radius)
        hs = CVaRSafeHalfspace(h, g_value)
        hs.info = _read_timing("cvar")
        return hs


class DRCVaRSafeHalfspace(SafeHalfspace):
    @staticmethod
    def create(samples, ego_ref_pos, alpha, delta, epsilon, robot_radius, obstacle_radius):
        """DR-CVaR halfspace (:155-194); stores ``g_tilde = g* - R_c|h|``."""
        h = compute_separating_vector(ego_ref_pos, np.mean(samples, axis=0))
        _g_star, g_tilde = dr_cvar_halfspace(samples, h, alpha, delta, epsilon, robot_radius,
                                             obstacle_radius)
        hs = DRCVaRSafeHalfspace(h, g_tilde)
        hs.info = _read_timing("drcvar")
        return hs


def _read_timing(key):
    import json
    try:
        with open(f"tmp/timing_info_{key}.json") as f:
            return json.load(f)
    except Exception:
        return None


@dataclass
class HalfspaceBatch:
    """All halfspaces of an ``[O, T]`` grid of units: ``record`` is the [O, T, 8] device tensor."""

    record: torch.Tensor
    setup_time: float = 0.0
    solve_time: float = 0.0

    @property
    def mean(self):
        return self.record[..., 0:2], self.record[..., 2]

    @property
    def cvar(self):
        return self.record[..., 3:5], self.record[..., 5]

    @property
    def dr_cvar(self):
        return self.record[..., 3:5], self.record[..., 7]

    def to_lists(self):
        """``{'mean','cvar','dr_cvar'}`` -> ``[T][O]`` lists of SafeHalfspace objects, the layout of
        ``compute_safe_halfspaces_for_trajectory`` (simulation/environment.py:75-104)."""
        rec = self.record.detach().cpu().numpy()
        O, T = rec.shape[:2]
        per = max(O * T, 1)
        info = {"setup_time": self.setup_time / per, "solve_time": self.solve_time / per,
                "solve_call_time": (self.setup_time + self.solve_time) / per}
        out = {"mean": [], "cvar": [], "dr_cvar": []}
        for t in range(T):
            ms, cs, ds = [], [], []
            for o in range(O):
                r = rec[o, t]
                m = MeanSafeHalfspace(r[0:2].copy(), float(r[2]))
                m.info = dict(_ZERO_INFO)
                c = CVaRSafeHalfspace(r[3:5].copy(), float(r[5]))
                c.info = dict(info)
                d = DRCVaRSafeHalfspace(r[3:5].copy(), float(r[7]))
                d.info = dict(info)
                ms.append(m)
                cs.append(c)
                ds.append(d)
            out["mean"].append(ms)
            out["cvar"].append(cs)
            out["dr_cvar"].append(ds)
        return out


def launch_with_singletons(launch, keys, shape, robot_radius, obstacle_radius):
    """Records of a grid of units whose CVaR / DR-CVaR parameters come from the reference's
    N-keyed optimiser singletons (``risk_metrics.plan_singletons``).

    ``launch(params) -> [*shape, 8]`` evaluates the whole grid with one parameter set; ``keys``
    lists ``((a_c, d_c), (a_d, d_d, e_d))`` per unit in row-major order of ``shape``.  Every
    column but ``g_cvar`` comes from the unit's DR-CVaR parameters (the directions and the mean
    halfspace do not depend on them), ``g_cvar`` from its CVaR parameters.  The usual case — one
    parameter set for the whole grid, CVaR equal to DR — is ONE launch; each further distinct
    set costs one more launch of the grid, and the rows are picked by one gather per column group
    (each unit mapped once to the index of its parameter set).
    """
    index: dict = {}
    dr_idx = np.empty(len(keys), dtype=np.int64)
    cv_idx = np.empty(len(keys), dtype=np.int64)
    for u, (ck, dk) in enumerate(keys):
        dr_idx[u] = index.setdefault(dk, len(index))
        cv_idx[u] = index.setdefault((ck[0], ck[1], dk[2]), len(index))
    needed = [RiskParams(robot_radius, obstacle_radius, *k) for k in index]
    recs = [launch(p) for p in needed]
    if len(needed) == 1:
        return recs[0]
    flat = torch.stack([r.reshape(-1, engine.OUT_WIDTH) for r in recs])   # [P, U, 8]
    dev = flat.device
    units = torch.arange(flat.shape[1], device=dev)
    out = flat[torch.as_tensor(dr_idx, device=dev), units]                 # whole rows: DR params
    out[:, _native.COL_G_CVAR] = flat[torch.as_tensor(cv_idx, device=dev), units, _native.COL_G_CVAR]
    return out.view(recs[0].shape)


def compute_safe_halfspaces_batched(samples, ego, robot_radius, obstacle_radius, alpha, delta,
                                    epsilon, stream=None) -> HalfspaceBatch:
    """Every (obstacle, step) unit of ``samples`` [O, T, N, 2] against ``ego`` [T, 2] in one launch.

    Accepts device tensors (no copy) or host arrays (staged to the current HIP device).  A build
    API (the reference has no batched call): the parameters given are the parameters used — the
    optimiser singletons are neither read nor changed.
    """
    params = RiskParams(robot_radius, obstacle_radius, alpha, delta, epsilon)
    t0 = time.time()
    dev = risk_metrics.device()
    if not (isinstance(samples, torch.Tensor) and samples.device.type == "cuda"):
        samples = torch.as_tensor(np.ascontiguousarray(samples, dtype=np.float64)).to(dev)
    if not (isinstance(ego, torch.Tensor) and ego.device.type == "cuda"):
        ego = torch.as_tensor(np.ascontiguousarray(ego, dtype=np.float64)).to(samples.device)
    t1 = time.time()
    rec = engine.safe_halfspaces(samples, ego, params, stream=stream)
    return HalfspaceBatch(rec, setup_time=t1 - t0, solve_time=0.0)


def compute_safe_halfspaces(obstacle_samples, ego_ref_pos, robot_radius, obstacle_radius, alpha,
                            delta, epsilon):
    """Safe halfspaces for a list of per-obstacle sample arrays ``[N_i, 2]`` (:196-248).

    Returns ``{'mean': [...], 'cvar': [...], 'dr_cvar': [...]}`` with one SafeHalfspace per
    obstacle, in input order.  Obstacles with equal N share one kernel launch.  Like the
    reference (which reaches its LPs through ``cvar_halfspace`` / ``dr_cvar_halfspace``), each
    obstacle is solved with the parameters of the optimiser singleton for its N
    (``risk_metrics.singleton_params``), and the singletons are left as the reference leaves them.
    ``.info`` of every CVaR / DR-CVaR object is this call's staging / kernel time divided evenly
    over the obstacles (the reference's is the JSON of that obstacle's own last LP solve).
    """
    RiskParams(robot_radius, obstacle_radius, alpha, delta, epsilon).validate()
    n_obstacles = len(obstacle_samples)
    result = {"mean": [None] * n_obstacles, "cvar": [None] * n_obstacles,
              "dr_cvar": [None] * n_obstacles}
    if n_obstacles == 0:
        return {"mean": [], "cvar": [], "dr_cvar": []}
    t0 = time.time()
    dev = risk_metrics.device()
    counts = [int(np.shape(s)[0]) for s in obstacle_samples]
    keys, final = risk_metrics.plan_singletons(counts, alpha, delta, epsilon)
    groups: dict[int, list[int]] = {}
    for i, n in enumerate(counts):
        groups.setdefault(n, []).append(i)
    ego = torch.as_tensor(np.asarray(ego_ref_pos, dtype=np.float64).reshape(1, 2)).to(dev)
    staged = []
    for n, idx in groups.items():
        host = np.stack([np.asarray(obstacle_samples[i], dtype=np.float64) for i in idx])
        staged.append((idx, torch.as_tensor(host).to(dev).reshape(len(idx), 1, n, 2)))
    t1 = time.time()
    recs = [(idx, launch_with_singletons(lambda p, s=s: engine.safe_halfspaces(s, ego, p),
                                         [keys[i] for i in idx], (len(idx), 1),
                                         robot_radius, obstacle_radius))
            for idx, s in staged]
    host_recs = [(idx, r.cpu().numpy()) for idx, r in recs]
    t2 = time.time()
    risk_metrics.commit_singletons(final)  # only once every launch has succeeded
    per = {"setup_time": (t1 - t0) / n_obstacles, "solve_time": (t2 - t1) / n_obstacles}
    per["solve_call_time"] = per["setup_time"] + per["solve_time"]
    for idx, rec in host_recs:
        for j, i in enumerate(idx):
            r = rec[j, 0]
            m = MeanSafeHalfspace(r[0:2].copy(), float(r[2]))
            m.info = dict(_ZERO_INFO)
            c = CVaRSafeHalfspace(r[3:5].copy(), float(r[5]))
            c.info = dict(per)
            d = DRCVaRSafeHalfspace(r[3:5].copy(), float(r[7]))
            d.info = dict(per)
            result["mean"][i], result["cvar"][i], result["dr_cvar"][i] = m, c, d
    if risk_metrics.WRITE_TIMING_FILES:
        risk_metrics.save_timing_info("cvar", per["setup_time"], per["solve_time"])
        risk_metrics.save_timing_info("drcvar", per["setup_time"], per["solve_time"])
    return result

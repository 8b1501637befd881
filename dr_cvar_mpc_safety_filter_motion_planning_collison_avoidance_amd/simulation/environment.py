"""``simulation/environment.py`` — the caller that feeds the hot path, batched.

Reference ``SafetyFilteringEnvironment.compute_safe_halfspaces_for_trajectory``
(``simulation/environment.py:60-106``) loops over the horizon and, per step, over the obstacles,
solving two LPs per (obstacle, step).  Here the whole horizon of every obstacle is ONE kernel
launch: the per-obstacle ``[N, S+1, 2]`` sample trajectories are staged to the device once and
handed to the kernel with their native strides (sample stride ``(S+1)*2``, step stride 2), so no
transpose is made; obstacles with different N are grouped, one launch per distinct N.
The return value keeps the reference's ``{'mean','cvar','dr_cvar'}`` -> ``[T][O]`` layout.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from .. import engine
from ..core import risk_metrics
from ..core import halfspaces as hs_mod
from ..core.halfspaces import HalfspaceBatch
from ..engine import RiskParams


def create_double_integrator_matrices(dt, dim=2):
    """``core/dynamics.py:7-33`` (only ``C`` touches the hot path: environment.py:92)."""
    A = np.block([[np.eye(dim), dt * np.eye(dim)], [np.zeros((dim, dim)), np.eye(dim)]])
    B = np.block([[0.5 * dt ** 2 * np.eye(dim)], [dt * np.eye(dim)]])
    C = np.block([np.eye(dim), np.zeros((dim, dim))])
    return A, B, C


class SafetyFilteringEnvironment:
    def __init__(self, ROBOT_RADIUS, OBSTACLE_RADIUS, HORIZON, DT, ALPHA, DELTA, EPSILON):
        self.ROBOT_RADIUS = ROBOT_RADIUS
        self.OBSTACLE_RADIUS = OBSTACLE_RADIUS
        self.HORIZON = HORIZON
        self.DT = DT
        self.ALPHA = ALPHA
        self.DELTA = DELTA
        self.EPSILON = EPSILON
        self.A, self.B, self.C = create_double_integrator_matrices(DT)
        self.n_states = self.A.shape[0]
        self.n_inputs = self.B.shape[1]
        self.n_outputs = self.C.shape[0]
        self.state_bounds = None
        self.input_bounds = None

    @property
    def params(self) -> RiskParams:
        return RiskParams(self.ROBOT_RADIUS, self.OBSTACLE_RADIUS, self.ALPHA, self.DELTA,
                          self.EPSILON)

    def set_bounds(self, state_bounds=None, input_bounds=None):
        self.state_bounds = state_bounds
        self.input_bounds = input_bounds

    def compute_halfspace_batch(self, obstacle_sample_trajectories, ego_ref_trajectory):
        """Device-side result: a HalfspaceBatch whose record is [O, T, 8] (T = min(len(ref), H)).

        Each unit is solved with the parameters of the reference's optimiser singleton for its N
        (``risk_metrics.plan_singletons`` over the reference's call order: steps outer,
        obstacles inner), so a previous call with the same N but other alpha/delta/epsilon
        carries over exactly as in the reference; usually that is one launch per distinct N.
        """
        n_obstacles = len(obstacle_sample_trajectories)
        n_steps = min(len(ego_ref_trajectory), self.HORIZON)               # environment.py:72
        self.params.validate()
        t0 = time.time()
        dev = risk_metrics.device()
        ego = np.asarray(ego_ref_trajectory, dtype=np.float64)[:n_steps] @ self.C.T  # :92
        ego_d = torch.as_tensor(np.ascontiguousarray(ego)).to(dev)
        record = torch.empty((n_obstacles, n_steps, engine.OUT_WIDTH), dtype=torch.float64,
                             device=dev)
        if n_obstacles == 0 or n_steps == 0:
            return HalfspaceBatch(record)
        counts = [int(np.shape(tr)[0]) for tr in obstacle_sample_trajectories]
        keys, final = risk_metrics.plan_singletons([counts[o] for _ in range(n_steps)
                                                    for o in range(n_obstacles)],
                                                   self.ALPHA, self.DELTA, self.EPSILON)
        groups: dict[int, list[int]] = {}
        for i, n in enumerate(counts):
            groups.setdefault(n, []).append(i)
        launches = []
        for n, idx in groups.items():
            # [G, N, n_steps, 2] slice of the reference layout, staged as-is (environment.py:88)
            host = np.stack([np.asarray(obstacle_sample_trajectories[i], dtype=np.float64)[:, :n_steps, :]
                             for i in idx])
            # one pinned staging buffer (cached, grown on demand), asynchronous H2D; the kernel
            # reads the reference's [G, N, T, 2] order through strides (no transpose pass)
            stage = self._pinned_stage(host.size).view(-1)[:host.size].view(host.shape)
            stage.copy_(torch.from_numpy(host))
            dev_s = stage.to(dev, non_blocking=True)
            self._stage_event = torch.cuda.Event()
            self._stage_event.record()
            view = dev_s.permute(0, 2, 1, 3)                                  # [G, T, N, 2] strided
            # unit (g, t) is call t * O + o of the reference's loop
            gkeys = [keys[t * n_obstacles + o] for o in idx for t in range(n_steps)]
            launches.append((idx, view, gkeys))
        t1 = time.time()
        params = self.params
        for idx, view, gkeys in launches:
            out = hs_mod.launch_with_singletons(
                lambda p, v=view: engine.safe_halfspaces(v, ego_d, p), gkeys,
                (len(idx), n_steps), params.robot_radius, params.obstacle_radius)
            if len(idx) == n_obstacles:
                record = out
            else:
                record[torch.as_tensor(idx, device=dev)] = out
        risk_metrics.commit_singletons(final)  # only once every launch was accepted
        return HalfspaceBatch(record, setup_time=t1 - t0)

    def _pinned_stage(self, n_doubles):
        """The cached pinned host buffer the trajectories are staged through (one allocation for
        the environment's lifetime unless a larger batch arrives).  Before it is refilled, the
        previous asynchronous copy out of it must have finished."""
        ev = getattr(self, "_stage_event", None)
        if ev is not None:
            ev.synchronize()
        buf = getattr(self, "_stage_buf", None)
        if buf is None or buf.numel() < n_doubles:
            buf = torch.empty(int(n_doubles), dtype=torch.float64).pin_memory()
            self._stage_buf = buf
        return buf

    def compute_safe_halfspaces_for_trajectory(self, obstacle_sample_trajectories,
                                               ego_ref_trajectory):
        """Reference layout: ``{'mean','cvar','dr_cvar'}`` -> ``[T][O]`` SafeHalfspace lists."""
        batch = self.compute_halfspace_batch(obstacle_sample_trajectories, ego_ref_trajectory)
        t1 = time.time()
        torch.cuda.synchronize()
        batch.solve_time = time.time() - t1
        return batch.to_lists()

    def compute_distance_to_collision(self, ego_trajectory, obstacle_trajectories):
        """Per-step minimum clearance (environment.py:108-140)."""
        n_steps = min(len(ego_trajectory), len(obstacle_trajectories[0]))
        distances = np.inf * np.ones(n_steps)
        for t in range(n_steps):
            ego_pos_t = self.C @ ego_trajectory[t]
            for obs in obstacle_trajectories:
                dist = np.linalg.norm(ego_pos_t - obs[t]) - self.ROBOT_RADIUS - self.OBSTACLE_RADIUS
                distances[t] = min(distances[t], dist)
        return distances

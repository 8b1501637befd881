"""Synthetic obstacle-sample workloads generated on the device (no host staging).

Shapes and distributions follow SURVEY.md §8d, i.e. the reference's own scenario generator:
obstacle o moves on a straight line from a start ~ U[-5, 5]^2 with heading ~ U[0, 2 pi) and speed
~ U[0.6, 1.5] m/s at DT = 0.2 s (``simulation/obstacles.py:7-41``, speeds as in
``config/scenarios.py:36-62``); the N samples at step t are the nominal position plus
N(0, diag(0.01, 0.01)) noise (``simulation/obstacles.py:62-74``, cov at :134), noise-free at t = 0
(:63).  The ego follows the straight line (-4, 0) -> (4, 0) at 1.5 m/s
(``simulation/planner.py:120-197``).  Output is the packed ``[O, T, N, 2]`` float64 layout the
kernel streams at full coalescing, and ego ``[T, 2]``.  The samples are drawn by the device
sampler (``drcvar_sample_trajectories_f64``, Philox4x32-10), so nothing is staged from the host.
"""
from __future__ import annotations

import math

import torch

from .simulation.obstacles import sample_trajectories_device

DT = 0.2
NOISE_STD = 0.1  # sqrt(0.01)


def straight_line_ego(n_steps: int, device, start=(-4.0, 0.0), goal=(4.0, 0.0), velocity=1.5,
                      dt: float = DT) -> torch.Tensor:
    """Ego positions of ``ReferenceTrajectoryPlanner.straight_line_trajectory`` for t < n_steps."""
    start_t = torch.tensor(start, dtype=torch.float64)
    goal_t = torch.tensor(goal, dtype=torch.float64)
    dist = float(torch.linalg.norm(goal_t - start_t))
    ego = start_t.repeat(n_steps, 1)
    if dist >= 1e-10:
        n_move = int((dist / velocity) / dt)
        for t in range(1, n_steps):
            ego[t] = start_t + (t / n_move) * (goal_t - start_t) if t <= n_move else goal_t
    return ego.to(device)


def nominal_paths(n_obstacles: int, n_steps: int, device, seed: int = 42) -> torch.Tensor:
    """Nominal obstacle positions ``[O, T, 2]`` f64 on ``device`` (deterministic for a seed): start
    ~ U[-5, 5]^2, heading ~ U[0, 2 pi), speed ~ U[0.6, 1.5] m/s, straight lines at DT."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    f64 = dict(dtype=torch.float64, device=device)
    start = (torch.rand((n_obstacles, 2), generator=g, **f64) * 10.0) - 5.0
    heading = torch.rand((n_obstacles,), generator=g, **f64) * (2.0 * math.pi)
    speed = 0.6 + torch.rand((n_obstacles,), generator=g, **f64) * 0.9
    vel = torch.stack([torch.cos(heading), torch.sin(heading)], dim=1) * speed[:, None]
    t = torch.arange(n_steps, **f64) * DT
    return (start[:, None, :] + t[None, :, None] * vel[:, None, :]).contiguous()


NOISE_COV = [[NOISE_STD ** 2, 0.0], [0.0, NOISE_STD ** 2]]


def obstacle_batch(n_obstacles: int, n_steps: int, n_samples: int, device, seed: int = 42):
    """(samples [O, T, N, 2] f64, ego [T, 2] f64) on ``device``, deterministic for a seed."""
    nominal = nominal_paths(n_obstacles, n_steps, device, seed)
    samples = sample_trajectories_device(nominal, n_samples, NOISE_COV, seed=seed,
                                         zero_first_step=True)                       # obstacles.py:63
    return samples, straight_line_ego(n_steps, device)

"""``simulation/obstacles.py`` — obstacle trajectories feeding the hot path, host and device.

Reference: ``generate_nominal_trajectory`` (:7-41), ``generate_obstacle_sample_trajectories``
(:43-77), ``generate_laplace_realization`` (:79-113), ``generate_obstacle_scenarios`` (:115-197).

Two paths:

* host (NumPy) — the reference's RNG stream exactly: the same ``np.random`` calls in the same order
  (multivariate normal per step, two exponential draws per realisation step), the nominal path by
  the same single-integrator recurrence ``p_{t+1} = p_t + dt v``.  Seeded runs reproduce the
  reference bit for bit (checked against the golden vectors); this is the parity path.
* device (``drcvar_sample_trajectories_f64``, ``include/drcvar_sampling.h``) — the same
  distribution drawn by Philox4x32-10 in HBM, directly in the engine's ``[O, T, N, 2]`` layout, so
  a GPU pipeline never stages Monte Carlo samples through the host.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from .. import _native

NOISE_COV = np.diag([0.01, 0.01])     # simulation/obstacles.py:134


def generate_nominal_trajectory(start_pos, direction, speed, n_steps, dt):
    """Constant-velocity path ``[n_steps + 1, dim]`` (:7-41); stationary if |direction| < 1e-10."""
    start_pos = np.asarray(start_pos, dtype=np.float64)
    direction = np.asarray(direction, dtype=np.float64)
    norm = np.linalg.norm(direction)
    if norm < 1e-10:
        return np.tile(start_pos, (n_steps + 1, 1))
    velocity = speed * (direction / norm)
    step = dt * velocity                      # B u of the single integrator (B = dt I)
    path = np.empty((n_steps + 1, start_pos.shape[0]))
    path[0] = start_pos
    for t in range(n_steps):
        path[t + 1] = path[t] + step
    return path


def generate_obstacle_sample_trajectories(nominal_trajectory, n_samples, noise_cov, dt=None):
    """``[n_samples, n_steps + 1, dim]``: nominal + N(0, noise_cov) per step, step 0 exact (:43-77)."""
    n_steps = nominal_trajectory.shape[0] - 1
    dim = nominal_trajectory.shape[1]
    out = np.zeros((n_samples, n_steps + 1, dim))
    out[:, 0, :] = nominal_trajectory[0, :]
    for t in range(1, n_steps + 1):
        noise = np.random.multivariate_normal(mean=np.zeros(dim), cov=noise_cov, size=n_samples)
        out[:, t, :] = nominal_trajectory[t, :] + noise
    return out


def generate_laplace_realization(nominal_trajectory, noise_cov, dt=None):
    """One Laplace-noise realisation (difference of two Exp(1) draws, scale sqrt(var/2)) (:79-113)."""
    n_steps = nominal_trajectory.shape[0] - 1
    dim = nominal_trajectory.shape[1]
    out = np.zeros_like(nominal_trajectory)
    out[0, :] = nominal_trajectory[0, :]
    scale = np.sqrt(np.diag(noise_cov) / 2)
    for t in range(1, n_steps + 1):
        e1 = np.random.exponential(scale=1.0, size=dim)
        e2 = np.random.exponential(scale=1.0, size=dim)
        out[t, :] = nominal_trajectory[t, :] + scale * (e1 - e2)
    return out


def _obstacle_specs(scenario_config):
    if "obstacles" in scenario_config:
        return [(ob["start"], ob["direction"], ob.get("speed", 1.0))
                for ob in scenario_config["obstacles"]]
    return [(scenario_config["obstacle_start"], scenario_config["obstacle_direction"],
             scenario_config.get("obstacle_speed", 1.0))]


def generate_obstacle_scenarios(scenario_config, horizon, dt, n_samples=100):
    """Nominal, sample and realisation trajectories of every obstacle (:115-197), host RNG."""
    n_steps = int(horizon / dt)
    nominal, samples, realizations = [], [], []
    for start, direction, speed in _obstacle_specs(scenario_config):
        nom = generate_nominal_trajectory(start, direction, speed, n_steps, dt)
        nominal.append(nom)
        samples.append(generate_obstacle_sample_trajectories(nom, n_samples, NOISE_COV, dt))
        realizations.append(generate_laplace_realization(nom, NOISE_COV, dt))
    return {"nominal_trajectories": nominal, "sample_trajectories": samples,
            "realization_trajectories": realizations}


# ------------------------------------------------------------------------------------ device

def sample_trajectories_device(nominal, n_samples, noise_cov=NOISE_COV, seed=0, stream_offset=0,
                               zero_first_step=True, out=None, stream=None):
    """Device samples ``[O, T, N, 2]`` float64 around ``nominal`` ``[O, T, 2]`` (device tensor).

    One ``drcvar_sample_trajectories_f64`` launch; ``out`` may be any float64 view with adjacent
    coordinates (e.g. a slice of a larger batch).  Deterministic in (seed, stream_offset).
    """
    if not isinstance(nominal, torch.Tensor) or nominal.device.type != "cuda":
        raise ValueError("nominal must be a device tensor (the sampler has no CPU path)")
    if nominal.dtype != torch.float64 or nominal.dim() != 3 or nominal.shape[2] != 2 or \
            nominal.stride(2) != 1:
        raise ValueError("nominal must be float64 [O, T, 2] with adjacent coordinates")
    O, T, _ = nominal.shape
    cov = np.asarray(noise_cov, dtype=np.float64).reshape(2, 2)
    L = np.linalg.cholesky(cov)
    if out is None:
        out = torch.empty((O, T, int(n_samples), 2), dtype=torch.float64, device=nominal.device)
    elif tuple(out.shape) != (O, T, int(n_samples), 2) or out.dtype != torch.float64 or \
            out.stride(3) != 1 or out.device != nominal.device:
        raise ValueError("out must be a float64 [O, T, N, 2] device view with adjacent coordinates")
    s = stream if stream is not None else torch.cuda.current_stream(nominal.device)
    _native.check(_native.lib().drcvar_sample_trajectories_f64(
        ctypes.c_void_p(nominal.data_ptr()), O, T, nominal.stride(0), nominal.stride(1),
        int(n_samples), float(L[0, 0]), float(L[1, 0]), float(L[1, 1]),
        ctypes.c_uint64(int(seed) & (2 ** 64 - 1)), ctypes.c_uint64(int(stream_offset) & (2 ** 64 - 1)),
        1 if zero_first_step else 0, ctypes.c_void_p(out.data_ptr()), out.stride(0), out.stride(1),
        out.stride(2), ctypes.c_void_p(int(s.cuda_stream))))
    return out


def sample_units_device(nominal, n_samples, unit_begin, unit_count, noise_cov=NOISE_COV, seed=0,
                        stream_offset=0, zero_first_step=True, out=None, stream=None):
    """Units ``[unit_begin, unit_begin + unit_count)`` of the global batch ``nominal`` ``[O, T, 2]``
    describes, as a flat ``[unit_count, N, 2]`` float64 device tensor (unit ``u = o * T + t``).

    Sample for sample the same values :func:`sample_trajectories_device` draws for the whole batch
    (``drcvar_sample_units_f64``): one rank draws its shard of a global batch and nothing else.
    ``out`` may be any ``[unit_count, N, 2]`` view with adjacent coordinates.
    """
    if not isinstance(nominal, torch.Tensor) or nominal.device.type != "cuda":
        raise ValueError("nominal must be a device tensor (the sampler has no CPU path)")
    if nominal.dtype != torch.float64 or nominal.dim() != 3 or nominal.shape[2] != 2 or \
            nominal.stride(2) != 1:
        raise ValueError("nominal must be float64 [O, T, 2] with adjacent coordinates")
    O, T, _ = nominal.shape
    unit_begin, unit_count, n_samples = int(unit_begin), int(unit_count), int(n_samples)
    if unit_begin < 0 or unit_count < 0 or unit_begin + unit_count > O * T:
        raise ValueError(f"unit range [{unit_begin}, {unit_begin + unit_count}) outside the "
                         f"{O} x {T} batch")
    L = np.linalg.cholesky(np.asarray(noise_cov, dtype=np.float64).reshape(2, 2))
    if out is None:
        out = torch.empty((unit_count, n_samples, 2), dtype=torch.float64, device=nominal.device)
    elif tuple(out.shape) != (unit_count, n_samples, 2) or out.dtype != torch.float64 or \
            out.stride(2) != 1 or out.device != nominal.device:
        raise ValueError("out must be a float64 [units, N, 2] device view with adjacent coordinates")
    s = stream if stream is not None else torch.cuda.current_stream(nominal.device)
    _native.check(_native.lib().drcvar_sample_units_f64(
        ctypes.c_void_p(nominal.data_ptr()), O, T, nominal.stride(0), nominal.stride(1),
        unit_begin, unit_count, n_samples, float(L[0, 0]), float(L[1, 0]), float(L[1, 1]),
        ctypes.c_uint64(int(seed) & (2 ** 64 - 1)), ctypes.c_uint64(int(stream_offset) & (2 ** 64 - 1)),
        1 if zero_first_step else 0, ctypes.c_void_p(out.data_ptr()), out.stride(0), out.stride(1),
        ctypes.c_void_p(int(s.cuda_stream))))
    return out


def generate_obstacle_scenarios_device(scenario_config, horizon, dt, n_samples=100, seed=0,
                                       device=None):
    """``generate_obstacle_scenarios`` with the samples drawn on the device.

    Returns the reference's dict, except ``sample_trajectories`` is ONE device tensor
    ``[O, n_steps + 1, N, 2]`` (the engine layout) instead of a list of ``[N, n_steps + 1, 2]``
    arrays; nominal paths and the (tiny) Laplace realisations stay on the host.
    """
    from ..core import risk_metrics
    dev = torch.device(device) if device is not None else risk_metrics.device()
    n_steps = int(horizon / dt)
    nominal, realizations = [], []
    for start, direction, speed in _obstacle_specs(scenario_config):
        nom = generate_nominal_trajectory(start, direction, speed, n_steps, dt)
        nominal.append(nom)
        realizations.append(generate_laplace_realization(nom, NOISE_COV, dt))
    nom_d = torch.as_tensor(np.stack(nominal)).to(dev)
    samples = sample_trajectories_device(nom_d, n_samples, NOISE_COV, seed=seed)
    return {"nominal_trajectories": nominal, "sample_trajectories": samples,
            "realization_trajectories": realizations}


def pack_sample_trajectories(sample_trajectories, n_steps, device, pin=True):
    """Reference layout (list of ``[N, S+1, 2]``, equal N) -> device ``[O, n_steps, N, 2]`` packed.

    The per-obstacle arrays are staged once through pinned host memory and copied asynchronously;
    the transpose to the engine's packed layout happens on the device.
    """
    host = np.stack([np.asarray(tr, dtype=np.float64)[:, :n_steps, :] for tr in sample_trajectories])
    staged = torch.from_numpy(np.ascontiguousarray(host))
    if pin:
        staged = staged.pin_memory()
    dev_t = staged.to(device, non_blocking=pin)                  # [O, N, T, 2]
    return dev_t.permute(0, 2, 1, 3).contiguous()                 # [O, T, N, 2]

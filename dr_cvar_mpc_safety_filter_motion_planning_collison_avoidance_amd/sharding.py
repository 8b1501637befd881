"""Multi-GPU sharding of the (obstacle x step) unit batch — one process per GPU.

Units are independent (no cross-unit data in ``core/halfspaces.py:225-246`` or
``simulation/environment.py:82-104``), so the batch is split into contiguous blocks of the
flattened unit index ``u = o*T + t`` with no data-path collective.  The only exchange is the one
the consumer needs: the MPC QP (``core/mpc_filter.py:116-144``) takes every halfspace of the
horizon, so :func:`gather_records` reassembles the ``[U, 8]`` records on every rank with ONE
``all_gather_into_tensor`` (RCCL over xGMI when the backend is ``nccl``; gloo in the CPU tests).
Each record is 64 B, so even the largest config (12 800 units, 800 KB) is latency-bound.

``compute`` is injectable so the partition/gather logic can be exercised with world_size 2 on
CPU (gloo) in the tests; the product path always passes the HIP engine.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import engine
from .engine import RiskParams


def shard_bounds(n_units: int, world_size: int, rank: int) -> tuple[int, int]:
    """Contiguous block ``[start, stop)`` of rank ``rank`` (blocks of ceil(U/W); the tail rank may
    get fewer or zero units)."""
    if world_size < 1 or not (0 <= rank < world_size):
        raise ValueError("invalid rank/world_size")
    per = -(-n_units // world_size) if n_units else 0
    start = min(rank * per, n_units)
    return start, min(start + per, n_units)


def shard_units(samples: torch.Tensor, ego: torch.Tensor, world_size: int, rank: int):
    """This rank's units of an [O, T, N, 2] batch, flattened: ``(samples [u, N, 2], ego [u, 2],
    start, stop)``.  Works on any device; no copy of the samples when they are contiguous."""
    O, T, N, _ = samples.shape
    start, stop = shard_bounds(O * T, world_size, rank)
    flat = samples.reshape(O * T, N, 2)
    ego_units = ego.repeat(O, 1)  # unit u -> ego[u % T]
    return flat[start:stop], ego_units[start:stop], start, stop


def engine_compute(samples_u: torch.Tensor, ego_u: torch.Tensor, params: RiskParams) -> torch.Tensor:
    """HIP engine on a flattened shard: [u, N, 2] x [u, 2] -> [u, 8] (one launch)."""
    u = samples_u.shape[0]
    if u == 0:
        return torch.empty((0, engine.OUT_WIDTH), dtype=torch.float64, device=samples_u.device)
    # one obstacle row with u steps, ego per step = ego per unit
    return engine.safe_halfspaces(samples_u.unsqueeze(0), ego_u, params).reshape(u, engine.OUT_WIDTH)


def gather_records(local: torch.Tensor, n_units: int, group=None) -> torch.Tensor:
    """All-gather every rank's ``[u_r, 8]`` block into the full ``[n_units, 8]`` on every rank."""
    world = dist.get_world_size(group)
    per = -(-n_units // world) if n_units else 0
    padded = torch.zeros((per, local.shape[1]), dtype=local.dtype, device=local.device)
    padded[: local.shape[0]] = local
    full = torch.empty((per * world, local.shape[1]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(full, padded, group=group)
    return full[:n_units]


def sharded_safe_halfspaces(samples: torch.Tensor, ego: torch.Tensor, params: RiskParams,
                            group=None, gather: bool = True, compute=engine_compute):
    """Evaluate this rank's share of an [O, T, N, 2] batch; with ``gather`` return the full
    [O, T, 8] record on every rank, else ``(local [u, 8], start, stop)``."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    O, T = samples.shape[:2]
    s_u, e_u, start, stop = shard_units(samples, ego, world, rank)
    local = compute(s_u, e_u, params)
    if not gather:
        return local, start, stop
    return gather_records(local, O * T, group).reshape(O, T, -1)

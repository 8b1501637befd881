"""CPU, world_size 2 over gloo: the multi-GPU partition + all-gather path
(sharding.sharded_safe_halfspaces) reassembles exactly the single-process result.  The per-shard
compute is the C oracle here (test-only injection); on the GPU box it is the HIP engine."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import sharding
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.engine import RiskParams


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_compute(samples, ego, p, out):
    from oracle import c_oracle
    out.copy_(torch.from_numpy(c_oracle.safe_halfspaces(
        samples.contiguous().numpy(), ego.contiguous().numpy(), p.robot_radius, p.obstacle_radius,
        p.alpha, p.delta, p.epsilon)))


def _worker(rank, world, port, O, T, N, strided, q, chunks=1):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(42)
        samples = torch.from_numpy(rng.normal(size=(O, T, N, 2)))
        ego = torch.from_numpy(rng.normal(size=(T, 2)))
        if strided:   # the reference's own [O, N, T, 2] order, consumed through views
            samples = samples.permute(0, 2, 1, 3).contiguous().permute(0, 2, 1, 3)
        full = sharding.sharded_safe_halfspaces(samples, ego, RiskParams(), compute=_oracle_compute,
                                                chunks=chunks)
        local, a, b = sharding.sharded_safe_halfspaces(samples, ego, RiskParams(), gather=False,
                                                       compute=_oracle_compute, chunks=chunks)
        q.put((rank, full.numpy(), a, b, local.shape[0]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("O,T,N,strided,chunks", [(3, 5, 40, False, 1), (1, 3, 17, False, 1),
                                                  (10, 20, 100, False, 1), (3, 5, 40, True, 1),
                                                  (5, 3, 12, True, 1),
                                                  # the pipelined exchange:
                                                  # chunk j's all-gather behind chunk j + 1's compute
                                                  (10, 20, 100, False, 2), (3, 5, 40, True, 3),
                                                  (7, 9, 30, False, 4), (1, 3, 17, False, 4)])
def test_two_rank_gather_matches_single_process(O, T, N, strided, chunks):
    from oracle import c_oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, O, T, N, strided, q, chunks)) for r in range(2)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(42)
    samples = rng.normal(size=(O, T, N, 2))
    ego = rng.normal(size=(T, 2))
    ref = c_oracle.safe_halfspaces(samples, ego, 0.3, 0.3, 0.2, 0.1, 0.15)
    spans = {}
    for rank, full, a, b, n_local in results:
        np.testing.assert_array_equal(full, ref)
        spans[rank] = (a, b)
        assert b - a == n_local
    assert spans[0][0] == 0 and spans[0][1] == spans[1][0] and spans[1][1] == O * T
    assert spans[0][1] % chunks == 0 or spans[0][1] == O * T   # blocks are whole chunks


def test_block_alignment():
    assert sharding.block_units(1920, 8, 1) == 240 and sharding.block_units(1920, 8, 3) == 240
    assert sharding.block_units(15, 2, 4) == 8 and sharding.shard_bounds(15, 2, 1, align=4) == (8, 15)
    assert sharding.shard_bounds(3, 2, 1, align=4) == (3, 3)

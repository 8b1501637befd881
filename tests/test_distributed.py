"""CPU, world sizes 2, 4 and 8 over gloo: the multi-GPU partition + all-gather path
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


# ---- ShardedBatch (the form bench.py times) at world sizes 2, 4 and 8, chunked and not ---------

def _global_batch(O, T, N):
    rng = np.random.default_rng(7)
    nominal = torch.from_numpy(rng.normal(size=(O, T, 2)) * 5)
    samples = nominal[:, :, None, :] + torch.from_numpy(rng.normal(size=(O, T, N, 2)))
    ego = torch.from_numpy(rng.normal(size=(T, 2)))
    return nominal, samples, ego


def _sharded_worker(rank, world, port, O, T, N, chunk_list, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        nominal, whole, ego = _global_batch(O, T, N)
        flat = whole.reshape(O * T, N, 2)

        def sample_fn(nom, n, start, count, cov, seed=0, stream_offset=0, zero_first_step=True):
            return flat[start:start + count].clone()          # this rank's units only

        def prepare_fn(samples, ego_u, p, out=None, stream=None):
            return (lambda: _oracle_compute(samples, ego_u, p, out)), out

        got = {}
        for chunks in chunk_list:
            sb = sharding.ShardedBatch(nominal, ego, N, RiskParams(), world, rank, chunks=chunks,
                                       sample_fn=sample_fn, prepare_fn=prepare_fn)
            for _ in range(2):                                 # repeated steps reuse the buffers
                sb.step()
            got[chunks] = (sb.records().clone().numpy(), sb.start, sb.stop, sb.local_records().numpy().copy())
        # graph-vs-eager agreement (bench.Stepper): one rank's failure makes every rank eager
        votes = (bench.agree(world, None, True), bench.agree(world, None, rank != world - 1))
        q.put((rank, got, votes))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,O,T,N,chunk_list", [
    (2, 3, 5, 40, [1, 2]), (4, 3, 5, 40, [1, 2, 4]),
    (4, 1, 5, 17, [1, 2, 3]),      # U = 5 over 4 ranks: the tail rank(s) hold zero units
    (4, 6, 7, 30, [1, 2]), (2, 1, 1, 9, [1, 2]),
    (8, 4, 6, 30, [1, 2]),         # the driver's largest N: 3 units per rank
    (8, 1, 5, 17, [1, 2]),         # U = 5 over 8 ranks: three ranks with zero units
])
def test_sharded_batch_steps_match_single_process(world, O, T, N, chunk_list):
    """bench.py's strong-scaling step (sharding.ShardedBatch: per-rank draw, the kernel into the
    all-gather input, the exchange — pipelined by chunks or not) at world sizes 2, 4 and 8 over gloo,
    with the C oracle as the shard compute: every rank ends with exactly the single-process
    records, every chunking gives the same bytes, blocks tile [0, U), and a rank with no units
    takes part in every collective; the graph-vs-eager vote is unanimous."""
    from oracle import c_oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, O, T, N, chunk_list, q))
             for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nominal, whole, ego = _global_batch(O, T, N)
    ref = c_oracle.safe_halfspaces(whole.numpy(), ego.numpy(), 0.3, 0.3, 0.2, 0.1, 0.15)
    empty_ranks = 0
    for rank, got, votes in results:
        assert votes == (True, False), (rank, votes)
        for chunks in chunk_list:
            rec, a, b, local = got[chunks]
            np.testing.assert_array_equal(rec, ref)
            np.testing.assert_array_equal(local, ref.reshape(O * T, 8)[a:b])
            empty_ranks += (a == b) and chunks == chunk_list[0]
    for chunks in chunk_list:
        spans = sorted((got[chunks][1], got[chunks][2]) for _, got, _ in results)
        assert spans[0][0] == 0 and spans[-1][1] == O * T
        assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
    if O * T < world * 2:
        assert empty_ranks >= 1

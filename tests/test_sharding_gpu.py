"""GPU: the multi-GPU partition with the real HIP engine (`engine_compute` was only
ever exercised with the C oracle injected).

* every (world, rank) split of a global batch — contiguous and the reference's strided order —
  evaluated through `shard_views` + `engine_compute` reassembles the single-launch result bit for
  bit and matches the C oracle within the north-star tolerance;
* `ShardedBatch` (per-rank device sampling of its units + the kernel writing into the all-gather
  input) gives, rank by rank, exactly the records of the whole batch;
* a world-size-1 RCCL (`nccl`) process group runs `sharded_safe_halfspaces` and
  `ShardedBatch.step` (launch + all_gather_into_tensor), eagerly and captured in a hipGraph.
"""
import os
import socket

import numpy as np
import pytest
import torch

from conftest import OFFSET_TOL
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import engine, sharding, synthetic
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.engine import RiskParams

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def _oracle(samples, ego, p=RiskParams()):
    from oracle import c_oracle
    return c_oracle.safe_halfspaces(np.ascontiguousarray(samples.cpu().numpy()), ego.cpu().numpy(),
                                    p.robot_radius, p.obstacle_radius, p.alpha, p.delta, p.epsilon)


@pytest.mark.parametrize("O,T,N", [(10, 20, 1000), (7, 9, 300), (3, 1, 64)])
@pytest.mark.parametrize("strided", [False, True])
def test_every_rank_split_reassembles_the_batch(dev, O, T, N, strided):
    s, ego = synthetic.obstacle_batch(O, T, N, dev, seed=3)
    if strided:  # the reference's [O, N, T, 2] order, consumed through views
        s = s.permute(0, 2, 1, 3).contiguous().permute(0, 2, 1, 3)
    whole = engine.safe_halfspaces(s, ego, RiskParams()).view(O * T, 8)
    ref = _oracle(s, ego).reshape(O * T, 8)
    for world in (2, 3, 8):
        parts = []
        for r in range(world):
            views, a, b = sharding.shard_views(s, ego, world, r)
            local = torch.full((b - a, 8), float("nan"), dtype=torch.float64, device=dev)
            for sv, ev, off, cnt in views:
                sharding.engine_compute(sv, ev, RiskParams(),
                                        local[off:off + cnt].view(sv.shape[0], sv.shape[1], 8))
            parts.append(local)
        got = torch.cat(parts)
        assert torch.equal(got, whole), world
        assert np.max(np.abs(got.cpu().numpy() - ref)) < OFFSET_TOL


def _nominal(O, T, dev, seed=5):
    return synthetic.nominal_paths(O, T, dev, seed=seed), synthetic.straight_line_ego(T, dev)


@pytest.mark.parametrize("O,T,N", [(10, 20, 1000), (6, 5, 2000), (4, 3, 100)])
def test_sharded_batch_ranks_match_whole_batch(dev, O, T, N):
    nominal, ego = _nominal(O, T, dev)
    whole_s, _ = synthetic.obstacle_batch(O, T, N, dev, seed=5)
    whole = engine.safe_halfspaces(whole_s, ego, RiskParams()).view(O * T, 8)
    for world in (1, 2, 4, 8):
        got = []
        for r in range(world):
            sb = sharding.ShardedBatch(nominal, ego, N, RiskParams(), world, r, seed=5)
            assert torch.equal(sb.samples, whole_s.reshape(O * T, N, 2)[sb.start:sb.stop])
            sb.compute()
            assert sb.send.shape[0] == sb.per
            got.append(sb.local_records().clone())
        assert torch.equal(torch.cat(got), whole), world
    ref = _oracle(whole_s, ego).reshape(O * T, 8)
    assert np.max(np.abs(whole.cpu().numpy() - ref)) < OFFSET_TOL


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


@pytest.fixture(scope="module")
def rccl_group(dev):
    import torch.distributed as dist
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1, device_id=dev)
    yield dist.group.WORLD
    dist.destroy_process_group()


def test_rccl_world1_sharded_safe_halfspaces(dev, rccl_group):
    s, ego = synthetic.obstacle_batch(6, 7, 500, dev, seed=11)
    full = sharding.sharded_safe_halfspaces(s, ego, RiskParams(), group=rccl_group)
    assert full.shape == (6, 7, 8) and full.device == dev
    assert torch.equal(full, engine.safe_halfspaces(s, ego, RiskParams()))
    assert np.max(np.abs(full.cpu().numpy() - _oracle(s, ego))) < OFFSET_TOL


def test_rccl_world1_sharded_batch_step_eager_and_graph(dev, rccl_group):
    """ShardedBatch with a (1-rank) RCCL group: the all-gather path runs (full buffer allocated),
    eagerly and inside a captured hipGraph (launch + all_gather_into_tensor per step)."""
    O, T, N = 8, 10, 1000
    nominal, ego = _nominal(O, T, dev, seed=9)
    sb = sharding.ShardedBatch(nominal, ego, N, RiskParams(), 1, 0, group=rccl_group, seed=9,
                               force_exchange=True)
    sb.full.fill_(float("nan"))
    sb.step()
    torch.cuda.synchronize()
    whole_s, _ = synthetic.obstacle_batch(O, T, N, dev, seed=9)
    want = engine.safe_halfspaces(whole_s, ego, RiskParams())
    assert torch.equal(sb.records(), want)
    sb.full.fill_(float("nan"))
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(dev)
    with torch.cuda.graph(g, stream=cap):
        launch = sb.prepare(torch.cuda.current_stream(dev))
        for _ in range(3):
            sb.step(launch)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(sb.records(), want)


@pytest.mark.parametrize("chunks", [1, 2, 3])
def test_rccl_world1_c4_leg_phases(dev, rccl_group, chunks):
    """bench.py's C4 strong-scaling leg (BASELINE config 4: 64 obstacles x T 30 x N 5000, the
    RCCL all-gather config) on a 1-rank RCCL group with the collective forced on: the stepper of
    the whole step, of the kernel alone and of the all-gather alone (the phase splits the leg
    reports), graph-captured; with chunks > 1 the step is the pipelined form (chunk j's
    all-gather issued behind chunk j + 1's kernel).  The gathered records equal the single-launch
    evaluation of the same batch, and the C oracle on a strided subset of units."""
    import bench
    O, T, N = bench.WORKLOADS["c4"][:3]
    nominal, ego = _nominal(O, T, dev, seed=11)
    sb = sharding.ShardedBatch(nominal, ego, N, RiskParams(), 1, 0, group=rccl_group, seed=11,
                               chunks=chunks, force_exchange=True)
    sb.full.fill_(float("nan"))
    whole_s, _ = synthetic.obstacle_batch(O, T, N, dev, seed=11)
    want = engine.safe_halfspaces(whole_s, ego, RiskParams())
    for kw in ({}, {"exchange": False}, {"compute": False}):
        st = bench.Stepper(sb, "graph", 10, 20, dev, warmup=5, **kw)
        assert st.fallback is None, st.fallback
        assert st.run(5) == 5 and st.run(20) == 20
        torch.cuda.synchronize()
        assert "step = " in st.describe()
    assert torch.equal(sb.records(), want)
    sub = slice(0, O, 9)
    ref = _oracle(whole_s[sub], ego)
    assert np.max(np.abs(sb.records()[sub].cpu().numpy() - ref)) < OFFSET_TOL

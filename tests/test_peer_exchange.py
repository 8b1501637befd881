"""GPU: the peer record exchange (include/drcvar_exchange.h, sharding.PeerExchange), in both forms:
push (the kernel writes every record into every rank's region) and pull (into its own region; the
small launch copies every rank's rows from that rank's region).

* one rank (the exchange with itself): ShardedBatch(exchange="peer") gives bitwise the records of
  the plain launch, step after step, eager and replayed from a hipGraph, the generation counts the
  steps and the error word stays 0;
* two processes on the one GPU of the box (gloo control group; each maps the other's region by
  IPC — the same code path as xGMI peers, minus the link): both ranks end with the whole batch's
  records, bitwise, for several steps and both parities, eager and graph-replayed;
* a wait whose peer never signals gives up at its spin limit and sets the error word (bit 63 and
  the silent rank's bit) instead of hanging.

The 8-GPU xGMI form is exercised only by the driver's multi-GPU bench (bench.py strong_scaling,
`exchanges.peer`, which checks its records against the RCCL all-gather's before using it).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import engine, sharding, synthetic
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.engine import RiskParams

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _whole(O, T, N, dev, seed):
    nominal, ego = synthetic.nominal_paths(O, T, dev, seed=seed), synthetic.straight_line_ego(T, dev)
    s, _ = synthetic.obstacle_batch(O, T, N, dev, seed=seed)
    return nominal, ego, engine.safe_halfspaces(s, ego, RiskParams())


@pytest.mark.parametrize("form", ["peer", "peer_pull"])
@pytest.mark.parametrize("O,T,N", [(10, 20, 1000), (7, 9, 300), (3, 5, 5000)])
def test_peer_exchange_one_rank_matches_plain_launch(dev, O, T, N, form):
    nominal, ego, whole = _whole(O, T, N, dev, seed=5)
    sb = sharding.ShardedBatch(nominal, ego, N, RiskParams(), 1, 0, seed=5, exchange=form,
                               force_exchange=True)
    assert sb.peer is not None and sb.peer.rows == O * T
    for k in range(3):                                  # both parities, then the first again
        sb.step()
        torch.cuda.synchronize(dev)
        assert torch.equal(sb.records(), whole), k
        assert sb.peer.generation() == k + 1 and sb.peer.error() == 0
    # graph capture and replay (the bench's form): the parity comes from the device counter
    g = torch.cuda.CUDAGraph()
    sb.full.fill_(float("nan"))
    with torch.cuda.graph(g, stream=torch.cuda.Stream(dev)):
        launch = sb.prepare(torch.cuda.current_stream(dev))
        for _ in range(3):
            sb.step(launch)
    for r in range(3):
        g.replay()
        torch.cuda.synchronize(dev)
        assert torch.equal(sb.records(), whole), r
    assert sb.peer.generation() == 3 + 9 and sb.peer.error() == 0
    sb.close()


def _two_rank_worker(rank, world, port, O, T, N, q, form="peer"):
    import sys
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    try:
        nominal, ego, whole = _whole(O, T, N, dev, seed=9)
        sb = sharding.ShardedBatch(nominal, ego, N, RiskParams(), world, rank, seed=9, exchange=form)
        ok = []
        for k in range(3):
            sb.step()
            torch.cuda.synchronize(dev)
            ok.append(bool(torch.equal(sb.records(), whole)))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=torch.cuda.Stream(dev)):
            launch = sb.prepare(torch.cuda.current_stream(dev))
            for _ in range(2):
                sb.step(launch)
        dist.barrier()
        for _ in range(2):
            sb.full.fill_(float("nan"))
            g.replay()
            torch.cuda.synchronize(dev)
            ok.append(bool(torch.equal(sb.records(), whole)))
        gen, err = sb.peer.generation(), sb.peer.error()
        sb.close()
        # the failure path: rank 1 never signals, rank 0's wait gives up at its spin limit
        px = sharding.PeerExchange(8, world, rank, dev, spin_limit_us=50_000,
                                   mode="pull" if form == "peer_pull" else "push")
        if rank == 0:
            px.signal_wait()
            torch.cuda.synchronize(dev)
        timeout_err = px.error()
        px.close()
        q.put((rank, ok, gen, err, timeout_err))
    except Exception as exc:  # noqa: BLE001 - reported to the parent
        q.put((rank, repr(exc), None, None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("form", ["peer", "peer_pull"])
@pytest.mark.parametrize("O,T,N", [(10, 20, 1000), (5, 3, 64)])
def test_peer_exchange_two_processes_one_gpu(dev, O, T, N, form):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_two_rank_worker, args=(r, 2, port, O, T, N, q, form)) for r in range(2)]
    for p in procs:
        p.start()
    results = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, gen, err, timeout_err in results:
        assert isinstance(ok, list), (rank, ok)
        assert all(ok), (rank, ok)
        assert gen == 3 + 4 and err == 0, (rank, gen, err)
        if rank == 0:
            assert timeout_err == (1 << 63) | (1 << 1), hex(timeout_err)
        else:
            assert timeout_err == 0

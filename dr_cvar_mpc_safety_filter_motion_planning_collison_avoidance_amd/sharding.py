"""Multi-GPU sharding of the (obstacle x step) unit batch — one process per GPU.

Units are independent (no cross-unit data in ``core/halfspaces.py:225-246`` or
``simulation/environment.py:82-104``), so the flattened unit index ``u = o*T + t`` is split into
contiguous blocks (:func:`shard_bounds`) and each rank evaluates its block with no data-path
collective.  The only exchange is the one the consumer needs: the MPC QP
(``core/mpc_filter.py:116-144``) takes every halfspace of the horizon, so the ``[U, 8]`` records
are reassembled on every rank with ONE ``all_gather_into_tensor`` (RCCL over xGMI when the
backend is ``nccl``; gloo in the CPU tests).  A record is 64 B, so even the largest config
(12 800 units, 800 KB) is a latency-bound exchange.

Two forms:

* :func:`sharded_safe_halfspaces` — the global ``[O, T, N, 2]`` batch exists on every rank (e.g.
  the reference's harness handed it over); a rank's block is addressed through at most three
  strided VIEWS of it (:func:`shard_views`: the tail of one obstacle, whole obstacles, the head of
  another), never a copy, whatever the batch's strides.
* :class:`ShardedBatch` — the global batch exists on NO rank: each rank draws only its own units
  with the device sampler (``drcvar_sample_units_f64``, the same Philox counters the whole batch
  would use), the kernel writes straight into its slice of the all-gather input, and
  :meth:`ShardedBatch.step` is one launch + one ``all_gather_into_tensor``.  This is the
  north-star multi-GPU form ``bench.py`` times.

Two exchanges for :class:`ShardedBatch`:

* ``"rccl"`` — the portable one: ``all_gather_into_tensor`` of the records (RCCL over xGMI with
  the ``nccl`` backend), optionally pipelined behind the kernel by chunks
  (:func:`chunked_all_gather`);
* ``"peer"`` — the MI355X-native one (:class:`PeerExchange`, ``include/drcvar_exchange.h``): each
  rank's halfspace launch writes every record straight into every rank's exchange region (mapped
  by IPC, written over xGMI), and one small launch per step publishes and awaits the step's
  generation and copies the gathered records out — the exchange rides inside the kernel and only
  a flag round trip is left after it.  Set up only when every rank can map every peer's memory;
  all ranks agree (over the control group) before any rank uses it, otherwise every rank keeps
  ``"rccl"``;
* ``"peer_pull"`` — the same regions and flags, but each rank's launch writes its records into its
  own region only and the small launch copies every rank's rows from that rank's region (reads
  over xGMI): no write round trip over xGMI inside the halfspace kernel's units.

``compute`` is injectable in :func:`sharded_safe_halfspaces`, and the sampler / launch preparation
in :class:`ShardedBatch`, so the partition/gather logic can be exercised with world_size 2 and 4
on CPU (gloo) in the tests; the product path always uses the HIP engine.
"""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist

from . import _native, engine
from .engine import RiskParams


class PeerExchangeUnavailable(RuntimeError):
    """Some rank cannot map or access some peer's exchange region (every rank raises it)."""


class PeerExchange:
    """The peer-push record exchange of one rank (``include/drcvar_exchange.h``).

    ``rows`` records per parity buffer (the padded global batch, ``world * per``).  Collective:
    every rank of ``group`` constructs it together.  The region handles and device indices go
    round the control group (``ctrl``: a gloo group; the default group when it is gloo itself);
    each rank maps every peer's region, checks that its device can access every peer's device,
    and all ranks agree on the outcome before any of them uses it — if anything fails on any rank,
    every rank raises :class:`PeerExchangeUnavailable` (and has released what it mapped).
    ``out`` (``[rows, 8]``, an ordinary device tensor) holds the gathered records after
    :meth:`signal_wait`.  ``spin_limit_us`` bounds every wait for a peer (then ``error()`` is
    non-zero instead of a hang)."""

    def __init__(self, rows: int, world: int, rank: int, device: torch.device, ctrl=None,
                 spin_limit_us: int = 2_000_000, mode: str = "push"):
        if mode not in ("push", "pull"):
            raise ValueError(f"mode must be 'push' or 'pull', not {mode!r}")
        if mode == "pull" and rows % world:
            raise ValueError(f"the pull form needs rows ({rows}) = world ({world}) * rows per rank")
        self.mode = mode
        if not (1 <= world <= _native.MAX_PEERS):
            raise PeerExchangeUnavailable(f"peer exchange supports 1..{_native.MAX_PEERS} ranks, not {world}")
        lib = _native.lib()
        self.rows, self.world, self.rank, self.device = int(rows), world, rank, device
        self.spin_limit_us = int(spin_limit_us)
        self._lib = lib
        self._ctrl = ctrl
        self._own = ctypes.c_void_p()
        self._opened = []
        handle = (ctypes.c_char * _native.PEER_HANDLE_BYTES)()
        doubles = lib.drcvar_peer_region_doubles(self.rows)
        with torch.cuda.device(device):
            rc = lib.drcvar_peer_alloc(doubles, ctypes.byref(self._own), handle)
        ok = rc == _native.OK
        why = None if ok else f"rank {rank}: drcvar_peer_alloc -> {rc}"
        bus = ctypes.create_string_buffer(64)
        if ok and lib.drcvar_peer_bus_id(device.index, bus, 64) != _native.OK:
            ok, why = False, f"rank {rank}: no PCI bus id for device {device.index}"
        mine = (bytes(handle), bus.value.decode() if ok else "")
        infos = [None] * world
        if world > 1:
            dist.all_gather_object(infos, mine, group=ctrl)
        else:
            infos = [mine]
        regions = [None] * world
        if ok:
            regions[rank] = self._own.value
            for j, (h, pbus) in enumerate(infos):
                if j == rank:
                    continue
                # the peer's GPU by its bus id, in this process's device numbering (the ranks' lists
                # of visible devices may differ); same device: the one-GPU rehearsal
                d, can = ctypes.c_int32(-1), ctypes.c_int32(0)
                if not pbus or lib.drcvar_peer_device_of(pbus.encode(), ctypes.byref(d)) != _native.OK:
                    ok, why = False, f"rank {rank}: rank {j}'s GPU {pbus or '?'} is not visible here"
                    break
                if lib.drcvar_peer_can_access(device.index, d.value, ctypes.byref(can)) != _native.OK \
                        or not can.value:
                    ok, why = False, f"rank {rank}: device {device.index} cannot access rank {j}'s GPU {pbus}"
                    break
                r = ctypes.c_void_p()
                with torch.cuda.device(device):
                    rc = lib.drcvar_peer_open((ctypes.c_char * _native.PEER_HANDLE_BYTES).from_buffer_copy(h),
                                              ctypes.byref(r))
                if rc != _native.OK:
                    ok, why = False, f"rank {rank}: drcvar_peer_open(rank {j}) -> {rc}"
                    break
                self._opened.append(r.value)
                regions[j] = r.value
        flag = torch.tensor([1 if ok else 0], dtype=torch.int64)
        if world > 1:
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=ctrl)
            reasons = [None] * world
            dist.all_gather_object(reasons, why, group=ctrl)
            why = "; ".join(r for r in reasons if r) or why
        if not int(flag.item()):
            self._release()   # nothing was ever written through a mapping: no barrier needed
            raise PeerExchangeUnavailable(why or "a peer rank could not set up the exchange")
        self.state = torch.zeros(3, dtype=torch.int64, device=device)   # generation, counter, error
        self.out = torch.empty((self.rows, engine.OUT_WIDTH), dtype=torch.float64, device=device)
        ps = _native.PeerSet()
        for j in range(world):
            ps.region[j] = regions[j]
        ps.rows, ps.state, ps.n_ranks, ps.rank = self.rows, self.state.data_ptr(), world, rank
        self.peers = ps
        self._ps_ref = ctypes.pointer(ps)
        # the pull form's halfspace launches write into the own region only: a one-rank set
        local = _native.PeerSet()
        local.region[0] = regions[rank]
        local.rows, local.state, local.n_ranks, local.rank = self.rows, self.state.data_ptr(), 1, 0
        self._local = local
        self._launch_ref = ctypes.pointer(local) if mode == "pull" else self._ps_ref
        self._signal = lib.drcvar_peer_signal_wait_pull if mode == "pull" else lib.drcvar_peer_signal_wait
        self._out_ptr = ctypes.c_void_p(self.out.data_ptr())
        self._spin = ctypes.c_int64(self.spin_limit_us)

    def signal_wait(self, stream=None) -> None:
        """Publish this rank's step, wait for every peer's, copy the gathered records to ``out``
        (one launch on ``stream``, default the current stream)."""
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        code = self._signal(self._ps_ref, self._out_ptr, self._spin, ctypes.c_void_p(int(s.cuda_stream)))
        if code != _native.OK:
            _native.check(code)

    def prepare_launch(self, samples: torch.Tensor, ego: torch.Tensor, params: RiskParams, row_base: int,
                       stream=None) -> engine.PreparedLaunch:
        """Freeze one ``drcvar_safe_halfspaces_f64_peer`` call over an ``[O, T, N, 2]`` block whose
        unit 0 is global row ``row_base``."""
        params.validate()
        engine._check_samples(samples, 4)
        O, T, N, _ = samples.shape
        engine._check_pairs(ego, "ego", T, samples.device)
        if row_base < 0 or row_base + O * T > self.rows:
            raise ValueError(f"rows [{row_base}, {row_base + O * T}) outside the exchange's {self.rows}")
        args = (ctypes.c_void_p(samples.data_ptr()), O, T, N, samples.stride(0), samples.stride(1),
                samples.stride(2), ctypes.c_void_p(ego.data_ptr()), ego.stride(0),
                params.robot_radius, params.obstacle_radius, params.alpha, params.delta, params.epsilon,
                self._launch_ref, int(row_base), ctypes.c_void_p(None),
                ctypes.c_void_p(engine._stream_handle(samples.device, stream)))
        return engine.PreparedLaunch(self._lib.drcvar_safe_halfspaces_f64_peer, args, (samples, ego, self))

    def generation(self) -> int:
        return int(self.state[0].item())

    def error(self) -> int:
        """0, or bit 63 | bit j for every rank j whose flag a wait gave up on."""
        return int(self.state[2].item()) & 0xFFFFFFFFFFFFFFFF

    def close(self) -> None:
        """Collective: wait until this device and (a barrier on the control group) every peer
        have finished writing, then unmap the peers' regions and free the own one — a region
        freed while a slower peer still writes into it would fault that peer."""
        if not (self._opened or self._own.value):
            return
        torch.cuda.synchronize(self.device)
        if self.world > 1:
            dist.barrier(group=self._ctrl)
        self._release()

    def _release(self) -> None:
        for r in self._opened:
            self._lib.drcvar_peer_close(ctypes.c_void_p(r))
        self._opened = []
        if self._own.value:
            self._lib.drcvar_peer_free(self._own)
            self._own = ctypes.c_void_p()

    def __del__(self):
        # one rank: nothing else writes the region, so it can go with the object; several: the
        # region stays mapped until close() or process exit (freeing it here, at a rank-local
        # moment, could fault a peer still writing into it)
        try:
            if self.world == 1:
                if self._own.value:
                    torch.cuda.synchronize(self.device)
                self._release()
        except Exception:  # noqa: BLE001 - interpreter teardown
            pass


def block_units(n_units: int, world_size: int, align: int = 1) -> int:
    """Units per rank block: ceil(U/W), rounded up to a multiple of ``align`` (the chunk count of a
    pipelined exchange, so every chunk of every block has the same length)."""
    per = -(-n_units // world_size) if n_units else 0
    return -(-per // align) * align


def shard_bounds(n_units: int, world_size: int, rank: int, align: int = 1) -> tuple[int, int]:
    """Contiguous block ``[start, stop)`` of rank ``rank`` (blocks of :func:`block_units`; the tail
    rank may get fewer or zero units)."""
    if world_size < 1 or not (0 <= rank < world_size) or align < 1:
        raise ValueError("invalid rank/world_size/align")
    per = block_units(n_units, world_size, align)
    start = min(rank * per, n_units)
    return start, min(start + per, n_units)


def chunked_all_gather(full: torch.Tensor, send: torch.Tensor, chunks: int, compute_chunk=None,
                       scratch: torch.Tensor | None = None, group=None) -> None:
    """The records exchange, pipelined behind the kernel: ``send [per, 8]`` (``per = chunks *
    cs``) is produced chunk by chunk (``compute_chunk(j)`` fills ``send[j cs:(j + 1) cs]``); each
    chunk's all-gather is issued asynchronously as soon as its kernel is queued (RCCL: on the
    communicator's stream, ordered after that kernel by an event), so chunk j's collective runs
    while chunk j + 1's kernel does.  The gathered chunks land in ``scratch [chunks, W cs, 8]``
    (chunk-major) and one copy puts them into ``full [W per, 8]`` in rank-major order — the same
    bytes, in the same ``[O, T, 8]`` order, as one all-gather of the whole block.
    ``chunks == 1``: compute, then one ``all_gather_into_tensor(full, send)``."""
    world = dist.get_world_size(group)
    per, width = send.shape
    if chunks == 1:
        if compute_chunk is not None:
            compute_chunk(0)
        _all_gather(full, send, group)
        return
    cs = per // chunks
    if cs * chunks != per or scratch is None or tuple(scratch.shape) != (chunks, world * cs, width):
        raise ValueError("chunked exchange: send must hold chunks * cs rows and scratch [chunks, W cs, 8]")
    works = []
    for j in range(chunks):
        if compute_chunk is not None:
            compute_chunk(j)
        src = send[j * cs:(j + 1) * cs]
        if src.device != scratch.device:             # gloo rehearsal: device records via the host
            src = src.to(scratch.device)
        works.append(dist.all_gather_into_tensor(scratch[j], src, group=group, async_op=True))
    for w in works:
        w.wait()
    full.view(world, chunks, cs, width).copy_(scratch.view(chunks, world, cs, width).transpose(0, 1))


def shard_pieces(n_obstacles: int, n_steps: int, start: int, stop: int):
    """Split the unit block ``[start, stop)`` of an ``[O, T]`` grid into at most three rectangles
    ``(o_lo, o_hi, t_lo, t_hi, offset)`` — the rest of one obstacle's steps, whole obstacles, the
    first steps of one more — each a strided view of any ``[O, T, ...]`` tensor; ``offset`` is
    the rectangle's first unit relative to ``start``."""
    O, T = n_obstacles, n_steps
    if not (0 <= start <= stop <= O * T):
        raise ValueError(f"unit block [{start}, {stop}) outside the {O} x {T} grid")
    pieces, u = [], start
    while u < stop:
        o, t = divmod(u, T)
        if t or stop - u < T:                       # a partial obstacle row
            t_hi = min(T, t + stop - u)
            pieces.append((o, o + 1, t, t_hi, u - start))
            u += t_hi - t
        else:                                       # whole obstacles
            n = (stop - u) // T
            pieces.append((o, o + n, 0, T, u - start))
            u += n * T
    return pieces


def shard_views(samples: torch.Tensor, ego: torch.Tensor, world_size: int, rank: int):
    """This rank's units of an ``[O, T, N, 2]`` batch (any strides) as strided views:
    ``([(samples [o, t, N, 2], ego [t, 2], offset, count)], start, stop)`` — no copies."""
    O, T = samples.shape[:2]
    start, stop = shard_bounds(O * T, world_size, rank)
    views = [(samples[o0:o1, t0:t1], ego[t0:t1], off, (o1 - o0) * (t1 - t0))
             for o0, o1, t0, t1, off in shard_pieces(O, T, start, stop)]
    return views, start, stop


def engine_compute(samples: torch.Tensor, ego: torch.Tensor, params: RiskParams,
                   out: torch.Tensor) -> None:
    """HIP engine on one rectangle: ``[o, t, N, 2]`` x ``[t, 2]`` -> ``out [o, t, 8]`` (one launch,
    strided samples consumed in place)."""
    engine.safe_halfspaces(samples, ego, params, out=out)


def _all_gather(full: torch.Tensor, send: torch.Tensor, group=None) -> None:
    if full.device == send.device:
        dist.all_gather_into_tensor(full, send, group=group)
    else:                                           # gloo rehearsal: device records via the host
        dist.all_gather_into_tensor(full, send.to(full.device), group=group)


def gather_records(send: torch.Tensor, n_units: int, group=None) -> torch.Tensor:
    """All-gather every rank's padded ``[ceil(U/W), 8]`` block into ``[n_units, 8]`` on every
    rank (one collective; the padding rows of the tail rank are dropped)."""
    world = dist.get_world_size(group)
    full = torch.empty((send.shape[0] * world, send.shape[1]), dtype=send.dtype, device=send.device)
    dist.all_gather_into_tensor(full, send, group=group)
    return full[:n_units]


def sharded_safe_halfspaces(samples: torch.Tensor, ego: torch.Tensor, params: RiskParams,
                            group=None, gather: bool = True, compute=engine_compute, chunks: int = 1):
    """Evaluate this rank's share of an ``[O, T, N, 2]`` batch; with ``gather`` return the full
    ``[O, T, 8]`` record on every rank, else ``(local [u, 8], start, stop)``.  ``chunks > 1``: the
    block is evaluated in that many pieces, each all-gathered while the next is computed
    (:func:`chunked_all_gather`; identical records)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    O, T = samples.shape[:2]
    start, stop = shard_bounds(O * T, world, rank, align=chunks)
    per = block_units(O * T, world, chunks)
    send = torch.zeros((per, engine.OUT_WIDTH), dtype=torch.float64, device=samples.device)
    cs = per // chunks if per else 0

    def compute_chunk(j):
        a, b = min(start + j * cs, stop), min(start + (j + 1) * cs, stop)
        for o0, o1, t0, t1, off in shard_pieces(O, T, a, b):
            cnt = (o1 - o0) * (t1 - t0)
            dst = send[a - start + off:a - start + off + cnt]
            compute(samples[o0:o1, t0:t1], ego[t0:t1], params, dst.view(o1 - o0, t1 - t0, engine.OUT_WIDTH))

    if not gather:
        for j in range(chunks):
            compute_chunk(j)
        return send[:stop - start], start, stop
    full = torch.empty((per * world, engine.OUT_WIDTH), dtype=torch.float64, device=samples.device)
    scratch = (torch.empty((chunks, world * cs, engine.OUT_WIDTH), dtype=torch.float64, device=samples.device)
               if chunks > 1 else None)
    chunked_all_gather(full, send, chunks, compute_chunk, scratch, group)
    return full[:O * T].reshape(O, T, engine.OUT_WIDTH)


class _Prepared(list):
    """The frozen launches of a rank's block (one per chunk) and the stream they are bound to."""

    def __init__(self, launches, stream):
        super().__init__(launches)
        self.stream = stream


class ShardedBatch:
    """One rank's block of a global ``[O, T, N, 2]`` obstacle-sample batch that no rank holds.

    ``nominal [O, T, 2]`` / ``ego [T, 2]`` describe the global batch (tiny; identical on every
    rank).  The rank's units ``[start, stop)`` are drawn once on its device
    (``drcvar_sample_units_f64``: sample for sample what the whole batch would hold), laid out flat
    ``[count, N, 2]`` and evaluated as ONE launch of a ``[1, count]`` grid whose per-unit ego is
    ``ego[u mod T]``.

    ``exchange="rccl"``: the kernel writes into ``send[:count]``, the all-gather input itself; with
    ``world > 1`` :meth:`step` then runs ``all_gather_into_tensor(full, send)`` — on RCCL the
    records go device to device, nothing is staged (``chunks > 1``: pipelined behind the kernel).
    ``exchange="peer"``: a :class:`PeerExchange` (collective set-up over ``ctrl``; raises
    :class:`PeerExchangeUnavailable` on every rank when any rank cannot use it) — the kernel writes
    every record into every rank's region and :meth:`step` adds the one publish/wait/copy launch;
    ``exchange="peer_pull"``: the kernel writes into the own region only and that launch copies
    every rank's rows from its region; ``full`` is the exchange's output.  ``records()`` is the global ``[O, T, 8]`` either way.

    ``sample_fn(nominal, n, start, count, cov, seed=, stream_offset=, zero_first_step=)`` and
    ``prepare_fn(samples [1, c, N, 2], ego [c, 2], params, out [1, c, 8], stream)`` are test-only
    injections (CPU rehearsal of the partition and exchange logic over gloo); the product path
    uses the device sampler and the HIP engine.  ``samples`` reuses another form's draw of the
    same block.
    """

    def __init__(self, nominal: torch.Tensor, ego: torch.Tensor, n_samples: int, params: RiskParams,
                 world_size: int = 1, rank: int = 0, group=None, seed: int = 42,
                 stream_offset: int = 0, noise_cov=None, zero_first_step: bool = True,
                 gather_device=None, chunks: int = 1, force_exchange: bool = False,
                 exchange: str = "rccl", ctrl=None, sample_fn=None, prepare_fn=None,
                 samples: torch.Tensor | None = None, peer_spin_us: int = 2_000_000):
        from .simulation import obstacles
        if exchange not in ("rccl", "peer", "peer_pull"):
            raise ValueError(f"exchange must be 'rccl', 'peer' or 'peer_pull', not {exchange!r}")
        if exchange != "rccl" and (chunks != 1 or gather_device is not None):
            raise ValueError("the peer exchange runs inside the kernel: one chunk, device records")
        O, T = int(nominal.shape[0]), int(nominal.shape[1])
        dev = nominal.device
        self.O, self.T, self.N = O, T, int(n_samples)
        self.U = O * T
        self.world, self.rank, self.group = world_size, rank, group
        self.params, self.nominal, self.seed = params, nominal, seed
        self.chunks = int(chunks)
        self.start, self.stop = shard_bounds(self.U, world_size, rank, align=self.chunks)
        self.count = self.stop - self.start
        self.per = block_units(self.U, world_size, self.chunks)
        self.cs = self.per // self.chunks if self.per else 0
        cov = obstacles.NOISE_COV if noise_cov is None else noise_cov
        if samples is not None:   # another form of the same block (bench.py: one draw, several exchanges)
            if tuple(samples.shape) != (self.count, self.N, 2):
                raise ValueError(f"samples must be this block's [{self.count}, {self.N}, 2]")
            self.samples = samples
        else:
            sample = sample_fn if sample_fn is not None else obstacles.sample_units_device
            self.samples = sample(nominal, self.N, self.start, self.count, cov, seed=seed,
                                  stream_offset=stream_offset, zero_first_step=zero_first_step)
        self._prepare_fn = prepare_fn if prepare_fn is not None else engine.prepare_safe_halfspaces
        idx = torch.arange(self.start, self.stop, device=dev) % T
        self.ego_units = ego.index_select(0, idx).contiguous()            # [count, 2], built once
        self.send = torch.zeros((self.per, engine.OUT_WIDTH), dtype=torch.float64, device=dev)
        gdev = dev if gather_device is None else torch.device(gather_device)
        # force_exchange: the collective runs at world 1 too (tests / the 1-rank rehearsals)
        do_exchange = world_size > 1 or force_exchange
        self.exchange_kind = exchange if do_exchange else None
        self.peer = None
        self.scratch = None
        if do_exchange and exchange != "rccl":
            self.peer = PeerExchange(self.per * world_size, world_size, rank, dev, ctrl=ctrl,
                                     spin_limit_us=peer_spin_us,
                                     mode="pull" if exchange == "peer_pull" else "push")
            self.full = self.peer.out
        else:
            self.full = (torch.empty((self.per * world_size, engine.OUT_WIDTH), dtype=torch.float64,
                                     device=gdev) if do_exchange else None)
            self.scratch = (torch.empty((self.chunks, world_size * self.cs, engine.OUT_WIDTH),
                                        dtype=torch.float64, device=gdev)
                            if do_exchange and self.chunks > 1 else None)
        self._launch = self.prepare()

    def prepare(self, stream=None) -> _Prepared:
        """Frozen launches of this rank's block on ``stream`` (default: the current stream), one
        per chunk — for hipGraph capture pass the capturing stream."""
        launches = []
        for j in range(self.chunks):
            a, b = min(j * self.cs, self.count), min((j + 1) * self.cs, self.count)
            if a == b:
                launches.append(None)
                continue
            if self.peer is not None:
                launch = self.peer.prepare_launch(self.samples[a:b].unsqueeze(0), self.ego_units[a:b],
                                                  self.params, self.start + a, stream=stream)
            else:
                launch, _ = self._prepare_fn(
                    self.samples[a:b].unsqueeze(0), self.ego_units[a:b], self.params,
                    out=self.send[a:b].view(1, b - a, engine.OUT_WIDTH), stream=stream)
            launches.append(launch)
        return _Prepared(launches, stream)

    def _compute_chunk(self, launches, j) -> None:
        if launches[j] is not None:
            launches[j]()

    def compute(self, launch=None) -> None:
        """The halfspace kernel over this rank's units (no collective; the peer form's kernel
        writes the records into every rank's region, but publishes nothing)."""
        launches = launch if launch is not None else self._launch
        for j in range(self.chunks):
            self._compute_chunk(launches, j)

    def exchange(self, launch=None) -> None:
        """The QP hand-off exchange: every rank's records to every rank (no-op without one)."""
        if self.peer is not None:
            launches = launch if launch is not None else self._launch
            self.peer.signal_wait(launches.stream)
        elif self.full is not None:
            chunked_all_gather(self.full, self.send, self.chunks, None, self.scratch, self.group)

    def step(self, launch=None) -> None:
        """One step: the kernel and the exchange — RCCL with ``chunks > 1`` pipelined (chunk j's
        all-gather behind chunk j + 1's kernel, :func:`chunked_all_gather`); peer: the kernel
        (records already pushed to every rank) and the publish/wait/copy launch."""
        launches = launch if launch is not None else self._launch
        if self.full is None:
            self.compute(launches)
            return
        if self.peer is not None:
            self.compute(launches)
            self.peer.signal_wait(launches.stream)
            return
        chunked_all_gather(self.full, self.send, self.chunks,
                           lambda j: self._compute_chunk(launches, j), self.scratch, self.group)

    def local_records(self) -> torch.Tensor:
        """``[count, 8]`` records of this rank's units (the peer form: after a step, from the
        gathered output)."""
        if self.peer is not None:
            return self.full[self.start:self.stop]
        return self.send[:self.count]

    def records(self) -> torch.Tensor:
        """Global ``[O, T, 8]`` records (after :meth:`step`; at world 1 the local block)."""
        src = self.full if self.full is not None else self.send
        return src[:self.U].view(self.O, self.T, engine.OUT_WIDTH)

    def close(self) -> None:
        """Collective for the peer exchange (see :meth:`PeerExchange.close`); no-op otherwise."""
        if self.peer is not None:
            self.peer.close()

    @property
    def algorithmic_bytes(self) -> int:
        """Bytes this rank's launch must move: its samples once, a 64-B record and the ego pair
        per unit (the ego is per unit here: ``[count, 2]``)."""
        return self.count * (16 * self.N + 64 + 16)

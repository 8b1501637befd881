"""Tensor-level entry points of the HIP engine (device-resident PyTorch-ROCm tensors).

These are the batched calls everything else is built on:

* :func:`safe_halfspaces`   — ``drcvar_safe_halfspaces_f64``: mean / CVaR / DR-CVaR halfspaces for
  every (obstacle, step) of a ``[O, T, N, 2]`` sample tensor (``core/halfspaces.py:196-248`` x the
  horizon loop of ``simulation/environment.py:82-104``).
* :func:`offsets_given_h`   — ``drcvar_offsets_given_h_f64``: ``cvar_halfspace`` /
  ``dr_cvar_halfspace`` for caller-supplied directions (``core/risk_metrics.py:267-338``).

Both enqueue one kernel on the current HIP stream and return without synchronising.  Inputs must
be float64 CUDA tensors whose two coordinates are adjacent (last stride 1); any other strides are
passed to the kernel as they are (no hidden copies).  :class:`PreparedLaunch` freezes the argument
tuple of a repeated call (bench loops, graph capture) so the per-launch host cost is one ctypes
call.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass

import torch

from . import _native

OUT_WIDTH = _native.OUT_WIDTH


@dataclass(frozen=True)
class RiskParams:
    """The five scalars the reference threads through every call (``config/parameters.py:11-29``)."""

    robot_radius: float = 0.3
    obstacle_radius: float = 0.3
    alpha: float = 0.2
    delta: float = 0.1
    epsilon: float = 0.15

    def validate(self) -> None:
        vals = (self.robot_radius, self.obstacle_radius, self.alpha, self.delta, self.epsilon)
        if not all(math.isfinite(v) for v in vals):
            raise ValueError(f"risk parameters must be finite: {self}")
        if self.alpha <= 0.0:
            # the reference divides by alpha while building its LPs (risk_metrics.py:105-107,212)
            raise ValueError(f"alpha must be > 0, got {self.alpha}")


def _stream_handle(device: torch.device, stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return int(s.cuda_stream)


def _check_samples(samples: torch.Tensor, ndim: int) -> None:
    if not isinstance(samples, torch.Tensor):
        raise TypeError("samples must be a torch.Tensor")
    if samples.device.type != "cuda":
        raise ValueError("samples must live on the GPU (HIP device tensor); the engine has no CPU path")
    if samples.dtype != torch.float64:
        raise TypeError(f"samples must be float64 (the reference computes in f64), got {samples.dtype}")
    if samples.dim() != ndim or samples.shape[-1] != 2:
        raise ValueError(f"samples must have shape {'[O, T, N, 2]' if ndim == 4 else '[U, N, 2]'}, "
                         f"got {tuple(samples.shape)}")
    if samples.stride(-1) != 1:
        raise ValueError("the two coordinates of a sample must be adjacent (last stride 1)")
    n = samples.shape[-2]
    if n < 1:
        raise ValueError("each unit needs at least one sample")
    if n > _native.MAX_SAMPLES_STREAM:
        raise ValueError(f"n_samples={n} exceeds the engine limit {_native.MAX_SAMPLES_STREAM}")


def _check_pairs(t: torch.Tensor, name: str, rows: int, device: torch.device) -> None:
    if t.device != device or t.dtype != torch.float64:
        raise ValueError(f"{name} must be a float64 tensor on {device}")
    if t.dim() != 2 or t.shape[0] != rows or t.shape[1] != 2 or t.stride(1) != 1:
        raise ValueError(f"{name} must have shape [{rows}, 2] with adjacent coordinates, got "
                         f"{tuple(t.shape)}")


def _check_out(out, shape, device: torch.device, what: str) -> None:
    """A caller-supplied output buffer must be exactly what the kernel writes: the engine writes
    ``prod(shape) * 8`` doubles through the raw pointer, so anything else is an out-of-bounds
    device write (checked before any ABI call)."""
    if not isinstance(out, torch.Tensor):
        raise TypeError("out must be a torch.Tensor")
    if (tuple(out.shape) != tuple(shape) or out.dtype != torch.float64 or not out.is_contiguous()
            or out.device != device):
        raise ValueError(f"out must be a contiguous float64 {what} tensor on {device}, got "
                         f"{tuple(out.shape)} {out.dtype} on {out.device}"
                         f"{'' if out.is_contiguous() else ' (non-contiguous)'}")


def _typed(args):
    """Pre-convert an argument tuple to ctypes objects (saves the per-call conversion)."""
    out = []
    for a in args:
        if isinstance(a, (ctypes._SimpleCData, ctypes._Pointer)):   # (a pointer: a struct argument)
            out.append(a)
        elif isinstance(a, bool) or not isinstance(a, (int, float)):
            raise TypeError(f"unexpected argument {a!r}")
        elif isinstance(a, int):
            out.append(ctypes.c_int64(a))
        else:
            out.append(ctypes.c_double(a))
    return tuple(out)


class PreparedLaunch:
    """A frozen engine call: same buffers, same parameters, relaunched by ``__call__``."""

    def __init__(self, fn, args, keepalive):
        self._fn = fn
        self._args = _typed(args)
        self._keepalive = keepalive  # tensors whose storage the pointers refer to

    def __call__(self) -> None:
        code = self._fn(*self._args)
        if code != _native.OK:
            _native.check(code)


def _check_status(status, n, device):
    if not isinstance(status, torch.Tensor) or status.dtype != torch.int32 or status.device != device \
            or status.numel() != n or not status.is_contiguous():
        raise ValueError(f"status must be a contiguous int32 tensor of {n} elements on {device}")


def prepare_safe_halfspaces(samples: torch.Tensor, ego: torch.Tensor, params: RiskParams,
                            out: torch.Tensor | None = None, stream=None,
                            geometry: tuple[int, int] | None = None,
                            status: torch.Tensor | None = None) -> tuple[PreparedLaunch, torch.Tensor]:
    """Freeze one ``drcvar_safe_halfspaces_f64`` call; ``geometry=(threads, per_thread)`` selects a
    specific compiled launch geometry, ``status`` (int32 ``[O, T]``) receives the per-unit status
    word (``_native.UNIT_*``) — both through ``drcvar_safe_halfspaces_f64_v2``."""
    params.validate()
    _check_samples(samples, 4)
    O, T, N, _ = samples.shape
    _check_pairs(ego, "ego", T, samples.device)
    if out is None:
        out = torch.empty((O, T, OUT_WIDTH), dtype=torch.float64, device=samples.device)
    else:
        _check_out(out, (O, T, OUT_WIDTH), samples.device, "[O, T, 8]")
    lib = _native.lib()
    so, st, sn = samples.stride(0), samples.stride(1), samples.stride(2)
    args = (ctypes.c_void_p(samples.data_ptr()), O, T, N, so, st, sn,
            ctypes.c_void_p(ego.data_ptr()), ego.stride(0),
            params.robot_radius, params.obstacle_radius, params.alpha, params.delta, params.epsilon,
            ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(_stream_handle(samples.device, stream)))
    if geometry is not None or status is not None:
        if status is not None:
            _check_status(status, O * T, samples.device)
        geo = tuple(ctypes.c_int32(int(g)) for g in (geometry or (0, 0)))
        st_ptr = ctypes.c_void_p(status.data_ptr() if status is not None else None)
        args2 = args[:-1] + (st_ptr, args[-1]) + geo
        return PreparedLaunch(lib.drcvar_safe_halfspaces_f64_v2, args2, (samples, ego, out, status)), out
    return PreparedLaunch(lib.drcvar_safe_halfspaces_f64, args, (samples, ego, out)), out


def safe_halfspaces(samples: torch.Tensor, ego: torch.Tensor, params: RiskParams = RiskParams(),
                    out: torch.Tensor | None = None, stream=None,
                    status: torch.Tensor | None = None) -> torch.Tensor:
    """Mean / CVaR / DR-CVaR halfspaces of every (obstacle, step) unit.

    samples [O, T, N, 2] float64 (device), ego [T, 2] float64 (device) -> [O, T, 8] float64 with
    columns (mean_h0, mean_h1, g_mean, h0, h1, g_cvar, g_dr_star, g_dr_tilde).  ``status``
    (optional int32 ``[O, T]`` device tensor) receives each unit's ``_native.UNIT_*`` bits.
    """
    launch, out = prepare_safe_halfspaces(samples, ego, params, out, stream, status=status)
    if samples.shape[0] * samples.shape[1] > 0:
        launch()
    return out


def offsets_given_h(samples: torch.Tensor, h: torch.Tensor, params: RiskParams = RiskParams(),
                    out: torch.Tensor | None = None, stream=None,
                    status: torch.Tensor | None = None) -> torch.Tensor:
    """``cvar_halfspace`` / ``dr_cvar_halfspace`` for U units with given directions.

    samples [U, N, 2] float64 (device), h [U, 2] float64 (device) -> [U, 8] float64 (same columns;
    h echoed in columns 3..4).  ``status`` (optional int32 ``[U]``) receives the ``UNIT_*`` bits.
    """
    params.validate()
    _check_samples(samples, 3)
    U, N, _ = samples.shape
    _check_pairs(h, "h", U, samples.device)
    if out is None:
        out = torch.empty((U, OUT_WIDTH), dtype=torch.float64, device=samples.device)
    else:
        _check_out(out, (U, OUT_WIDTH), samples.device, "[U, 8]")
    if status is not None:
        _check_status(status, U, samples.device)
    if U == 0:
        return out
    lib = _native.lib()
    _native.check(lib.drcvar_offsets_given_h_f64_v2(
        ctypes.c_void_p(samples.data_ptr()), U, N, samples.stride(0), samples.stride(1),
        ctypes.c_void_p(h.data_ptr()), h.stride(0),
        params.robot_radius, params.obstacle_radius, params.alpha, params.delta, params.epsilon,
        ctypes.c_void_p(out.data_ptr()),
        ctypes.c_void_p(status.data_ptr() if status is not None else None),
        ctypes.c_void_p(_stream_handle(samples.device, stream))))
    return out

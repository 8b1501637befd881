"""``core/mpc_filter.py`` surface backed by the HIP interior-point kernel (the halfspace hand-off).

Reference: ``MPCSafetyFilter`` (``core/mpc_filter.py:9-219``).  ``filter_trajectory`` keeps its
signature and return value ``(x_filtered [H+1, nx], u_filtered [H, nu], info)``; instead of a CVXPY
problem per call, the condensed model (``drcvar_mpc_model_init``) is built once per (A, B, C, Q, R,
horizon, bounds) and each call is ONE kernel launch (``drcvar_mpc_filter_f64``) that solves the QP
and, when it does not converge, rolls out the reference's fallback inputs (``_fallback``,
``:180-219``) on the device.

Two input forms for ``safe_halfspaces``:

* the reference's ``[T][O]`` lists of ``SafeHalfspace`` objects (``get_constraint_params()`` ->
  ``(h, g)``, ``:130``) — packed once into a device tensor (ragged steps padded with the
  always-satisfied row ``h = 0, g = -1``);
* a :class:`~.halfspaces.HalfspaceBatch` (or its ``[O, T, 8]`` record) plus ``metric`` — consumed
  in place on the device, no host round trip (the hand-off the engine is built for).

:func:`filter_batch` is the batched device API: B independent problems, one workgroup each.
"""
from __future__ import annotations

import ctypes
import time
import warnings

import numpy as np
import torch

from .. import _native
from . import risk_metrics

STATUS_NAMES = {_native.MPC_STATUS_OPTIMAL: "optimal", _native.MPC_STATUS_MAX_ITER: "max_iter",
                _native.MPC_STATUS_NUMERICAL: "numerical_error",
                _native.MPC_STATUS_OPTIMAL_INACCURATE: "optimal_inaccurate",
                _native.MPC_STATUS_CLUSTER_TIMEOUT: "cluster_timeout",
                _native.MPC_STATUS_CLUSTER_DIVERGED: "cluster_diverged"}
SOLVED = ("optimal", "optimal_inaccurate")   # core/mpc_filter.py:154
# record columns of each metric's (h, g): core/halfspaces.py get_constraint_params
METRIC_COLUMNS = {"mean": (_native.COL_MEAN_H0, _native.COL_G_MEAN),
                  "cvar": (_native.COL_H0, _native.COL_G_CVAR),
                  "dr_cvar": (_native.COL_H0, _native.COL_G_DR_TILDE)}
DEFAULT_MAX_ITER = 60
# interior-point tolerance before the active-set polish, which makes the answer exact: 1e-7 saves
# the last interior-point iteration on C5 (11 -> 10) with no polish failure on any measured shape
# (answers within 1.6e-9 of 1e-8's); 1e-6 made three-problem C5 launches need up to five polish
# attempts
DEFAULT_TOL = 1e-7


def _bounds(bounds, dim):
    """(min, max) truncated to ``dim`` entries (``core/mpc_filter.py:103-110``); None passes."""
    if bounds is None:
        return None, None
    lo, hi = bounds
    lo = np.ascontiguousarray(np.asarray(lo, dtype=np.float64).reshape(-1)[:dim])
    hi = np.ascontiguousarray(np.asarray(hi, dtype=np.float64).reshape(-1)[:dim])
    if lo.shape[0] != dim or hi.shape[0] != dim:
        raise ValueError(f"bounds need {dim} entries, got {lo.shape[0]} and {hi.shape[0]}")
    return lo, hi


def _host(m):
    return np.ascontiguousarray(np.asarray(m, dtype=np.float64))


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def make_options(cluster_size=0, spin_limit_us=0, debug_force_resume=False, debug_perturb_group=None,
                 debug_perturb_iteration=0, debug_stall_group=None) -> _native.MpcOptions:
    """``drcvar_mpc_options`` (include/drcvar_mpc.h).  ``cluster_size`` 0 = automatic, 1 = one
    workgroup per problem; the ``debug_*`` hooks exist for the tests (groups are 0-based here)."""
    o = _native.MpcOptions()
    o.cluster_size = int(cluster_size)
    o.spin_limit_us = int(spin_limit_us)
    o.debug_force_resume = int(bool(debug_force_resume))
    o.debug_perturb_group = 0 if debug_perturb_group is None else int(debug_perturb_group) + 1
    o.debug_perturb_iteration = int(debug_perturb_iteration)
    if debug_stall_group is not None and int(debug_stall_group) < 1:
        raise ValueError("debug_stall_group must be >= 1 (workgroup 0 writes the problem's outputs)")
    o.debug_stall_group = 0 if debug_stall_group is None else int(debug_stall_group) + 1
    return o


def _opt_ref(options):
    return ctypes.byref(options) if options is not None else None


class MPCModel:
    """Condensed (A, B, C, Q, R, horizon, bounds) resident on one device."""

    def __init__(self, A, B, C, Q, R, horizon, input_constraints=None, position_constraints=None,
                 device=None):
        A, B, C, Q, R = (_host(m) for m in (A, B, C, Q, R))
        nx, nu, ny = A.shape[0], B.shape[1], C.shape[0]
        if A.shape != (nx, nx) or B.shape != (nx, nu) or C.shape != (ny, nx) or \
                Q.shape != (nx, nx) or R.shape != (nu, nu):
            raise ValueError("inconsistent model shapes")
        if ny != 2:
            raise ValueError("the output matrix C must select the 2-D position (n_outputs == 2)")
        umin, umax = _bounds(input_constraints, nu)
        pmin, pmax = _bounds(position_constraints, ny)
        lib = _native.lib()
        model = _native.MpcModel()
        args = (_ptr(A), _ptr(B), _ptr(C), _ptr(Q), _ptr(R), nx, nu, ny, int(horizon),
                _ptr(umin), _ptr(umax), _ptr(pmin), _ptr(pmax), ctypes.byref(model))
        _native.check(lib.drcvar_mpc_model_init(*args, None))
        blob = np.empty(model.blob_doubles, dtype=np.float64)
        _native.check(lib.drcvar_mpc_model_init(*args, _ptr(blob)))
        self.model = model
        self.host_blob = blob
        self.device = torch.device(device) if device is not None else risk_metrics.device()
        self.blob = torch.as_tensor(blob).to(self.device)
        self.A, self.B = A, B
        self.nx, self.nu, self.horizon = nx, nu, int(horizon)

    def launch_groups(self, n_problems, n_obstacles, options=None):
        """Workgroups per problem a launch of this batch shape uses (drcvar_mpc_launch_groups_ex)."""
        return int(_native.lib().drcvar_mpc_launch_groups_ex(ctypes.byref(self.model), n_problems,
                                                             n_obstacles, _opt_ref(options)))

    def workspace_doubles(self, n_problems, n_obstacles):
        return int(_native.lib().drcvar_mpc_workspace_doubles(ctypes.byref(self.model), n_problems,
                                                             n_obstacles))


def _check_dev(t, name, shape, device):
    if not isinstance(t, torch.Tensor) or t.device != device or t.dtype != torch.float64:
        raise ValueError(f"{name} must be a float64 tensor on {device}")
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} must have shape {tuple(shape)}, got {tuple(t.shape)}")
    if t.numel() and t.stride(-1) != 1:
        raise ValueError(f"{name}: last dimension must be contiguous")


def filter_batch(model: MPCModel, hs_h: torch.Tensor, hs_g: torch.Tensor, x0: torch.Tensor,
                 x_ref: torch.Tensor, u_fallback: torch.Tensor, max_iter: int = DEFAULT_MAX_ITER,
                 tol: float = DEFAULT_TOL, polish: bool = True,
                 workspace: torch.Tensor | None = None, stream=None, options=None):
    """Solve B safety-filter QPs on the device (one ``drcvar_mpc_filter_f64_ex`` launch).

    hs_h [B, O, K, 2] (any strides, last 1), hs_g [B, O, K]; x0 [B, nx]; x_ref [B, H+1, nx];
    u_fallback [B, H, nu].  Returns (x [B, H+1, nx], u [B, H, nu], info [B, 10]) device tensors
    (columns ``_native.MPC_INFO_*``); nothing is synchronised.  ``polish`` finishes each solve
    with the active-set polish (exact optimum when it succeeds).  ``options``: :func:`make_options`.
    A clustered problem whose workgroups could not all stay resident, or disagreed, ends
    CLUSTER_TIMEOUT / CLUSTER_DIVERGED with the fallback rolled out; this function does not retry
    it — batch callers call :func:`retry_cluster_failures` on the result themselves (the
    MPCSafetyFilter wrapper does).
    """
    dev = model.device
    B = x0.shape[0]
    H, nx, nu = model.horizon, model.nx, model.nu
    if hs_h.dim() != 4 or hs_h.shape[0] != B or hs_h.shape[-1] != 2:
        raise ValueError(f"hs_h must be [B, O, K, 2], got {tuple(hs_h.shape)}")
    O, K = hs_h.shape[1], hs_h.shape[2]
    _check_dev(hs_h, "hs_h", (B, O, K, 2), dev)
    if hs_g.device != dev or hs_g.dtype != torch.float64 or tuple(hs_g.shape) != (B, O, K):
        raise ValueError(f"hs_g must be a float64 [{B}, {O}, {K}] tensor on {dev}")
    _check_dev(x0, "x0", (B, nx), dev)
    _check_dev(x_ref, "x_ref", (B, H + 1, nx), dev)
    _check_dev(u_fallback, "u_fallback", (B, H, nu), dev)
    x = torch.empty((B, H + 1, nx), dtype=torch.float64, device=dev)
    u = torch.empty((B, H, nu), dtype=torch.float64, device=dev)
    info = torch.empty((B, _native.MPC_INFO_WIDTH), dtype=torch.float64, device=dev)
    need = model.workspace_doubles(B, O)
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(max(need, 1), dtype=torch.float64, device=dev)
    if B == 0:
        return x, u, info
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    vp = ctypes.c_void_p
    _native.check(_native.lib().drcvar_mpc_filter_f64_ex(
        ctypes.byref(model.model), vp(model.blob.data_ptr()), B,
        vp(hs_h.data_ptr()), vp(hs_g.data_ptr()), O, K,
        hs_h.stride(0), hs_h.stride(1), hs_h.stride(2), hs_g.stride(0), hs_g.stride(1), hs_g.stride(2),
        vp(x0.data_ptr()), x0.stride(0), vp(x_ref.data_ptr()), x_ref.stride(0), x_ref.stride(1),
        vp(u_fallback.data_ptr()), u_fallback.stride(0), u_fallback.stride(1),
        int(max_iter), float(tol), int(bool(polish)), vp(x.data_ptr()), vp(u.data_ptr()), vp(info.data_ptr()),
        vp(workspace.data_ptr()), workspace.numel(), _opt_ref(options), vp(int(s.cuda_stream))))
    return x, u, info


CLUSTER_FAILURES = (_native.MPC_STATUS_CLUSTER_TIMEOUT, _native.MPC_STATUS_CLUSTER_DIVERGED)


def retry_cluster_failures(model: MPCModel, hs_h, hs_g, x0, x_ref, u_fallback, x, u, info,
                           max_iter: int = DEFAULT_MAX_ITER, tol: float = DEFAULT_TOL,
                           polish: bool = True, stream=None):
    """Re-solve, on one workgroup each, the problems of a :func:`filter_batch` result that ended
    CLUSTER_TIMEOUT or CLUSTER_DIVERGED (a cluster whose workgroups could not all stay resident, or
    disagreed), so that the caller gets the optimum the reference would return rather than the
    fallback rollout.  Synchronises (reads the status column); patches x / u / info in place and
    warns once per call that retried.  Returns the indices retried."""
    status = info[:, _native.MPC_INFO_STATUS].cpu()
    bad = torch.nonzero((status == CLUSTER_FAILURES[0]) | (status == CLUSTER_FAILURES[1])).flatten()
    if bad.numel() == 0:
        return []
    warnings.warn(f"{bad.numel()} clustered QP solve(s) ended "
                  f"{sorted({STATUS_NAMES.get(int(status[i])) for i in bad})}; re-solving them on one "
                  "workgroup each", RuntimeWarning, stacklevel=2)
    idx = bad.to(x.device)
    pick = lambda t: t.index_select(0, idx)
    x1, u1, info1 = filter_batch(model, pick(hs_h), pick(hs_g), pick(x0), pick(x_ref),
                                 pick(u_fallback), max_iter, tol, polish, stream=stream,
                                 options=make_options(cluster_size=1))
    x.index_copy_(0, idx, x1)
    u.index_copy_(0, idx, u1)
    info.index_copy_(0, idx, info1)
    return bad.tolist()


def record_views(record: torch.Tensor, metric: str):
    """(h [1, O, T, 2], g [1, O, T]) views of an ``[O, T, 8]`` halfspace record for ``metric``."""
    ch, cg = METRIC_COLUMNS[metric]
    return record[None, :, :, ch:ch + 2], record[None, :, :, cg]


def pack_halfspace_lists(safe_halfspaces, horizon):
    """Reference ``[T][O]`` SafeHalfspace lists -> host (h [O, K, 2], g [O, K]), K = min(T, H).

    Steps with fewer halfspaces are padded with ``h = 0, g = -1`` (a row ``-1 <= s`` that no
    input can violate, so the optimum is unchanged).
    """
    K = min(len(safe_halfspaces), horizon)
    O = max((len(safe_halfspaces[k]) for k in range(K)), default=0)
    h = np.zeros((O, K, 2))
    g = np.full((O, K), -1.0)
    for k in range(K):
        for o, hs in enumerate(safe_halfspaces[k]):
            hv, gv = hs.get_constraint_params()
            h[o, k] = np.asarray(hv, dtype=np.float64).reshape(2)
            g[o, k] = float(gv)
    return h, g


class MPCSafetyFilter:
    """MPC-based safety filter (``core/mpc_filter.py:9-38``)."""

    def __init__(self, A, B, C, Q, R, horizon, dt):
        self.A = np.asarray(A, dtype=np.float64)
        self.B = np.asarray(B, dtype=np.float64)
        self.C = np.asarray(C, dtype=np.float64)
        self.Q = np.asarray(Q, dtype=np.float64)
        self.R = np.asarray(R, dtype=np.float64)
        self.horizon = horizon
        self.dt = dt
        self.n_states = self.A.shape[0]
        self.n_inputs = self.B.shape[1]
        self.n_outputs = self.C.shape[0]
        self.last_optimal_u = None
        self.max_iter = DEFAULT_MAX_ITER
        self.tol = DEFAULT_TOL
        self._models = {}

    def model(self, input_constraints=None, position_constraints=None) -> MPCModel:
        """The condensed model for these bounds (built once, cached)."""
        key = tuple(None if b is None else
                    tuple(tuple(np.asarray(v, dtype=np.float64).reshape(-1).tolist()) for v in b)
                    for b in (input_constraints, position_constraints))
        m = self._models.get(key)
        if m is None:
            m = MPCModel(self.A, self.B, self.C, self.Q, self.R, self.horizon, input_constraints,
                         position_constraints)
            self._models[key] = m
        return m

    def _fallback_inputs(self, u_ref):
        """``_fallback`` input sequence (``core/mpc_filter.py:197-210``)."""
        u_ref = np.asarray(u_ref, dtype=np.float64)
        if self.last_optimal_u is None:
            return u_ref.copy()
        u = np.zeros((self.horizon, self.n_inputs))
        remaining = min(self.horizon - 1, len(self.last_optimal_u) - 1)
        u[:remaining] = self.last_optimal_u[1:remaining + 1]
        if remaining < self.horizon:
            u[remaining:] = u_ref[remaining:]
        return u

    def filter_trajectory(self, x0, x_ref, u_ref, safe_halfspaces, input_constraints=None,
                          position_constraints=None, metric="dr_cvar"):
        """Filter a reference trajectory (``core/mpc_filter.py:40-178``).

        ``safe_halfspaces``: the reference's ``[T][O]`` SafeHalfspace lists, or a HalfspaceBatch /
        ``[O, T, 8]`` device record together with ``metric`` ('mean' | 'cvar' | 'dr_cvar').
        Returns ``(x_filtered, u_filtered, info)`` as NumPy arrays + dict.
        """
        start = time.time()
        m = self.model(input_constraints, position_constraints)
        dev = m.device
        H, nx = self.horizon, self.n_states
        record = getattr(safe_halfspaces, "record", safe_halfspaces)
        if isinstance(record, torch.Tensor):
            if record.device != dev:
                record = record.to(dev)
            hs_h, hs_g = record_views(record[:, :H], metric)
        else:
            h, g = pack_halfspace_lists(safe_halfspaces, H)
            hs_h = torch.as_tensor(h[None]).to(dev)
            hs_g = torch.as_tensor(g[None]).to(dev)
        x0_d = torch.as_tensor(_host(x0).reshape(1, nx)).to(dev)
        xr_d = torch.as_tensor(_host(x_ref)[None, :H + 1]).to(dev)
        uf_d = torch.as_tensor(self._fallback_inputs(u_ref)[None]).to(dev)
        x, u, info = filter_batch(m, hs_h, hs_g, x0_d, xr_d, uf_d, self.max_iter, self.tol)
        retry_cluster_failures(m, hs_h, hs_g, x0_d, xr_d, uf_d, x, u, info, self.max_iter, self.tol)
        x, u, info = x[0].cpu().numpy(), u[0].cpu().numpy(), info[0].cpu().numpy()
        status = STATUS_NAMES.get(int(info[_native.MPC_INFO_STATUS]), "error")
        if status in SOLVED:                                       # :154-167
            self.last_optimal_u = u
            return x, u, {"status": status, "solve_time": time.time() - start,
                          "objective": float(info[_native.MPC_INFO_OBJECTIVE]),
                          "iterations": int(info[_native.MPC_INFO_ITERATIONS])}
        return x, u, {"status": status, "error": "Problem could not be solved optimally",  # :168-173
                      "used_fallback": True, "iterations": int(info[_native.MPC_INFO_ITERATIONS])}

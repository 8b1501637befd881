"""Loader for the HIP engine (``_lib/libdrcvar_halfspace.so``) — the C ABI of
``include/drcvar_halfspace.h`` bound with ctypes.

There is deliberately no fallback: if the shared library is missing or cannot be loaded every
entry point raises :class:`NativeLibraryError`.  ``build()`` compiles it for gfx950 in-tree.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_DIR = os.path.join(PKG_DIR, "_lib")
LIB_PATH = os.path.join(LIB_DIR, "libdrcvar_halfspace.so")
# diagnostic builds only (scripts/diag_stages.sh); the product always loads LIB_PATH
LIB_PATH = os.environ.get("DRCVAR_DIAG_LIB", LIB_PATH)
SOURCES = [os.path.join(PKG_DIR, "csrc", "drcvar_halfspace.hip"),
           os.path.join(PKG_DIR, "csrc", "drcvar_mpc.hip"),
           os.path.join(PKG_DIR, "csrc", "drcvar_sampling.hip")]
INCLUDE_DIR = os.path.join(REPO_DIR, "include")
HEADERS = [os.path.join(INCLUDE_DIR, h) for h in ("drcvar_halfspace.h", "drcvar_mpc.h",
                                                  "drcvar_sampling.h")]
OFFLOAD_ARCH = os.environ.get("DRCVAR_OFFLOAD_ARCH", "gfx950")

ABI_VERSION = 1
OUT_WIDTH = 8
MAX_SAMPLES = 16384               # largest unit held on chip (register plans)
MAX_SAMPLES_STREAM = 2 ** 31 - 1  # larger units run the streaming kernel
COL_MEAN_H0, COL_MEAN_H1, COL_G_MEAN, COL_H0, COL_H1, COL_G_CVAR, COL_G_DR_STAR, COL_G_DR_TILDE = range(8)

# return codes (include/drcvar_halfspace.h)
OK, ERR_INVALID_ARGUMENT, ERR_UNSUPPORTED, ERR_LAUNCH = 0, 1, 2, 3

# MPC hand-off (include/drcvar_mpc.h)
MPC_MAX_STATES, MPC_MAX_INPUTS, MPC_MAX_HORIZON, MPC_MAX_DECISION = 8, 4, 64, 120
MPC_INFO_WIDTH = 10
(MPC_INFO_STATUS, MPC_INFO_ITERATIONS, MPC_INFO_OBJECTIVE, MPC_INFO_MU, MPC_INFO_PRIMAL_RES,
 MPC_INFO_DUAL_RES, MPC_INFO_MAX_SLACK, MPC_INFO_USED_FALLBACK, MPC_INFO_POLISHED,
 MPC_INFO_POLISH_ATTEMPTS) = range(10)
MPC_STATUS_OPTIMAL, MPC_STATUS_MAX_ITER, MPC_STATUS_NUMERICAL, MPC_STATUS_OPTIMAL_INACCURATE = 0, 1, 2, 3


class MpcModel(ctypes.Structure):
    """``drcvar_mpc_model`` (include/drcvar_mpc.h)."""

    _fields_ = [("n_states", ctypes.c_int32), ("n_inputs", ctypes.c_int32),
                ("n_outputs", ctypes.c_int32), ("horizon", ctypes.c_int32),
                ("has_input_bounds", ctypes.c_int32), ("has_position_bounds", ctypes.c_int32),
                ("u_min", ctypes.c_double * MPC_MAX_INPUTS), ("u_max", ctypes.c_double * MPC_MAX_INPUTS),
                ("p_min", ctypes.c_double * 2), ("p_max", ctypes.c_double * 2),
                ("blob_doubles", ctypes.c_int64)]


# Every symbol include/*.h declares (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = (
    "drcvar_abi_version",
    "drcvar_strerror",
    "drcvar_safe_halfspaces_f64",
    "drcvar_safe_halfspaces_f64_ex",
    "drcvar_offsets_given_h_f64",
    "drcvar_launch_plan",
    "drcvar_mpc_model_init",
    "drcvar_mpc_workspace_doubles",
    "drcvar_mpc_launch_groups",
    "drcvar_mpc_filter_f64",
    "drcvar_sample_trajectories_f64",
    "drcvar_sample_units_f64",
)


class NativeLibraryError(RuntimeError):
    """The HIP engine is not built or cannot be loaded (there is no CPU fallback)."""


class EngineError(RuntimeError):
    """A DRCVAR_* error code returned by the engine."""

    def __init__(self, code: int, message: str):
        super().__init__(f"drcvar error {code}: {message}")
        self.code = code


_lock = threading.Lock()
_lib = None


def build(verbose: bool = False, extra_flags=()) -> str:
    """Compile the engine for gfx950 with hipcc into ``_lib/`` (works without a GPU)."""
    os.makedirs(LIB_DIR, exist_ok=True)
    # one hipcc per source, concurrently (the halfspace kernel's template plans dominate), then
    # one link: the library is the same as a single-command build
    objs = [os.path.join(LIB_DIR, os.path.basename(src) + ".o") for src in SOURCES]
    procs = []
    for src, obj in zip(SOURCES, objs):
        cmd = ["hipcc", f"--offload-arch={OFFLOAD_ARCH}", "-O3", "-std=c++17", "-fPIC", "-c",
               "-I", INCLUDE_DIR, *extra_flags, src, "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append((cmd, subprocess.Popen(cmd)))
    failed = [cmd for cmd, p in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    link = ["hipcc", f"--offload-arch={OFFLOAD_ARCH}", "-shared", "-fPIC", *objs,
            "-o", LIB_PATH + ".tmp"]
    if verbose:
        print(" ".join(link))
    subprocess.run(link, check=True)
    for obj in objs:
        os.remove(obj)
    os.replace(LIB_PATH + ".tmp", LIB_PATH)
    return LIB_PATH


def _bind(lib):
    i64, dbl, ptr, i32p = ctypes.c_int64, ctypes.c_double, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)
    lib.drcvar_abi_version.argtypes = []
    lib.drcvar_abi_version.restype = ctypes.c_int
    lib.drcvar_strerror.argtypes = [ctypes.c_int]
    lib.drcvar_strerror.restype = ctypes.c_char_p
    lib.drcvar_safe_halfspaces_f64.argtypes = [
        ptr, i64, i64, i64, i64, i64, i64, ptr, i64, dbl, dbl, dbl, dbl, dbl, ptr, ptr]
    lib.drcvar_safe_halfspaces_f64.restype = ctypes.c_int
    lib.drcvar_safe_halfspaces_f64_ex.argtypes = [
        ptr, i64, i64, i64, i64, i64, i64, ptr, i64, dbl, dbl, dbl, dbl, dbl, ptr, ptr,
        ctypes.c_int32, ctypes.c_int32]
    lib.drcvar_safe_halfspaces_f64_ex.restype = ctypes.c_int
    lib.drcvar_offsets_given_h_f64.argtypes = [
        ptr, i64, i64, i64, i64, ptr, i64, dbl, dbl, dbl, dbl, dbl, ptr, ptr]
    lib.drcvar_offsets_given_h_f64.restype = ctypes.c_int
    lib.drcvar_launch_plan.argtypes = [i64, i32p, i32p, i32p]
    lib.drcvar_launch_plan.restype = ctypes.c_int
    i32, modelp = ctypes.c_int32, ctypes.POINTER(MpcModel)
    lib.drcvar_mpc_model_init.argtypes = [ptr, ptr, ptr, ptr, ptr, i32, i32, i32, i32,
                                          ptr, ptr, ptr, ptr, modelp, ptr]
    lib.drcvar_mpc_model_init.restype = ctypes.c_int
    lib.drcvar_mpc_workspace_doubles.argtypes = [modelp, i64, i64]
    lib.drcvar_mpc_workspace_doubles.restype = i64
    lib.drcvar_mpc_launch_groups.argtypes = [modelp, i64, i64]
    lib.drcvar_mpc_launch_groups.restype = ctypes.c_int32
    lib.drcvar_mpc_filter_f64.argtypes = [
        modelp, ptr, i64, ptr, ptr, i64, i64, i64, i64, i64, i64, i64, i64, ptr, i64, ptr, i64,
        i64, ptr, i64, i64, i32, dbl, i32, ptr, ptr, ptr, ptr, i64, ptr]
    lib.drcvar_mpc_filter_f64.restype = ctypes.c_int
    u64 = ctypes.c_uint64
    lib.drcvar_sample_trajectories_f64.argtypes = [
        ptr, i64, i64, i64, i64, i64, dbl, dbl, dbl, u64, u64, i32, ptr, i64, i64, i64, ptr]
    lib.drcvar_sample_trajectories_f64.restype = ctypes.c_int
    lib.drcvar_sample_units_f64.argtypes = [
        ptr, i64, i64, i64, i64, i64, i64, i64, dbl, dbl, dbl, u64, u64, i32, ptr, i64, i64, ptr]
    lib.drcvar_sample_units_f64.restype = ctypes.c_int
    return lib


def lib():
    """The loaded engine library (raises NativeLibraryError if unavailable)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise NativeLibraryError(
                    f"HIP engine not built: {LIB_PATH} is missing (run __graft_entry__.build() or "
                    f"python -m dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.build)")
            try:
                handle = ctypes.CDLL(LIB_PATH)
            except OSError as exc:  # pragma: no cover - depends on the ROCm install
                raise NativeLibraryError(f"cannot load {LIB_PATH}: {exc}") from exc
            _bind(handle)
            if handle.drcvar_abi_version() != ABI_VERSION:
                raise NativeLibraryError("engine ABI version mismatch; rebuild the library")
            _lib = handle
    return _lib


def check(code: int) -> None:
    if code != OK:
        raise EngineError(code, lib().drcvar_strerror(code).decode())


def launch_plan(n_samples: int):
    """(threads_per_unit, samples_per_thread, bins) chosen for ``n_samples`` (host-only query)."""
    b, p, nb = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    check(lib().drcvar_launch_plan(int(n_samples), ctypes.byref(b), ctypes.byref(p), ctypes.byref(nb)))
    return b.value, p.value, nb.value

"""Loader for the HIP engine (``_lib/libdrcvar_halfspace.so``) — the C ABI of
``include/drcvar_halfspace.h`` (+ ``drcvar_mpc.h``, ``drcvar_sampling.h``, ``drcvar_exchange.h``)
bound with ctypes.

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
SOURCES = [os.path.join(PKG_DIR, "csrc", "drcvar_halfspace.hip"),
           os.path.join(PKG_DIR, "csrc", "drcvar_mpc.hip"),
           os.path.join(PKG_DIR, "csrc", "drcvar_sampling.hip"),
           os.path.join(PKG_DIR, "csrc", "drcvar_exchange.hip")]
INCLUDE_DIR = os.path.join(REPO_DIR, "include")
HEADERS = [os.path.join(INCLUDE_DIR, h) for h in ("drcvar_halfspace.h", "drcvar_mpc.h",
                                                  "drcvar_sampling.h", "drcvar_exchange.h")]
OFFLOAD_ARCH = "gfx950"  # CDNA4 only

ABI_VERSION = 3
OUT_WIDTH = 8
MAX_SAMPLES = 16384               # largest unit held on chip (register plans)
MAX_SAMPLES_STREAM = 2 ** 31 - 1  # larger units run the streaming kernel
COL_MEAN_H0, COL_MEAN_H1, COL_G_MEAN, COL_H0, COL_H1, COL_G_CVAR, COL_G_DR_STAR, COL_G_DR_TILDE = range(8)
# per-unit status word (DRCVAR_UNIT_*), a bit set
UNIT_OK, UNIT_NONFINITE, UNIT_UNBOUNDED, UNIT_DR_UNBOUNDED = 0, 1, 2, 4

# return codes (include/drcvar_halfspace.h)
OK, ERR_INVALID_ARGUMENT, ERR_UNSUPPORTED, ERR_LAUNCH = 0, 1, 2, 3

# MPC hand-off (include/drcvar_mpc.h)
MPC_MAX_STATES, MPC_MAX_INPUTS, MPC_MAX_HORIZON, MPC_MAX_DECISION = 8, 4, 64, 120
MPC_INFO_WIDTH = 10
(MPC_INFO_STATUS, MPC_INFO_ITERATIONS, MPC_INFO_OBJECTIVE, MPC_INFO_MU, MPC_INFO_PRIMAL_RES,
 MPC_INFO_DUAL_RES, MPC_INFO_MAX_SLACK, MPC_INFO_USED_FALLBACK, MPC_INFO_POLISHED,
 MPC_INFO_POLISH_ATTEMPTS) = range(10)
(MPC_STATUS_OPTIMAL, MPC_STATUS_MAX_ITER, MPC_STATUS_NUMERICAL, MPC_STATUS_OPTIMAL_INACCURATE,
 MPC_STATUS_CLUSTER_TIMEOUT, MPC_STATUS_CLUSTER_DIVERGED) = range(6)


class MpcModel(ctypes.Structure):
    """``drcvar_mpc_model`` (include/drcvar_mpc.h)."""

    _fields_ = [("n_states", ctypes.c_int32), ("n_inputs", ctypes.c_int32),
                ("n_outputs", ctypes.c_int32), ("horizon", ctypes.c_int32),
                ("has_input_bounds", ctypes.c_int32), ("has_position_bounds", ctypes.c_int32),
                ("u_min", ctypes.c_double * MPC_MAX_INPUTS), ("u_max", ctypes.c_double * MPC_MAX_INPUTS),
                ("p_min", ctypes.c_double * 2), ("p_max", ctypes.c_double * 2),
                ("blob_doubles", ctypes.c_int64)]


class MpcOptions(ctypes.Structure):
    """``drcvar_mpc_options`` (include/drcvar_mpc.h): per-call options, all 0 = the defaults."""

    _fields_ = [("cluster_size", ctypes.c_int32), ("spin_limit_us", ctypes.c_int32),
                ("debug_force_resume", ctypes.c_int32), ("debug_perturb_group", ctypes.c_int32),
                ("debug_perturb_iteration", ctypes.c_int32), ("debug_stall_group", ctypes.c_int32),
                ("reserved", ctypes.c_int32 * 2)]


# peer-push exchange (include/drcvar_exchange.h)
MAX_PEERS = 8
PEER_HANDLE_BYTES = 64


class PeerSet(ctypes.Structure):
    """``drcvar_peer_set`` (include/drcvar_exchange.h)."""

    _fields_ = [("region", ctypes.c_void_p * MAX_PEERS), ("rows", ctypes.c_int64),
                ("state", ctypes.c_void_p), ("n_ranks", ctypes.c_int32), ("rank", ctypes.c_int32)]


# Every symbol include/*.h declares (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = (
    "drcvar_abi_version",
    "drcvar_strerror",
    "drcvar_safe_halfspaces_f64",
    "drcvar_safe_halfspaces_f64_ex",
    "drcvar_safe_halfspaces_f64_v2",
    "drcvar_offsets_given_h_f64",
    "drcvar_offsets_given_h_f64_v2",
    "drcvar_launch_plan",
    "drcvar_mpc_model_init",
    "drcvar_mpc_workspace_doubles",
    "drcvar_mpc_launch_groups",
    "drcvar_mpc_launch_groups_ex",
    "drcvar_mpc_filter_f64",
    "drcvar_mpc_filter_f64_ex",
    "drcvar_sample_trajectories_f64",
    "drcvar_sample_units_f64",
    "drcvar_peer_region_doubles",
    "drcvar_peer_alloc",
    "drcvar_peer_free",
    "drcvar_peer_open",
    "drcvar_peer_close",
    "drcvar_peer_can_access",
    "drcvar_peer_bus_id",
    "drcvar_peer_device_of",
    "drcvar_peer_signal_wait",
    "drcvar_peer_signal_wait_pull",
    "drcvar_safe_halfspaces_f64_peer",
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
_lib_path = LIB_PATH  # what lib() loads; only use_library() changes it


def use_library(path: str) -> None:
    """Load ``path`` (a diagnostic variant build, e.g. a stamps build) instead of the product library.

    Diagnostic scripts call this explicitly before the first engine call; nothing in the package
    reads the environment to pick a library.  Raises if another library is already loaded."""
    global _lib_path
    path = os.path.abspath(path)
    with _lock:
        if _lib is not None and path != _lib_path:
            raise NativeLibraryError(f"{_lib_path} is already loaded; use_library({path!r}) must come first")
        _lib_path = path


def _compile_units():
    """(source, extra defines) per object: the MPC source is compiled as five parts (host code,
    then the kernels of the 1..4-input models: csrc/drcvar_mpc.hip, DRCVAR_MPC_PART) so that its
    template instantiations build concurrently."""
    units = []
    for src in SOURCES:
        if src.endswith("drcvar_mpc.hip"):
            units += [(src, (f"-DDRCVAR_MPC_PART={k}",)) for k in range(5)]
        elif src.endswith("drcvar_halfspace.hip"):
            # the latency-bound halfspace kernel: its first 16 kernarg dwords arrive preloaded in
            # SGPRs (gfx950 kernarg preload; the code object keeps a loading prologue for firmware
            # without it), so the sample addresses do not wait for a scalar-memory round trip:
            # C3 4.04 -> 3.97 us per step (scripts/micro/gpu_hs_ab.sh)
            units.append((src, ("-mllvm", "-amdgpu-kernarg-preload-count=16")))
        else:
            units.append((src, ()))
    return units


def _quoted_includes(path: str, seen=None) -> list:
    """The files a source pulls in through ``#include "..."`` (include/ or csrc/), transitively."""
    import re
    seen = set() if seen is None else seen
    out = []
    for name in re.findall(r'^\s*#\s*include\s+"([^"]+)"', open(path).read(), re.M):
        for d in (INCLUDE_DIR, os.path.join(PKG_DIR, "csrc")):
            f = os.path.join(d, name)
            if os.path.exists(f) and f not in seen:
                seen.add(f)
                out.append(f)
                out.extend(_quoted_includes(f, seen))
                break
    return out


_toolchain_id = None
TOOLCHAIN_PATH = os.path.join(LIB_DIR, "toolchain.id")


def _toolchain(probe: bool = False) -> bytes:
    """The compiler's identity (``hipcc --version``): part of every object key and source key.
    build() probes hipcc (probe=True) and records the answer next to the library it links;
    everything else reads that record — the identity of the compiler that built the loaded
    library — and never starts a process: bench.py asks for source_key() after the GPU is
    initialised, where forking a child to exec hipcc is not allowed."""
    global _toolchain_id
    if probe:
        tid = subprocess.run(["hipcc", "--version"], capture_output=True, check=True).stdout
        os.makedirs(LIB_DIR, exist_ok=True)
        with open(TOOLCHAIN_PATH + ".tmp", "wb") as f:
            f.write(tid)
        os.replace(TOOLCHAIN_PATH + ".tmp", TOOLCHAIN_PATH)
        _toolchain_id = tid
    elif _toolchain_id is None:
        try:
            with open(TOOLCHAIN_PATH, "rb") as f:
                _toolchain_id = f.read()
        except OSError:
            return b"unrecorded (library not built)"
    return _toolchain_id


def _unit_flags(defs=(), extra_flags=()) -> list:
    """The full hipcc flag list of one translation unit (what build() compiles it with)."""
    return [f"--offload-arch={OFFLOAD_ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", "-I", INCLUDE_DIR,
            *defs, *extra_flags]


def source_key(basename: str = "drcvar_halfspace.hip") -> str:
    """A hash of one translation unit's inputs (its source, the headers and .inc tables it
    includes, the toolchain's identity and its full compile flags, as build() keys its object):
    profiles/ evidence is tied to the kernel build it measured, and bench.py uses it only while
    all of these still match."""
    import hashlib
    src = os.path.join(PKG_DIR, "csrc", basename)
    h = hashlib.sha256(open(src, "rb").read())
    for f in _quoted_includes(src):
        h.update(open(f, "rb").read())
    h.update(_toolchain())
    for s, defs in _compile_units():
        if s == src:
            h.update(" ".join(_unit_flags(defs)).replace(INCLUDE_DIR, "include").encode())
    return h.hexdigest()[:16]


def build(verbose: bool = False, extra_flags=()) -> str:
    """Compile the engine for gfx950 with hipcc into ``_lib/`` (works without a GPU).

    One hipcc per translation unit, concurrently, then one link.  Objects are cached under
    ``_lib/obj`` by a hash of the unit's source, the headers and the flags, so a rebuild after an
    edit recompiles only the units it touched."""
    import hashlib
    os.makedirs(LIB_DIR, exist_ok=True)
    obj_dir = os.path.join(LIB_DIR, "obj")
    os.makedirs(obj_dir, exist_ok=True)
    import glob
    incs = sorted(glob.glob(os.path.join(PKG_DIR, "csrc", "*.inc")))  # tables the sources include
    headers = b"".join(open(h, "rb").read() for h in HEADERS + incs)
    # the compiler's identity is part of every key: objects of an older hipcc / ROCm are rebuilt
    toolchain = _toolchain(probe=True)
    objs, procs = [], []
    for src, defs in _compile_units():
        flags = _unit_flags(defs, extra_flags)
        key = hashlib.sha256(open(src, "rb").read() + headers + toolchain
                             + " ".join(flags).encode()).hexdigest()[:16]
        tag = "".join(d.replace("-D", ".") for d in defs if d.startswith("-D"))
        obj = os.path.join(obj_dir, f"{os.path.basename(src)}{tag}.{key}.o")
        objs.append(obj)
        if os.path.exists(obj):
            continue
        cmd = ["hipcc", *flags, src, "-o", obj + ".tmp"]
        if verbose:
            print(" ".join(cmd))
        procs.append((cmd, obj, subprocess.Popen(cmd)))
    failed = [cmd for cmd, _, p in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    for _, obj, _ in procs:
        os.replace(obj + ".tmp", obj)
    link = ["hipcc", f"--offload-arch={OFFLOAD_ARCH}", "-shared", "-fPIC", *objs,
            "-o", LIB_PATH + ".tmp"]
    if verbose:
        print(" ".join(link))
    subprocess.run(link, check=True)
    os.replace(LIB_PATH + ".tmp", LIB_PATH)
    keep = set(objs)  # drop stale cached objects (not *.tmp: another build may be writing them)
    for f in os.listdir(obj_dir):
        if f.endswith(".o") and os.path.join(obj_dir, f) not in keep:
            os.remove(os.path.join(obj_dir, f))
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
    lib.drcvar_safe_halfspaces_f64_v2.argtypes = [
        ptr, i64, i64, i64, i64, i64, i64, ptr, i64, dbl, dbl, dbl, dbl, dbl, ptr, ptr, ptr,
        ctypes.c_int32, ctypes.c_int32]
    lib.drcvar_safe_halfspaces_f64_v2.restype = ctypes.c_int
    lib.drcvar_offsets_given_h_f64_v2.argtypes = [
        ptr, i64, i64, i64, i64, ptr, i64, dbl, dbl, dbl, dbl, dbl, ptr, ptr, ptr]
    lib.drcvar_offsets_given_h_f64_v2.restype = ctypes.c_int
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
    optp = ctypes.POINTER(MpcOptions)
    lib.drcvar_mpc_launch_groups_ex.argtypes = [modelp, i64, i64, optp]
    lib.drcvar_mpc_launch_groups_ex.restype = ctypes.c_int32
    lib.drcvar_mpc_filter_f64_ex.argtypes = lib.drcvar_mpc_filter_f64.argtypes[:-1] + [optp, ptr]
    lib.drcvar_mpc_filter_f64_ex.restype = ctypes.c_int
    u64 = ctypes.c_uint64
    lib.drcvar_sample_trajectories_f64.argtypes = [
        ptr, i64, i64, i64, i64, i64, dbl, dbl, dbl, u64, u64, i32, ptr, i64, i64, i64, ptr]
    lib.drcvar_sample_trajectories_f64.restype = ctypes.c_int
    lib.drcvar_sample_units_f64.argtypes = [
        ptr, i64, i64, i64, i64, i64, i64, i64, dbl, dbl, dbl, u64, u64, i32, ptr, i64, i64, ptr]
    lib.drcvar_sample_units_f64.restype = ctypes.c_int
    peerp = ctypes.POINTER(PeerSet)
    lib.drcvar_peer_region_doubles.argtypes = [i64]
    lib.drcvar_peer_region_doubles.restype = i64
    lib.drcvar_peer_alloc.argtypes = [i64, ctypes.POINTER(ctypes.c_void_p), ptr]
    lib.drcvar_peer_alloc.restype = ctypes.c_int
    lib.drcvar_peer_free.argtypes = [ptr]
    lib.drcvar_peer_free.restype = ctypes.c_int
    lib.drcvar_peer_open.argtypes = [ptr, ctypes.POINTER(ctypes.c_void_p)]
    lib.drcvar_peer_open.restype = ctypes.c_int
    lib.drcvar_peer_close.argtypes = [ptr]
    lib.drcvar_peer_close.restype = ctypes.c_int
    lib.drcvar_peer_can_access.argtypes = [i32, i32, i32p]
    lib.drcvar_peer_can_access.restype = ctypes.c_int
    lib.drcvar_peer_bus_id.argtypes = [i32, ctypes.c_char_p, i32]
    lib.drcvar_peer_bus_id.restype = ctypes.c_int
    lib.drcvar_peer_device_of.argtypes = [ctypes.c_char_p, i32p]
    lib.drcvar_peer_device_of.restype = ctypes.c_int
    lib.drcvar_peer_signal_wait.argtypes = [peerp, ptr, i64, ptr]
    lib.drcvar_peer_signal_wait.restype = ctypes.c_int
    lib.drcvar_peer_signal_wait_pull.argtypes = [peerp, ptr, i64, ptr]
    lib.drcvar_peer_signal_wait_pull.restype = ctypes.c_int
    lib.drcvar_safe_halfspaces_f64_peer.argtypes = [
        ptr, i64, i64, i64, i64, i64, i64, ptr, i64, dbl, dbl, dbl, dbl, dbl, peerp, i64, ptr, ptr]
    lib.drcvar_safe_halfspaces_f64_peer.restype = ctypes.c_int
    return lib


def lib():
    """The loaded engine library (raises NativeLibraryError if unavailable)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(_lib_path):
                raise NativeLibraryError(
                    f"HIP engine not built: {_lib_path} is missing (run __graft_entry__.build() or "
                    f"python -m dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.build)")
            try:
                handle = ctypes.CDLL(_lib_path)
            except OSError as exc:  # pragma: no cover - depends on the ROCm install
                raise NativeLibraryError(f"cannot load {_lib_path}: {exc}") from exc
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

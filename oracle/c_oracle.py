"""CPU ORACLE — test infrastructure only.  ctypes binding of oracle/drcvar_oracle.c.

Used by tests/ as a second checker and by bench.py as the timed cpu_baseline ("port").
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libdrcvar_oracle.so")
_lib = None

_i64 = ctypes.c_int64
_dbl = ctypes.c_double
_ptr = ctypes.c_void_p


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        lib = ctypes.CDLL(_LIB_PATH)
        lib.oracle_safe_halfspaces_f64.argtypes = [
            _ptr, _i64, _i64, _i64, _i64, _i64, _i64, _ptr, _i64,
            _dbl, _dbl, _dbl, _dbl, _dbl, _ptr, ctypes.c_int]
        lib.oracle_safe_halfspaces_f64.restype = ctypes.c_int
        lib.oracle_offsets_given_h_f64.argtypes = [
            _ptr, _i64, _i64, _i64, _i64, _ptr, _dbl, _dbl, _dbl, _dbl, _dbl, _ptr]
        lib.oracle_offsets_given_h_f64.restype = ctypes.c_int
        _lib = lib
    return _lib


def safe_halfspaces(samples, ego, robot_radius, obstacle_radius, alpha, delta, epsilon,
                    nthreads=1):
    """samples [O,T,N,2] f64 (any strides, coordinate stride 1), ego [T,2] -> out [O,T,8]."""
    lib = _load()
    samples = np.asarray(samples, dtype=np.float64)
    if samples.strides[-1] != 8:
        samples = np.ascontiguousarray(samples)
    ego = np.ascontiguousarray(ego, dtype=np.float64)
    O, T, N, _ = samples.shape
    so, st, sn = (s // 8 for s in samples.strides[:3])
    out = np.empty((O, T, 8), dtype=np.float64)
    rc = lib.oracle_safe_halfspaces_f64(
        samples.ctypes.data, O, T, N, so, st, sn, ego.ctypes.data, 2,
        robot_radius, obstacle_radius, alpha, delta, epsilon, out.ctypes.data, int(nthreads))
    if rc != 0:
        raise ValueError("oracle_safe_halfspaces_f64: invalid arguments")
    return out


def offsets_given_h(samples, h, robot_radius, obstacle_radius, alpha, delta, epsilon):
    """samples [U,N,2], h [U,2] -> out [U,8] (columns 5..7 are g_cvar, g_star, g_tilde)."""
    lib = _load()
    samples = np.ascontiguousarray(samples, dtype=np.float64)
    h = np.ascontiguousarray(h, dtype=np.float64)
    U, N, _ = samples.shape
    out = np.empty((U, 8), dtype=np.float64)
    rc = lib.oracle_offsets_given_h_f64(samples.ctypes.data, U, N, N * 2, 2, h.ctypes.data,
                                        robot_radius, obstacle_radius, alpha, delta, epsilon,
                                        out.ctypes.data)
    if rc != 0:
        raise ValueError("oracle_offsets_given_h_f64: invalid arguments")
    return out

"""Diagnostic scripts only: run against a variant build of the engine (stamps, truncated stages,
A/B candidates) named by DRCVAR_DIAG_LIB.  The product loader reads no environment; a script that
wants a variant calls apply() before its first engine call."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def apply():
    path = os.environ.get("DRCVAR_DIAG_LIB")
    if path:
        from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import _native
        _native.use_library(path)
    return path

"""MI355X-native DR-CVaR safe-halfspace engine.

A from-scratch HIP/CDNA4 implementation of the safe-halfspace hot path of the DR-CVaR MPC safety
filter (reference: core/halfspaces.py, core/risk_metrics.py, simulation/environment.py), behind
the C ABI in include/drcvar_halfspace.h and the reference's Python call surface:

    from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.core.halfspaces import (
        compute_safe_halfspaces, CVaRSafeHalfspace, DRCVaRSafeHalfspace, MeanSafeHalfspace)

Batched device API: ``engine.safe_halfspaces`` / ``core.risk_metrics.RiskMetric``.
"""
from . import _native
from .engine import RiskParams, offsets_given_h, safe_halfspaces

__all__ = ["RiskParams", "safe_halfspaces", "offsets_given_h", "build", "native_available"]


def build(verbose: bool = False) -> str:
    """Compile the HIP engine for gfx950 into the package (``_lib/``)."""
    return _native.build(verbose=verbose)


def native_available() -> bool:
    try:
        _native.lib()
        return True
    except _native.NativeLibraryError:
        return False

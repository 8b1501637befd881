import glob
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN_DIR = os.path.join(REPO, "tests", "golden")

# Parity tolerance stated by the north star: offsets within 1e-6 absolute of the reference.
OFFSET_TOL = 1e-6


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    # A/B runs of the suite against a variant build (scripts/micro/*.sh): the test harness, not the
    # package, chooses the library
    if os.environ.get("DRCVAR_DIAG_LIB"):
        from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import _native
        _native.use_library(os.environ["DRCVAR_DIAG_LIB"])


def golden_files():
    """Halfspace fixtures (the mpc_*.npz hand-off fixtures and the qp_*.npz QP instances are loaded
    by tests/test_mpc.py, the singleton_*.npz call sequences by tests/test_singletons.py)."""
    return sorted(p for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz"))
                  if not os.path.basename(p).startswith(("mpc_", "qp_", "singleton_")))


def load_golden(path):
    z = np.load(path, allow_pickle=False)
    return {k: z[k] for k in z.files}


@pytest.fixture(params=golden_files(), ids=lambda p: os.path.basename(p)[:-4])
def golden(request):
    return load_golden(request.param)

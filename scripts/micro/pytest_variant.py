"""pytest on a variant build of the engine: python scripts/micro/pytest_variant.py <lib.so> <pytest args...>"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd import _native  # noqa: E402

_native.use_library(sys.argv[1])
import pytest  # noqa: E402

sys.exit(pytest.main(sys.argv[2:]))

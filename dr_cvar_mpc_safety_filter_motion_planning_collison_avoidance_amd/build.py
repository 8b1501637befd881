"""``python -m dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd.build``"""
from ._native import build

if __name__ == "__main__":
    print(build(verbose=True))

#!/usr/bin/env bash
# Build the -DDRCVAR_MPC_STAMPS diagnostic library and print the MPC kernel's phase totals.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -DDRCVAR_MPC_STAMPS -I include \
  dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd/csrc/drcvar_halfspace.hip \
  dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd/csrc/drcvar_mpc.hip \
  dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd/csrc/drcvar_sampling.hip -o /tmp/mpc_stamps.so || exit 1
DRCVAR_DIAG_LIB=/tmp/mpc_stamps.so timeout -k 10 300 python3 scripts/mpc_stamps.py ${MPC_SHAPES:-30,3,1 20,10,1 50,256,1} 2>&1 | grep -v amdgpu.ids

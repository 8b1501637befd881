#!/usr/bin/env bash
# Entry/exit spread of the halfspace kernel's workgroups on the shared 100 MHz clock
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd/csrc
hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -I include -DDRCVAR_STAMPS -DDRCVAR_STAMPS_REALTIME \
  $D/drcvar_halfspace.hip $D/drcvar_mpc.hip $D/drcvar_sampling.hip -o /tmp/spread.so || exit 1
for shape in ${SHAPES:-10,20,1000}; do
  DRCVAR_STAMPS_REALTIME=1 DRCVAR_DIAG_LIB=/tmp/spread.so timeout -k 10 120 python3 scripts/stamps.py --shape $shape 2>&1 | grep -v amdgpu.ids || exit 2
done

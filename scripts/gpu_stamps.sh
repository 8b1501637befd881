#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
SRC="dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd/csrc/drcvar_halfspace.hip dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd/csrc/drcvar_mpc.hip dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd/csrc/drcvar_sampling.hip"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -I include -DDRCVAR_STAMPS $SRC -o /tmp/stamps.so 2>/dev/null || exit 1
for spec in ${STAMP_SPECS:-10,20,1000: 256,50,10000: 64,30,5000:}; do
  shape=${spec%%:*}; geo=${spec#*:}
  DRCVAR_DIAG_LIB=/tmp/stamps.so timeout -k 10 300 python3 scripts/stamps.py --shape $shape ${geo:+--geometry $geo} || exit 2
done

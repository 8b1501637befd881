#!/usr/bin/env bash
# Build scripts/micro/variants/$VARIANT.hip into its own library and run scripts/micro/diag_one.py
# against it: ARGS="dyn H O i,j,..."
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
D=dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd/csrc
hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -I include $D/drcvar_halfspace.hip scripts/micro/variants/$VARIANT.hip $D/drcvar_sampling.hip -o /tmp/var_diag.so || exit 1
for a in "${ARGS[@]:-}"; do :; done
IFS=';' read -ra CASES <<< "$ARGS"
for c in "${CASES[@]}"; do
  echo "== $c"
  DRCVAR_DIAG_LIB=/tmp/var_diag.so timeout -k 10 120 python scripts/micro/diag_one.py $c 2>&1 | grep -v amdgpu.ids || exit 2
done

#!/usr/bin/env bash
# A/B of sampler variants: VARIANTS="name:file.hip ..." (each linked with the tree's other
# sources into its own library); runs scripts/micro/sampler_bench.py against each.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
D=dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd/csrc
for v in $VARIANTS; do
  name=${v%%:*}; src=${v#*:}
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -I include $D/drcvar_halfspace.hip $D/drcvar_mpc.hip $src -o /tmp/var_$name.so || exit 1
  echo "== $name"
  DRCVAR_DIAG_LIB=/tmp/var_$name.so timeout -k 10 120 python scripts/micro/sampler_bench.py 2>&1 | grep -v amdgpu.ids || exit 2
done

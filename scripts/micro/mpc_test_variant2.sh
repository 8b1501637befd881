#!/usr/bin/env bash
# Runs one pytest selection against MPC kernel variants: VARIANTS="name:file.hip ..." TESTS="..."
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
D=dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd/csrc
for v in $VARIANTS; do
  name=${v%%:*}; src=${v#*:}
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -I include $D/drcvar_halfspace.hip $src $D/drcvar_sampling.hip -o /tmp/var_$name.so || exit 1
  echo "== $name"
  DRCVAR_DIAG_LIB=/tmp/var_$name.so timeout -k 10 300 python -m pytest $TESTS -m gpu -q --timeout 120 --timeout-method thread 2>&1 | grep -E "passed|failed|^E  " | head -8
done

#!/usr/bin/env bash
# A/B of halfspace-kernel variants: VARIANTS="name:file.hip ..." (each linked with the tree's MPC
# and sampler sources into its own library); runs the C3 parity tests and scripts/tune.py
# (automatic geometry, graph-free launches) against each.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
D=dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd/csrc
for v in $VARIANTS; do
  name=${v%%:*}; src=${v#*:}
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -I include $src $D/drcvar_mpc.hip $D/drcvar_sampling.hip -o /tmp/var_$name.so || exit 1
done
for v in $VARIANTS; do
  name=${v%%:*}
  echo "== $name"
  DRCVAR_DIAG_LIB=/tmp/var_$name.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q -x 2>&1 | tail -1 || exit 2
  DRCVAR_DIAG_LIB=/tmp/var_$name.so timeout -k 10 120 python scripts/tune.py --shape ${SHAPE:-10,20,1000} --launches 3000 --only-auto 2>&1 | grep geometry || exit 3
done

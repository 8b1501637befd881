#!/usr/bin/env bash
# Round-3 iteration: sampler (tests, refill bench, VALU pass), then the cluster gather width A/B
# (scripts/mpc_bench.py on the product library and on scripts/micro/variants/mpc_g16.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash scripts/micro/gpu_sampler_quick.sh || exit $?
for rep in 1 2; do
  echo "product gather 8:"; timeout -k 10 200 python3 -u scripts/mpc_bench.py --shapes 50,256,1 50,256,3 20,100,3 || exit $?
  echo "variant gather 16:"; DRCVAR_DIAG_LIB=scripts/micro/variants/mpc_g16.so timeout -k 10 200 python3 -u scripts/mpc_bench.py --shapes 50,256,1 50,256,3 20,100,3 || exit $?
done

#!/usr/bin/env bash
# Round 4: the factorisation overlapped with the affine rhs (product) against the start-only build,
# and the interior-point tolerance before the polish (1e-8 default vs 1e-7 / 1e-6 / 1e-5).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4c; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_mpc.py tests/test_mpc_cluster.py > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit 2
S="30,3,1 30,3,1024 20,10,3 50,256,1 50,256,3"
for v in product start; do
  lib=""; [ $v != product ] && lib=scripts/micro/variants/mpc_$v.so
  echo "== mpc_bench $v"
  DRCVAR_DIAG_LIB=$lib timeout -k 10 300 python3 -u scripts/mpc_bench.py --shapes $S 2>&1 | grep -v amdgpu.ids || exit 3
done
for tol in 1e-7 1e-6 1e-5; do
  echo "== mpc_bench product tol $tol"
  timeout -k 10 300 python3 -u scripts/mpc_bench.py --tol $tol --shapes $S 2>&1 | grep -v amdgpu.ids || exit 3
done

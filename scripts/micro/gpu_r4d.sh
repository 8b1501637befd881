#!/usr/bin/env bash
# Round 4: the matrix-core Riccati factorisation (product) against the VALU form (overlap build):
# MPC GPU tests, then mpc_bench at the default tolerance and at 1e-7; and the permlane probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4d; mkdir -p $OUT
timeout -k 5 60 ./scripts/micro/mfma_f64_probe | tail -3
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_mpc.py tests/test_mpc_cluster.py > $OUT/tests.log 2>&1; rc=$?
tail -15 $OUT/tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit 2
S="30,3,1 30,3,1024 20,10,3 50,256,1 50,256,3"
for v in product overlap; do
  lib=""; [ $v != product ] && lib=scripts/micro/variants/mpc_$v.so
  for tol in 1e-8 1e-7; do
    echo "== mpc_bench $v tol $tol"
    DRCVAR_DIAG_LIB=$lib timeout -k 10 300 python3 -u scripts/mpc_bench.py --tol $tol --shapes $S 2>&1 | grep -v amdgpu.ids | cut -c1-150 || exit 3
  done
done

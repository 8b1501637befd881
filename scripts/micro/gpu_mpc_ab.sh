#!/usr/bin/env bash
# gpu_mpc_ab.sh <outdir> [variant.so ...]: MPC GPU tests on the in-tree library, then mpc_bench of
# the in-tree library and of each variant, interleaved twice, and bench.py's MPC hand-off legs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-mpcab}; shift; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mpc or smoke" > $OUT/pytest_mpc.log 2>&1
rc=$?; tail -2 $OUT/pytest_mpc.log; [ $rc -eq 0 ] || exit $rc
SH="npz:tests/golden/qp_c5_degenerate.npz 50,256,1 50,256,3 30,3,1024 20,10,3 30,3,1"
for r in 1 2; do
  timeout -k 10 300 python3 scripts/mpc_bench.py --shapes $SH > $OUT/bench_product_$r.log 2>&1 || exit $?
  for v in "$@"; do
    DRCVAR_DIAG_LIB=$v timeout -k 10 300 python3 scripts/mpc_bench.py --shapes $SH > $OUT/bench_$(basename $v .so)_$r.log 2>&1 || exit $?
  done
done
grep -H "ms/launch" $OUT/bench_*.log | sed 's/max|u.*//'

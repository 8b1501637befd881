#!/usr/bin/env bash
# A/B of the pipelined affine solve: stamps builds with and without it, interleaved twice
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5j}; mkdir -p $OUT
for r in 1 2; do for v in stamps_nopipe stamps_pipe; do
  DRCVAR_DIAG_LIB=scripts/micro/variants/$v.so timeout -k 10 300 python3 scripts/mpc_stamps.py npz:tests/golden/qp_c5_degenerate.npz:fixture > $OUT/${v}_$r.log 2>&1 || exit $?
  DRCVAR_DIAG_LIB=scripts/micro/variants/$v.so timeout -k 10 300 python3 scripts/mpc_bench.py --shapes npz:tests/golden/qp_c5_degenerate.npz 30,3,1024 > $OUT/bench_${v}_$r.log 2>&1 || exit $?
done; done
for f in $OUT/stamps_*; do echo $f; grep "total\|P1 span\|P1 resid\|solves (ipm)" $f; done
grep -H "ms/launch" $OUT/bench_* | sed 's/iters.*//'

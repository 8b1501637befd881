#!/usr/bin/env bash
# A/B of the follower with cached progress words and a one-block prefetch (fol) against the
# committed follower (base), interleaved; the follower's stamps; the MPC GPU tests on fol
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5folab}; mkdir -p $OUT
DRCVAR_DIAG_LIB=scripts/micro/variants/fol.so timeout -k 10 600 python3 -u -m pytest tests/test_mpc_cluster.py tests/test_mpc.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_fol.log 2>&1
rc=$?; tail -2 $OUT/pytest_fol.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for v in base fol; do
  DRCVAR_DIAG_LIB=scripts/micro/variants/$v.so timeout -k 10 300 python3 scripts/mpc_bench.py --shapes npz:tests/golden/qp_c5_degenerate.npz 50,256,3 30,3,1024 > $OUT/bench_${v}_$r.log 2>&1 || exit $?
done; done
for v in; do
  DRCVAR_DIAG_LIB=scripts/micro/variants/$v.so timeout -k 10 300 python3 scripts/mpc_stamps.py npz:tests/golden/qp_c5_degenerate.npz:fixture > $OUT/${v}.log 2>&1 || exit $?
done
for f in $OUT/stamps_*; do echo $f; grep "total\|P1 span\|P1 resid" $f; done
grep -H "ms/launch" $OUT/bench_* | sed 's/iters.*max polish/max polish/; s/polished.*//; s/.*bench_//'

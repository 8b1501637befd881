#!/usr/bin/env bash
# setup breakdown (stamps) and the polish penalty A/B (rho 1e6 vs 1e8): MPC tests on the variant,
# stamps of both on the C5 fixture and two C5 problems, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5k}; mkdir -p $OUT
timeout -k 10 600 python3 -u scripts/micro/pytest_variant.py scripts/micro/variants/stamps_rho8.so tests -m gpu -q --timeout 120 --timeout-method thread -k "mpc" > $OUT/pytest_rho8.log 2>&1; echo rho8; tail -2 $OUT/pytest_rho8.log
for r in 1 2; do for v in stamps_pipe stamps_rho8; do
  DRCVAR_DIAG_LIB=scripts/micro/variants/$v.so timeout -k 10 300 python3 scripts/mpc_stamps.py npz:tests/golden/qp_c5_degenerate.npz:fixture 50,256,3 > $OUT/${v}_$r.log 2>&1 || exit $?
  DRCVAR_DIAG_LIB=scripts/micro/variants/$v.so timeout -k 10 300 python3 scripts/mpc_bench.py --shapes npz:tests/golden/qp_c5_degenerate.npz 50,256,3 30,3,1024 > $OUT/bench_${v}_$r.log 2>&1 || exit $?
done; done
cat $OUT/stamps_pipe_1.log
grep -H "ms/launch" $OUT/bench_* | sed 's/iters.*max polish/ max polish/; s/polished.*//'

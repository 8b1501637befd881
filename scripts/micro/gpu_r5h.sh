#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5h}; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mpc or smoke" > $OUT/pytest_mpc.log 2>&1
rc=$?; echo mpc; tail -2 $OUT/pytest_mpc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/mpc_bench.py --shapes npz:tests/golden/qp_c5_degenerate.npz 50,256,1 50,256,3 30,3,1024 20,10,3 30,3,1 > $OUT/bench.log 2>&1 || exit $?
grep -v amdgpu $OUT/bench.log | sed 's/max|u.*//'
for sh in npz:tests/golden/qp_c5_degenerate.npz:fixture 30,3,1024; do
  DRCVAR_DIAG_LIB=scripts/micro/variants/stamps_pipe.so timeout -k 10 300 python3 scripts/mpc_stamps.py $sh > $OUT/stamps_$(echo $sh | tr ':/,' '___').log 2>&1 || exit $?
done
grep -h "total\|P1 span\|P1 resid\|solves (ipm)\|exchanges " $OUT/stamps_*.log

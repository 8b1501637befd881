#!/usr/bin/env bash
# Round 4: the blocked Riccati factorisation (variants mpc_blk: barrier-separated phases,
# mpc_blk_pipe: phase 3 of each block starts when wave 0 publishes its end value) against the
# product: MPC GPU tests on each variant, mpc_bench interleaved, phase stamps (single-unit builds).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4h; mkdir -p $OUT
V=scripts/micro/variants
S="30,3,1 30,3,1024 20,10,3 50,256,1 50,256,3"
for v in blk blk_pipe; do
  echo "== mpc tests on mpc_$v"
  DRCVAR_DIAG_LIB=$V/mpc_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_mpc.py tests/test_mpc_cluster.py > $OUT/tests_$v.log 2>&1; rc=$?
  tail -4 $OUT/tests_$v.log
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit 2
done
for r in 1 2; do
  for v in product blk blk_pipe; do
    lib=""; [ $v != product ] && lib=$V/mpc_$v.so
    echo "== mpc_bench $v run $r"
    DRCVAR_DIAG_LIB=$lib timeout -k 10 300 python3 -u scripts/mpc_bench.py --shapes $S > $OUT/bench_${v}_$r.log 2>&1 \
      || { tail -20 $OUT/bench_${v}_$r.log; exit 3; }
    grep -v amdgpu.ids $OUT/bench_${v}_$r.log | cut -c1-150
  done
done
for v in stamps blk_stamps blk_pipe_stamps; do
  echo "== mpc stamps $v"
  DRCVAR_DIAG_LIB=$V/mpc_$v.so timeout -k 10 300 python3 scripts/mpc_stamps.py npz:tests/golden/qp_c5_degenerate.npz:fixture \
    50,256,1 > $OUT/stamps_$v.log 2>&1 || { tail -20 $OUT/stamps_$v.log; exit 4; }
  grep -v amdgpu.ids $OUT/stamps_$v.log
done

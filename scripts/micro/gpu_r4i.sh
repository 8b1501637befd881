#!/usr/bin/env bash
# Round 4: the blocked factorisation's per-wave phase costs (stamps builds with 8 and 4 blocks),
# and mpc_bench of 4-block variants against the product and the 8-block pipelined variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4i; mkdir -p $OUT
V=scripts/micro/variants
S="30,3,1 20,10,3 50,256,1 50,256,3"
echo "== mpc tests on mpc_blk4p"
DRCVAR_DIAG_LIB=$V/mpc_blk4p.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_mpc.py tests/test_mpc_cluster.py > $OUT/tests_blk4p.log 2>&1; rc=$?
tail -3 $OUT/tests_blk4p.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit 2
for r in 1 2; do
  for v in product blk4 blk4p blk_pipe; do
    lib=""; [ $v != product ] && lib=$V/mpc_$v.so
    echo "== mpc_bench $v run $r"
    DRCVAR_DIAG_LIB=$lib timeout -k 10 300 python3 -u scripts/mpc_bench.py --shapes $S > $OUT/bench_${v}_$r.log 2>&1 \
      || { tail -20 $OUT/bench_${v}_$r.log; exit 3; }
    grep -v amdgpu.ids $OUT/bench_${v}_$r.log | cut -c1-60
  done
done
for v in blk8p_stamps blk4p_stamps blk4_stamps; do
  echo "== mpc stamps $v"
  DRCVAR_DIAG_LIB=$V/mpc_$v.so timeout -k 10 300 python3 scripts/mpc_stamps.py 50,256,1 30,3,1 > $OUT/stamps_$v.log 2>&1 \
    || { tail -20 $OUT/stamps_$v.log; exit 4; }
  grep -v amdgpu.ids $OUT/stamps_$v.log
done

#!/usr/bin/env bash
# Round 4: the blocked factorisation with the affine-rhs rows' H0 u through the dynamics
# (mpc_dyn: 2 (Gx' Q (Gx u) + R u) as two parallel convolutions before phase 1, the rows' partial
# sums on wave 0 during phase 1) against mpc_p (rows over H0T) and the product.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4q; mkdir -p $OUT
V=scripts/micro/variants
S="30,3,1 30,3,1024 20,10,3 50,256,1 50,256,3"
for v in dyn p; do
  echo "== mpc tests on mpc_$v"
  DRCVAR_DIAG_LIB=$V/mpc_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_mpc.py tests/test_mpc_cluster.py > $OUT/tests_$v.log 2>&1; rc=$?
  tail -3 $OUT/tests_$v.log
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit 2
done
for r in 1 2; do
  for v in product p dyn; do
    lib=""; [ $v != product ] && lib=$V/mpc_$v.so
    echo "== mpc_bench $v run $r"
    DRCVAR_DIAG_LIB=$lib timeout -k 10 300 python3 -u scripts/mpc_bench.py --shapes $S > $OUT/bench_${v}_$r.log 2>&1 \
      || { tail -20 $OUT/bench_${v}_$r.log; exit 3; }
    grep -v amdgpu.ids $OUT/bench_${v}_$r.log | cut -c1-60
  done
done
for v in dyn_stamps; do
  echo "== mpc stamps $v"
  DRCVAR_DIAG_LIB=$V/mpc_$v.so timeout -k 10 300 python3 scripts/mpc_stamps.py 50,256,1 npz:tests/golden/qp_c5_degenerate.npz:fixture 30,3,1 \
    > $OUT/stamps_$v.log 2>&1 || { tail -20 $OUT/stamps_$v.log; exit 4; }
  grep -v amdgpu.ids $OUT/stamps_$v.log
done

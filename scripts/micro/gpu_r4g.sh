#!/usr/bin/env bash
# Round 4 (re-entry): (1) VERDICT r3 item 2b on the current tree — the per-wave bitonic sort's price
# by stamps, its parity, C3 per step in bench.py's graph form against the product; (2) the MPC
# phase stamps of the C5 QP after this round's overlapped factorisation (what the factorisation
# still costs on the chain), and mpc_bench of the product.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4g; mkdir -p $OUT
V=scripts/micro/variants
for v in stamps bitonic_stamps; do
  echo "== stamps $v"
  DRCVAR_DIAG_LIB=$V/hs_$v.so timeout -k 10 300 python3 scripts/stamps.py --shape 10,20,1000 > $OUT/stamps_$v.log 2>&1 \
    || { tail -20 $OUT/stamps_$v.log; exit 2; }
  grep -v amdgpu.ids $OUT/stamps_$v.log | tail -14
done
DRCVAR_DIAG_LIB=$V/hs_bitonic.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > $OUT/bitonic_tests.log 2>&1 || { tail -30 $OUT/bitonic_tests.log; exit 3; }
tail -1 $OUT/bitonic_tests.log
for r in 1 2 3; do
  for v in product bitonic; do
    lib=""; [ $v != product ] && lib="--lib $V/hs_$v.so"
    timeout -k 10 300 python3 bench.py --steps 2000 --warmup 50 --no-large --no-cpu-baseline --no-strong --no-mpc $lib \
      > $OUT/c3_${v}_$r.json 2> $OUT/c3_${v}_$r.err || { tail -20 $OUT/c3_${v}_$r.err; exit 4; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('$v', round(d['ms_per_step']*1e3,3))" $OUT/c3_${v}_$r.json
  done
done
echo "== mpc stamps"
DRCVAR_DIAG_LIB=$V/mpc_stamps.so timeout -k 10 300 python3 scripts/mpc_stamps.py npz:tests/golden/qp_c5_degenerate.npz:fixture \
  50,256,1 20,10,1 > $OUT/mpc_stamps.log 2>&1 || { tail -20 $OUT/mpc_stamps.log; exit 5; }
grep -v amdgpu.ids $OUT/mpc_stamps.log
echo "== mpc_bench product"
timeout -k 10 300 python3 -u scripts/mpc_bench.py --shapes 30,3,1 30,3,1024 20,10,3 50,256,1 50,256,3 > $OUT/mpc_bench.log 2>&1 \
  || { tail -20 $OUT/mpc_bench.log; exit 6; }
grep -v amdgpu.ids $OUT/mpc_bench.log | cut -c1-160
# (3) the blocked Riccati factorisation (variant mpc_blk): MPC GPU tests, mpc_bench, stamps
echo "== mpc tests on mpc_blk"
DRCVAR_DIAG_LIB=$V/mpc_blk.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_mpc.py tests/test_mpc_cluster.py > $OUT/blk_tests.log 2>&1; rc=$?
tail -15 $OUT/blk_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit 7
echo "== mpc_bench mpc_blk"
DRCVAR_DIAG_LIB=$V/mpc_blk.so timeout -k 10 300 python3 -u scripts/mpc_bench.py --shapes 30,3,1 30,3,1024 20,10,3 50,256,1 50,256,3 > $OUT/mpc_bench_blk.log 2>&1 \
  || { tail -20 $OUT/mpc_bench_blk.log; exit 8; }
grep -v amdgpu.ids $OUT/mpc_bench_blk.log | cut -c1-160
echo "== mpc stamps mpc_blk"
DRCVAR_DIAG_LIB=$V/mpc_blk_stamps.so timeout -k 10 300 python3 scripts/mpc_stamps.py npz:tests/golden/qp_c5_degenerate.npz:fixture \
  50,256,1 20,10,1 > $OUT/mpc_stamps_blk.log 2>&1 || { tail -20 $OUT/mpc_stamps_blk.log; exit 9; }
grep -v amdgpu.ids $OUT/mpc_stamps_blk.log

#!/usr/bin/env bash
# Round 4, VERDICT r3 item 2b/2c: (1) the per-wave bitonic sort's price by stamps (a stamps build
# of the product against the same build with -DDRCVAR_DIAG_BITONIC), its parity (the GPU engine
# tests on the sorting build: the rest of the kernel reads d[] as a multiset) and C3 per step in
# bench.py's graph form; (2) rocprofv3 --kernel-trace --stats of the driver's bench command, whose
# C3 kernel mean goes to profiles/rocprof_kernel_time.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4f; mkdir -p $OUT
V=scripts/micro/variants
for v in stamps bitonic_stamps; do
  echo "== stamps $v"
  DRCVAR_DIAG_LIB=$V/hs_$v.so timeout -k 10 300 python3 scripts/stamps.py --shape 10,20,1000 2>&1 | grep -v amdgpu.ids || exit 2
done
DRCVAR_DIAG_LIB=$V/hs_bitonic.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > $OUT/bitonic_tests.log 2>&1 || { tail -30 $OUT/bitonic_tests.log; exit 3; }
tail -1 $OUT/bitonic_tests.log
for r in 1 2 3; do
  for v in product bitonic; do
    lib=""; [ $v != product ] && lib="--lib $V/hs_$v.so"
    timeout -k 10 300 python3 bench.py --steps 2000 --warmup 50 --no-large --no-cpu-baseline $lib > $OUT/c3_$v.json 2> $OUT/c3_$v.err \
      || { tail -20 $OUT/c3_$v.err; exit 4; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('$v', round(d['ms_per_step']*1e3,3), round(d['roofline']['kernel_ms']*1e3,3))" $OUT/c3_$v.json
  done
done
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$OUT/prof_bench.json 2> $GRAFT_REPO_ROOT/$OUT/prof_bench.err \
  || { tail -20 $GRAFT_REPO_ROOT/$OUT/prof_bench.err; exit 5; }
echo "rocprof run exit 0"
cd $GRAFT_REPO_ROOT
DRCVAR_BENCH_DUMP_QP=$OUT/bench_qp.npz timeout -k 10 600 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/dump_bench.json 2> $OUT/dump_bench.err \
  || { tail -20 $OUT/dump_bench.err; exit 6; }
echo "bench QP dumped"

#!/usr/bin/env bash
# Round 4: the fused draw + evaluate launch without the paired draws' 80 KB LDS staging
# (hs_nopair: every slot its own Philox call; two workgroups per CU instead of one) against the
# product: the sampling GPU tests on the variant, bench.py's sampling leg interleaved; then the
# multi-rank rehearsal of the final tree (gloo, ranks sharing the GPU).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4p; mkdir -p $OUT
V=scripts/micro/variants
DRCVAR_DIAG_LIB=$V/hs_nopair.so timeout -k 10 600 python -u -m pytest tests/test_sampling.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > $OUT/tests_nopair.log 2>&1; rc=$?
tail -2 $OUT/tests_nopair.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit 2
for r in 1 2; do
  for v in product nopair; do
    lib=""; [ $v != product ] && lib="--lib $V/hs_$v.so"
    timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --strong-workloads c5 --no-mpc $lib \
      > $OUT/bench_${v}_$r.json 2> $OUT/bench_${v}_$r.err || { tail -20 $OUT/bench_${v}_$r.err; exit 3; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); s=d['sampling']; print('$v', 'refill', round(s['kernel_ms'],4), 'fused', round(s['fused_draw_evaluate']['kernel_ms'],4), s['fused_draw_evaluate']['records_equal_to_refill_then_evaluate'], 'evaluate', round(d['roofline_large']['kernel_ms'],4))" $OUT/bench_${v}_$r.json
  done
done
timeout -k 10 900 bash scripts/gpu_dist.sh || exit 4
cp gpurun_out/dist_2.log gpurun_out/dist_4.log $OUT/

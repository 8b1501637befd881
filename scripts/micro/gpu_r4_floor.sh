#!/usr/bin/env bash
# Round 4, VERDICT r3 item 2a: the C3 floor by truncated builds under bench.py's own graph form
# (stage 0 = dispatch + one store, 1 = + loads and mean sums, 2 = + direction, window histogram and
# scan, product = whole kernel), at the driver's K = 20 and at K = 2000, interleaved; then item 4
# (pipeline_c5.py under rocprofv3 must exit 0) and the new GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4floor; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_sampling.py::test_device_sampler_radius_tail tests/test_mpc_cluster.py -k "tail or stall" \
  > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 2; }
tail -3 $OUT/tests.log
one() {  # one <label> <lib or ""> <steps> <warmup>
  timeout -k 10 200 python3 bench.py ${2:+--lib $2} --steps $3 --warmup $4 --no-large --no-cpu-baseline > $OUT/one.json 2>$OUT/one.err || return 3
  python3 -c "import json; d=json.loads([l for l in open('$OUT/one.json') if l.startswith('{')][-1]); print('$1 K=$3 ms_per_step_us', round(d['ms_per_step']*1e3,3), 'events_us', round(d['roofline']['kernel_ms']*1e3,3))" | tee -a $OUT/floor.txt
}
for r in 1 2 3; do
  for v in stage0 stage1 stage2 product; do
    lib=""; [ $v != product ] && lib=scripts/micro/variants/hs_$v.so
    one $v "$lib" 2000 200 || exit 3
    one $v "$lib" 20 5 || exit 3
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/pipe -o run --output-format csv -- python3 scripts/micro/pipeline_c5.py > $OUT/pipe_prof.log 2>&1
echo "pipeline_c5 under rocprofv3 exit $?" | tee -a $OUT/floor.txt
tail -5 $OUT/pipe_prof.log

#!/usr/bin/env bash
# Sampler iteration: its GPU tests, the refill bench, one VALU counter pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/spmc2
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_sampling.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; echo "tests rc=$?"; tail -2 $OUT/tests.log
timeout -k 10 120 python3 scripts/micro/sampler_bench.py > $OUT/plain.log 2>&1 || exit $?
cat $OUT/plain.log
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d $OUT/valu -o run --output-format csv -- python3 scripts/micro/sampler_bench.py > $OUT/valu.log 2>&1
echo "pmc rc=$?"

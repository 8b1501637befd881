#!/usr/bin/env bash
# Sampler A/B: its GPU tests, the refill bench (product library, then the arithmetic-only
# variant scripts/micro/variants/samp_nostore.so), one VALU counter pass of the product.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/spmc3
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_sampling.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; echo "tests rc=$?"; tail -2 $OUT/tests.log
for rep in 1 2; do
  timeout -k 10 120 python3 scripts/micro/sampler_bench.py 2>&1 | grep sampler || exit 3
  DRCVAR_DIAG_LIB=scripts/micro/variants/samp_nostore.so timeout -k 10 120 python3 scripts/micro/sampler_bench.py 2>&1 | grep sampler | sed 's/^/nostore /' || exit 4
done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d $OUT/valu -o run --output-format csv -- python3 scripts/micro/sampler_bench.py > $OUT/valu.log 2>&1
echo "pmc rc=$?"

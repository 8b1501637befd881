#!/usr/bin/env bash
# C3 A/B of a variant library (VARIANT=scripts/micro/variants/<name>.so) against the product: the
# halfspace parity tests on the variant first, then the bench's metric line at K = 2000 and K = 20,
# interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
DRCVAR_DIAG_LIB=$VARIANT timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_reference_surface.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/abv_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/abv_pytest.log; [ $rc -eq 0 ] || exit $rc
one() {  # one <label> <lib or ""> <steps> <warmup>
  local lib=$2
  if [ -n "$lib" ]; then export DRCVAR_DIAG_LIB=$lib; else unset DRCVAR_DIAG_LIB; fi
  timeout -k 10 200 python3 bench.py ${DRCVAR_DIAG_LIB:+--lib $DRCVAR_DIAG_LIB} --steps $3 --warmup $4 --no-large --no-cpu-baseline 2>&1 | grep "^{" | \
    python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 K=$3', round(d['ms_per_step']*1e3,3), round(d['roofline']['kernel_ms']*1e3,3))"
}
for r in 1 2 3; do
  one product "" 2000 200 || exit 3
  one variant $VARIANT 2000 200 || exit 3
done
for r in 1 2 3; do
  one product "" 20 5 || exit 3
  one variant $VARIANT 20 5 || exit 3
done

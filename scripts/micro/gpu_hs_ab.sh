#!/usr/bin/env bash
# C3 A/B: a baseline library (scripts/micro/variants/hs_base.so) against the product, and a variant
# (hs_preload.so) — the bench's metric line at K = 2000 and K = 20, interleaved; then the halfspace
# parity tests on the variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
one() {  # one <label> <lib or ""> <steps> <warmup>
  local lib=$2
  timeout -k 10 200 python3 bench.py ${lib:+--lib $lib} --steps $3 --warmup $4 --no-large --no-cpu-baseline 2>&1 | grep "^{" | \
    python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 K=$3', round(d['ms_per_step']*1e3,3), round(d['roofline']['kernel_ms']*1e3,3))"
}
for r in 1 2 3; do
  one base scripts/micro/variants/hs_base.so 2000 200 || exit 3
  one product "" 2000 200 || exit 3
  one preload scripts/micro/variants/hs_preload.so 2000 200 || exit 3
done
for r in 1 2; do
  one base scripts/micro/variants/hs_base.so 20 5 || exit 3
  one product "" 20 5 || exit 3
  one preload scripts/micro/variants/hs_preload.so 20 5 || exit 3
done
DRCVAR_DIAG_LIB=scripts/micro/variants/hs_preload.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
if [ -f scripts/micro/variants/hs_stamps.so ]; then
  DRCVAR_STAMPS_WAVES=1 DRCVAR_DIAG_LIB=scripts/micro/variants/hs_stamps.so timeout -k 10 120 python3 scripts/stamps.py 2>&1 | grep -v amdgpu.ids
fi

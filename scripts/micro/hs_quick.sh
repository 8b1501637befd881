#!/usr/bin/env bash
# halfspace kernel iteration loop: parity tests, phase stamps, short bench (no MPC / CPU legs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_abi.py -m gpu -q -x > gpurun_out/pytest_hs.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_hs.log
[ $rc -eq 0 ] || exit 1
STAMP_SPECS="${STAMP_SPECS:-10,20,1000: 256,50,10000:}" bash scripts/gpu_stamps.sh 2>&1 | grep -v amdgpu.ids || exit 2
timeout -k 10 300 python bench.py --no-mpc --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1 || exit 3
python3 - <<'PY'
import json
r = json.loads(open('gpurun_out/bench_quick.log').read().strip().splitlines()[-1])
print('value', r['value'], 'ms', r['ms_per_step'], 'err', r.get('max_abs_err'))
print('roofline', r['roofline']['frac'], r['roofline']['kernel_ms'])
print('large', r['roofline_large']['frac'], r['roofline_large']['kernel_ms'])
PY

#!/usr/bin/env bash
# Iteration loop on the GPU box: parity tests, phase stamps and a geometry sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
bash scripts/gpu_stamps.sh 2>&1 | grep -v amdgpu.ids || exit 3
for shape in ${TUNE_SHAPES:-10,20,1000 256,50,10000}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tune_${shape//,/x} -o run --output-format csv -- python3 scripts/tune.py --shape $shape --launches 50 > gpurun_out/tune_${shape//,/x}.log 2>&1 || exit 4
  python3 - "$shape" <<'PY'
import csv, sys
shape = sys.argv[1].replace(',', 'x')
for r in csv.DictReader(open(f'gpurun_out/tune_{shape}/run_kernel_stats.csv')):
    n = r['Name']
    if 'safe_halfspace' in n:
        print(shape, n[n.index('<'):n.index('>') + 1], 'avg_us %.2f min_us %.2f' % (float(r['AverageNs']) / 1e3, float(r['MinNs']) / 1e3))
PY
done

#!/usr/bin/env bash
# MPC hand-off timing on the GPU box, plus a rocprof kernel-stats pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/mpc_bench.py ${MPC_SHAPES:+--shapes $MPC_SHAPES} > gpurun_out/mpc_bench.log 2>&1; rc=$?
cat gpurun_out/mpc_bench.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mpc_prof -o run --output-format csv -- python3 scripts/mpc_bench.py --reps 5 > gpurun_out/mpc_prof.log 2>&1 || exit 2
python3 - <<'PY'
import csv, glob
for f in glob.glob('gpurun_out/mpc_prof/**/run_kernel_stats.csv', recursive=True) + glob.glob('gpurun_out/mpc_prof/run_kernel_stats.csv'):
    for r in csv.DictReader(open(f)):
        print(r['Name'][:60], r['Calls'], 'avg_us %.1f' % (float(r['AverageNs']) / 1e3), 'min_us %.1f' % (float(r['MinNs']) / 1e3), 'max_us %.1f' % (float(r['MaxNs']) / 1e3))
    break
PY

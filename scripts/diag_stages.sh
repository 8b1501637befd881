#!/usr/bin/env bash
# Diagnostic: kernel time by truncation stage (0 = dispatch only, 1 = +load/moments,
# 2 = +histogram/scan, 3 = full), for C3 and C5 shapes, under rocprofv3 kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/diag; mkdir -p $OUT
SRC="dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd/csrc/drcvar_halfspace.hip dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd/csrc/drcvar_mpc.hip dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd/csrc/drcvar_sampling.hip"
for st in 0 1 2 3; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -I include -DDRCVAR_DIAG_STAGE=$st $SRC -o /tmp/diag_s$st.so || exit 1
done
for shape in ${SHAPES:-10,20,1000 256,50,10000}; do
  for st in 0 1 2 3; do
    DRCVAR_DIAG_LIB=/tmp/diag_s$st.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/s${st}_${shape//,/x} -o run --output-format csv -- python3 scripts/tune.py --shape $shape --launches 50 --only-auto > $OUT/s${st}_${shape//,/x}.log 2>&1 || exit 2
  done
done
python3 - <<'PY'
import csv, glob, os
for f in sorted(glob.glob('gpurun_out/diag/*/run_kernel_stats.csv')):
    for r in csv.DictReader(open(f)):
        if 'safe_halfspace' in r['Name']:
            print(os.path.basename(os.path.dirname(f)), r['Calls'], 'avg_us', float(r['AverageNs'])/1e3, 'min_us', float(r['MinNs'])/1e3)
PY

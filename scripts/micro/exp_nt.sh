#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SRC="dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd/csrc/drcvar_halfspace.hip dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd/csrc/drcvar_mpc.hip dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd/csrc/drcvar_sampling.hip"
for v in base nt; do
  if [ $v = nt ]; then F=-DDRCVAR_NT_LOADS; else F=; fi
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -I include $F $SRC -o /tmp/exp_$v.so || exit 1
done
for w in c5 c3 c5 c3; do for v in base nt; do
  timeout -k 10 200 python bench.py --lib /tmp/exp_$v.so --workload $w --steps 200 --warmup 10 --graph-batch 10 --no-large --no-cpu-baseline --no-mpc > gpurun_out/exp_${v}_$w.log 2>&1 || exit 2
  python3 -c "import json,sys; r=json.loads(open('gpurun_out/exp_${v}_$w.log').read().strip().splitlines()[-1]); print('$v $w', r['value'], r['roofline']['frac'], r['roofline']['kernel_ms'])"
done; done

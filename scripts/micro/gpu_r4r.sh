#!/usr/bin/env bash
# Round 4: cluster-size sweep of the clustered QP on the final tree (mpc_bench --cluster): with the
# round-4 iteration, are 16 workgroups per C5 problem still the right count?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4r; mkdir -p $OUT
for r in 1 2; do
  for c in 4 6 8 12 16 24 32; do
    echo "== cluster $c run $r"
    timeout -k 10 300 python3 -u scripts/mpc_bench.py --cluster $c --shapes 50,256,1 50,256,3 20,100,1 > $OUT/c${c}_$r.log 2>&1 \
      || { tail -20 $OUT/c${c}_$r.log; exit 2; }
    grep -v amdgpu.ids $OUT/c${c}_$r.log | cut -c1-70
  done
done

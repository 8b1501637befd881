#!/usr/bin/env bash
# Round 4: interior-point tolerance sweep on the final tree (mpc_bench --tol; the polish makes the
# answer exact, so the interior-point phase may stop earlier if the polish still succeeds at once).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4t; mkdir -p $OUT
for tol in 1e-7 2e-7 3e-7 5e-7; do
  echo "== tol $tol"
  timeout -k 10 300 python3 -u scripts/mpc_bench.py --tol $tol --shapes 30,3,1 30,3,1024 20,10,3 50,256,1 50,256,3 \
    > $OUT/tol_$tol.log 2>&1 || { tail -20 $OUT/tol_$tol.log; exit 2; }
  grep -v amdgpu.ids $OUT/tol_$tol.log | cut -c1-200
done

#!/usr/bin/env bash
# gpu_r5_cl.sh <outdir>: cluster-size sweep of the C5 QP on the round-5 iteration (two passes)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5cl}; mkdir -p $OUT
for r in 1 2; do for c in 8 12 16 20 24 32; do
  timeout -k 10 200 python3 scripts/mpc_bench.py --cluster $c --shapes npz:tests/golden/qp_c5_degenerate.npz 50,256,3 > $OUT/cl${c}_$r.log 2>&1 || exit $?
done; done
for c in 8 12 16 20 24 32; do echo "cluster $c"; grep -h "ms/launch" $OUT/cl${c}_*.log | sed 's/QPs\/s.*//'; done

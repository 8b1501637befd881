#!/usr/bin/env bash
# gpu_r5_tag.sh <outdir>: the clustered-form tests and the C5 shapes (tagged scalar exchanges)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5tag}; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_mpc_cluster.py tests/test_mpc.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/mpc_bench.py --shapes npz:tests/golden/qp_c5_degenerate.npz 50,256,1 50,256,3 30,3,1024 > $OUT/mpc_bench.log 2>&1 || exit $?
grep -v amdgpu $OUT/mpc_bench.log | sed 's/iters.*max polish/ max polish/; s/polished.*//'

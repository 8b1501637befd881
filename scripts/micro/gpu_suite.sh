#!/usr/bin/env bash
# gpu_suite.sh <outdir> [pytest -k expr]: the GPU test suite (or a subset) on the in-tree library,
# then the MPC bench shapes.  Every GPU step under its own time limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-suite}; mkdir -p $OUT
K=${2:-}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/mpc_bench.py --shapes 50,256,1 50,256,3 30,3,1024 20,10,3 > $OUT/mpc_bench.log 2>&1 || exit $?
cat $OUT/mpc_bench.log | grep -v amdgpu.ids

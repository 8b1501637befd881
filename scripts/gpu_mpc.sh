#!/usr/bin/env bash
# MPC hand-off on the GPU box: its parity tests, then the rest of the GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_mpc.py -m gpu -q -x > gpurun_out/pytest_mpc.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_mpc.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
exit $rc

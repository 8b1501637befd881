#!/usr/bin/env bash
# Sampler tests + refill bench; MPC phase stamps of the degenerate C5 fixture (stamps variant).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
: timeout -k 10 300 python -u -m pytest tests/test_sampling.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
for r in 1; do timeout -k 10 120 python3 scripts/micro/sampler_bench.py 2>&1 | grep sampler || exit 3; done
DRCVAR_DIAG_LIB=scripts/micro/variants/mpc_stamps.so timeout -k 10 300 python3 scripts/mpc_stamps.py npz:tests/golden/qp_c5_degenerate.npz:fixture 50,256,1 30,3,1 2>&1 | grep -v amdgpu.ids

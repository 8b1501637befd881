#!/usr/bin/env bash
# Round 5 baseline: MPC bench shapes and per-phase stamps of the current kernel on bench.py's C5 fixture.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5a; mkdir -p $OUT
timeout -k 10 300 python3 scripts/mpc_bench.py --shapes 50,256,1 50,256,3 30,3,1024 20,10,3 > $OUT/mpc_bench.log 2>&1 || exit $?
DRCVAR_DIAG_LIB=scripts/micro/variants/stamps_head.so timeout -k 10 300 python3 scripts/mpc_stamps.py \
  npz:tests/golden/qp_c5_degenerate.npz:fixture 50,256,1 > $OUT/stamps.log 2>&1 || exit $?
echo done

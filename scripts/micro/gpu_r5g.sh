#!/usr/bin/env bash
# per-phase and per-wave stamps of the pipelined build: the bench's C5 fixture, a C5 problem, the batch
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5g; mkdir -p $OUT
for sh in npz:tests/golden/qp_c5_degenerate.npz:fixture 30,3,1024 30,3,1; do
  DRCVAR_DIAG_LIB=scripts/micro/variants/stamps_pipe.so timeout -k 10 300 python3 scripts/mpc_stamps.py $sh > $OUT/stamps_$(echo $sh | tr ':/,' '___').log 2>&1 || exit $?
done
grep -h -v amdgpu $OUT/stamps_*.log

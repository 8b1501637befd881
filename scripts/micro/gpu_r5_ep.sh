#!/usr/bin/env bash
# gpu_r5_ep.sh <outdir>: early polish on stall: MPC GPU tests, mpc_bench (with the straggler fixture),
# stamps of the C5 fixture, bench.py's MPC hand-off legs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5ep}; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mpc or smoke" > $OUT/pytest_mpc.log 2>&1
rc=$?; tail -3 $OUT/pytest_mpc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/mpc_bench.py --shapes npz:tests/golden/qp_c5_degenerate.npz npz:tests/golden/qp_h30_straggler.npz 50,256,1 50,256,3 30,3,1024 20,10,3 30,3,1 > $OUT/mpc_bench.log 2>&1 || exit $?
grep -v amdgpu $OUT/mpc_bench.log | sed 's/max|u.*//'
DRCVAR_DIAG_LIB=scripts/micro/variants/stamps_iso.so timeout -k 10 300 python3 scripts/mpc_stamps.py npz:tests/golden/qp_c5_degenerate.npz:fixture > $OUT/stamps_c5.log 2>&1 || exit $?
grep "total\|P1 span\|exchanges  \|polish" $OUT/stamps_c5.log
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20.json 2> $OUT/bench20.err || exit $?
echo bench ok

#!/usr/bin/env bash
# gpu_r5_base.sh <outdir>: the whole GPU suite, smoke, the driver's bench command and the MPC
# bench shapes on the in-tree library.  Each GPU step under its own limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5base}; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 300 python3 scripts/mpc_bench.py --shapes npz:tests/golden/qp_c5_degenerate.npz 50,256,1 50,256,3 30,3,1024 20,10,3 30,3,1 > $OUT/mpc_bench.log 2>&1 || exit $?
grep -v amdgpu $OUT/mpc_bench.log | sed 's/max|u.*//'

#!/usr/bin/env bash
# gpu_r5_final.sh <outdir>: the round's final-tree evidence in one call: the whole GPU suite, smoke,
# the driver's bench command, the default bench (2000 timed steps) and the MPC bench shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5final}; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_steps20.json 2> $OUT/bench_steps20.err || exit $?
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit $?
timeout -k 10 300 python3 scripts/mpc_bench.py --shapes npz:tests/golden/qp_c5_degenerate.npz npz:tests/golden/qp_h30_straggler.npz 50,256,1 50,256,3 30,3,1024 20,10,3 30,3,1 > $OUT/mpc_bench.log 2>&1 || exit $?
grep -v amdgpu $OUT/mpc_bench.log | sed 's/iters.*max polish/ max polish/; s/polished.*//'

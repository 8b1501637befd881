#!/usr/bin/env bash
# Dump bench.py's C5 QP hand-off problem and re-solve it with several cluster sizes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
DRCVAR_BENCH_DUMP_QP=gpurun_out/c5qp.npz timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/c5qp_bench.log 2>&1 || { tail -20 gpurun_out/c5qp_bench.log; exit 2; }
grep -o '"full_loop_c5": {[^}]*}' gpurun_out/c5qp_bench.log
timeout -k 10 300 python -u scripts/micro/c5_qp_check.py gpurun_out/c5qp.npz

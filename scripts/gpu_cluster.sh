#!/usr/bin/env bash
# Clustered QP session: the cluster parity tests, then the MPC timings clustered and on one
# workgroup (--cluster 1), then the rest of the MPC GPU suite.  Each GPU step is bounded
# and a failure other than "tests failed" stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/cl
mkdir -p $OUT
run() {  # run <name> <timeout> <cmd...>
  local name=$1 limit=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return $rc
}
SHAPES="50,256,1 50,256,3 20,100,1 30,64,2 30,3,1 30,3,1024"
run cluster_tests 400 python -u -m pytest tests/test_mpc_cluster.py -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
run bench_cl 200 python -u scripts/mpc_bench.py --shapes $SHAPES
run bench_one 200 python -u scripts/mpc_bench.py --cluster 1 --shapes $SHAPES
run mpc_tests 600 python -u -m pytest tests/test_mpc.py -m gpu -x -q --timeout 120 --timeout-method thread
grep -h "ms/launch" $OUT/bench_cl.log $OUT/bench_one.log
MPC_SHAPES="50,256,1 30,3,1" timeout -k 10 400 bash scripts/gpu_mpc_stamps.sh > $OUT/stamps.log 2>&1; tail -42 $OUT/stamps.log

#!/usr/bin/env bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel trace.
# Every GPU step has its own time limit; anything but "tests failed" (rc 1) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 limit=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-"pytest smoke bench prof"}
for s in $STEPS; do
  case $s in
    pytest) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    cluster) step pytest_cluster 600 python -u -m pytest tests/test_mpc_cluster.py tests/test_mpc.py -m gpu -x -v --timeout 120 --timeout-method thread ;;
    mpcbench) step mpc_bench 300 python -u scripts/mpc_bench.py --shapes 30,3,1 30,3,1024 50,256,1 50,256,3 ;;
    bench20) step bench20 600 python bench.py --steps 20 --warmup 5 ;;
    cold) step cold_start 300 python -u scripts/micro/cold_start.py ;;
    dist) step dist 900 bash scripts/gpu_dist.sh ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    bench_all) for w in c2 c3 c4 c5; do step bench_$w 600 python bench.py --workload $w --no-cpu-baseline; done ;;
    prof) step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline ;;
  esac
done
echo "=== done"

#!/usr/bin/env bash
# Round-end GPU session: parity tests, smoke, benches, rocprof kernel trace and PMC traffic passes.
# Every GPU step has its own time limit; anything but "tests failed" stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
step() {  # step <name> <timeout> <cmd...>
  local name=$1 limit=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in ${STEPS:-pytest smoke bench bench_c5 prof mpcprof pmc}; do
  case $s in
    pytest) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    bench_eager) step bench_eager 600 python bench.py --launch eager --no-large --no-cpu-baseline ;;
    bench_c5) step bench_c5 600 python bench.py --workload c5 --steps 200 --warmup 10 --graph-batch 10 --no-large --no-cpu-baseline ;;
    prof) step rocprof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 2000 --no-cpu-baseline ;;
    prof20) step rocprof20 600 rocprofv3 --kernel-trace --stats -d $OUT/prof20 -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench20) step bench20 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    samppmc) step sampler_pmc 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sampler_pmc -o run --output-format csv -- python3 scripts/micro/sampler_bench.py ;;
    dist) step dist 900 bash scripts/gpu_dist.sh ;;
    mpcprof) step mpc_bench 300 rocprofv3 --kernel-trace --stats -d $OUT/mpcprof -o run --output-format csv -- python3 scripts/mpc_bench.py ;;
    pmc)
      for w in c3 c5; do
        step pmc_fetch_$w 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 20 --warmup 2 --graph-batch 10 --no-large --no-cpu-baseline
        step pmc_write_$w 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 20 --warmup 2 --graph-batch 10 --no-large --no-cpu-baseline
        python3 scripts/pmc_traffic.py $w $OUT/pmc_fetch_$w $OUT/pmc_write_$w
      done ;;
  esac
done
echo "=== done"

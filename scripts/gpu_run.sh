#!/usr/bin/env bash
# gpu_run.sh <outdir> [step ...]: the one parameterised GPU-box runner (replaces the per-session
# one-offs of rounds 1-5, which stay in git history).  Every GPU step runs under its own time
# limit; a failing step stops the script (nothing further touches the GPU in that call).
#
#   suite        pytest -m gpu (K="<expr>" narrows it)          smoke      __graft_entry__.smoke()
#   bench20      the driver's command (bench_steps20.json)      bench      the default bench.py
#   mpc          scripts/mpc_bench.py on the product library, then on each VARIANTS=<a.so b.so>,
#                interleaved ROUNDS=<n> times
#   mpctests     the MPC GPU tests only (on DRCVAR_DIAG_LIB when LIB=<a.so> is given)
#   stamps       MPC phase stamps of STAMPS=<stamps build .so> on the C5 fixture and the batch
#   kernel_time  the driver's command under a GRBM counter pass and a kernel trace
#                (scripts/kernel_time.py turns them into profiles/kernel_time.json)
#   pmc          FETCH_SIZE / WRITE_SIZE passes of c3 c4 c5 (profiles/pmc_traffic.json)
#   sampler      scripts/micro/sampler_bench.py (VARIANTS as for mpc)
#   dist         scripts/gpu_dist.sh (gloo, 2 and 4 ranks sharing cuda:0)
#   shard        scripts/micro/shard_kernel_times.py (per-rank shard kernels of the strong legs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:?outdir}; shift; mkdir -p $OUT
MPC_SHAPES=${MPC_SHAPES:-"npz:tests/golden/qp_c5_degenerate.npz npz:tests/golden/qp_h30_straggler.npz 50,256,1 50,256,3 30,3,1024 20,10,3 30,3,1"}
CMD="python3 bench.py --gpus 1 --steps 20 --warmup 5"
# counter passes go through an input file: rocprofv3 then runs the program as a child process
# (with --pmc on the command line its launcher replaces itself by the program after touching the
# GPU, which the box refuses and reports)
pmcfile() { local f=$OUT/pmc_$(echo "$*" | tr ' ' '_').txt; echo "pmc: $*" > $f; echo $f; }
fail() { echo "stopping: $1"; exit ${2:-2}; }
for s in "$@"; do
  echo "=== $s ($(date +%T))"
  case $s in
    suite)
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} \
        > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; fail suite; }
      tail -1 $OUT/pytest_gpu.log ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; fail smoke; }
      tail -1 $OUT/smoke.log ;;
    bench20)
      timeout -k 10 600 $CMD > $OUT/bench_steps20.json 2> $OUT/bench_steps20.err || { tail $OUT/bench_steps20.err; fail bench20; } ;;
    bench)
      timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; fail bench; } ;;
    mpc)
      for r in $(seq 1 ${ROUNDS:-1}); do
        timeout -k 10 300 python3 scripts/mpc_bench.py --shapes $MPC_SHAPES > $OUT/mpc_product_$r.log 2>&1 || fail mpc
        for v in ${VARIANTS:-}; do
          DRCVAR_DIAG_LIB=$v timeout -k 10 300 python3 scripts/mpc_bench.py --shapes $MPC_SHAPES \
            > $OUT/mpc_$(basename $v .so)_$r.log 2>&1 || fail "mpc $v"
        done
      done
      grep -H "ms/launch" $OUT/mpc_*.log | sed 's/max|u.*//' ;;
    mpctests)
      DRCVAR_DIAG_LIB=${LIB:-} timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        -k "mpc or smoke" > $OUT/pytest_mpc.log 2>&1 || { tail -30 $OUT/pytest_mpc.log; fail mpctests; }
      tail -1 $OUT/pytest_mpc.log ;;
    stamps)
      for sh in npz:tests/golden/qp_c5_degenerate.npz:fixture 30,3,1024; do
        DRCVAR_DIAG_LIB=${STAMPS:?STAMPS=<stamps .so>} timeout -k 10 300 python3 scripts/mpc_stamps.py $sh \
          > $OUT/stamps_$(echo $sh | tr ':/,' '___').log 2>&1 || fail stamps
      done
      grep -h "total\|P1 span\|solves (ipm)\|exchanges \|factor" $OUT/stamps_*.log ;;
    kernel_time)
      timeout -s KILL 600 rocprofv3 -i $(pmcfile GRBM_COUNT GRBM_GUI_ACTIVE) --kernel-trace -d $OUT/busy -o run \
        --output-format csv -- $CMD > $OUT/busy_bench.json 2> $OUT/busy_bench.err || fail kernel_time
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv \
        -- $CMD > $OUT/trace_bench.json 2> $OUT/trace_bench.err || fail kernel_time ;;
    pmc)
      for w in c3 c4 c5; do
        for k in FETCH_SIZE WRITE_SIZE; do
          timeout -s KILL 600 rocprofv3 -i $(pmcfile $k) -d $OUT/pmc_${k}_$w -o run --output-format csv -- python3 bench.py \
            --workload $w --steps 20 --warmup 2 --graph-batch 10 --no-large --no-cpu-baseline > $OUT/pmc_${k}_$w.log 2>&1 || fail pmc
        done
        python3 scripts/pmc_traffic.py $w $OUT/pmc_FETCH_SIZE_$w $OUT/pmc_WRITE_SIZE_$w || fail pmc
      done
      cp profiles/pmc_traffic.json $OUT/ ;;
    sampler)
      for v in "" ${VARIANTS:-}; do
        DRCVAR_DIAG_LIB=$v timeout -k 10 300 python3 scripts/micro/sampler_bench.py > $OUT/sampler_$(basename ${v:-product} .so).log 2>&1 || fail sampler
      done
      grep -H . $OUT/sampler_*.log | grep -v amdgpu ;;
    dist)
      OUTDIR=$OUT timeout -k 10 1000 bash scripts/gpu_dist.sh || fail dist ;;
    shard)
      timeout -k 10 300 python3 scripts/micro/shard_kernel_times.py > $OUT/shard_kernel_times.json 2> $OUT/shard.err \
        || { tail $OUT/shard.err; fail shard; } ;;
    *) fail "unknown step $s" ;;
  esac
done
echo "=== done"

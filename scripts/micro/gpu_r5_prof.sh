#!/usr/bin/env bash
# gpu_r5_prof.sh <outdir>: (1) MPC phase stamps of the current kernel (stamps build) on the bench's
# C5 fixture and the 1024-problem batch; (2) the driver's bench command under a GRBM counter pass
# and under a plain kernel trace (scripts/kernel_time.py -> profiles/kernel_time.json); (3) the
# FETCH_SIZE / WRITE_SIZE passes of C3, C4 and C5 (profiles/pmc_traffic.json).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
R=$PWD
OUT=gpurun_out/${1:-r5prof}; mkdir -p $OUT
for sh in npz:tests/golden/qp_c5_degenerate.npz:fixture 30,3,1024; do
  DRCVAR_DIAG_LIB=scripts/micro/variants/stamps_cur.so timeout -k 10 300 python3 scripts/mpc_stamps.py $sh > $OUT/stamps_$(echo $sh | tr ':/,' '___').log 2>&1 || exit $?
done
echo stamps done
CMD="python3 bench.py --gpus 1 --steps 20 --warmup 5"
timeout -s KILL 600 rocprofv3 --pmc GRBM_COUNT GRBM_GUI_ACTIVE --kernel-trace -d $OUT/busy -o run --output-format csv -- $CMD > $OUT/busy_bench.json 2> $OUT/busy_bench.err || exit $?
echo busy done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $CMD > $OUT/trace_bench.json 2> $OUT/trace_bench.err || exit $?
echo trace done
for w in c3 c4 c5; do
  timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 20 --warmup 2 --graph-batch 10 --no-large --no-cpu-baseline > $OUT/pmc_fetch_$w.log 2>&1 || exit $?
  timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 20 --warmup 2 --graph-batch 10 --no-large --no-cpu-baseline > $OUT/pmc_write_$w.log 2>&1 || exit $?
  python3 scripts/pmc_traffic.py $w $OUT/pmc_fetch_$w $OUT/pmc_write_$w || exit $?
done
cp profiles/pmc_traffic.json $OUT/
echo pmc done
grep -h "total\|P1 span\|P1 resid\|solves (ipm)\|exchanges \|factor" $OUT/stamps_*.log

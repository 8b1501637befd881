#!/usr/bin/env bash
# Counter passes over the device sampler (scripts/micro/sampler_bench.py: 23 refills of a resident
# 256 x 50 x 10000 batch, 2.05 GB each), one pass per counter group, plus the C3 launch-geometry
# sweep (scripts/tune.py, HIP events).  Summaries: python3 scripts/pmc_sampler.py gpurun_out/spmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/spmc
mkdir -p $OUT
rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
timeout -k 10 120 python3 scripts/micro/sampler_bench.py > $OUT/plain.log 2>&1 || exit $?
pass() {  # pass <name> <counters...>
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $OUT/$name -o run --output-format csv -- \
    python3 scripts/micro/sampler_bench.py > $OUT/$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
pass valu SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE && \
pass f64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_VMEM_WR && \
pass fetch FETCH_SIZE && \
pass write WRITE_SIZE && \
timeout -k 10 300 python3 scripts/tune.py --shape 10,20,1000 --launches 2000 > $OUT/tune_c3.log 2>&1
rc=$?
grep -h geometry $OUT/tune_c3.log
cat $OUT/plain.log
exit $rc

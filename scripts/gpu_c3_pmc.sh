#!/usr/bin/env bash
# Counter passes over the C3 launches of the halfspace kernel (bench.py --workload c3), one pass per
# counter group (at most 8 SQ counters each), to back the "latency-bound" reading of the headline
# kernel with counters: how much of each wave's life is spent waiting, and on what.
# Summary: python3 scripts/pmc_c3.py gpurun_out/c3pmc  (-> profiles/r02/c3_latency_pmc.json)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/c3pmc
mkdir -p $OUT
rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
pass() {  # pass <name> <counters...>; a counter this box does not list skips the pass
  local name=$1; shift
  for c in "$@"; do
    grep -qw "$c" $OUT/avail.txt || { echo "pass $name skipped: $c not listed"; return 0; }
  done
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $OUT/$name -o run --output-format csv -- \
    python3 bench.py --workload c3 --steps 200 --warmup 10 --graph-batch 10 --no-large --no-cpu-baseline \
    > $OUT/$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
pass wait SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE && \
pass mix SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT

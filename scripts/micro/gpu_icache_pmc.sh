#!/usr/bin/env bash
# Instruction-fetch counters of the C3 launches: the counters the box offers for the SQ/SQC
# instruction path, then one --pmc pass over a short bench run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/pmc_list.txt 2>&1
grep -i -E "icache|ifetch|SQC_INST|INST_LEVEL|WAIT_INST" gpurun_out/pmc_list.txt | head -40
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_IFETCH SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES \
  -d gpurun_out/pmc_icache -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --graph-batch 10 --no-large --no-cpu-baseline > gpurun_out/pmc_icache.log 2>&1
echo "pmc rc=$?"

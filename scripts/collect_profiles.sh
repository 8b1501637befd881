#!/usr/bin/env bash
# Copy the judged summaries of a scripts/gpu_run.sh session from gpurun_out/ (scratch) into
# profiles/<round>/ (tracked):  bash scripts/collect_profiles.sh r01
set -eu
cd "$(dirname "$0")/.."
R=${1:?round tag, e.g. r01}
D=profiles/$R
mkdir -p "$D"
O=gpurun_out
[ -f $O/bench.log ] && grep '^{' $O/bench.log | tail -1 > $D/bench_c3.json
[ -f $O/bench_c5.log ] && grep '^{' $O/bench_c5.log | tail -1 > $D/bench_c5.json
[ -f $O/prof/run_kernel_stats.csv ] && cp $O/prof/run_kernel_stats.csv $D/bench_c3_graph_kernel_stats.csv
[ -f $O/prof/run_domain_stats.csv ] && cp $O/prof/run_domain_stats.csv $D/bench_c3_graph_domain_stats.csv
[ -f $O/mpc_bench.log ] && grep -v amdgpu.ids $O/mpc_bench.log > $D/mpc_bench.log
[ -f $O/mpcprof/run_kernel_stats.csv ] && cp $O/mpcprof/run_kernel_stats.csv $D/mpc_bench_kernel_stats.csv
for w in c3 c5; do
  for k in fetch write; do
    f=$(find $O/pmc_${k}_$w -name '*counter_collection.csv' 2>/dev/null | head -1)
    [ -n "$f" ] && cp "$f" $D/pmc_${k}_$w.csv
  done
  [ -d $O/pmc_fetch_$w ] && python3 scripts/pmc_traffic.py $w $O/pmc_fetch_$w $O/pmc_write_$w
done
ls -la "$D"

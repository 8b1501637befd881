#!/usr/bin/env bash
# Round 4 MPC A/B: GPU MPC tests on the product, then scripts/mpc_bench.py and bench.py's hand-off
# legs for the product against variants (scripts/micro/variants/<name>.so; VARIANTS="r3 start").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4mpc; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_mpc.py tests/test_mpc_cluster.py > $OUT/tests.log 2>&1; rc=$?
tail -15 $OUT/tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit 2
for v in product ${VARIANTS:-}; do
  lib=""; [ $v != product ] && lib=scripts/micro/variants/mpc_$v.so
  echo "== mpc_bench $v"
  DRCVAR_DIAG_LIB=$lib timeout -k 10 300 python3 -u scripts/mpc_bench.py --shapes 30,3,1 30,3,1024 20,10,3 50,256,1 50,256,3 2>&1 | grep -v amdgpu.ids || exit 3
done
for v in product ${VARIANTS:-}; do
  lib=""; [ $v != product ] && lib=scripts/micro/variants/mpc_$v.so
  timeout -k 10 400 python3 bench.py ${lib:+--lib $lib} --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_$v.json 2>$OUT/bench_$v.err || exit 4
  python3 - $OUT/bench_$v.json $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
m = d["mpc_handoff"]
c5 = m["full_loop_c5"]
print(sys.argv[2], "C5 full", round(c5["full_step_ms"], 4), "qp", round(c5["qp_ms"], 4), "iters", c5["qp_iterations"],
      c5["qp_status"], "polish", c5["polish_attempts"], "main_flow", round(m["main_flow_c5"]["step_ms"], 4),
      m["main_flow_c5"]["qp_iterations"], "batched", round(m["batched_reference"]["launch_ms"], 4),
      m["batched_reference"]["mean_iterations"], m["batched_reference"]["optimal_frac"])
PY
done

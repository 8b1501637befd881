#!/usr/bin/env bash
# Round 4 checkpoint: the whole GPU suite, smoke(), mpc_bench against the overlap build (at the new
# default tolerance), and bench.py at the driver's command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4e; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 2; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 3; }
tail -1 $OUT/smoke.log
S="30,3,1 30,3,1024 20,10,3 50,256,1 50,256,3"
for v in product overlap; do
  lib=""; [ $v != product ] && lib=scripts/micro/variants/mpc_$v.so
  echo "== mpc_bench $v (tol 1e-7)"
  DRCVAR_DIAG_LIB=$lib timeout -k 10 300 python3 -u scripts/mpc_bench.py --tol 1e-7 --shapes $S 2>&1 | grep -v amdgpu.ids | cut -c1-120 || exit 4
done
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 5; }
python3 - $OUT/bench_driver.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
m = d["mpc_handoff"]
print("value", round(d["value"] / 1e6, 2), "M/s  ms_per_step", round(d["ms_per_step"] * 1e3, 3), "us  frac", round(d["roofline"]["frac"], 4),
      "| C5 full", round(m["full_loop_c5"]["full_step_ms"], 4), "qp", round(m["full_loop_c5"]["qp_ms"], 4), m["full_loop_c5"]["qp_iterations"],
      "err_u", m["full_loop_c5"].get("max_abs_err_u_vs_oracle"), "| main_flow", round(m["main_flow_c5"]["step_ms"], 4), m["main_flow_c5"]["qp_iterations"],
      "| batched", round(m["batched_reference"]["launch_ms"], 4), "| max_abs_err", d.get("max_abs_err"))
sm = d["sampling"]
print("sampler", round(sm["kernel_ms"], 4), "ms; C5 evaluate", round(d["roofline_large"]["kernel_ms"], 4),
      "ms; fused draw+evaluate", sm["fused_draw_evaluate"])
PY

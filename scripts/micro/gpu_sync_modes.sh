#!/usr/bin/env bash
# K = 20 / K = 2000 timed regions (scripts/micro/c_loop.py) under the runtime's completion-wait
# modes: default, HSA_ENABLE_INTERRUPT=0 (signal waits poll instead of sleeping on an interrupt).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for r in 1 2; do
  echo "== default"; timeout -k 10 200 python3 scripts/micro/c_loop.py 2>&1 | grep "warm=graph" || exit 3
  echo "== HSA_ENABLE_INTERRUPT=0"; HSA_ENABLE_INTERRUPT=0 timeout -k 10 200 python3 scripts/micro/c_loop.py 2>&1 | grep "warm=graph" || exit 3
done
echo "== bench.py --steps 20 --warmup 5, default then HSA_ENABLE_INTERRUPT=0"
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-large --no-cpu-baseline | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', round(d['ms_per_step']*1e3,3))" || exit 3
  HSA_ENABLE_INTERRUPT=0 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-large --no-cpu-baseline | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('polling', round(d['ms_per_step']*1e3,3))" || exit 3
done

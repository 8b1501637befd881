#!/usr/bin/env bash
# Rehearse the multi-rank bench path on a one-GPU box: gloo, ranks sharing cuda:0.  2 ranks: the
# metric line (each rank its own C3 block) and the strong_scaling line (the global C5 batch
# sharded over the ranks + the all-gather + the full MPC loop); 4 ranks: the metric line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29502 bench.py --gpus 2 --steps 400 --warmup 50 --dist-backend gloo --no-cpu-baseline \
  > gpurun_out/dist_2.log 2>&1 || { tail -30 gpurun_out/dist_2.log; exit 2; }
grep '^{' gpurun_out/dist_2.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); s = d['strong_scaling']
print(2, d['value'], d['ms_per_step'], d['config']['parallelism'], d['n_gpus'])
print(2, 'strong', s['value'], s['ms_per_step'], s['parallelism'], s['units_per_rank'], s.get('full_loop'))"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29504 bench.py --gpus 4 --steps 400 --warmup 50 --dist-backend gloo --no-large \
  > gpurun_out/dist_4.log 2>&1 || { tail -30 gpurun_out/dist_4.log; exit 3; }
grep '^{' gpurun_out/dist_4.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print(4, d['value'], d['ms_per_step'], d['config']['parallelism'], d['n_gpus'])"

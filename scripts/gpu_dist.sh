#!/usr/bin/env bash
# Rehearse the multi-rank bench path on a one-GPU box: gloo, 2 and 4 ranks sharing cuda:0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 2 4; do
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 400 --warmup 50 --dist-backend gloo --no-large > gpurun_out/dist_$n.log 2>&1 || { tail -30 gpurun_out/dist_$n.log; exit 2; }
  grep '^{' gpurun_out/dist_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, d['value'], d['ms_per_step'], d['config']['parallelism'], d['n_gpus'])"
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 100 --warmup 10 --dist-backend gloo --no-large --gather > gpurun_out/dist_gather_$n.log 2>&1 || { tail -30 gpurun_out/dist_gather_$n.log; exit 3; }
  grep '^{' gpurun_out/dist_gather_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, 'gather', d['value'], d['ms_per_step'], d['config']['parallelism'])"
done
# full MPC loop (config 5 shape reduced to N=1000 for the rehearsal), 1 and 2 ranks
timeout -k 10 600 python bench.py --full-loop --workload c5 --steps 10 --warmup 2 > gpurun_out/full_1.log 2>&1 || { tail -20 gpurun_out/full_1.log; exit 4; }
grep '^{' gpurun_out/full_1.log
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29710 bench.py --gpus 2 --full-loop --workload c5 --steps 10 --warmup 2 --dist-backend gloo > gpurun_out/full_2.log 2>&1 || { tail -20 gpurun_out/full_2.log; exit 5; }
grep '^{' gpurun_out/full_2.log

#!/usr/bin/env bash
# Bench rehearsal: the driver's N=1 command, then a 2-rank gloo rehearsal of the N>1 path (two
# ranks on the one GPU), each step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/b_n1.log 2>&1; rc=$?
echo "n1 rc=$rc"; tail -c 3000 $OUT/b_n1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --no-cpu-baseline \
  --strong-steps 4 > $OUT/b_gloo2.log 2>&1; rc=$?
echo "gloo2 rc=$rc"; tail -c 2500 $OUT/b_gloo2.log; exit $rc

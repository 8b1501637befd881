#!/usr/bin/env bash
# Rehearse the multi-rank bench path on a one-GPU box: gloo, ranks sharing cuda:0.  2 ranks: the
# metric line (each rank its own C3 block) and both strong_scaling legs (the global C4 and C5
# batches sharded over the ranks, every exchange form — the RCCL-style all-gather (here gloo,
# through the host), the same pipelined by chunks, and the peer-push exchange (IPC-mapped regions,
# the ranks sharing the one GPU) — with their rank-max phase splits; C5 also the full MPC loop);
# 4 ranks: the metric line and both legs without the MPC loops; 8 ranks (the driver's largest N):
# everything, main.py's three filters on ranks 0-2 and ranks 3-7 with none (RANKS="2 4 8" default).
# Logs: $OUTDIR (default gpurun_out/dist)/dist_{2,4,8}.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUTDIR:-gpurun_out/dist}; mkdir -p $OUT
show() {  # show <ranks> <log>
  grep '^{' "$2" | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print($1, 'metric', round(d['value']), d['ms_per_step'], d['config']['parallelism'], d['scaling'], d['config']['launch'])
for w, s in (d.get('strong_scaling') or {}).items():
    print($1, 'strong', w, round(s['value']), round(s['ms_per_step'], 4), s['exchange'], s['units_per_rank'],
          s['phases_rank_max'], s.get('full_loop', {}).get('ms_per_step'))
    for k, v in (s.get('exchanges') or {}).items():
        print($1, '   ', w, k, {a: b for a, b in v.items() if a not in ('what',)})
    if s.get('main_flow'):
        print($1, 'strong', w, 'main_flow', s['main_flow']['ms_per_step'], s['main_flow']['rank0_filters'], s['main_flow']['rank0_qp_iterations'])"
}
for n in ${RANKS:-2 4 8}; do
  extra=""
  [ "$n" = 4 ] && extra="--no-mpc"
  timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 400 --warmup 50 --dist-backend gloo $extra \
    --no-cpu-baseline > $OUT/dist_$n.log 2>&1 || { tail -30 $OUT/dist_$n.log; exit $n; }
  show $n $OUT/dist_$n.log
done

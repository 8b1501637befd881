#!/usr/bin/env bash
# order_ab.sh <outdir>: the halfspace kernel's launch time per shape (scripts/tune.py, automatic
# plan, graph replays of 10) for the product library and each VARIANTS=<a.so ...> library,
# interleaved ROUNDS=<n> times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:?outdir}; mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in product ${VARIANTS:-}; do
    lib=""; [ "$v" != product ] && lib=$v
    for sh in ${SHAPES:-64,30,5000 256,50,10000 10,20,1000 32,50,10000 8,30,5000}; do
      DRCVAR_DIAG_LIB=$lib timeout -k 10 200 python3 scripts/tune.py --shape $sh --graph 10 --launches 400 --only-auto 2>&1 \
        | grep "rep 1" | sed "s|^|$(basename $v .so) r$r |" >> $OUT/order_ab.log || exit 3
    done
  done
done
cat $OUT/order_ab.log

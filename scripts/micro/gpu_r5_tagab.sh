#!/usr/bin/env bash
# A/B of the tagged scalar exchange (cluster_scalars) against the counter exchange at the scalar
# sites: product-flag builds and stamps builds of both, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5tagab}; mkdir -p $OUT
for r in 1 2 3; do for v in base tag; do
  DRCVAR_DIAG_LIB=scripts/micro/variants/$v.so timeout -k 10 300 python3 scripts/mpc_bench.py --shapes npz:tests/golden/qp_c5_degenerate.npz 50,256,1 50,256,3 > $OUT/bench_${v}_$r.log 2>&1 || exit $?
done; done
for v in stamps_base stamps_tag; do
  DRCVAR_DIAG_LIB=scripts/micro/variants/$v.so timeout -k 10 300 python3 scripts/mpc_stamps.py npz:tests/golden/qp_c5_degenerate.npz:fixture > $OUT/${v}.log 2>&1 || exit $?
done
for f in $OUT/stamps_*; do echo $f; grep "total\|cluster exch" $f; done
grep -H "ms/launch" $OUT/bench_* | sed 's/iters.*//; s/.*bench_//'

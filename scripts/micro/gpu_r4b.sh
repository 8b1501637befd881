#!/usr/bin/env bash
# Round 4: MPC phase stamps (C5 shapes), the batched-QP distribution against round 3, and the C4
# kernel against residency / nontemporal-load variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4b; mkdir -p $OUT
DRCVAR_DIAG_LIB=scripts/micro/variants/mpc_stamps.so timeout -k 10 300 python3 scripts/mpc_stamps.py \
  50,256,1 npz:tests/golden/qp_c5_degenerate.npz:fixture 30,3,1 2>&1 | grep -v amdgpu.ids | tee $OUT/stamps.log || exit 2
for v in product r3; do
  lib=""; [ $v != product ] && lib=scripts/micro/variants/mpc_$v.so
  echo "== mpc_bench $v"
  DRCVAR_DIAG_LIB=$lib timeout -k 10 300 python3 -u scripts/mpc_bench.py --shapes 30,3,1024 20,10,3 2>&1 | grep -v amdgpu.ids || exit 3
done
for r in 1 2; do
  for v in product nt occ2 occ3; do
    lib=""; [ $v != product ] && lib=scripts/micro/variants/hs_$v.so
    DRCVAR_DIAG_LIB=$lib timeout -k 10 200 python3 scripts/tune.py --shape 64,30,5000 --only-auto --graph 10 --launches 200 2>&1 | grep "rep 1" | sed "s/^/$v /" || exit 4
  done
done

#!/usr/bin/env bash
# Sampler A/B: product refill vs the nontemporal-store variant (scripts/micro/variants/samp_nt.so),
# three interleaved repetitions.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for rep in 1 2 3; do
  timeout -k 10 120 python3 scripts/micro/sampler_bench.py 2>&1 | grep sampler || exit 3
  DRCVAR_DIAG_LIB=scripts/micro/variants/samp_nt.so timeout -k 10 120 python3 scripts/micro/sampler_bench.py 2>&1 | grep sampler | sed 's/^/nt /' || exit 4
done

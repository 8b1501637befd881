#!/usr/bin/env bash
# Round 4, final tree: rocprofv3 kernel trace of mpc_bench (the QP kernels' durations) and the PMC
# HBM-traffic passes of C3 / C5 (profiles/pmc_traffic.json, copied back under gpurun_out/r4s).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
STEPS="mpcprof pmc" bash scripts/gpu_round.sh || exit $?
mkdir -p gpurun_out/r4s && cp profiles/pmc_traffic.json gpurun_out/r4s/

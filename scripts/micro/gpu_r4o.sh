#!/usr/bin/env bash
# Round 4: the blocked-factorisation / blocked-solve A/B (gpu_r4n.sh), then the round's product
# validation (gpu_round.sh: GPU suite, smoke, default bench, the driver's command, its rocprof trace).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/micro/gpu_r4n.sh || exit $?
STEPS="pytest smoke bench bench20 prof20" bash scripts/gpu_round.sh

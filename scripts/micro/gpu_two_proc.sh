#!/usr/bin/env bash
# One process alone, then two processes at once on the same GPU (scripts/micro/two_proc_qp.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
timeout -k 10 120 python3 scripts/micro/two_proc_qp.py alone || exit 3
timeout -k 10 180 python3 scripts/micro/two_proc_qp.py rankA &
pa=$!
timeout -k 10 180 python3 scripts/micro/two_proc_qp.py rankB &
pb=$!
wait $pa; ra=$?
wait $pb; rb=$?
echo "rc $ra $rb"

#!/usr/bin/env bash
# usage: run_micro.sh name.hip ...   (diagnostic microbenchmarks)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for f in "$@"; do
  hipcc --offload-arch=gfx950 -O3 scripts/micro/$f -o /tmp/${f%.hip} 2>/dev/null || exit 1
  timeout -k 10 60 /tmp/${f%.hip} || exit 2
done

#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
hipcc --offload-arch=gfx950 -O3 scripts/micro/calib.hip -o /tmp/calib || exit 1
timeout -k 10 60 /tmp/calib

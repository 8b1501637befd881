#!/usr/bin/env bash
# build_mpc_stamps.sh <name> <flags...>: a -DDRCVAR_MPC_STAMPS diagnostic library as ONE translation
# unit (the drcvar_diag_mpc_stamps export exists only in the single-unit build; build_variant.sh
# compiles the MPC source in parts), written to scripts/micro/variants/<name>.so.
set -eu
cd "$(dirname "$0")/../.."
name=$1; shift
PKG=dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd
mkdir -p scripts/micro/variants
hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -DDRCVAR_MPC_STAMPS -I include "$@" \
  $PKG/csrc/drcvar_halfspace.hip $PKG/csrc/drcvar_mpc.hip $PKG/csrc/drcvar_sampling.hip \
  -o scripts/micro/variants/$name.so
echo scripts/micro/variants/$name.so

#!/usr/bin/env bash
# build_mpc_stamps.sh <name> <flags...>: a -DDRCVAR_MPC_STAMPS diagnostic library (the product
# library with the MPC source rebuilt as its five parts, concurrently; the stamps exports live in
# the 2-input part), written to scripts/micro/variants/<name>.so.
set -eu
cd "$(dirname "$0")/../.."
name=$1; shift
exec bash scripts/micro/build_variant.sh "$name" drcvar_mpc -DDRCVAR_MPC_STAMPS "$@"

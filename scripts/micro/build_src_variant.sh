#!/usr/bin/env bash
# build_src_variant.sh <name> <path to a modified drcvar_mpc.hip> [flags...]: the product library
# with the MPC source replaced by the given file (compiled as its five parts, concurrently; the
# other sources from the cached objects of _native.build()), written to
# scripts/micro/ab/<name>.so for DRCVAR_DIAG_LIB runs.
set -eu
cd "$(dirname "$0")/../.."
name=$1; src=$2; shift 2
PKG=dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd
mkdir -p scripts/micro/ab
tmp=$(mktemp -d)
new=()
for k in 0 1 2 3 4; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -I include -I $PKG/csrc -DDRCVAR_MPC_PART=$k "$@" \
    "$src" -o $tmp/part_$k.o &
  new+=($tmp/part_$k.o)
done
for j in $(jobs -p); do wait $j || { echo "a part failed to compile" >&2; exit 1; }; done
objs=$(ls $PKG/_lib/obj/*.o | grep -v "/drcvar_mpc.hip")
hipcc --offload-arch=gfx950 -shared -fPIC $objs "${new[@]}" -o scripts/micro/ab/$name.so
rm -rf $tmp
echo scripts/micro/ab/$name.so

#!/usr/bin/env bash
# build_variant.sh <name> <source-basename> <flags...>: the product library with one source
# rebuilt with extra flags (the other sources from the cached objects of _native.build(); the MPC
# source as its five parts, concurrently), written to scripts/micro/ab/<name>.so for
# DRCVAR_DIAG_LIB runs.  The product sources carry only the stamp hooks; the other diagnostic
# switches (-DDRCVAR_DIAG_STAGE, -DDRCVAR_NO_PIPE, -DDRCVAR_POLISH_RHO, -DDRCVAR_NT_BYTES,
# -DDRCVAR_HS_LDS_PAD, -DDRCVAR_SAMPLER_NO_STORE) live in patches/diag_switches.diff, applied here
# to a temporary copy of the sources; PATCHES="<a.diff> ..." applies more (e.g.
# patches/early_polish_knobs.diff: the early polish's thresholds as -D switches).
set -eu
cd "$(dirname "$0")/../.."
name=$1; src=$2; shift 2
PKG=dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd
mkdir -p scripts/micro/ab
tmp=$(mktemp -d)
trap 'rm -rf $tmp' EXIT
cp $PKG/csrc/*.hip $PKG/csrc/*.inc $tmp/
patch -s -p1 -d $tmp < scripts/micro/patches/diag_switches.diff
for p in ${PATCHES:-}; do patch -s -p1 -d $tmp < $p; done
new=()
if [ "$src" = drcvar_mpc ]; then
  for k in 0 1 2 3 4; do
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -I include -I $tmp -DDRCVAR_MPC_PART=$k "$@" \
      $tmp/$src.hip -o $tmp/variant_${name}_$k.o &
    new+=($tmp/variant_${name}_$k.o)
  done
  for j in $(jobs -p); do wait $j || { echo "a part failed to compile" >&2; exit 1; }; done
else
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -I include -I $tmp "$@" $tmp/$src.hip -o $tmp/variant_$name.o
  new+=($tmp/variant_$name.o)
fi
objs=$(ls $PKG/_lib/obj/*.o | grep -v "/$src.hip")
hipcc --offload-arch=gfx950 -shared -fPIC $objs "${new[@]}" -o scripts/micro/ab/$name.so
echo scripts/micro/ab/$name.so

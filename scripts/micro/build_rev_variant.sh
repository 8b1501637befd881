#!/usr/bin/env bash
# build_rev_variant.sh <git-rev> <name> [source-basename, default drcvar_mpc]: the product library
# with one source taken from an earlier commit (A/B against the working tree), written to
# scripts/micro/variants/<name>.so (the other sources from the cached objects of _native.build()).
set -eu
cd "$(dirname "$0")/../.."
rev=$1; name=$2; src=${3:-drcvar_mpc}
PKG=dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd
tmp=$(mktemp -d)
mkdir -p $tmp/csrc $tmp/include
git show $rev:$PKG/csrc/$src.hip > $tmp/csrc/$src.hip
for h in include/*.h; do git show $rev:$h > $tmp/$h 2>/dev/null || cp $h $tmp/$h; done
cp $PKG/csrc/*.inc $tmp/csrc/ 2>/dev/null || true
mkdir -p scripts/micro/variants
new=()
if [ "$src" = drcvar_mpc ]; then
  for k in 0 1 2 3 4; do
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -I $tmp/include -DDRCVAR_MPC_PART=$k \
      $tmp/csrc/$src.hip -o $tmp/part_$k.o &
    new+=($tmp/part_$k.o)
  done
  for j in $(jobs -p); do wait $j || { echo "a part failed to compile" >&2; exit 1; }; done
else
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -I $tmp/include $tmp/csrc/$src.hip -o $tmp/one.o
  new+=($tmp/one.o)
fi
objs=$(ls $PKG/_lib/obj/*.o | grep -v "/$src.hip")
hipcc --offload-arch=gfx950 -shared -fPIC $objs "${new[@]}" -o scripts/micro/variants/$name.so
rm -rf $tmp
echo scripts/micro/variants/$name.so

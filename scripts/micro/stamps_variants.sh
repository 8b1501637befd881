set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=dr_cvar_mpc_safety_filter_motion_planning_collison_avoidance_amd/csrc
for v in $VARIANTS; do
  name=${v%%:*}; src=${v#*:}
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -DDRCVAR_MPC_STAMPS -I include $D/drcvar_halfspace.hip $src $D/drcvar_sampling.hip -o /tmp/st_$name.so || exit 1
  echo "== $name"
  DRCVAR_DIAG_LIB=/tmp/st_$name.so timeout -k 10 120 python3 scripts/mpc_stamps.py $SHAPES 2>&1 | grep -E "total|Riccati|groups" || exit 2
done

set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_mpc.py -m gpu -q -x > gpurun_out/pytest_mpc.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_mpc.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python scripts/mpc_bench.py > gpurun_out/mpc_bench.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/mpc_bench.log
exit $rc

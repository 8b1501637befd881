set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5e
for v in var_d var_e; do
timeout -k 10 300 python3 -u scripts/micro/pytest_variant.py scripts/micro/variants/$v.so tests/test_mpc.py -m gpu -q --timeout 120 --timeout-method thread -k "generic4 or generic8" > gpurun_out/r5e/$v.log 2>&1; echo $v; tail -3 gpurun_out/r5e/$v.log
done
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mpc or smoke" > gpurun_out/r5e/pytest_mpc_pipe.log 2>&1; echo pipe; tail -3 gpurun_out/r5e/pytest_mpc_pipe.log
timeout -k 10 300 python3 scripts/mpc_bench.py --shapes npz:tests/golden/qp_c5_degenerate.npz 50,256,1 50,256,3 30,3,1024 20,10,3 30,3,1 > gpurun_out/r5e/bench_pipe.log 2>&1; grep -v amdgpu gpurun_out/r5e/bench_pipe.log | sed 's/max|u.*//'

set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/micro/timed_overhead.py > gpurun_out/ovh_default.log 2>&1 && \
DRCVAR_SCHED=spin timeout -k 10 300 python -u scripts/micro/timed_overhead.py > gpurun_out/ovh_spin.log 2>&1 && \
DRCVAR_SCHED=yield timeout -k 10 300 python -u scripts/micro/timed_overhead.py > gpurun_out/ovh_yield.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20.log 2>&1
echo rc=$?

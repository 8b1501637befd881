cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tune3 -o run --output-format csv -- python3 scripts/tune.py --shape 10,20,1000 > gpurun_out/tune3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tune5 -o run --output-format csv -- python3 scripts/tune.py --shape 256,50,10000 --launches 30 > gpurun_out/tune5.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1; cat gpurun_out/tune3.log | grep geometry; grep geometry gpurun_out/tune5.log; cat gpurun_out/bench.log | tail -1

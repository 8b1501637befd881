#!/usr/bin/env bash
# round 5: the pipelined affine solve — generic-model tests first (isolated), then every MPC test,
# then the MPC bench; the committed tree's library (var_head) on the new generic44 cases for reference
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5f; mkdir -p $OUT
timeout -k 10 300 python3 -u scripts/micro/pytest_variant.py scripts/micro/variants/var_head.so tests/test_mpc.py -m gpu -q --timeout 120 --timeout-method thread -k "generic44" > $OUT/head_generic44.log 2>&1; echo head; tail -2 $OUT/head_generic44.log
timeout -k 10 300 python3 -u -m pytest tests/test_mpc.py -m gpu -x -q --timeout 120 --timeout-method thread -k "generic" > $OUT/generic.log 2>&1
rc=$?; echo generic; tail -2 $OUT/generic.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mpc or smoke" > $OUT/pytest_mpc.log 2>&1
rc=$?; echo mpc; tail -2 $OUT/pytest_mpc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/mpc_bench.py --shapes npz:tests/golden/qp_c5_degenerate.npz 50,256,1 50,256,3 30,3,1024 20,10,3 30,3,1 > $OUT/bench.log 2>&1 || exit $?
grep -v amdgpu $OUT/bench.log | sed 's/max|u.*//'
timeout -k 10 300 python3 scripts/micro/dump_qp_problems.py benchbatch > $OUT/dump_batch.log 2>&1; tail -1 $OUT/dump_batch.log

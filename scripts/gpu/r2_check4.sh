#!/bin/bash
# round 2: model-parallel GPU test, full GPU suite, headline bench
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_model_parallel_gpu.py -v --timeout 200 --timeout-method thread > gpurun_out/r2c4_mp.log 2>&1
rc=$?; echo "mp tests rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/r2c4_mp.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2c4_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r2c4_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r2c4_bench.log 2>&1
rc=$?; tail -c 600 gpurun_out/r2c4_bench.log; exit $rc

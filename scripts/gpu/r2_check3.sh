#!/bin/bash
# round 2: compile/opcheck tests + full GPU suite
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_compile_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/r2c3_compile.log 2>&1
echo "compile tests rc=$?"; grep -E "passed|failed|Error|error" gpurun_out/r2c3_compile.log | tail -30
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread --deselect tests/test_compile_gpu.py > gpurun_out/r2c3_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r2c3_tests.log; exit $rc

#!/bin/bash
# round 2: precision modes (fp16 autocast + loss scaling, fp32) + full GPU suite
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_amp.py -v --timeout 200 --timeout-method thread > gpurun_out/r2c5_amp.log 2>&1
rc=$?; echo "amp rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/r2c5_amp.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r2c5_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" gpurun_out/r2c5_tests.log | tail -20; exit $rc

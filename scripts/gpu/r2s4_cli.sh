#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_cli_gpu.py -q -x -v --timeout 400 --timeout-method thread > gpurun_out/cli_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/cli_tests.log | tail -8; exit $rc

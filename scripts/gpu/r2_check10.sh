#!/bin/bash
# round 2: attention GPU tests after removing the losing backward variants + same-box A/B
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "attn or attention" -x -q --timeout 200 --timeout-method thread > gpurun_out/r2c10_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r2c10_tests.log; [ $rc -ne 0 ] && exit $rc
CFG=64x12x1024x64,8x16x4096x64,16x16x2048x64,4x12x1024x64 bash scripts/gpu/r2_attnab.sh

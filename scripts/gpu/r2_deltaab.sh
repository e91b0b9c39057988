#!/bin/bash
# attention tests on the current build, then same-box A/B vs xso/ variants
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "attention or attn" > gpurun_out/r2_delta_tests.log 2>&1 || { tail -30 gpurun_out/r2_delta_tests.log; exit 1; }
tail -2 gpurun_out/r2_delta_tests.log
CFG=${CFG:-64x12x1024x64,8x16x4096x64,4x8x2048x32} bash scripts/gpu/r2_attnab.sh

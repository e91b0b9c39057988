#!/bin/bash
# D=128 forward with 8 waves per workgroup (PLLM_FWD128_NW=8 build) vs the 4-wave default
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PLLM_SO=$R/pretraining_llm_amd/_C_fwd8.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/r4a1_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error|assert" gpurun_out/r4a1_tests.log | tail -12; [ $rc -ne 0 ] && exit $rc
for round in 1 2; do
  for so in "" fwd8; do
    s=""; [ -n "$so" ] && s="$R/pretraining_llm_amd/_C_$so.so"
    PLLM_SO=$s timeout -k 10 120 python bench/attn_bench.py --ours --configs 16x16x2048x128,8x16x4096x128 --rounds 3 2>&1 | grep -v amdgpu.ids | sed "s/^/[${so:-base}] /" || exit 1
  done
done
PLLM_SO=$R/pretraining_llm_amd/_C_qspread.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/r4a1_tests_q.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error|assert" gpurun_out/r4a1_tests_q.log | tail -12; [ $rc -ne 0 ] && exit $rc
for round in 1 2; do
  for so in "" qspread; do
    s=""; [ -n "$so" ] && s="$R/pretraining_llm_amd/_C_$so.so"
    PLLM_SO=$s timeout -k 10 120 python bench/attn_bench.py --ours --configs 64x12x1024x64,8x16x4096x64 --rounds 3 2>&1 | grep -v amdgpu.ids | sed "s/^/[${so:-base}] /" || exit 1
  done
done

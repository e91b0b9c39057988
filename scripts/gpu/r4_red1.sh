#!/bin/bash
# slab reduce with the slab loop unrolled: wgrad tests, GPT-2 / llama step A/B vs the previous build
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_gpu.py -k "wgrad or fused_mlp" > gpurun_out/r4_red1_tests.log 2>&1 || { tail -20 gpurun_out/r4_red1_tests.log; exit 1; }
tail -1 gpurun_out/r4_red1_tests.log
for i in 1 2; do
  for so in xso/_C_base.so pretraining_llm_amd/_C.so; do
    PLLM_SO=$so timeout -k 10 300 python bench.py > gpurun_out/r4_red1_gpt2.log 2>&1 || exit 1
    echo "gpt2 $so $(tail -1 gpurun_out/r4_red1_gpt2.log | grep -o '"value": [0-9.]*')"
  done
done

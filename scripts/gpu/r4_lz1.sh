#!/bin/bash
# lazy gradient zeroing: tests, then GPT-2 / llama step A/B (PLLM_LAZY_ZERO 0 / 1, two interleaved rounds)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_lazy_zero_gpu.py tests/test_compile_gpu.py tests/test_kernels_gpu.py -k "lazy or wgrad or trainer or lm_head" > gpurun_out/r4_lz1_tests.log 2>&1 || { tail -40 gpurun_out/r4_lz1_tests.log; exit 1; }
tail -1 gpurun_out/r4_lz1_tests.log
for i in 1 2; do
  for v in 0 1; do
    PLLM_LAZY_ZERO=$v timeout -k 10 300 python bench.py > gpurun_out/r4_lz1_gpt2_${v}_$i.log 2>&1 || { tail -3 gpurun_out/r4_lz1_gpt2_${v}_$i.log; exit 1; }
    echo "gpt2 lazy=$v $(tail -1 gpurun_out/r4_lz1_gpt2_${v}_$i.log | grep -o '"value": [0-9.]*')"
  done
done
for i in 1 2; do
  for v in 0 1; do
    PLLM_LAZY_ZERO=$v timeout -k 10 400 python bench.py --model llama-1.3b --batch 16 --seq 2048 --steps 5 --warmup 2 > gpurun_out/r4_lz1_llama_${v}_$i.log 2>&1 || { tail -3 gpurun_out/r4_lz1_llama_${v}_$i.log; exit 1; }
    echo "llama lazy=$v $(tail -1 gpurun_out/r4_lz1_llama_${v}_$i.log | grep -o '"value": [0-9.]*')"
  done
done

#!/bin/bash
# hipBLASLt ReLU epilogue (csrc/blaslt.cpp): GPU tests, then ref-3b A/B (PLLM_LT_RELU 1 / 0, twice each)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k "gemm_lt or relu_mlp or fused_mlp" > gpurun_out/r4_lt1_tests.log 2>&1 || { tail -20 gpurun_out/r4_lt1_tests.log; exit 1; }
tail -2 gpurun_out/r4_lt1_tests.log
for i in 1 2; do
  for v in 1 0; do
    PLLM_LT_RELU=$v timeout -k 10 400 python bench.py --model ref-3b --batch 32 --seq 512 --steps 8 --warmup 3 > gpurun_out/r4_lt1_ref3b_$v.log 2>&1 || { tail -3 gpurun_out/r4_lt1_ref3b_$v.log; exit 1; }
    echo "PLLM_LT_RELU=$v $(tail -1 gpurun_out/r4_lt1_ref3b_$v.log | cut -c1-160)"
  done
done

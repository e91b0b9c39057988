#!/bin/bash
# hybrid weight gradients (whole tiles + sliced last round): tests, per-shape A/B, step A/B vs the previous
# build (xso/_C_base.so) with the hybrid off and on
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad" > gpurun_out/r4_hy1_tests.log 2>&1 || { tail -30 gpurun_out/r4_hy1_tests.log; exit 1; }
tail -1 gpurun_out/r4_hy1_tests.log
timeout -k 10 300 python -u bench/wgrad_hy_bench.py > gpurun_out/r4_hy1_bench.log 2>&1 || { tail -5 gpurun_out/r4_hy1_bench.log; exit 1; }
grep "{" gpurun_out/r4_hy1_bench.log
for i in 1 2; do
  for v in base off on; do
    so=pretraining_llm_amd/_C.so; hy=0
    [ $v = base ] && so=xso/_C_base.so
    [ $v = on ] && hy=1
    PLLM_SO=$so PLLM_WGRAD_HY=$hy timeout -k 10 300 python bench.py > gpurun_out/r4_hy1_gpt2_$v.log 2>&1 || { tail -3 gpurun_out/r4_hy1_gpt2_$v.log; exit 1; }
    echo "gpt2 $v $(tail -1 gpurun_out/r4_hy1_gpt2_$v.log | grep -o '"value": [0-9.]*')"
  done
done
for i in 1 2; do
  for v in base off on; do
    so=pretraining_llm_amd/_C.so; hy=0
    [ $v = base ] && so=xso/_C_base.so
    [ $v = on ] && hy=1
    PLLM_SO=$so PLLM_WGRAD_HY=$hy timeout -k 10 400 python bench.py --model llama-1.3b --batch 16 --seq 2048 --steps 5 --warmup 2 > gpurun_out/r4_hy1_llama_$v.log 2>&1 || { tail -3 gpurun_out/r4_hy1_llama_$v.log; exit 1; }
    echo "llama $v $(tail -1 gpurun_out/r4_hy1_llama_$v.log | grep -o '"value": [0-9.]*')"
  done
done

#!/bin/bash
# weight gradients: slice 0 straight into the gradient (one slab less).  Tests, per-shape times and
# GPT-2 / llama step A/B against the previous build (xso/_C_base.so), interleaved
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad" > gpurun_out/r4_slab1_tests.log 2>&1 || { tail -20 gpurun_out/r4_slab1_tests.log; exit 1; }
tail -1 gpurun_out/r4_slab1_tests.log
for so in xso/_C_base.so pretraining_llm_amd/_C.so; do
  PLLM_SO=$so timeout -k 10 200 python -u bench/wgrad_time.py > gpurun_out/r4_slab1_wt_$(basename $so .so).jsonl 2>&1 || exit 1
done
for i in 1 2; do
  for so in xso/_C_base.so pretraining_llm_amd/_C.so; do
    PLLM_SO=$so timeout -k 10 300 python bench.py > gpurun_out/r4_slab1_gpt2_$i_$(basename $so .so).log 2>&1 || exit 1
    echo "gpt2 $so $(tail -1 gpurun_out/r4_slab1_gpt2_$i_$(basename $so .so).log | cut -c1-150)"
  done
done
for i in 1 2; do
  for so in xso/_C_base.so pretraining_llm_amd/_C.so; do
    PLLM_SO=$so timeout -k 10 400 python bench.py --model llama-1.3b --batch 16 --seq 2048 --steps 5 --warmup 2 > gpurun_out/r4_slab1_llama_$(basename $so .so).log 2>&1 || exit 1
    echo "llama $so $(tail -1 gpurun_out/r4_slab1_llama_$(basename $so .so).log | cut -c1-150)"
  done
done

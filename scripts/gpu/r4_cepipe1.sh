#!/bin/bash
# LM head + CE pipelined over two streams (PLLM_CE_PIPE=K): test, then GPT-2 step A/B (0 / 4 / 8), interleaved
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "lm_head_ce" > gpurun_out/r4_cepipe1_tests.log 2>&1 || { tail -20 gpurun_out/r4_cepipe1_tests.log; exit 1; }
tail -1 gpurun_out/r4_cepipe1_tests.log
for i in 1 2; do
  for k in 0 4 8 2; do
    PLLM_CE_PIPE=$k timeout -k 10 300 python bench.py > gpurun_out/r4_cepipe1_$k.log 2>&1 || { tail -3 gpurun_out/r4_cepipe1_$k.log; exit 1; }
    echo "PLLM_CE_PIPE=$k $(tail -1 gpurun_out/r4_cepipe1_$k.log | cut -c1-140)"
  done
done

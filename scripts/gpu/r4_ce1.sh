#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PLLM_SO=$R/pretraining_llm_amd/_C_ceon.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "cross_entropy or lm_head" --timeout 120 --timeout-method thread > gpurun_out/r4ce_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error|assert" gpurun_out/r4ce_tests.log | tail -6; [ $rc -ne 0 ] && exit $rc
for round in 1 2 3; do
  for so in "" ceon; do
    s=""; [ -n "$so" ] && s="$R/pretraining_llm_amd/_C_$so.so"
    PLLM_SO=$s timeout -k 10 120 python bench/ce_bench.py 2>&1 | grep median || exit 1
  done
done

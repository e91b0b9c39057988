#!/bin/bash
# full-grid streaming kernels: GPU tests, HBM probe and GPT-2 / llama steps vs xso/_C_head.so
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2_gridab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2_gridab_tests.log; [ $rc -ne 0 ] && exit $rc
for v in cur head; do
  so="$R/pretraining_llm_amd/_C.so"; [ "$v" != cur ] && so="$R/xso/_C_$v.so"
  echo "$v $(PLLM_SO=$so timeout -k 10 120 python bench/hbm_probe.py 2>&1 | grep '^{')"
done
for round in 1 2; do
  for v in cur head; do
    so="$R/pretraining_llm_amd/_C.so"; [ "$v" != cur ] && so="$R/xso/_C_$v.so"
    PLLM_SO=$so timeout -k 10 300 python bench.py --steps 12 --warmup 4 > gpurun_out/r2_gridab_$v.log 2>&1 || { tail -3 gpurun_out/r2_gridab_$v.log; exit 1; }
    echo "$round $v gpt2 $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r2_gridab_$v.log | tr '\n' ' ')"
  done
done
for v in cur head; do
  so="$R/pretraining_llm_amd/_C.so"; [ "$v" != cur ] && so="$R/xso/_C_$v.so"
  PLLM_SO=$so timeout -k 10 300 python bench.py --model llama-1.3b --batch 16 --seq 2048 --steps 4 --warmup 2 > gpurun_out/r2_gridab_llama_$v.log 2>&1 || { tail -3 gpurun_out/r2_gridab_llama_$v.log; exit 1; }
  echo "$v llama $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r2_gridab_llama_$v.log | tr '\n' ' ')"
done

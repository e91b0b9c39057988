#!/bin/bash
# GPT-2 headline step with the LM-head/CE sub-chunks (PLLM_CE_SUBCHUNK) vs one chunk
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for sc in 0 2048 4096 1024 0; do
  PLLM_CE_SUBCHUNK=$sc timeout -k 10 300 python bench.py --steps 12 --warmup 4 > gpurun_out/r2_cesub_$sc.log 2>&1 || { tail -5 gpurun_out/r2_cesub_$sc.log; exit 1; }
  echo "sub=$sc $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r2_cesub_$sc.log | tr '\n' ' ')"
done

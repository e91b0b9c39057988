#!/bin/bash
# GPT-2 headline step: shipped TunableOp tables vs the previous ones (xtune/), interleaved
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in new old new old; do
  d=""; [ $v = old ] && d="$R/xtune"
  PLLM_TUNING_DIR=$d timeout -k 10 300 python bench.py --steps 12 --warmup 4 > gpurun_out/r2_tuneab_$v.log 2>&1 || { tail -5 gpurun_out/r2_tuneab_$v.log; exit 1; }
  echo "$v $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r2_tuneab_$v.log | tr '\n' ' ')"
done

#!/bin/bash
# desynchronising tile split on the llama step (long-K SwiGLU epilogues 5 / 7) A/B
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for round in 1 2; do
  for v in 0 1; do
    PLLM_GEMM_SPLIT=$v timeout -k 10 400 python bench.py --model llama-1.3b --batch 16 --seq 2048 --steps 5 --warmup 2 > gpurun_out/r4sp2_llama_${v}_$round.log 2>&1 || { tail -3 gpurun_out/r4sp2_llama_${v}_$round.log; exit 1; }
    echo "llama split=$v $(tail -1 gpurun_out/r4sp2_llama_${v}_$round.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
  done
done

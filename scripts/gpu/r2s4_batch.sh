#!/bin/bash
# per-GPU batch sweep for the llama-1.3B and GPT-2-small bench configs
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/batch
export HSA_ENABLE_IPC_MODE_LEGACY=0
for b in 16 24 32; do
  timeout -k 10 400 python bench.py --model llama-1.3b --batch $b --seq 2048 --steps 5 --warmup 2 > gpurun_out/batch/llama_$b.log 2>&1 || { tail -5 gpurun_out/batch/llama_$b.log; exit 1; }
  echo "llama b=$b $(tail -1 gpurun_out/batch/llama_$b.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"])')"
done
for b in 64 128; do
  timeout -k 10 400 python bench.py --batch $b --steps 20 --warmup 5 > gpurun_out/batch/gpt2_$b.log 2>&1 || { tail -5 gpurun_out/batch/gpt2_$b.log; exit 1; }
  echo "gpt2 b=$b $(tail -1 gpurun_out/batch/gpt2_$b.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"])')"
done

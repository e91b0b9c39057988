#!/bin/bash
# GPT-2 small, 1500 steps, HIP vs stock PyTorch ops (same seed / batches): numerics over a longer run
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1100 python -u scripts/convergence.py --model gpt2-small --steps 1500 --batch 16 --seq 1024 --lr 6e-4 \
  --out gpurun_out/conv_gpt2_long.jsonl 2> gpurun_out/conv_gpt2_long.log || { tail -5 gpurun_out/conv_gpt2_long.log; exit 1; }
grep final gpurun_out/conv_gpt2_long.log

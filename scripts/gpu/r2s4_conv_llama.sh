#!/bin/bash
# llama-1.3B numerics at scale: HIP kernels vs stock PyTorch ops, same seed / batches, 300 steps
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u scripts/convergence.py --model llama-1.3b --steps 300 --batch 4 --seq 2048 --lr 3e-4 \
  --out gpurun_out/conv_llama.jsonl 2>&1 | grep -v amdgpu.ids
tail -1 gpurun_out/conv_llama.jsonl

#!/bin/bash
# llama-1.3B: stock PyTorch ops in fp32 as the numerics ground truth for the HIP-vs-bf16-torch curves
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1100 python -u scripts/convergence.py --model llama-1.3b --steps 300 --batch 4 --seq 2048 --lr 3e-4 \
  --backends torch:float32 --out gpurun_out/conv_llama_fp32.jsonl 2> gpurun_out/conv_llama_fp32.log || { tail -5 gpurun_out/conv_llama_fp32.log; exit 1; }
tail -3 gpurun_out/conv_llama_fp32.log

#!/bin/bash
# BASELINE.json configs 4 and 5 on one GPU (per-GPU throughput; DP=8 is the driver's scaling run)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python bench.py --model llama-1.3b --batch 8 --steps 5 --warmup 2 --verbose > gpurun_out/b7_llama.log 2>&1 || { echo "llama failed"; tail -20 gpurun_out/b7_llama.log; exit 4; }
tail -1 gpurun_out/b7_llama.log | cut -c1-500
timeout -k 10 400 python bench.py --model gpt2-medium --batch 8 --steps 5 --warmup 2 --verbose > gpurun_out/b7_med.log 2>&1 || { echo "medium failed"; tail -20 gpurun_out/b7_med.log; exit 5; }
tail -1 gpurun_out/b7_med.log | cut -c1-500
timeout -k 10 400 python bench.py --backend torch --model llama-1.3b --batch 8 --steps 5 --warmup 2 --verbose > gpurun_out/b7_llama_torch.log 2>&1 || { echo "llama torch failed"; tail -20 gpurun_out/b7_llama_torch.log; exit 6; }
tail -1 gpurun_out/b7_llama_torch.log | cut -c1-300
timeout -k 10 400 python bench.py --backend torch --batch 64 --steps 5 --warmup 2 --verbose > gpurun_out/b7_small_torch.log 2>&1 || { echo "small torch failed"; tail -20 gpurun_out/b7_small_torch.log; exit 7; }
tail -1 gpurun_out/b7_small_torch.log | cut -c1-300

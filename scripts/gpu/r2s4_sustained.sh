#!/bin/bash
# sustained throughput: 300 timed headline steps (~20 s of continuous training) and 40 llama steps
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python bench.py --steps 300 --warmup 5 > gpurun_out/sus_gpt2.log 2>&1 || { tail -5 gpurun_out/sus_gpt2.log; exit 1; }
tail -1 gpurun_out/sus_gpt2.log | cut -c1-220
timeout -k 10 500 python bench.py --model llama-1.3b --batch 16 --seq 2048 --steps 40 --warmup 2 > gpurun_out/sus_llama.log 2>&1 || { tail -5 gpurun_out/sus_llama.log; exit 1; }
tail -1 gpurun_out/sus_llama.log | cut -c1-220

#!/bin/bash
# round 2: headline + llama + ref-3b step benches with the llama / ref-3b TunableOp tables
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python bench.py --model llama-1.3b --batch 16 --seq 2048 --steps 5 --warmup 2 > gpurun_out/r2b6_llama.log 2>&1 || { tail -5 gpurun_out/r2b6_llama.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"mfu": [0-9.]*' gpurun_out/r2b6_llama.log | tr '\n' ' '; echo
timeout -k 10 400 python bench.py --model ref-3b --batch 32 --seq 512 --steps 5 --warmup 2 > gpurun_out/r2b6_ref3b.log 2>&1 || { tail -5 gpurun_out/r2b6_ref3b.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"mfu": [0-9.]*' gpurun_out/r2b6_ref3b.log | tr '\n' ' '; echo

#!/bin/bash
# headline bench: per-GPU micro-batch sweep (tokens/s vs sequences per GPU), 1x MI355X
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
: > gpurun_out/bsweep.jsonl
for b in 64 96 128 32; do
  timeout -k 10 300 python bench.py --batch $b --steps 12 --warmup 4 > gpurun_out/bs_$b.log 2>&1 || { echo "bench failed b=$b"; tail -20 gpurun_out/bs_$b.log; exit 4; }
  tail -1 gpurun_out/bs_$b.log >> gpurun_out/bsweep.jsonl
  echo "b=$b $(tail -1 gpurun_out/bs_$b.log | grep -o '"value": [0-9.]*') $(tail -1 gpurun_out/bs_$b.log | grep -o '"peak_mem_gb": [0-9.]*')"
done

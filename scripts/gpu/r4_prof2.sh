#!/bin/bash
# fresh kernel tables of the current build (GPT-2 small headline, llama-1.3B) + the counter list
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu/prof.sh r4b_prof_gpt2 --steps 8 --warmup 3 || exit 1
python scripts/prof_summary.py gpurun_out/r4b_prof_gpt2/run_kernel_stats.csv 13 "GPT-2 small B=64 T=1024 step (round 4: ping-pong fused-epilogue GEMM)" > gpurun_out/r4b_prof_gpt2.md
head -40 gpurun_out/r4b_prof_gpt2.md
bash scripts/gpu/prof.sh r4b_prof_llama --model llama-1.3b --batch 16 --seq 2048 --steps 3 --warmup 2 || exit 1
python scripts/prof_summary.py gpurun_out/r4b_prof_llama/run_kernel_stats.csv 7 "llama-1.3B B=16 T=2048 step (round 4)" > gpurun_out/r4b_prof_llama.md
head -40 gpurun_out/r4b_prof_llama.md
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > "$R/gpurun_out/r4b_counters.txt" 2>&1 || true
grep -c . "$R/gpurun_out/r4b_counters.txt"

#!/bin/bash
# round 2: kernel-time profiles of the GPT-2 small headline and llama-1.3B b16 steps
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
bash scripts/gpu/prof.sh r2_prof5_gpt2 --steps 5 --warmup 3 || exit 1
python scripts/prof_summary.py gpurun_out/r2_prof5_gpt2/run_kernel_stats.csv 8 "GPT-2 small B=64 T=1024 step" > gpurun_out/r2_prof5_gpt2.md
head -45 gpurun_out/r2_prof5_gpt2.md
bash scripts/gpu/prof.sh r2_prof5_llama --model llama-1.3b --batch 16 --steps 3 --warmup 2 || exit 1
python scripts/prof_summary.py gpurun_out/r2_prof5_llama/run_kernel_stats.csv 5 "llama-1.3B B=16 T=2048 step" > gpurun_out/r2_prof5_llama.md
head -30 gpurun_out/r2_prof5_llama.md

#!/bin/bash
# round-3 kernel-time profiles: GPT-2 small headline, GPT-2 medium seq4096 (BASELINE config 5), llama-1.3B
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
bash scripts/gpu/prof.sh r3prof_gpt2 --steps 8 --warmup 3 || exit 1
bash scripts/gpu/prof.sh r3prof_med --model gpt2-medium --seq 4096 --batch 8 --act-ckpt auto --steps 5 --warmup 2 || exit 1
bash scripts/gpu/prof.sh r3prof_llama --model llama-1.3b --batch 16 --steps 4 --warmup 2 || exit 1

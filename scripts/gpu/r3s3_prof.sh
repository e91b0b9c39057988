#!/bin/bash
# session-3 kernel-time profiles + un-profiled benches: GPT-2 medium seq4096 (BASELINE config 5), llama-1.3B
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench.py --model gpt2-medium --seq 4096 --batch 8 --act-ckpt auto --steps 10 --warmup 3 > gpurun_out/s3_med.log 2>&1 || { tail -5 gpurun_out/s3_med.log; exit 1; }
grep -h '^{' gpurun_out/s3_med.log | cut -c1-200
timeout -k 10 300 python bench.py --model llama-1.3b --batch 16 --steps 10 --warmup 3 > gpurun_out/s3_llama.log 2>&1 || { tail -5 gpurun_out/s3_llama.log; exit 1; }
grep -h '^{' gpurun_out/s3_llama.log | cut -c1-200
bash scripts/gpu/prof.sh s3prof_med --model gpt2-medium --seq 4096 --batch 8 --act-ckpt auto --steps 5 --warmup 2 || exit 1
python scripts/prof_summary.py gpurun_out/s3prof_med/run_kernel_stats.csv 7 "GPT-2 medium B=8 T=4096 step, --act-ckpt auto (round 3, session 3)" > gpurun_out/s3prof_med.md
bash scripts/gpu/prof.sh s3prof_llama --model llama-1.3b --batch 16 --steps 4 --warmup 2 || exit 1
python scripts/prof_summary.py gpurun_out/s3prof_llama/run_kernel_stats.csv 6 "llama-1.3b B=16 T=2048 step (round 3, session 3)" > gpurun_out/s3prof_llama.md
head -16 gpurun_out/s3prof_med.md; head -16 gpurun_out/s3prof_llama.md

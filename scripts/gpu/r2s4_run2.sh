#!/bin/bash
# batched norm-backward column reductions: GPU suite, headline bench x2, step profile, refreshed
# GPT-2-medium seq4096 (auto checkpointing) and llama-1.3B numbers
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/s4r2_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|error" gpurun_out/s4r2_tests.log | tail -15; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/s4r2_gpt2_$i.log 2>&1 || { tail -5 gpurun_out/s4r2_gpt2_$i.log; exit 1; }
  tail -1 gpurun_out/s4r2_gpt2_$i.log | cut -c1-220
done
bash scripts/gpu/prof.sh s4_prof_gpt2 --steps 5 --warmup 3 || exit 1
python scripts/prof_summary.py gpurun_out/s4_prof_gpt2/run_kernel_stats.csv 8 "GPT-2 small B=64 T=1024 step" > gpurun_out/s4_prof_gpt2.md
head -24 gpurun_out/s4_prof_gpt2.md
timeout -k 10 500 python bench.py --model gpt2-medium --seq 4096 --batch 8 --act-ckpt auto --steps 8 --warmup 3 > gpurun_out/s4r2_med.log 2>&1 || { tail -5 gpurun_out/s4r2_med.log; exit 1; }
tail -1 gpurun_out/s4r2_med.log | cut -c1-300
timeout -k 10 400 python bench.py --model llama-1.3b --batch 16 --seq 2048 --steps 5 --warmup 2 > gpurun_out/s4r2_llama.log 2>&1 || { tail -5 gpurun_out/s4r2_llama.log; exit 1; }
tail -1 gpurun_out/s4r2_llama.log | cut -c1-300

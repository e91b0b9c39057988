#!/bin/bash
# round 2 close-out: full GPU suite + smoke, headline / llama / ref-3b benches, step profiles
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r2f1_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|error" gpurun_out/r2f1_tests.log | tail -15; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2f1_smoke.log 2>&1 || { tail -5 gpurun_out/r2f1_smoke.log; exit 1; }
tail -1 gpurun_out/r2f1_smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r2f1_gpt2.log 2>&1 || { tail -5 gpurun_out/r2f1_gpt2.log; exit 1; }
tail -1 gpurun_out/r2f1_gpt2.log
timeout -k 10 400 python bench.py --model llama-1.3b --batch 16 --seq 2048 --steps 5 --warmup 2 > gpurun_out/r2f1_llama.log 2>&1 || { tail -5 gpurun_out/r2f1_llama.log; exit 1; }
tail -1 gpurun_out/r2f1_llama.log
timeout -k 10 400 python bench.py --model ref-3b --batch 32 --seq 512 --steps 5 --warmup 2 > gpurun_out/r2f1_ref3b.log 2>&1 || { tail -5 gpurun_out/r2f1_ref3b.log; exit 1; }
tail -1 gpurun_out/r2f1_ref3b.log
bash scripts/gpu/prof.sh r2_prof6_gpt2 --steps 5 --warmup 3 || exit 1
python scripts/prof_summary.py gpurun_out/r2_prof6_gpt2/run_kernel_stats.csv 8 "GPT-2 small B=64 T=1024 step" > gpurun_out/r2_prof6_gpt2.md
head -30 gpurun_out/r2_prof6_gpt2.md
bash scripts/gpu/prof.sh r2_prof6_llama --model llama-1.3b --batch 16 --steps 3 --warmup 2 || exit 1
python scripts/prof_summary.py gpurun_out/r2_prof6_llama/run_kernel_stats.csv 5 "llama-1.3B B=16 T=2048 step" > gpurun_out/r2_prof6_llama.md
head -30 gpurun_out/r2_prof6_llama.md

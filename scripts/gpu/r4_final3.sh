#!/bin/bash
# round-4 close: GPT-2 / llama / ref-3b / GPT-2 medium numbers + kernel tables of the final build
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4x_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|error" gpurun_out/r4x_tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4x_smoke.log 2>&1 || { tail -5 gpurun_out/r4x_smoke.log; exit 1; }
tail -1 gpurun_out/r4x_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r4x_gpt2.log 2>&1 || { tail -3 gpurun_out/r4x_gpt2.log; exit 1; }
tail -1 gpurun_out/r4x_gpt2.log | cut -c1-200
timeout -k 10 400 python bench.py --model llama-1.3b --batch 16 --seq 2048 --steps 5 --warmup 2 > gpurun_out/r4x_llama.log 2>&1 || { tail -3 gpurun_out/r4x_llama.log; exit 1; }
tail -1 gpurun_out/r4x_llama.log | cut -c1-200
timeout -k 10 400 python bench.py --model ref-3b --batch 32 --seq 512 --steps 5 --warmup 2 > gpurun_out/r4x_ref3b.log 2>&1 || { tail -3 gpurun_out/r4x_ref3b.log; exit 1; }
tail -1 gpurun_out/r4x_ref3b.log | cut -c1-200
timeout -k 10 400 python bench.py --model gpt2-medium --seq 4096 --batch 8 --act-ckpt auto --steps 5 --warmup 2 > gpurun_out/r4x_medium.log 2>&1 || { tail -3 gpurun_out/r4x_medium.log; exit 1; }
tail -1 gpurun_out/r4x_medium.log | cut -c1-200
bash scripts/gpu/prof.sh r4x_prof_gpt2 --steps 8 --warmup 3 || exit 1
python scripts/prof_summary.py gpurun_out/r4x_prof_gpt2/run_kernel_stats.csv 13 "GPT-2 small B=64 T=1024 step (round-4 final build, session 2 close: ping-pong GEMM + ping-pong weight gradients)" > gpurun_out/r4x_prof_gpt2.md
head -12 gpurun_out/r4x_prof_gpt2.md
bash scripts/gpu/prof.sh r4x_prof_llama --model llama-1.3b --batch 16 --seq 2048 --steps 3 --warmup 2 || exit 1
python scripts/prof_summary.py gpurun_out/r4x_prof_llama/run_kernel_stats.csv 7 "llama-1.3B B=16 T=2048 step (round-4 final build, session 2 close)" > gpurun_out/r4x_prof_llama.md
head -12 gpurun_out/r4x_prof_llama.md

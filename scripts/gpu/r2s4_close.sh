#!/bin/bash
# session close-out: full GPU suite, smoke, benches (headline, llama-1.3B, ref-3b, GPT-2-medium 4K)
# and the kernel-time profiles of the headline and llama steps
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/s4c_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|error" gpurun_out/s4c_tests.log | tail -15; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s4c_smoke.log 2>&1 || { tail -5 gpurun_out/s4c_smoke.log; exit 1; }
tail -1 gpurun_out/s4c_smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/s4c_gpt2.log 2>&1 || { tail -5 gpurun_out/s4c_gpt2.log; exit 1; }
tail -1 gpurun_out/s4c_gpt2.log | cut -c1-200
timeout -k 10 400 python bench.py --model llama-1.3b --batch 16 --seq 2048 --steps 5 --warmup 2 > gpurun_out/s4c_llama.log 2>&1 || { tail -5 gpurun_out/s4c_llama.log; exit 1; }
tail -1 gpurun_out/s4c_llama.log | cut -c1-200
timeout -k 10 400 python bench.py --model ref-3b --batch 32 --seq 512 --steps 5 --warmup 2 > gpurun_out/s4c_ref3b.log 2>&1 || { tail -5 gpurun_out/s4c_ref3b.log; exit 1; }
tail -1 gpurun_out/s4c_ref3b.log | cut -c1-200
timeout -k 10 500 python bench.py --model gpt2-medium --seq 4096 --batch 8 --act-ckpt auto --steps 8 --warmup 3 > gpurun_out/s4c_med.log 2>&1 || { tail -5 gpurun_out/s4c_med.log; exit 1; }
tail -1 gpurun_out/s4c_med.log | cut -c1-200
bash scripts/gpu/prof.sh s4c_prof_gpt2 --steps 5 --warmup 3 || exit 1
python scripts/prof_summary.py gpurun_out/s4c_prof_gpt2/run_kernel_stats.csv 8 "GPT-2 small B=64 T=1024 step" > gpurun_out/s4c_prof_gpt2.md
bash scripts/gpu/prof.sh s4c_prof_llama --model llama-1.3b --batch 16 --steps 3 --warmup 2 || exit 1
python scripts/prof_summary.py gpurun_out/s4c_prof_llama/run_kernel_stats.csv 5 "llama-1.3B B=16 T=2048 step" > gpurun_out/s4c_prof_llama.md
head -12 gpurun_out/s4c_prof_gpt2.md

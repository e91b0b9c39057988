#!/bin/bash
# round-4 start on a fresh box: GPU suite, headline, the reference's own config (ref-3b), and a
# fresh GPT-2 medium seq4096 kernel table (VERDICT r3 weak #7 / missing #3)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4a_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|error" gpurun_out/r4a_tests.log | tail -15; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r4a_gpt2.log 2>&1 || { tail -5 gpurun_out/r4a_gpt2.log; exit 1; }
tail -1 gpurun_out/r4a_gpt2.log | cut -c1-250
timeout -k 10 400 python bench.py --model ref-3b --batch 32 --seq 512 --steps 5 --warmup 2 > gpurun_out/r4a_ref3b.log 2>&1 || { tail -5 gpurun_out/r4a_ref3b.log; exit 1; }
tail -1 gpurun_out/r4a_ref3b.log | cut -c1-250
bash scripts/gpu/prof.sh r4a_prof_med --model gpt2-medium --seq 4096 --batch 8 --act-ckpt auto --steps 3 --warmup 2 || exit 1
python scripts/prof_summary.py gpurun_out/r4a_prof_med/run_kernel_stats.csv 3 "GPT-2 medium B=8 T=4096 step" > gpurun_out/r4a_prof_med.md
head -30 gpurun_out/r4a_prof_med.md

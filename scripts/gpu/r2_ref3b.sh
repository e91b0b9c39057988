#!/bin/bash
# round 2: the reference's own configured workload (arch=ref, V=50304 T=512 C=2048 H=16 L=64, B=32)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python bench.py --model ref-3b --batch 32 --steps 10 --warmup 3 > gpurun_out/r2_ref3b_bench.log 2>&1
rc=$?; tail -1 gpurun_out/r2_ref3b_bench.log | cut -c1-2000; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu/prof.sh r2_prof_ref3b --model ref-3b --batch 32 --steps 3 --warmup 2 || exit 1
python scripts/prof_summary.py gpurun_out/r2_prof_ref3b/run_kernel_stats.csv 5 "ref-3b kernel stats" > gpurun_out/r2_prof_ref3b.md
head -40 gpurun_out/r2_prof_ref3b.md

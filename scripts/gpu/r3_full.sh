#!/bin/bash
# full GPU suite + smoke + headline bench + GPT-2 step kernel profile (tag = $1)
R="${GRAFT_REPO_ROOT:-/root/repo}"
T="${1:-r3}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu/r3_check.sh $T || exit 1
bash scripts/gpu/prof.sh ${T}_prof --steps 5 --warmup 3 || exit 1
python scripts/prof_summary.py gpurun_out/${T}_prof/run_kernel_stats.csv 8 "GPT-2 small B=64 T=1024 step" > gpurun_out/${T}_prof.md
head -24 gpurun_out/${T}_prof.md

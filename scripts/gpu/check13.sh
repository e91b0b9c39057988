#!/bin/bash
# headline bench (committed state, 32x32 wgrad default) + kernel profile
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench.py > gpurun_out/b13.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/b13.log; exit 4; }
tail -1 gpurun_out/b13.log | cut -c1-300
bash scripts/gpu/prof.sh prof7 --steps 10 --warmup 3

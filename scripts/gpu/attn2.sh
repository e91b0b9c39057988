#!/bin/bash
# attention backward tiling variants A/B + attention GPU tests under each variant
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench/attn_bench.py --ours --configs 64x12x1024x64,8x16x4096x64,16x12x1024x64 --rounds 3 > gpurun_out/attn2.log 2>&1 || { echo "attn bench failed"; tail -20 gpurun_out/attn2.log; exit 3; }
grep -v amdgpu.ids gpurun_out/attn2.log | cut -c1-700

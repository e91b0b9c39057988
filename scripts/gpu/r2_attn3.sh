#!/bin/bash
# round 2: attention kernels with the pre-loop vmcnt fix + unconditional lse/delta prefetch
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention or attn" -x -q --timeout 200 --timeout-method thread > gpurun_out/r2a3_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2a3_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench/attn_bench.py --configs 64x12x1024x64,16x16x2048x128,8x16x4096x64 --rounds 3 > gpurun_out/r2a3_bench.jsonl 2>&1
rc=$?; cut -c1-700 gpurun_out/r2a3_bench.jsonl; exit $rc

#!/bin/bash
# round 2: attention backward rewrite (KH=2 variants, fp32 slabs in bounded passes)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 200 --timeout-method thread > gpurun_out/r2a1_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2a1_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench/attn_bench.py --configs 64x12x1024x64,8x16x4096x64,32x16x512x64 --ours --rounds 3 > gpurun_out/r2a1_d64.jsonl 2>&1
rc=$?; cut -c1-600 gpurun_out/r2a1_d64.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench/attn_bench.py --configs 16x16x2048x128,32x16x512x128 --ours --rounds 3 > gpurun_out/r2a1_d128.jsonl 2>&1
rc=$?; cut -c1-600 gpurun_out/r2a1_d128.jsonl; [ $rc -ne 0 ] && exit $rc
PLLM_ATTN_BWD_WS_MB=64 timeout -k 10 300 python bench/attn_bench.py --configs 64x12x1024x64,8x16x4096x64 --ours --rounds 2 > gpurun_out/r2a1_passes.jsonl 2>&1
rc=$?; cut -c1-600 gpurun_out/r2a1_passes.jsonl; exit $rc

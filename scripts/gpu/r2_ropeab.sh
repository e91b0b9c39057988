#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "rope" -x -q --timeout 200 --timeout-method thread > gpurun_out/r2_ropeab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2_ropeab_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench/attn_bench.py --configs 16x16x2048x128,64x12x1024x64 --rope-ab --rounds 3 > gpurun_out/r2_ropeab.jsonl 2>&1; rc=$?
grep "^{" gpurun_out/r2_ropeab.jsonl; tail -2 gpurun_out/r2_ropeab.jsonl; exit $rc

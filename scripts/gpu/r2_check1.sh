#!/bin/bash
# round 2: GPU test suite + headline bench (fp32 gradient path) + kernel-time profile
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2c1_tests.log 2>&1
rc=$?; tail -25 gpurun_out/r2c1_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2c1_bench.log 2>&1
rc=$?; tail -2 gpurun_out/r2c1_bench.log | cut -c1-1500; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --model llama-1.3b --batch 16 > gpurun_out/r2c1_bench_llama.log 2>&1
rc=$?; tail -1 gpurun_out/r2c1_bench_llama.log | cut -c1-1500; exit $rc

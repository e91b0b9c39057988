#!/bin/bash
# stream-K weight gradients: tests, per-shape A/B, then GPT-2 / llama step A/B (env PLLM_WGRAD_SK)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad" > gpurun_out/r4_sk1_tests.log 2>&1 || { tail -30 gpurun_out/r4_sk1_tests.log; exit 1; }
tail -1 gpurun_out/r4_sk1_tests.log
timeout -k 10 300 python -u bench/wgrad_sk_bench.py > gpurun_out/r4_sk1_bench.log 2>&1 || { tail -5 gpurun_out/r4_sk1_bench.log; exit 1; }
grep "{" gpurun_out/r4_sk1_bench.log

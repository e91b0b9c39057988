#!/bin/bash
# round 2: phased wgrad kernel -- tests + A/B vs the two-stage kernel and hipBLASLt
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad and (32 or 8)" -v --timeout 120 --timeout-method thread > gpurun_out/r2wg1_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert" gpurun_out/r2wg1_tests.log | tail -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench/gemm_bench.py --shapes gpt2 --variants 32,8,9,10,11 --rounds 3 > gpurun_out/r2wg1_gpt2.jsonl 2>&1
rc=$?; cut -c1-330 gpurun_out/r2wg1_gpt2.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench/gemm_bench.py --shapes llama --M 32768 --variants 32,8,9,10,11 --rounds 3 > gpurun_out/r2wg1_llama.jsonl 2>&1
rc=$?; cut -c1-330 gpurun_out/r2wg1_llama.jsonl; exit $rc

#!/bin/bash
# ping-pong GEMM (csrc/gemm_pp.hip): numerics tests, then the interleaved A/B bench
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4pp1_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|error|Error" gpurun_out/r4pp1_tests.log | tail -15; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench/gemm_pp_bench.py --fused > gpurun_out/r4pp1_bench.jsonl 2>&1
rc=$?; cat gpurun_out/r4pp1_bench.jsonl; exit $rc

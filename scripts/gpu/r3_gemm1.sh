#!/bin/bash
# fused-epilogue TN GEMM: numerics tests, then timing vs hipBLASLt (both MFMA shapes)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/gemm
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm/tests.log 2>&1
rc=$?; tail -3 gpurun_out/gemm/tests.log; [ $rc -ne 0 ] && exit $rc
for mf in 32 16; do
  timeout -k 10 300 python bench/gemm_tn_bench.py --mf $mf --fused > gpurun_out/gemm/bench_$mf.log 2>&1 || { tail -3 gpurun_out/gemm/bench_$mf.log; exit 1; }
  cat gpurun_out/gemm/bench_$mf.log
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/gemm/bench_fused.log 2>&1 || { tail -5 gpurun_out/gemm/bench_fused.log; exit 1; }
tail -1 gpurun_out/gemm/bench_fused.log | cut -c1-200
PLLM_FUSED_MLP=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/gemm/bench_unfused.log 2>&1 || { tail -5 gpurun_out/gemm/bench_unfused.log; exit 1; }
tail -1 gpurun_out/gemm/bench_unfused.log | cut -c1-200

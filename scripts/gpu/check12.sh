#!/bin/bash
# wgrad MFMA-shape A/B microbench + DP engine GPU test + headline bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench/gemm_bench.py --rounds 3 > gpurun_out/gemm12.log 2>&1 || { echo "gemm bench failed"; tail -20 gpurun_out/gemm12.log; exit 3; }
grep -v amdgpu.ids gpurun_out/gemm12.log | cut -c1-600
timeout -k 10 300 python -u -m pytest tests/test_dp_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t12.log 2>&1
rc=$?; tail -3 gpurun_out/t12.log
if [ $rc -gt 1 ]; then exit $rc; fi
if [ $rc -eq 1 ]; then grep -E "^E |FAILED" gpurun_out/t12.log | head -30; fi
timeout -k 10 300 python bench.py > gpurun_out/b12.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/b12.log; exit 4; }
tail -1 gpurun_out/b12.log | cut -c1-300

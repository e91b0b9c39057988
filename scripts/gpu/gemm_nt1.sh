#!/bin/bash
# NT GEMM + fused MLP epilogue kernel: numerics tests, then A/B microbench vs hipBLASLt
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k gemm_nt > gpurun_out/tnt1.log 2>&1
rc=$?; tail -3 gpurun_out/tnt1.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/tnt1.log | head -30; exit $rc; fi
timeout -k 10 300 python bench/gemm_nt_bench.py --rounds 3 > gpurun_out/gnt1.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/gnt1.log; exit 3; }
grep -v amdgpu.ids gpurun_out/gnt1.log | cut -c1-900

#!/bin/bash
# wgrad v2 validation: numerics first, then microbench, then the full GPU suite and the step bench (hip vs blas).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -p no:cacheprovider -k wgrad > gpurun_out/t9a.log 2>&1
rc=$?; tail -3 gpurun_out/t9a.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/t9a.log | head -20; exit $rc; fi
timeout -k 10 400 python bench/gemm_bench.py > gpurun_out/gemm2.log 2>&1 || { echo "gemm bench failed"; tail -20 gpurun_out/gemm2.log; exit 3; }
grep "^{" gpurun_out/gemm2.log | cut -c1-400
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -x -p no:cacheprovider > gpurun_out/t9.log 2>&1
rc=$?; tail -3 gpurun_out/t9.log
if [ $rc -gt 1 ]; then exit $rc; fi
if [ $rc -eq 1 ]; then grep -E "^E |FAILED" gpurun_out/t9.log | head -20; fi
for w in hip blas; do
PLLM_WGRAD=$w timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/b9_$w.log 2>&1 || { echo "bench $w failed"; tail -20 gpurun_out/b9_$w.log; exit 4; }
tail -1 gpurun_out/b9_$w.log | cut -c1-200
done

#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python bench/gemm_bench.py > gpurun_out/gemm1.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/gemm1.log | cut -c1-400
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -q -x -p no:cacheprovider > gpurun_out/t8.log 2>&1
rc=$?
tail -3 gpurun_out/t8.log
if [ $rc -gt 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
if [ $rc -eq 1 ]; then grep -E "^E |FAILED" gpurun_out/t8.log | head -20; fi
for w in hip blas; do
PLLM_WGRAD=$w timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/b8_$w.log 2>&1 || { echo "bench $w failed"; tail -20 gpurun_out/b8_$w.log; exit 4; }
tail -1 gpurun_out/b8_$w.log | cut -c1-200
done
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --cuda-graph > gpurun_out/b8_graph.log 2>&1 || { echo "graph bench failed"; tail -20 gpurun_out/b8_graph.log; exit 5; }
tail -1 gpurun_out/b8_graph.log | cut -c1-200
timeout -k 10 600 python bench/attn_bench.py > gpurun_out/attn1.log 2>&1 || { echo "attn bench failed"; tail -20 gpurun_out/attn1.log; exit 6; }
grep -v amdgpu.ids gpurun_out/attn1.log | cut -c1-600

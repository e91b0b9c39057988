#!/bin/bash
# attention numerics (pytest -k attention) + fwd/bwd microbench vs SDPA, then the 1-GPU headline bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "attention or model" -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/attn1_t.log 2>&1
rc=$?; tail -3 gpurun_out/attn1_t.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/attn1_t.log | head -20; exit $rc; fi
timeout -k 10 300 python bench/attn_bench.py --configs 64x12x1024x64,8x16x2048x128 > gpurun_out/attn1_b.log 2>&1 || { tail -20 gpurun_out/attn1_b.log; exit 3; }
cut -c1-400 gpurun_out/attn1_b.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/attn1_bench.log 2>&1 || { tail -20 gpurun_out/attn1_bench.log; exit 4; }
tail -1 gpurun_out/attn1_bench.log | cut -c1-300

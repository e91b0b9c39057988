#!/bin/bash
# bf16 dQ slabs + static wave priority: attention tests, attention microbench, headline bench
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "attention or model" > gpurun_out/ta3.log 2>&1
rc=$?; tail -3 gpurun_out/ta3.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/ta3.log | head -30; exit $rc; fi
timeout -k 10 300 python bench/attn_bench.py --ours --configs 64x12x1024x64,8x16x4096x64 --rounds 3 > gpurun_out/attn3.log 2>&1 || { echo "attn bench failed"; tail -20 gpurun_out/attn3.log; exit 3; }
grep -v amdgpu.ids gpurun_out/attn3.log | cut -c1-400
timeout -k 10 300 python bench.py > gpurun_out/b16.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/b16.log; exit 4; }
tail -1 gpurun_out/b16.log | cut -c1-250

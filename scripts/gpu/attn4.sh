#!/bin/bash
# D=128 attention-bwd BQ=64 variant A/B + attention tests under it
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench/attn_bench.py --ours --configs 8x16x2048x128,2x16x1000x128,8x16x4096x128 --rounds 3 > gpurun_out/attn4.log 2>&1 || { echo "attn bench failed"; tail -20 gpurun_out/attn4.log; exit 3; }
grep -v amdgpu.ids gpurun_out/attn4.log | cut -c1-500
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "attention or model" > gpurun_out/ta4.log 2>&1
rc=$?; tail -2 gpurun_out/ta4.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/ta4.log | head -30; exit $rc; fi

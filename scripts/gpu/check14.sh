#!/bin/bash
# decode attention kernel + graphed decode tests, decode/serving bench
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "decode or graph" > gpurun_out/t14.log 2>&1
rc=$?; tail -3 gpurun_out/t14.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/t14.log | head -30; exit $rc; fi
timeout -k 10 300 python bench/decode_bench.py > gpurun_out/dec14.log 2>&1 || { echo "decode bench failed"; tail -20 gpurun_out/dec14.log; exit 3; }
grep -v amdgpu.ids gpurun_out/dec14.log

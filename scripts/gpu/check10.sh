#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -x -p no:cacheprovider > gpurun_out/t10.log 2>&1
rc=$?; tail -3 gpurun_out/t10.log
if [ $rc -gt 1 ]; then exit $rc; fi
if [ $rc -eq 1 ]; then grep -E "^E |FAILED" gpurun_out/t10.log | head -20; fi
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/b10.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/b10.log; exit 4; }
tail -1 gpurun_out/b10.log | cut -c1-200
bash scripts/gpu/prof.sh prof6 --steps 10 --warmup 3

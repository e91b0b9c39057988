#!/bin/bash
# GPU session 1: kernel numerics, then stock-torch baseline and HIP-path bench (gpt2-small, 1 GPU).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -q -x -p no:cacheprovider > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/t1.log
if [ $rc -gt 1 ] && [ $rc -ne 5 ]; then echo "stopping after pytest rc=$rc"; tail -30 gpurun_out/t1.log; exit $rc; fi
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --backend torch > gpurun_out/b_torch.log 2>&1 || { echo "torch bench failed"; tail -30 gpurun_out/b_torch.log; exit 3; }
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/b_auto.log 2>&1 || { echo "auto bench failed"; tail -30 gpurun_out/b_auto.log; exit 4; }
tail -5 gpurun_out/t1.log; cat gpurun_out/b_torch.log gpurun_out/b_auto.log

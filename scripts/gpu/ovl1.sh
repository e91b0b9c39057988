#!/bin/bash
# A/B: weight gradients on a side stream (PLLM_WGRAD_STREAM) -- numerics + headline bench
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PLLM_WGRAD_STREAM=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_dp_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "model or dp_engine or graphed_train" > gpurun_out/tovl.log 2>&1
rc=$?; tail -2 gpurun_out/tovl.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/tovl.log | head -20; exit $rc; fi
for i in 1 2; do
for f in 0 1; do
  PLLM_WGRAD_STREAM=$f timeout -k 10 300 python bench.py > gpurun_out/bovl_$f.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bovl_$f.log; exit 4; }
  echo "stream=$f $(tail -1 gpurun_out/bovl_$f.log | cut -c90-180)"
done
done

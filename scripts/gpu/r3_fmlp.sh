#!/bin/bash
# fused-MLP modes, whole GPT-2 step A/B/A/B (bwd = default)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/fmlp
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fmlp/tests.log 2>&1
rc=$?; tail -1 gpurun_out/fmlp/tests.log; [ $rc -ne 0 ] && exit $rc
for mode in 0 bwd all 0 bwd all; do
  PLLM_FUSED_MLP=$mode timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/fmlp/$mode.log 2>&1 || { tail -5 gpurun_out/fmlp/$mode.log; exit 1; }
  echo "$mode $(tail -1 gpurun_out/fmlp/$mode.log | cut -c100-190)"
done

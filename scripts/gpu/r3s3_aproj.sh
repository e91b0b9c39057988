#!/bin/bash
# fused attention-output projection backward (gemm_tn epilogue 6): full GPU suite, then the headline
# step with PLLM_ATTN_PROJ_FUSED=1 / 0 (A B B A A B)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/aproj_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/aproj_tests.log | tail -2; [ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/aproj_tests.log | head -20; exit $rc; }
bash scripts/gpu/r3s3_envab.sh aproj PLLM_ATTN_PROJ_FUSED 1 0 --steps 20 --warmup 5

#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python bench/gemm_bench.py > gpurun_out/gemm1.log 2>&1; rc=$?
cat gpurun_out/gemm1.log | grep -v amdgpu.ids
exit $rc

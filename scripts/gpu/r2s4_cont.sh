#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python scripts/gpu/cont_check.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python bench/serve_bench.py > gpurun_out/serve_bench.jsonl 2> gpurun_out/serve_bench.err || { tail -5 gpurun_out/serve_bench.err; exit 1; }
cat gpurun_out/serve_bench.jsonl

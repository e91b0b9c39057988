#!/bin/bash
# LM-head GEMM -> CE in Infinity-Cache-sized sub-chunks (PLLM_CE_SUB_ROWS), backward GEMMs once
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for sub in 0 1024 2048 4096 8192 0 2048 4096; do
  PLLM_CE_SUB_ROWS=$sub timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/cesub_$sub.log 2>&1 || { tail -5 gpurun_out/cesub_$sub.log; exit 1; }
  echo "sub=$sub $(tail -1 gpurun_out/cesub_$sub.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done

#!/bin/bash
# TunableOp tables for the llama-1.3B b16 and ref-3b b32 training GEMM shapes
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python scripts/tune_gemms.py --model llama-1.3b --batch 16 --steps 2 --tune-ms 40 --out gpurun_out/llama13b_b16_gfx950.csv > gpurun_out/r2_tune_llama.log 2>&1 || { tail -5 gpurun_out/r2_tune_llama.log; exit 1; }
tail -2 gpurun_out/r2_tune_llama.log
timeout -k 10 500 python scripts/tune_gemms.py --model ref-3b --batch 32 --steps 2 --tune-ms 40 --out gpurun_out/ref3b_b32_gfx950.csv > gpurun_out/r2_tune_ref3b.log 2>&1 || { tail -5 gpurun_out/r2_tune_ref3b.log; exit 1; }
tail -2 gpurun_out/r2_tune_ref3b.log

#!/bin/bash
# re-tune the GPT-2 small b64 GEMM shapes from scratch with a larger per-shape budget
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python scripts/tune_gemms.py --model gpt2-small --batch 64 --steps 2 --tune-ms 60 --fresh --out gpurun_out/gpt2small_b64_gfx950_v2.csv > gpurun_out/r2_tune2.log 2>&1 || { tail -5 gpurun_out/r2_tune2.log; exit 1; }
tail -2 gpurun_out/r2_tune2.log

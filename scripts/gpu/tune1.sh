#!/bin/bash
# TunableOp pass over the GPT-2-small B=64 training step (covers the W^T-shadow dgrad layouts)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u scripts/tune_gemms.py --model gpt2-small --batch 64 --out gpurun_out/tuned_gpt2small_b64.csv > gpurun_out/tune1.log 2>&1 || { echo "tune failed"; tail -20 gpurun_out/tune1.log; exit 3; }
tail -3 gpurun_out/tune1.log
grep -c . gpurun_out/tuned_gpt2small_b64.csv

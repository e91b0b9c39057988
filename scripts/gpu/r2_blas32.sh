#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python bench/wgrad_blas32.py > gpurun_out/r2_blas32.jsonl 2>&1; rc=$?
grep "^{" gpurun_out/r2_blas32.jsonl | cut -c1-300; tail -2 gpurun_out/r2_blas32.jsonl | cut -c1-300; exit $rc

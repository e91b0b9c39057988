#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PLLM_SO=$R/pretraining_llm_amd/_C_ppexp64.so timeout -k 10 120 python bench/gemm_pp_stamps.py --M 65536 --N 3072 --K 768 > gpurun_out/r4pp4_stamps_k768.jsonl 2>&1 || { tail -5 gpurun_out/r4pp4_stamps_k768.jsonl; exit 1; }
PLLM_SO=$R/pretraining_llm_amd/_C_ppexp64.so timeout -k 10 120 python bench/gemm_pp_stamps.py --M 32768 --N 2048 --K 2048 > gpurun_out/r4pp4_stamps_k2048.jsonl 2>&1 || { tail -5 gpurun_out/r4pp4_stamps_k2048.jsonl; exit 1; }
head -4 gpurun_out/r4pp4_stamps_k768.jsonl

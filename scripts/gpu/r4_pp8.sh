#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for shape in "65536 3072 768" "65536 2304 768" "65536 768 3072"; do
  set -- $shape
  for round in 1 2; do
    for v in "" 1 32; do
      so=""; [ -n "$v" ] && so="$R/pretraining_llm_amd/_C_ppexp$v.so"
      PLLM_SO=$so timeout -k 10 120 python bench/gemm_one.py --M $1 --N $2 --K $3 --phased 4 --no-blas --time 2>&1 | grep median || exit 1
    done
  done
done

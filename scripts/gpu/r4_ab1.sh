#!/bin/bash
# whole-step A/B: GEMM kernel (r3 vs ping-pong) and the forward GELU epilogue, GPT-2 small; llama
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python bench/gemm_tn_bench.py --swiglu > gpurun_out/r4ab1_swiglu.jsonl 2>&1 || { tail -3 gpurun_out/r4ab1_swiglu.jsonl; exit 1; }
cat gpurun_out/r4ab1_swiglu.jsonl
for round in 1 2 3; do
  for v in "r3 bwd" "pp bwd" "pp all"; do
    set -- $v
    PLLM_GEMM_KERNEL=$1 PLLM_FUSED_MLP=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4ab1_$1_$2_$round.log 2>&1 || { tail -3 gpurun_out/r4ab1_$1_$2_$round.log; exit 1; }
    echo "$1 $2 $(tail -1 gpurun_out/r4ab1_$1_$2_$round.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
  done
done
for v in r3 pp r3 pp; do
  PLLM_GEMM_KERNEL=$v timeout -k 10 400 python bench.py --model llama-1.3b --batch 16 --seq 2048 --steps 5 --warmup 2 > gpurun_out/r4ab1_llama_$v.log 2>&1 || { tail -3 gpurun_out/r4ab1_llama_$v.log; exit 1; }
  echo "llama $v $(tail -1 gpurun_out/r4ab1_llama_$v.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
done

#!/bin/bash
# numerics bisection on llama-1.3B (150 steps, same seed / batches): HIP path with one op family at a
# time moved to stock PyTorch ops (PLLM_TORCH_OPS), against the fp32 and bf16 stock-op curves
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/bisect
export HSA_ENABLE_IPC_MODE_LEGACY=0
A="--model llama-1.3b --steps 150 --batch 4 --seq 2048 --lr 3e-4"
timeout -k 10 400 python -u scripts/convergence.py $A --backends torch:float32,torch,auto --out gpurun_out/bisect/base.jsonl 2> gpurun_out/bisect/base.log || { tail -5 gpurun_out/bisect/base.log; exit 1; }
grep "final" gpurun_out/bisect/base.log
for ops in attn ce norm,act linear embed; do
  PLLM_TORCH_OPS=$ops timeout -k 10 300 python -u scripts/convergence.py $A --backends auto --out gpurun_out/bisect/$ops.jsonl 2> gpurun_out/bisect/$ops.log || { tail -5 gpurun_out/bisect/$ops.log; exit 2; }
  echo "torch ops=$ops: $(grep final gpurun_out/bisect/$ops.log)"
done

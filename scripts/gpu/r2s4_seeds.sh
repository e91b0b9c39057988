#!/bin/bash
# is the HIP-vs-stock-bf16 loss gap on llama-1.3B systematic or trajectory noise?  3 more seeds x both paths
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/seeds
export HSA_ENABLE_IPC_MODE_LEGACY=0
A="--model llama-1.3b --steps 150 --batch 4 --seq 2048 --lr 3e-4"
for seed in 1 2 3; do
  timeout -k 10 300 python -u scripts/convergence.py $A --seed $seed --backends auto,torch --out gpurun_out/seeds/s$seed.jsonl 2> gpurun_out/seeds/s$seed.log || { tail -5 gpurun_out/seeds/s$seed.log; exit 1; }
  echo "seed $seed: $(grep 'final' gpurun_out/seeds/s$seed.log | tr '\n' ' ')"
done

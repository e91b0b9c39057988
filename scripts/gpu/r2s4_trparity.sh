#!/bin/bash
# Trainer (reference CLI, Markov/Zipf synthetic shard) vs bench.py at the llama-1.3B (B=16, T=2048)
# and GPT-2-medium seq4096 (B=8, auto checkpointing) configs
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python scripts/train_transformer.py --preset=llama-1.3b --t_batch_size=16 --t_train_steps=13 \
  --t_eval_steps=1000 --eval_at_start=False --log_interval=6 --synthetic_data=True --synthetic_dir=/tmp/pllm_syn \
  --t_out_path=None > gpurun_out/s4_tr_llama.log 2>&1 || { echo "llama trainer failed"; tail -20 gpurun_out/s4_tr_llama.log; exit 3; }
grep -E "Step|model:" gpurun_out/s4_tr_llama.log | cut -c1-200
timeout -k 10 500 python scripts/train_transformer.py --preset=gpt2-medium-4k --t_train_steps=13 \
  --t_eval_steps=1000 --eval_at_start=False --log_interval=6 --synthetic_data=True --synthetic_dir=/tmp/pllm_syn \
  --t_out_path=None > gpurun_out/s4_tr_med.log 2>&1 || { echo "medium trainer failed"; tail -20 gpurun_out/s4_tr_med.log; exit 4; }
grep -E "Step|model:" gpurun_out/s4_tr_med.log | cut -c1-200

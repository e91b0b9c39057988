#!/bin/bash
# End-to-end on the GPU: reference-compatible trainer CLI (GPT-2 small, synthetic shards, eval,
# periodic checkpoint, resume), then generate_text.py from the saved checkpoint.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/e2e
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python scripts/train_transformer.py --run=gpt2-small --t_train_steps=40 --t_eval_steps=20 \
  --log_interval=10 --t_eval_iters=2 --synthetic_data=True --synthetic_dir=/tmp/pllm_syn --ckpt_interval=20 \
  --t_out_path=/tmp/pllm_ck/gpt2s.pt --metrics_path=gpurun_out/e2e/metrics.jsonl > gpurun_out/e2e/train.log 2>&1 \
  || { echo "train failed"; tail -20 gpurun_out/e2e/train.log; exit 3; }
grep -E "Step|saved|model:" gpurun_out/e2e/train.log | cut -c1-200
timeout -k 10 300 python scripts/train_transformer.py --run=gpt2-small --t_train_steps=50 --t_eval_steps=20 \
  --log_interval=10 --t_eval_iters=2 --synthetic_data=True --synthetic_dir=/tmp/pllm_syn --resume=/tmp/pllm_ck/gpt2s.latest.pt \
  --t_out_path=/tmp/pllm_ck/gpt2s_b.pt > gpurun_out/e2e/resume.log 2>&1 || { echo "resume failed"; tail -20 gpurun_out/e2e/resume.log; exit 4; }
grep -E "resumed|Step" gpurun_out/e2e/resume.log | cut -c1-200
timeout -k 10 300 python scripts/generate_text.py --model_path /tmp/pllm_ck/gpt2s.pt --input_text "The MI355X" \
  --max_new_tokens 32 --seed 1 > gpurun_out/e2e/gen.log 2>&1 || { echo "generate failed"; tail -20 gpurun_out/e2e/gen.log; exit 5; }
tail -3 gpurun_out/e2e/gen.log | cut -c1-300

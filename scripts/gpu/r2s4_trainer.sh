#!/bin/bash
# Trainer (reference CLI) throughput vs bench.py at the same config (GPT-2 small, 64 x 1024),
# then the 2-rank TP+SP trainer run (gloo on the one GPU) and the ZeRO-1 bench path
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python scripts/train_transformer.py --preset=gpt2-small --t_batch_size=64 --t_train_steps=41 \
  --t_eval_steps=1000 --eval_at_start=False --log_interval=10 --synthetic_data=True --synthetic_dir=/tmp/pllm_syn \
  --t_out_path=None > gpurun_out/s4_trainer.log 2>&1 || { echo "trainer failed"; tail -20 gpurun_out/s4_trainer.log; exit 3; }
grep -E "Step|model:" gpurun_out/s4_trainer.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/s4_bench_t.log 2>&1 || { tail -5 gpurun_out/s4_bench_t.log; exit 4; }
tail -1 gpurun_out/s4_bench_t.log | cut -c1-200
PLLM_DIST_BACKEND=gloo PLLM_DIST_ONE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 scripts/train_transformer.py --preset=llama-1.3b \
  --override_preset_dims=True --n_blocks=2 --t_batch_size=2 --tp_size=2 --sequence_parallel=True --t_train_steps=6 \
  --t_eval_steps=3 --log_interval=2 --t_eval_iters=1 --synthetic_data=True --synthetic_dir=/tmp/pllm_syn_l \
  --t_out_path=/tmp/pllm_ck/llama_tp.pt > gpurun_out/s4_tp.log 2>&1 || { echo "tp train failed"; tail -20 gpurun_out/s4_tp.log; exit 6; }
grep -E "Step|model:" gpurun_out/s4_tp.log | cut -c1-200
timeout -k 10 300 python bench.py --zero 1 --steps 10 --warmup 3 > gpurun_out/s4_zero.log 2>&1 || { tail -5 gpurun_out/s4_zero.log; exit 7; }
tail -1 gpurun_out/s4_zero.log | cut -c1-200

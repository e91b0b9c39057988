#!/bin/bash
# kernel-time profile of the Trainer path (reference CLI) at the bench config, to find what makes
# it slower than bench.py; plus the TP+SP trainer run and the ZeRO-1 bench path
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/s4_trprof
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/s4_trprof" -o run --output-format csv -- \
  python3 "$R/scripts/train_transformer.py" --preset=gpt2-small --t_batch_size=64 --t_train_steps=21 \
  --t_eval_steps=1000 --eval_at_start=False --log_interval=10 --synthetic_data=True --synthetic_dir=/tmp/pllm_syn \
  --t_out_path=None > "$R/gpurun_out/s4_trprof/train.log" 2>&1 || { echo "prof failed"; tail -20 "$R/gpurun_out/s4_trprof/train.log"; exit 3; }
cd "$R"
grep -E "Step" gpurun_out/s4_trprof/train.log | cut -c1-200
python scripts/prof_summary.py gpurun_out/s4_trprof/run_kernel_stats.csv 21 "Trainer GPT-2 small B=64 T=1024" > gpurun_out/s4_trprof.md
head -40 gpurun_out/s4_trprof.md
PLLM_DIST_BACKEND=gloo PLLM_DIST_ONE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 scripts/train_transformer.py --preset=llama-1.3b \
  --override_preset_dims=True --n_blocks=2 --t_batch_size=2 --tp_size=2 --sequence_parallel=True --t_train_steps=6 \
  --t_eval_steps=3 --log_interval=2 --t_eval_iters=1 --synthetic_data=True --synthetic_dir=/tmp/pllm_syn_l \
  --t_out_path=/tmp/pllm_ck/llama_tp.pt > gpurun_out/s4_tp.log 2>&1 || { echo "tp train failed"; grep -v "^\s*$" gpurun_out/s4_tp.log | grep -B5 Error | head -30; exit 6; }
grep -E "Step|model:" gpurun_out/s4_tp.log | cut -c1-200
timeout -k 10 300 python bench.py --zero 1 --steps 10 --warmup 3 > gpurun_out/s4_zero.log 2>&1 || { tail -5 gpurun_out/s4_zero.log; exit 7; }
tail -1 gpurun_out/s4_zero.log | cut -c1-200

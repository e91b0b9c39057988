#!/bin/bash
# RCCL / DP-bucket sweep for an 8-GPU MI355X node (xGMI, 7 links per GPU).  NOT for the 1-GPU
# boxes: run it on a whole node, e.g.  bash scripts/gpu/rccl_sweep.sh 8 > rccl_sweep.jsonl
#   1. collective bus bandwidth vs message size at RCCL's default channel count and pinned ones
#      (bench/comm_bench.py): where the busbw knee sits = the smallest bucket that stops paying latency
#   2. the headline training step (bench.py) over channel counts x bucket sizes x comm-stream
#      priority, each line carrying exposed_comm_ms / bucket_launch_ms / rank_step_ms_{min,max}
# Every step runs under its own time limit; the sweep stops at the first failure.
set -eo pipefail
N="${1:-8}"
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R"
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { timeout -k 10 600 "$@" || { echo "{\"failed\": \"$*\"}"; exit 1; }; }
TR=(python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1)
for ch in default 8 16 32; do
  extra=(); [ "$ch" != default ] && extra=(--rccl-channels "$ch")
  run "${TR[@]}" --master-port $((29500 + RANDOM % 1000)) bench/comm_bench.py --dtype float32 --ops all_reduce,reduce_scatter,all_gather \
      --sizes-mb 4,16,32,64,128,256 "${extra[@]}" | sed "s/^{/{\"channels\": \"$ch\", /"
done
for ch in default 16 32; do
  for bmb in 32 64 128; do
    for prio in 0 1; do
      extra=(--bucket-mb "$bmb" --rccl-env "TORCH_NCCL_HIGH_PRIORITY=$prio")
      [ "$ch" != default ] && extra+=(--rccl-channels "$ch")
      run "${TR[@]}" --master-port $((29500 + RANDOM % 1000)) bench.py --gpus "$N" --steps 20 --warmup 5 "${extra[@]}" | sed "s/^{/{\"sweep\": \"ch=$ch bucket=$bmb prio=$prio\", /"
    done
  done
done

#!/bin/bash
# 2-rank bench.py rehearsal on a one-GPU box: bench.py launches its own ranks for --gpus 2 (no
# hand-written torchrun); both ranks on device 0 with gloo collectives on the CUDA tensors --
# exercises the multi-rank path (self-launch, DP engine hooks, per-rank loaders, timing max over
# ranks, rank-0 JSON) end to end; the tokens/s it prints is NOT a scaling measurement.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PLLM_DIST_BACKEND=gloo PLLM_DIST_ONE_DEVICE=1
timeout -k 10 400 python bench.py --gpus 2 --steps 4 --warmup 2 --batch 16 > gpurun_out/dpr.log 2>&1
rc=$?; tail -3 gpurun_out/dpr.log | cut -c1-600; exit $rc

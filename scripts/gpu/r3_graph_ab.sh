#!/bin/bash
# headline bench: eager step vs the whole step replayed as one hipGraph, A/B/A/B
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/graph
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in eager graph eager graph; do
  if [ $v = graph ]; then F=--cuda-graph; else F=; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 $F > gpurun_out/graph/$v.log 2>&1 || { tail -5 gpurun_out/graph/$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/graph/$v.log | cut -c80-200)"
done

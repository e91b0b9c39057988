#!/bin/bash
# phase-removal timing experiments of the fused attention backward (xso/_C_<X>.so builds)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in base NODQ NOEXP NOSTAGE NOSUB; do
  so="$R/pretraining_llm_amd/_C.so"; [ "$v" != base ] && so="$R/xso/_C_$v.so"
  PLLM_SO=$so timeout -k 10 120 python bench/attn_bench.py --configs 64x12x1024x64,8x16x4096x64 --ours --rounds 3 > gpurun_out/r2ax_$v.jsonl 2>&1 || { echo "$v failed"; tail -3 gpurun_out/r2ax_$v.jsonl; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/r2ax_$v.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('$v', d['cfg'], round(min(d['bwd_us']),1))"
done

#!/bin/bash
# A/B: global vs buffer loads (PLLM_SO) x grid order (PLLM_ATTN_ORDER)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for so in _C.so _C_buf.so; do
  for ord in 0 1; do
    PLLM_SO="$R/pretraining_llm_amd/$so" PLLM_ATTN_ORDER=$ord timeout -k 10 200 python bench/attn_bench.py --configs 64x12x1024x64,16x16x2048x128 --rounds 3 > gpurun_out/r2a4_${so}_$ord.jsonl 2>&1 || exit 1
    echo "$so order=$ord"; python3 -c "
import json
for l in open('gpurun_out/r2a4_${so}_$ord.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d['cfg'], 'fwd', round(min(d['ours_fwd_us']),1), 'bwd', round(min(d['ours_bwd_us']),1))"
  done
done

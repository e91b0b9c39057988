#!/bin/bash
# same-box A/B of attention builds: current _C.so vs xso/_C_<tag>.so, interleaved rounds
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
CFG=${CFG:-64x12x1024x64,16x16x2048x128,8x16x4096x64}
for round in 1 2; do
  for v in cur $(ls xso | sed -e 's/^_C_//' -e 's/\.so$//'); do
    so="$R/pretraining_llm_amd/_C.so"; [ "$v" != cur ] && so="$R/xso/_C_$v.so"
    PLLM_SO=$so timeout -k 10 120 python bench/attn_bench.py --configs $CFG --ours --rounds 3 > gpurun_out/r2ab_$v.jsonl 2>&1 || { echo "$v failed"; tail -3 gpurun_out/r2ab_$v.jsonl; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/r2ab_$v.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('$round $v', d['cfg'], 'bwd', round(min(d['bwd_us']),1), 'fwd', round(min(d['fwd_us']),1))"
  done
done

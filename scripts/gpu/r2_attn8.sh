#!/bin/bash
# round 2: backward sub-block without per-element branches, explicit swizzle addressing, no spills
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention or attn" -x -q --timeout 200 --timeout-method thread > gpurun_out/r2a8_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r2a8_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench/attn_bench.py --configs 64x12x1024x64,16x16x2048x128,8x16x4096x64,32x16x512x128 --ours --rounds 3 > gpurun_out/r2a8_bench.jsonl 2>&1
rc=$?; python3 -c "
import json
for l in open('gpurun_out/r2a8_bench.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d['cfg'], {k: round(min(v),1) if isinstance(v,list) else round(v,4) for k,v in d.items() if k!='cfg'})"
exit $rc

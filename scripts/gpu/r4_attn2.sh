#!/bin/bash
# asymmetric Q/dO DMA in the D<=64 attention backward (PLLM_BWD_QASYM=1 build) vs default
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PLLM_SO=$R/pretraining_llm_amd/_C_qasym.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/r4a2_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error|assert" gpurun_out/r4a2_tests.log | tail -6; [ $rc -ne 0 ] && exit $rc
for round in 1 2 3; do
  for so in "" qasym; do
    s=""; [ -n "$so" ] && s="$R/pretraining_llm_amd/_C_$so.so"
    PLLM_SO=$s timeout -k 10 120 python bench/attn_bench.py --ours --configs 64x12x1024x64,8x16x4096x64 --rounds 3 2>&1 | grep -v amdgpu.ids | python -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print('[${so:-base}]', r['cfg'], 'bwd', round(min(r['bwd_us']),1))" || exit 1
  done
done
for v in "" qasym; do
  s=""; [ -n "$v" ] && s="$R/pretraining_llm_amd/_C_$v.so"
  PLLM_SO=$s timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r4a2_gpt2_${v:-base}.log 2>&1 || { tail -3 gpurun_out/r4a2_gpt2_${v:-base}.log; exit 1; }
  echo "gpt2 ${v:-base} $(tail -1 gpurun_out/r4a2_gpt2_${v:-base}.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
done

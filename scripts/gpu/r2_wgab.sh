#!/bin/bash
# same-box A/B of wgrad builds: current _C.so vs xso/_C_<tag>.so (gemm_bench, hand-written kernel only)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for shapes in gpt2 llama; do
  M=65536; [ $shapes = llama ] && M=32768
  for v in cur $(ls xso | sed -e 's/^_C_//' -e 's/\.so$//'); do
    so="$R/pretraining_llm_amd/_C.so"; [ "$v" != cur ] && so="$R/xso/_C_$v.so"
    PLLM_SO=$so timeout -k 10 200 python bench/gemm_bench.py --shapes $shapes --M $M --variants 32 --rounds 2 > gpurun_out/r2wg_${v}_$shapes.jsonl 2>&1 || { echo "$v failed"; tail -3 gpurun_out/r2wg_${v}_$shapes.jsonl; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/r2wg_${v}_$shapes.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('$v', d['P'], d['Q'], d['M'], 'hip', round(min(d['hip32_us']),1), round(d['hip32_tflops']), 'blas', round(d['blas_tflops']), 'err', round(d['rel_err32'],5))"
  done
done

#!/bin/bash
# 4-wave (128x128 per wave) wgrad variant: numerics, then kernel A/B vs the 8-wave default on the
# GPT-2 / llama training shapes (fp32 gradient targets), then the headline step with each
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k wgrad --timeout 120 --timeout-method thread > gpurun_out/wg4_tests.log 2>&1
rc=$?; tail -2 gpurun_out/wg4_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench/gemm_bench.py --f32 --variants 32,4 --rounds 3 > gpurun_out/wg4_gpt2.jsonl 2>&1 || { tail -5 gpurun_out/wg4_gpt2.jsonl; exit 1; }
timeout -k 10 300 python bench/gemm_bench.py --f32 --variants 32,4 --rounds 2 --shapes llama --M 32768 > gpurun_out/wg4_llama.jsonl 2>&1 || { tail -5 gpurun_out/wg4_llama.jsonl; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/wg4_gpt2.jsonl", "gpurun_out/wg4_llama.jsonl"):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); print(d["P"], d["Q"], d["M"], "v32 %.0f" % d["hip32_tflops"], "v4 %.0f" % d["hip4_tflops"], "err4 %.2e" % d["rel_err4"])
PY
for v in 32 4 32 4; do
  PLLM_WGRAD_VARIANT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/wg4_bench_$v.log 2>&1 || { tail -5 gpurun_out/wg4_bench_$v.log; exit 1; }
  echo "variant $v: $(tail -1 gpurun_out/wg4_bench_$v.log | cut -c1-200)"
done

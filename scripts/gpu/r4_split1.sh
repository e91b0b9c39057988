#!/bin/bash
# GEMM tests (incl. epilogue 7 and the tile split), split A/B on the training shapes, llama
# SwiGLU-forward epilogue A/B
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4s1_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error" gpurun_out/r4s1_tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench/gemm_pp_bench.py --fused --no-r3 --rounds 5 > gpurun_out/r4s1_bench.jsonl 2>&1 || { tail -5 gpurun_out/r4s1_bench.jsonl; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r4s1_bench.jsonl"):
    if l.startswith("{"):
        r = json.loads(l); print({k: v for k, v in r.items() if k.endswith("_us") and "min" not in k} | {"shape": (r["M"], r["N"], r["K"])})
PY
for v in 0 1; do
  PLLM_GEMM_SPLIT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r4s1_gpt2_$v.log 2>&1 || { tail -3 gpurun_out/r4s1_gpt2_$v.log; exit 1; }
  echo "gpt2 split=$v $(tail -1 gpurun_out/r4s1_gpt2_$v.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
done
for v in 0 1; do
  PLLM_FUSED_SWIGLU_FWD=$v timeout -k 10 400 python bench.py --model llama-1.3b --batch 16 --seq 2048 --steps 5 --warmup 2 > gpurun_out/r4s1_llama_$v.log 2>&1 || { tail -3 gpurun_out/r4s1_llama_$v.log; exit 1; }
  echo "llama swiglu_fwd_epi=$v $(tail -1 gpurun_out/r4s1_llama_$v.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
done

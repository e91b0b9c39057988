#!/bin/bash
# K-tile DMA pieces among the phase's own MFMAs (PLLM_PP_DMA_MFMA / PLLM_WP_DMA_MFMA builds) vs the LOAD segment
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PLLM_SO=$R/pretraining_llm_amd/_C_ppdm.so timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4dm_tests1.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error|assert" gpurun_out/r4dm_tests1.log | tail -6; [ $rc -ne 0 ] && exit $rc
PLLM_SO=$R/pretraining_llm_amd/_C_wpdm.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k wgrad --timeout 120 --timeout-method thread > gpurun_out/r4dm_tests2.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error|assert" gpurun_out/r4dm_tests2.log | tail -6; [ $rc -ne 0 ] && exit $rc
for round in 1 2; do
  for so in "" ppdm; do
    s=""; [ -n "$so" ] && s="$R/pretraining_llm_amd/_C_$so.so"
    PLLM_SO=$s timeout -k 10 200 python bench/gemm_pp_bench.py --no-r3 --rounds 3 --fused > gpurun_out/r4dm_pp_${so:-base}_$round.jsonl 2>&1 || { tail -3 gpurun_out/r4dm_pp_${so:-base}_$round.jsonl; exit 1; }
  done
  for so in "" wpdm; do
    s=""; [ -n "$so" ] && s="$R/pretraining_llm_amd/_C_$so.so"
    PLLM_SO=$s timeout -k 10 200 python bench/wgrad_time.py > gpurun_out/r4dm_wg_${so:-base}_$round.jsonl 2>&1 || { tail -3 gpurun_out/r4dm_wg_${so:-base}_$round.jsonl; exit 1; }
  done
done
python - <<'PY'
import json, glob
def load(pat):
    out = {}
    for f in sorted(glob.glob(pat)):
        for l in open(f):
            if l.startswith("{"):
                r = json.loads(l)
                key = tuple(r.get(k) for k in ("M", "N", "K", "P", "Q"))
                out.setdefault(key, []).append(r)
    return out
for tag in ("pp", "wg"):
    b = load(f"gpurun_out/r4dm_{tag}_base_*.jsonl")
    v = load(f"gpurun_out/r4dm_{tag}_{'ppdm' if tag == 'pp' else 'wpdm'}_*.jsonl")
    for k in b:
        if tag == "pp":
            f = lambda rs, n: [r.get(n) for r in rs]
            print(tag, k, "pp_ns", f(b[k], "pp_ns_us"), "->", f(v.get(k, []), "pp_ns_us"), "| gelu", f(b[k], "pp_ns_gelu_us"), "->", f(v.get(k, []), "pp_ns_gelu_us"), "| dgelu", f(b[k], "pp_dgelu_us"), "->", f(v.get(k, []), "pp_dgelu_us"), "| blas", f(b[k], "blas_us"))
        else:
            print(tag, k, [r["us"] for r in b[k]], "->", [r["us"] for r in v.get(k, [])])
PY

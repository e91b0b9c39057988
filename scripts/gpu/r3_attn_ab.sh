#!/bin/bash
# attention A/B: in-tree _C.so ("new") vs pretraining_llm_amd/_C_base.so ("base"): attention
# tests, kernel times at the GPT-2 / llama / GPT-2-medium shapes, headline bench.  $1 = tag,
# $2 = "bench" to also run the headline A/B, $3 = extra pytest -k filter
R="${GRAFT_REPO_ROOT:-/root/repo}"
T="${1:-ab}"
cd "$R"; mkdir -p gpurun_out/$T
O="$R/gpurun_out/$T"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_cp_gpu.py -q -x -k "${3:-attn or attention or flash or rope}" --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^E " $O/tests.log | head -20; exit $rc; }
for so in base new base new; do
  if [ $so = base ]; then export PLLM_SO=$R/pretraining_llm_amd/_C_base.so; else unset PLLM_SO; fi
  timeout -k 10 300 python bench/attn_bench.py --ours --configs 64x12x1024x64,16x16x2048x128,8x16x4096x64 --rounds 3 > $O/attn_$so.log 2>&1 || { tail -5 $O/attn_$so.log; exit 1; }
  echo "$so: $(grep -h '^{' $O/attn_$so.log | python -c 'import sys,json; [print(json.loads(l)["cfg"], "fwd", round(min(json.loads(l)["fwd_us"]),1), "bwd", round(min(json.loads(l)["bwd_us"])), end=" | ") for l in sys.stdin]')"
done
if [ "$2" = bench ]; then
for so in base new base new; do
  if [ $so = base ]; then export PLLM_SO=$R/pretraining_llm_amd/_C_base.so; else unset PLLM_SO; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_$so.log 2>&1 || { tail -5 $O/bench_$so.log; exit 1; }
  echo "$so bench: $(tail -1 $O/bench_$so.log | cut -c80-135)"
done
fi

#!/bin/bash
# attention forward: P row sums by MFMA against an all-ones operand (variant .so) vs VALU adds
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
V=$R/pretraining_llm_amd/_C_rowsum.so
PLLM_SO=$V timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "attn or attention or flash" --timeout 120 --timeout-method thread > gpurun_out/rowsum_tests.log 2>&1
rc=$?; tail -2 gpurun_out/rowsum_tests.log; [ $rc -ne 0 ] && exit $rc
for so in base var base var; do
  if [ $so = var ]; then export PLLM_SO=$V; else unset PLLM_SO; fi
  timeout -k 10 300 python bench/attn_bench.py --ours --configs 64x12x1024x64,16x16x2048x128 --rounds 3 > gpurun_out/rowsum_attn_$so.log 2>&1 || { tail -5 gpurun_out/rowsum_attn_$so.log; exit 1; }
  echo "$so: $(grep -h '^{' gpurun_out/rowsum_attn_$so.log | python -c 'import sys,json; [print(json.loads(l)["cfg"], [round(x) for x in json.loads(l)["fwd_us"]], round(min(json.loads(l)["bwd_us"])), end=" | ") for l in sys.stdin]')"
done
for so in base var base var; do
  if [ $so = var ]; then export PLLM_SO=$V; else unset PLLM_SO; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/rowsum_bench_$so.log 2>&1 || { tail -5 gpurun_out/rowsum_bench_$so.log; exit 1; }
  echo "$so bench: $(tail -1 gpurun_out/rowsum_bench_$so.log | cut -c80-135)"
done

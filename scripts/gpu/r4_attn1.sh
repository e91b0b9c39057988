#!/bin/bash
# D=128 forward with 8 waves per workgroup (PLLM_FWD128_NW=8 build) vs the 4-wave default
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PLLM_SO=$R/pretraining_llm_amd/_C_fwd8.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/r4a1_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error|assert" gpurun_out/r4a1_tests.log | tail -12; [ $rc -ne 0 ] && exit $rc
for round in 1 2; do
  for so in "" fwd8; do
    s=""; [ -n "$so" ] && s="$R/pretraining_llm_amd/_C_$so.so"
    PLLM_SO=$s timeout -k 10 120 python bench/attn_bench.py --ours --configs 16x16x2048x128,8x16x4096x128 --rounds 3 2>&1 | grep -v amdgpu.ids | sed "s/^/[${so:-base}] /" || exit 1
  done
done
PLLM_SO=$R/pretraining_llm_amd/_C_qspread.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/r4a1_tests_q.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error|assert" gpurun_out/r4a1_tests_q.log | tail -12; [ $rc -ne 0 ] && exit $rc
for round in 1 2; do
  for so in "" qspread; do
    s=""; [ -n "$so" ] && s="$R/pretraining_llm_amd/_C_$so.so"
    PLLM_SO=$s timeout -k 10 120 python bench/attn_bench.py --ours --configs 64x12x1024x64,8x16x4096x64 --rounds 3 2>&1 | grep -v amdgpu.ids | sed "s/^/[${so:-base}] /" || exit 1
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q -k "attn_proj or attn_delta" --timeout 120 --timeout-method thread > gpurun_out/r4a1_tests_p.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error|assert" gpurun_out/r4a1_tests_p.log | tail -12; [ $rc -ne 0 ] && exit $rc
for v in 0 1; do
  PLLM_ATTN_PROJ_D128=$v timeout -k 10 400 python bench.py --model llama-1.3b --batch 16 --seq 2048 --steps 5 --warmup 2 > gpurun_out/r4a1_llama_$v.log 2>&1 || { tail -3 gpurun_out/r4a1_llama_$v.log; exit 1; }
  echo "llama attn_proj_d128=$v $(tail -1 gpurun_out/r4a1_llama_$v.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
done

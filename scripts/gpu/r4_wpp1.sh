#!/bin/bash
# ping-pong wgrad: tests, A/B against the one-barrier kernel, long-K ceiling, GPT-2 step A/B
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "wgrad" --timeout 120 --timeout-method thread > gpurun_out/r4w1_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error|assert" gpurun_out/r4w1_tests.log | tail -12; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench/wgrad_time.py --variants 0,100 > gpurun_out/r4w1_wgrad.jsonl 2>&1 || { tail -5 gpurun_out/r4w1_wgrad.jsonl; exit 1; }
cat gpurun_out/r4w1_wgrad.jsonl
for v in 100 0; do
  PLLM_WGRAD_VARIANT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r4w1_gpt2_$v.log 2>&1 || { tail -3 gpurun_out/r4w1_gpt2_$v.log; exit 1; }
  echo "gpt2 wgrad=$v $(tail -1 gpurun_out/r4w1_gpt2_$v.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
done
timeout -k 10 300 python bench/gemm_longk.py > gpurun_out/r4w1_longk.jsonl 2>&1 || { tail -5 gpurun_out/r4w1_longk.jsonl; exit 1; }
cat gpurun_out/r4w1_longk.jsonl

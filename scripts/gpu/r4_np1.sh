#!/bin/bash
# non-persistent GEMM grids (one workgroup per tile): tests + whole-step cost at world 1
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q -k "persistent or reserved" --timeout 120 --timeout-method thread > gpurun_out/r4np_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error|assert" gpurun_out/r4np_tests.log | tail -6; [ $rc -ne 0 ] && exit $rc
for round in 1 2; do
  for v in 1 0; do
    PLLM_GEMM_PERSISTENT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r4np_gpt2_${v}_$round.log 2>&1 || { tail -3 gpurun_out/r4np_gpt2_${v}_$round.log; exit 1; }
    echo "gpt2 persistent=$v $(tail -1 gpurun_out/r4np_gpt2_${v}_$round.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
  done
done
for v in 1 0; do
  PLLM_GEMM_PERSISTENT=$v timeout -k 10 400 python bench.py --model llama-1.3b --batch 16 --seq 2048 --steps 5 --warmup 2 > gpurun_out/r4np_llama_$v.log 2>&1 || { tail -3 gpurun_out/r4np_llama_$v.log; exit 1; }
  echo "llama persistent=$v $(tail -1 gpurun_out/r4np_llama_$v.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
done

#!/bin/bash
# LayerNorm forward: half-wave rows for C = 768 (default build) vs one row per wave (_C_fullwave.so)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "norm" --timeout 120 --timeout-method thread > gpurun_out/ln_tests.log 2>&1
rc=$?; tail -1 gpurun_out/ln_tests.log; [ $rc -ne 0 ] && exit $rc
for so in base full base full; do
  if [ $so = full ]; then export PLLM_SO=$R/pretraining_llm_amd/_C_fullwave.so; else unset PLLM_SO; fi
  echo "$so: $(timeout -k 10 120 python scripts/gpu/ln_mb.py 2>&1 | tail -1)"
done
for so in base full base full; do
  if [ $so = full ]; then export PLLM_SO=$R/pretraining_llm_amd/_C_fullwave.so; else unset PLLM_SO; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ln_bench_$so.log 2>&1 || { tail -5 gpurun_out/ln_bench_$so.log; exit 1; }
  echo "$so bench: $(tail -1 gpurun_out/ln_bench_$so.log | cut -c80-135)"
done

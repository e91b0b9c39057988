#!/bin/bash
# round 2: convergence HIP vs stock torch, transpose fix, benches of the three training configs
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_convergence_gpu.py tests/test_kernels_gpu.py -k "convergence or transpose or tracks" -x -q --timeout 300 --timeout-method thread > gpurun_out/r2c2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2c2_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python scripts/convergence.py --model gpt2-small --steps 400 --batch 16 --out gpurun_out/r2_convergence_gpt2small.jsonl > gpurun_out/r2c2_conv.log 2>&1
rc=$?; tail -3 gpurun_out/r2c2_conv.log; [ $rc -ne 0 ] && exit $rc
for m in "ref-3b --batch 32" "gpt2-small" "llama-1.3b --batch 16"; do
  timeout -k 10 400 python bench.py --model $m --steps 10 --warmup 3 > gpurun_out/r2c2_bench.log 2>&1
  rc=$?; tail -1 gpurun_out/r2c2_bench.log | cut -c1-700; [ $rc -ne 0 ] && exit $rc
done
exit 0

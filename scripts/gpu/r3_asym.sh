#!/bin/bash
# asymmetric-DMA (waves 0-3 load, 4-7 compute first) A/B for the TN GEMM and the wgrad GEMM
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/asym
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_kernels_gpu.py -k "gemm or wgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/asym/tests.log 2>&1
rc=$?; tail -2 gpurun_out/asym/tests.log; [ $rc -ne 0 ] && exit $rc
for round in 1 2; do
for cfg in "0 16" "2 16" "0 32" "2 32"; do
  set -- $cfg
  timeout -k 10 300 python bench/gemm_tn_bench.py --phased $1 --mf $2 > gpurun_out/asym/g_$1_$2_$round.log 2>&1 || { tail -3 gpurun_out/asym/g_$1_$2_$round.log; exit 1; }
  echo "gemm ph$1 mf$2: $(grep '^{' gpurun_out/asym/g_$1_$2_$round.log | python -c 'import sys,json; print(" | ".join("%d %d %.0f/%.0f" % (d["N"], d["K"], d["ours_tflops"], d["blas_tflops"]) for d in map(json.loads, sys.stdin)))')"
done
for v in 32 132 16 116; do
  PLLM_WGRAD_VARIANT=$v timeout -k 10 300 python bench/wgrad_time.py > gpurun_out/asym/w_${v}_$round.log 2>&1 || { tail -3 gpurun_out/asym/w_${v}_$round.log; exit 1; }
  echo "wgrad $v: $(python -c 'import sys,json; [print(d["P"], d["Q"], d["tflops"], end=" | ") for d in map(json.loads, [l for l in open(sys.argv[1]) if l.startswith("{")])]' gpurun_out/asym/w_${v}_$round.log)"
done
done

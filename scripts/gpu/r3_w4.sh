#!/bin/bash
# one-wave-per-SIMD (W4) TN GEMM vs the 8-wave kernel vs hipBLASLt
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/w4
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/w4/tests.log 2>&1
rc=$?; tail -2 gpurun_out/w4/tests.log; [ $rc -ne 0 ] && exit $rc
for round in 1 2; do
for cfg in "0 16" "3 16"; do
  set -- $cfg
  timeout -k 10 300 python bench/gemm_tn_bench.py --phased $1 --mf $2 --fused > gpurun_out/w4/g_$1_$2_$round.log 2>&1 || { tail -3 gpurun_out/w4/g_$1_$2_$round.log; exit 1; }
  echo "gemm ph$1 mf$2: $(grep '^{' gpurun_out/w4/g_$1_$2_$round.log | python -c 'import sys,json; print(" | ".join("%d %d %.0f/%.0f %s %s" % (d["N"], d["K"], d["ours_tflops"], d["blas_tflops"], d.get("fused_gelu_us",""), d.get("fused_dgelu_us","")) for d in map(json.loads, sys.stdin)))')"
done
done

#!/bin/bash
# phased vs single-phase TN GEMM: numerics tests, then timing vs hipBLASLt, then whole-step fused-MLP modes
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/gemm2
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm2/tests.log 2>&1
rc=$?; tail -3 gpurun_out/gemm2/tests.log; [ $rc -ne 0 ] && exit $rc
for cfg in "1 16" "1 32" "0 16"; do
  set -- $cfg
  timeout -k 10 300 python bench/gemm_tn_bench.py --phased $1 --mf $2 --fused > gpurun_out/gemm2/bench_$1_$2.log 2>&1 || { tail -3 gpurun_out/gemm2/bench_$1_$2.log; exit 1; }
  grep '^{' gpurun_out/gemm2/bench_$1_$2.log | python -c 'import sys,json; [print(d["phased"], d["mf"], d["N"], d["K"], "ours", d["ours_tflops"], "blas", d["blas_tflops"], "fgelu", d.get("fused_gelu_us"), d.get("blas_plus_gelu_us"), "fdgelu", d.get("fused_dgelu_us"), d.get("blas_plus_dgelu_us")) for d in map(json.loads, sys.stdin)]'
done

#!/bin/bash
# ping-pong GEMM v2 (balanced reads, per-K-tile descriptors): tests, A/B bench, stamps
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4pp7_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|error|Error" gpurun_out/r4pp7_tests.log | tail -15; [ $rc -ne 0 ] && exit $rc
for shape in "65536 3072 768" "65536 768 3072" "32768 2048 2048"; do
  set -- $shape
  for round in 1 2; do
    for v in ""; do
      so=""; [ -n "$v" ] && so="$R/pretraining_llm_amd/_C_ppexp$v.so"
      PLLM_SO=$so timeout -k 10 120 python bench/gemm_one.py --M $1 --N $2 --K $3 --phased 4 --no-blas --time 2>&1 | grep median || exit 1
    done
  done
done
timeout -k 10 400 python -u bench/gemm_pp_bench.py --fused > gpurun_out/r4pp7_bench.jsonl 2>&1
rc=$?; cat gpurun_out/r4pp7_bench.jsonl | cut -c1-400; exit $rc

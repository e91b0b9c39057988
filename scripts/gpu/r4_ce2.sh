#!/bin/bash
# CE block size / non-temporal store variants (bench/ce_bench.py), 3 interleaved rounds
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "cross_entropy" > gpurun_out/r4_ce2_tests.log 2>&1 || { tail -20 gpurun_out/r4_ce2_tests.log; exit 1; }
tail -1 gpurun_out/r4_ce2_tests.log
for r in 1 2 3; do
  for v in "512 0" "256 0" "1024 0" "512 1" "256 1"; do
    set -- $v
    PLLM_CE_THREADS=$1 PLLM_CE_NT=$2 timeout -k 10 120 python -u bench/ce_bench.py 2>&1 | grep median | sed "s/^/threads=$1 nt=$2 /" || exit 1
  done
done

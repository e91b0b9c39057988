#!/bin/bash
# round 2: chunked LM-head + CE -- GPU tests, then the headline bench at several chunk sizes
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2ce_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r2ce_tests.log; [ $rc -ne 0 ] && exit $rc
for c in 2048 4096 8192 16384 65536; do
  PLLM_CE_CHUNK_ROWS=$c timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2ce_bench_$c.log 2>&1
  rc=$?; echo "chunk $c"; tail -1 gpurun_out/r2ce_bench_$c.log | cut -c1-420; [ $rc -ne 0 ] && exit $rc
done
exit 0

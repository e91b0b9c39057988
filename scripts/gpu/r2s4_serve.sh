#!/bin/bash
# batched generation service: GPU test + serving throughput (batched vs one request at a time)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_server_gpu.py tests/test_server.py tests/test_kernels_gpu.py -k "server or decode or gemv or generate or continuous" -q -x --timeout 120 --timeout-method thread > gpurun_out/serve_tests.log 2>&1
rc=$?; tail -2 gpurun_out/serve_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench/serve_bench.py > gpurun_out/serve_bench.jsonl 2> gpurun_out/serve_bench.err || { tail -5 gpurun_out/serve_bench.err; exit 1; }
cat gpurun_out/serve_bench.jsonl

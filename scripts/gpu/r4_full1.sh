#!/bin/bash
# full GPU suite + smoke + headline bench (current build)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4f1_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|error" gpurun_out/r4f1_tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f1_smoke.log 2>&1 || { tail -5 gpurun_out/r4f1_smoke.log; exit 1; }
tail -1 gpurun_out/r4f1_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r4f1_bench.log 2>&1 || { tail -5 gpurun_out/r4f1_bench.log; exit 1; }
tail -1 gpurun_out/r4f1_bench.log | cut -c1-400

#!/bin/bash
# round 2: full GPU suite + smoke after the attention rewrite and full-grid streaming kernels
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r2c11_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|error" gpurun_out/r2c11_tests.log | tail -15; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2c11_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/r2c11_smoke.log; exit $rc

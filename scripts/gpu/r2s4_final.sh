#!/bin/bash
# session close-out: full GPU suite + smoke, headline bench, step profile
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/s4f_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|error" gpurun_out/s4f_tests.log | tail -15; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s4f_smoke.log 2>&1 || { tail -5 gpurun_out/s4f_smoke.log; exit 1; }
tail -1 gpurun_out/s4f_smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/s4f_gpt2.log 2>&1 || { tail -5 gpurun_out/s4f_gpt2.log; exit 1; }
tail -1 gpurun_out/s4f_gpt2.log | cut -c1-250

#!/bin/bash
# round 3: full GPU suite + smoke + headline bench (tag = $1)
R="${GRAFT_REPO_ROOT:-/root/repo}"
T="${1:-r3}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|error" gpurun_out/${T}_tests.log | tail -15; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -5 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${T}_gpt2.log 2>&1 || { tail -5 gpurun_out/${T}_gpt2.log; exit 1; }
tail -1 gpurun_out/${T}_gpt2.log | cut -c1-250

#!/bin/bash
# Re-validation after container restore: GPU kernel tests + 1-GPU headline bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t11.log 2>&1
rc=$?; tail -3 gpurun_out/t11.log
if [ $rc -gt 1 ]; then exit $rc; fi
if [ $rc -eq 1 ]; then grep -E "^E |FAILED" gpurun_out/t11.log | head -20; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s11.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/s11.log; exit 5; }
tail -1 gpurun_out/s11.log
timeout -k 10 400 python bench.py > gpurun_out/b11.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/b11.log; exit 4; }
tail -1 gpurun_out/b11.log | cut -c1-400

#!/bin/bash
# full GPU suite, smoke, headline bench after the decode skinny-GEMM change
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t23.log 2>&1
rc=$?; tail -2 gpurun_out/t23.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/t23.log | head -30; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s23.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/s23.log; exit 5; }
tail -1 gpurun_out/s23.log
timeout -k 10 400 python bench.py > gpurun_out/b23.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/b23.log; exit 4; }
tail -1 gpurun_out/b23.log

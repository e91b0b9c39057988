#!/bin/bash
# full GPU suite + headline bench + llama bench after the wgrad split-plan change
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t19.log 2>&1
rc=$?; tail -3 gpurun_out/t19.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/t19.log | head -30; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/b19.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/b19.log; exit 4; }
tail -1 gpurun_out/b19.log | cut -c1-250
timeout -k 10 400 python bench.py --model llama-1.3b --batch 8 --steps 10 --warmup 3 > gpurun_out/b19_llama.log 2>&1 || { echo "llama bench failed"; tail -20 gpurun_out/b19_llama.log; exit 4; }
tail -1 gpurun_out/b19_llama.log | cut -c1-220

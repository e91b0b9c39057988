#!/bin/bash
# side-stream weight gradients ON by default: full GPU suite, smoke, headline / llama / medium / ZeRO benches
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t21.log 2>&1
rc=$?; tail -2 gpurun_out/t21.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/t21.log | head -30; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s21.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/s21.log; exit 5; }
for args in "" "--zero 1" "--model llama-1.3b --batch 8 --steps 10 --warmup 3" "--model gpt2-medium --batch 8 --steps 10 --warmup 3"; do
  timeout -k 10 400 python bench.py $args > gpurun_out/b21x.log 2>&1 || { echo "bench failed: $args"; tail -20 gpurun_out/b21x.log; exit 4; }
  echo "[$args] $(tail -1 gpurun_out/b21x.log | cut -c1-40) $(tail -1 gpurun_out/b21x.log | grep -o '"value": [0-9.]*') $(tail -1 gpurun_out/b21x.log | grep -o '"final_loss": [0-9.]*')"
done

#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -q -x -p no:cacheprovider > gpurun_out/t4.log 2>&1
rc=$?
tail -3 gpurun_out/t4.log
if [ $rc -gt 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
if [ $rc -eq 1 ]; then grep -E "^E |FAILED" gpurun_out/t4.log | head -20; fi
# tune B=64 shapes (tables for B=32 already shipped), keep the result
PLLM_TUNE_OUT=$PWD/gpurun_out timeout -k 10 900 python - <<'PY' > gpurun_out/tune64.log 2>&1 || { echo tune failed; tail -20 gpurun_out/tune64.log; exit 5; }
import os, sys, torch
sys.argv = ["bench.py", "--steps", "1", "--warmup", "2", "--batch", "64", "--tune-missing"]
import bench
bench.main()
from pretraining_llm_amd.utils.gemm_tuning import save_tuned
save_tuned("gpt2small_b64_gfx950.csv")
import shutil; shutil.copy("pretraining_llm_amd/tuning/gpt2small_b64_gfx950.csv", "gpurun_out/gpt2small_b64_gfx950.csv")
PY
tail -2 gpurun_out/tune64.log | cut -c1-300
for b in 32 64; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --batch $b > gpurun_out/b4_$b.log 2>&1 || { echo "bench $b failed"; tail -20 gpurun_out/b4_$b.log; exit 4; }
  tail -1 gpurun_out/b4_$b.log | cut -c1-420
done
bash scripts/gpu/prof.sh prof4 --steps 4 --warmup 2 --batch 64

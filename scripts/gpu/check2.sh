#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -q -x -p no:cacheprovider > gpurun_out/t2.log 2>&1
rc=$?
tail -3 gpurun_out/t2.log
if [ $rc -gt 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
for b in 8 32; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --batch $b > gpurun_out/b_auto_$b.log 2>&1 || { echo "bench $b failed"; tail -20 gpurun_out/b_auto_$b.log; exit 4; }
  tail -1 gpurun_out/b_auto_$b.log
done
bash scripts/gpu/prof.sh prof1 --steps 5 --warmup 2 --batch 16

#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -q -x -p no:cacheprovider > gpurun_out/t3.log 2>&1
rc=$?
tail -3 gpurun_out/t3.log
if [ $rc -gt 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
for b in 16 32 64; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --batch $b > gpurun_out/b3_$b.log 2>&1 || { echo "bench $b failed"; tail -20 gpurun_out/b3_$b.log; exit 4; }
  tail -1 gpurun_out/b3_$b.log | cut -c1-200
done
# TunableOp: tune the GEMM shapes of the B=32 step, then re-bench with the tuned table
export PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tunableop_b32.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 timeout -k 10 900 python bench.py --steps 2 --warmup 2 --batch 32 > gpurun_out/b3_tune.log 2>&1 || { echo "tune failed"; tail -20 gpurun_out/b3_tune.log; exit 5; }
ls -la gpurun_out/tunableop_b32*
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 timeout -k 10 400 python bench.py --steps 10 --warmup 3 --batch 32 > gpurun_out/b3_tuned.log 2>&1 || { echo "tuned bench failed"; tail -20 gpurun_out/b3_tuned.log; exit 6; }
tail -1 gpurun_out/b3_tuned.log | cut -c1-200
unset PYTORCH_TUNABLEOP_FILENAME
bash scripts/gpu/prof.sh prof3 --steps 5 --warmup 2 --batch 32

#!/bin/bash
# runtime knob A/B on the headline bench: HIP_FORCE_DEV_KERNARG=1 (kernel arguments in device memory)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in 0 1 0 1 0 1; do
  if [ $v = 1 ]; then export HIP_FORCE_DEV_KERNARG=1; else unset HIP_FORCE_DEV_KERNARG; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/env_$v.log 2>&1 || { tail -5 gpurun_out/env_$v.log; exit 1; }
  echo "devkernarg=$v $(tail -1 gpurun_out/env_$v.log | cut -c80-140)"
done

#!/bin/bash
# wgrad A/B: in-tree build vs xso/_C_wglob.so (global_load_lds DMA), + stamps + wgrad tests
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/wg
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "wgrad" --timeout 120 --timeout-method thread > gpurun_out/wg/tests.log 2>&1
rc=$?; tail -1 gpurun_out/wg/tests.log; [ $rc -ne 0 ] && exit $rc

for so in glob new glob new; do
  if [ $so = glob ]; then export PLLM_SO=$R/xso/_C_wglob.so; else unset PLLM_SO; fi
  timeout -k 10 300 python bench/wgrad_time.py > gpurun_out/wg/$so.log 2>&1 || { tail -3 gpurun_out/wg/$so.log; exit 1; }
  echo "$so: $(python -c 'import sys,json; [print(d["P"], d["Q"], d["tflops"], end=" | ") for d in map(json.loads, [l for l in open(sys.argv[1]) if l.startswith("{")])]' gpurun_out/wg/$so.log)"
done

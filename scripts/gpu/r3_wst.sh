#!/bin/bash
# wgrad A/B: stagger of the SIMD partners' DMA bursts (xso/_C_wst{1,2,3}.so) and the 16x16x32 MFMA shape, vs in-tree
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/wst
export HSA_ENABLE_IPC_MODE_LEGACY=0
for so in base wst2 base16 wst2_16 wst1 wst3 base wst2 base16 wst2_16; do
  unset PLLM_SO PLLM_WGRAD_VARIANT
  case $so in
    base) ;;
    base16) export PLLM_WGRAD_VARIANT=16 ;;
    wst2_16) export PLLM_SO=$R/xso/_C_wst2.so PLLM_WGRAD_VARIANT=16 ;;
    *) export PLLM_SO=$R/xso/_C_$so.so ;;
  esac
  timeout -k 10 300 python bench/wgrad_time.py > gpurun_out/wst/$so.log 2>&1 || { tail -3 gpurun_out/wst/$so.log; exit 1; }
  echo "$so: $(python -c 'import sys,json; [print(d["P"], d["Q"], d["tflops"], end=" | ") for d in map(json.loads, [l for l in open(sys.argv[1]) if l.startswith("{")])]' gpurun_out/wst/$so.log)"
done

#!/bin/bash
# attention diagnostics: kernel times of the in-tree build vs variant builds in xso/
R="${GRAFT_REPO_ROOT:-/root/repo}"
CF="${1:-64x12x1024x64,8x16x4096x64,16x16x2048x128}"
cd "$R"; mkdir -p gpurun_out/abl
export HSA_ENABLE_IPC_MODE_LEGACY=0
for round in 1 2; do
for so in main $(ls xso | sed 's/.so$//'); do
  if [ $so = main ]; then unset PLLM_SO; else export PLLM_SO=$R/xso/$so.so; fi
  timeout -k 10 200 python bench/attn_bench.py --ours --configs $CF --rounds 3 > gpurun_out/abl/$so.log 2>&1 || { tail -3 gpurun_out/abl/$so.log; exit 1; }
  echo "$so: $(grep -h '^{' gpurun_out/abl/$so.log | python -c 'import sys,json; [print(json.loads(l)["cfg"], "fwd", round(min(json.loads(l)["fwd_us"]),1), "bwd", round(min(json.loads(l)["bwd_us"]),1), end=" | ") for l in sys.stdin]')"
done
done

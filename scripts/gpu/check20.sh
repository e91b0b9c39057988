#!/bin/bash
# wgrad staging-ring A/B (gpt2 + llama shapes), with per-variant numerics
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for sh in gpt2 llama; do
  M=65536; [ $sh = llama ] && M=16384
  timeout -k 10 300 python bench/gemm_bench.py --rounds 3 --shapes $sh --M $M > gpurun_out/gemm20_$sh.log 2>&1 || { echo "gemm bench failed"; tail -20 gpurun_out/gemm20_$sh.log; exit 3; }
  grep -v amdgpu.ids gpurun_out/gemm20_$sh.log | python -c "import sys,json; [print({k: (round(v,4) if isinstance(v,float) else v) for k, v in json.loads(l).items() if 'tflops' in k or 'rel' in k or k in 'PQ'}) for l in sys.stdin if l.startswith('{')]"
done

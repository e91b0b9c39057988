#!/bin/bash
# wgrad split-plan A/B (gpt2 + llama shapes), D=128 attention-bwd 8-wave variant A/B, attention tests
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench/attn_bench.py --ours --configs 8x16x2048x128,64x12x1024x64 --rounds 3 > gpurun_out/attn18.log 2>&1 || { echo "attn bench failed"; tail -20 gpurun_out/attn18.log; exit 3; }
grep -v amdgpu.ids gpurun_out/attn18.log | cut -c1-500
for sh in gpt2 llama; do
  M=65536; [ $sh = llama ] && M=16384
  timeout -k 10 300 python bench/gemm_bench.py --rounds 3 --shapes $sh --M $M > gpurun_out/gemm18_$sh.log 2>&1 || { echo "gemm bench failed"; tail -20 gpurun_out/gemm18_$sh.log; exit 3; }
  grep -v amdgpu.ids gpurun_out/gemm18_$sh.log | python -c "import sys,json; [print({k: (round(v,1) if isinstance(v,float) else v) for k, v in json.loads(l).items() if 'tflops' in k or k in 'PQ'}) for l in sys.stdin if l.startswith('{')]"
done

#!/bin/bash
# wgrad priority A/B, then the other BASELINE configs and the stock-torch baseline, current code
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench/gemm_bench.py --rounds 3 > gpurun_out/gemm17.log 2>&1 || { echo "gemm bench failed"; tail -20 gpurun_out/gemm17.log; exit 3; }
grep -v amdgpu.ids gpurun_out/gemm17.log | python -c "import sys,json; [print({k: v for k, v in json.loads(l).items() if 'tflops' in k or k in 'PQ'}) for l in sys.stdin if l.startswith('{')]"
timeout -k 10 400 python bench.py --model llama-1.3b --batch 8 --steps 10 --warmup 3 > gpurun_out/b17_llama.log 2>&1 || { echo "llama bench failed"; tail -20 gpurun_out/b17_llama.log; exit 4; }
tail -1 gpurun_out/b17_llama.log | cut -c1-220
timeout -k 10 400 python bench.py --model gpt2-medium --batch 8 --steps 10 --warmup 3 > gpurun_out/b17_medium.log 2>&1 || { echo "medium bench failed"; tail -20 gpurun_out/b17_medium.log; exit 4; }
tail -1 gpurun_out/b17_medium.log | cut -c1-220
timeout -k 10 400 python bench.py --backend torch --steps 10 --warmup 3 > gpurun_out/b17_torch.log 2>&1 || { echo "torch bench failed"; tail -20 gpurun_out/b17_torch.log; exit 4; }
tail -1 gpurun_out/b17_torch.log | cut -c1-220

#!/bin/bash
# SwiGLU-backward epilogue: GEMM GPU tests, kernel-pair timing, llama bench A/B (PLLM_FUSED_MLP=0 vs default)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/swiglu
O="$R/gpurun_out/swiglu"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^E |Error" $O/tests.log | head -20; exit $rc; }
timeout -k 10 200 python bench/gemm_tn_bench.py --swiglu > $O/kern.jsonl 2>&1 || { tail -5 $O/kern.jsonl; exit 1; }
grep '^{' $O/kern.jsonl
for f in 0 bwd 0 bwd; do
  timeout -k 10 300 env PLLM_FUSED_MLP=$f python bench.py --model llama-1.3b --batch 16 --steps 6 --warmup 3 > $O/llama_$f.log 2>&1 || { tail -5 $O/llama_$f.log; exit 1; }
  echo "fused=$f: $(tail -1 $O/llama_$f.log | cut -c80-140)"
done

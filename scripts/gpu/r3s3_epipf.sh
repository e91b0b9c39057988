#!/bin/bash
# TN-GEMM epilogue aux prefetch: GEMM GPU tests, fused-epilogue kernel times base/new, headline A/B
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/epipf
O="$R/gpurun_out/epipf"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for so in base new; do
  if [ $so = base ]; then export PLLM_SO=$R/pretraining_llm_amd/_C_base.so; else unset PLLM_SO; fi
  timeout -k 10 200 python bench/gemm_tn_bench.py --fused > $O/kern_$so.jsonl 2>&1 || { tail -5 $O/kern_$so.jsonl; exit 1; }
  timeout -k 10 200 python bench/gemm_tn_bench.py --swiglu > $O/sw_$so.jsonl 2>&1 || { tail -5 $O/sw_$so.jsonl; exit 1; }
  echo "$so: $(grep -h '^{' $O/kern_$so.jsonl | python -c 'import sys,json; [print((d:=json.loads(l))["N"], d["K"], d.get("fused_dgelu_us"), end=" | ") for l in sys.stdin]') swiglu: $(grep -h '^{' $O/sw_$so.jsonl | python -c 'import sys,json; [print(json.loads(l)["fused_swiglu_bwd_us"], end=" ") for l in sys.stdin]')"
done
unset PLLM_SO
bash scripts/gpu/r3s3_ab.sh epipf "" tests/test_gemm_gpu.py

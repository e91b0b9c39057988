#!/bin/bash
# attention forward: half-wave row-statistic exchange by v_permlane32_swap (default) vs ds_bpermute (_C_bperm.so)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "attn or attention or flash or rope" --timeout 120 --timeout-method thread > gpurun_out/perm_tests.log 2>&1
rc=$?; tail -1 gpurun_out/perm_tests.log; [ $rc -ne 0 ] && exit $rc
for so in base bperm base bperm; do
  if [ $so = bperm ]; then export PLLM_SO=$R/pretraining_llm_amd/_C_bperm.so; else unset PLLM_SO; fi
  timeout -k 10 300 python bench/attn_bench.py --ours --configs 64x12x1024x64,16x16x2048x128 --rounds 3 > gpurun_out/perm_attn_$so.log 2>&1 || { tail -5 gpurun_out/perm_attn_$so.log; exit 1; }
  echo "$so: $(grep -h '^{' gpurun_out/perm_attn_$so.log | python -c 'import sys,json; [print(json.loads(l)["cfg"], "fwd", round(min(json.loads(l)["fwd_us"]),1), "bwd", round(min(json.loads(l)["bwd_us"])), end=" | ") for l in sys.stdin]')"
done
for so in base bperm base bperm; do
  if [ $so = bperm ]; then export PLLM_SO=$R/pretraining_llm_amd/_C_bperm.so; else unset PLLM_SO; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/perm_bench_$so.log 2>&1 || { tail -5 gpurun_out/perm_bench_$so.log; exit 1; }
  echo "$so bench: $(tail -1 gpurun_out/perm_bench_$so.log | cut -c80-135)"
done

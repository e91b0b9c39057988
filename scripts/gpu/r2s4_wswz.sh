#!/bin/bash
# attention D=64: ds_write_b128 staging order (Img<64>::st_pair, odd rows upper half first) vs
# the previous order (_C_base.so): tests, LDS-conflict PMC pass, kernel A/B, headline A/B
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/wswz
O="$R/gpurun_out/wswz"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "attn or attention or flash or rope" --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_WAVES"
for so in new base; do
  if [ $so = base ]; then export PLLM_SO=$R/pretraining_llm_amd/_C_base.so; else unset PLLM_SO; fi
  for only in fwd bwd; do
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C2 -d "$O/${so}_$only" -o run --output-format csv -- \
      python3 "$R/bench/attn_bench.py" --configs 64x12x1024x64 --only $only --rounds 1 > "$O/${so}_$only.log" 2>&1) || { echo "pmc $so $only failed"; tail -5 "$O/${so}_$only.log"; exit 1; }
    python3 "$R/scripts/pmc_kernels.py" "attention $only $so" "$O/${so}_$only" > "$O/${so}_$only.md" 2>&1 || true
  done
done
unset PLLM_SO
for so in base new base new; do
  if [ $so = base ]; then export PLLM_SO=$R/pretraining_llm_amd/_C_base.so; else unset PLLM_SO; fi
  timeout -k 10 300 python bench/attn_bench.py --ours --configs 64x12x1024x64,16x16x2048x128 --rounds 3 > $O/attn_$so.log 2>&1 || { tail -5 $O/attn_$so.log; exit 1; }
  echo "$so: $(grep -h '^{' $O/attn_$so.log | python -c 'import sys,json; [print(json.loads(l)["cfg"], "fwd", round(min(json.loads(l)["fwd_us"]),1), "bwd", round(min(json.loads(l)["bwd_us"])), end=" | ") for l in sys.stdin]')"
done
for so in base new base new; do
  if [ $so = base ]; then export PLLM_SO=$R/pretraining_llm_amd/_C_base.so; else unset PLLM_SO; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_$so.log 2>&1 || { tail -5 $O/bench_$so.log; exit 1; }
  echo "$so bench: $(tail -1 $O/bench_$so.log | cut -c80-135)"
done

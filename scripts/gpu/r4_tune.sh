#!/bin/bash
# fresh TunableOp table for the GPT-2 headline step (longer per-candidate timing), then a same-box A/B
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out/tune_alt
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python scripts/tune_gemms.py --model gpt2-small --batch 64 --fresh --tune-ms 60 --out gpurun_out/tune_alt/gpt2small_b64_gfx950.csv > gpurun_out/r4tune.log 2>&1 || { tail -5 gpurun_out/r4tune.log; exit 1; }
tail -2 gpurun_out/r4tune.log
wc -l gpurun_out/tune_alt/gpt2small_b64_gfx950.csv pretraining_llm_amd/tuning/gpt2small_b64_gfx950.csv
for round in 1 2; do
  for t in shipped fresh; do
    if [ $t = fresh ]; then export PLLM_TUNING_DIR=$R/gpurun_out/tune_alt; else unset PLLM_TUNING_DIR; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r4tune_${t}_$round.log 2>&1 || { tail -3 gpurun_out/r4tune_${t}_$round.log; exit 1; }
    echo "tuning=$t $(tail -1 gpurun_out/r4tune_${t}_$round.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["config"]["tuned_gemms"])')"
  done
done

#!/bin/bash
# GPT-2 step: graph vs eager (the world > 1 step mode), fused GELU forward epilogue A/B
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 $BARGS > gpurun_out/r4ab3_$tag.log 2>&1 || { tail -3 gpurun_out/r4ab3_$tag.log; return 1; }
  echo "$tag $(tail -1 gpurun_out/r4ab3_$tag.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["config"].get("step_mode"))')"
}
for round in 1 2; do
  BARGS="" run graph_$round PLLM_FUSED_MLP=bwd || exit 1
  BARGS="--cuda-graph 0" run eager_$round PLLM_FUSED_MLP=bwd || exit 1
  BARGS="" run gelufwd_$round PLLM_FUSED_MLP=all || exit 1
done

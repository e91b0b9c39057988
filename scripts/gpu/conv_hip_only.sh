#!/bin/bash
# HIP-path-only plateau re-run of scripts/convergence.py for a list of seeds (the stock-ops baseline of the same seeds
# does not depend on the HIP kernels, so it is reused from the earlier pair runs).
# usage: bash scripts/gpu/conv_hip_only.sh <tag> <model> <steps> <batch> <seq> <lr> <seed> [<seed> ...]
set -o pipefail
TAG=$1 MODEL=$2 STEPS=$3 BATCH=$4 SEQ=$5 LR=$6; shift 6
O=gpurun_out/$TAG; mkdir -p $O
for seed in "$@"; do
  timeout -k 10 500 python -u scripts/convergence.py --model $MODEL --steps $STEPS --batch $BATCH --seq $SEQ --lr $LR \
    --seed $seed --backends auto --out $O/${MODEL}_${STEPS}_s$seed.jsonl > $O/${MODEL}_s$seed.log 2>&1 \
    || { tail -5 $O/${MODEL}_s$seed.log; exit 1; }
  python - "$O/${MODEL}_${STEPS}_s$seed.jsonl" "$seed" "$STEPS" <<'PY'
import json, sys
recs = [json.loads(l) for l in open(sys.argv[1]) if '"step"' in l]
steps = int(sys.argv[3])
tail = [r["train_loss"] for r in recs if r["step"] > steps - 100]
print(json.dumps({"seed": int(sys.argv[2]), "tail_mean": round(sum(tail) / len(tail), 5), "final": recs[-1]["train_loss"]}))
PY
done

#!/bin/bash
# Numerics bisection over op families: the HIP path with one family at a time on stock PyTorch ops
# (PLLM_TORCH_OPS, ops/__init__.py), same seed / data as scripts/convergence.py's reference pair.
# usage: bash scripts/gpu/bisect_numerics.sh <tag> <model> <steps> <batch> <seq> <lr> <seed> <family> [<family> ...]
set -o pipefail
TAG=$1 MODEL=$2 STEPS=$3 BATCH=$4 SEQ=$5 LR=$6 SEED=$7; shift 7
O=gpurun_out/$TAG; mkdir -p $O
for fam in "$@"; do
  PLLM_TORCH_OPS=$fam timeout -k 10 500 python -u scripts/convergence.py --model $MODEL --steps $STEPS --batch $BATCH \
    --seq $SEQ --lr $LR --seed $SEED --backends auto --out $O/bisect_$fam.jsonl > $O/bisect_$fam.log 2>&1 \
    || { tail -5 $O/bisect_$fam.log; exit 1; }
  python - "$O/bisect_$fam.jsonl" "$fam" "$STEPS" <<'PY'
import json, sys
recs = [json.loads(l) for l in open(sys.argv[1]) if '"step"' in l]
steps = int(sys.argv[3])
tail = [r["train_loss"] for r in recs if r["step"] > steps - 100]
print(json.dumps({"torch_ops": sys.argv[2], "tail_mean": round(sum(tail) / len(tail), 5), "final": recs[-1]["train_loss"]}))
PY
done

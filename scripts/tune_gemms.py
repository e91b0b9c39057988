"""Tune the library (hipBLASLt / rocBLAS) GEMM selections of one training configuration with
PyTorch TunableOp on the MI355X and write the merged table.

Runs a few full training steps of the bench model with TunableOp tuning enabled, so every
GEMM shape the step issues (forward, data-gradient through the W^T shadows, LM head) gets
its fastest candidate measured, then writes the shipped tables plus the new results as one
CSV (copy it into ``pretraining_llm_amd/tuning/``).

  python scripts/tune_gemms.py --model gpt2-small --batch 64 --out gpurun_out/gpt2small_b64_gfx950.csv
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--out", required=True)
    ap.add_argument("--tune-ms", default="30")
    ap.add_argument("--fresh", action="store_true", help="ignore the shipped tables (re-tune every shape)")
    args = ap.parse_args()
    from pretraining_llm_amd.ab import ab, ab_set
    ab_set("tune_ms", args.tune_ms)
    ab_set("tune_iters", ab("tune_iters", 20))
    import torch
    import torch.cuda.tunable as tunable
    from pretraining_llm_amd import ops
    from pretraining_llm_amd.models import GPT, get_preset
    from pretraining_llm_amd.train.optim import FlatAdamW, no_decay_1d
    from pretraining_llm_amd.utils.gemm_tuning import enable_tuned_gemms
    ops._lib.require()
    enable_tuned_gemms(0, tune_missing=True, load_tables=not args.fresh)
    dev = torch.device("cuda", 0)
    cfg = get_preset(args.model)
    model = GPT(cfg).to(dev, torch.bfloat16)
    opt = FlatAdamW(model, lr=1e-4, betas=(0.9, 0.95), weight_decay=0.1, decay_filter=no_decay_1d, max_grad_norm=1.0)
    T = cfg.context_length
    for step in range(args.steps):
        x = torch.randint(0, cfg.vocab_size, (args.batch, T), device=dev)
        _, loss = model(x, x, return_logits=False)
        loss.backward()
        opt.step()
        opt.zero_grad()
        torch.cuda.synchronize()
        print(f"step {step} loss {float(loss):.3f}", flush=True)
    lines = [f"Validator,{k},{v}" for k, v in tunable.get_validators()]
    for res in tunable.get_results():
        lines.append(",".join(str(x) for x in res))
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print(f"wrote {len(lines)} lines to {args.out}", flush=True)


if __name__ == "__main__":
    main()

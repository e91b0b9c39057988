#!/usr/bin/env python
"""Numerics at scale: train the same model on the same synthetic Markov token stream with the
hand-written gfx950 kernels (``--backend auto``) and with stock PyTorch ops (``--backend torch``:
SDPA, F.layer_norm, fp32 F.cross_entropy, torch-op AdamW), same seed, same batches, and write
both loss curves.  A HIP path that drifts from the stock-op path over hundreds of steps shows
up here even when every kernel passes its single-call oracle test.

usage: python scripts/convergence.py --steps 400 --batch 16 [--model gpt2-small] --out profiles/X.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def train_curve(backend: str, model: str, steps: int, batch: int, seq: int, lr: float, log_every: int = 10,
                tokens: int = 4_000_000, data_dir: str = None, overrides: dict = None, device: str = "auto",
                seed: int = 1234):
    """Run ``steps`` optimizer steps; returns [(step, train_loss, val_loss)] every ``log_every``."""
    import torch
    from pretraining_llm_amd import ops
    from pretraining_llm_amd.train.trainer import Trainer
    from config.config import default_config
    ops.set_backend(backend)
    data_dir = data_dir or os.path.join(tempfile.gettempdir(), "pllm_convergence")
    cfg = dict(default_config)
    cfg.update(model_preset=model, t_batch_size=batch, seq_len=seq, t_train_steps=steps, t_lr=lr, t_lr_decayed=lr / 10,
               warmup_steps=max(1, steps // 10), lr_schedule="cosine", weight_decay=0.1, weight_decay_all=False,
               betas=(0.9, 0.95), max_grad_norm=1.0, log_interval=log_every, t_eval_steps=max(log_every, steps // 4),
               t_eval_iters=4, eval_at_start=False, synthetic_data=True, synthetic_tokens=tokens,
               synthetic_kind="markov", synthetic_dir=data_dir, seed=seed, t_out_path=None, device=device,
               ddp_backend="auto")
    cfg.update(overrides or {})
    recs = []
    tr = Trainer(cfg, log=lambda *_: None)
    def keep(rec):  # keep the records in memory; one progress line per record (long runs stay visibly alive)
        recs.append(rec)
        print(f"[convergence] {backend} step {rec['step']} loss {rec['train_loss']:.4f}", file=sys.stderr, flush=True)
    tr.metrics.log = keep
    t0 = time.perf_counter()
    try:
        tr.train()
    finally:
        tr.train_loader.close()
        if tr.val_loader is not None:
            tr.val_loader.close()
        ops.set_backend("auto")
    wall = time.perf_counter() - t0
    return [(r["step"], r["train_loss"], r["val_loss"]) for r in recs], wall


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--lr", type=float, default=6e-4)
    ap.add_argument("--backends", default="auto,torch", help="comma list of backend[:dtype] (auto = HIP kernels)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--tail", type=int, default=100, help="steps averaged for the plateau summary (tail_mean)")
    ap.add_argument("--seed", type=int, default=1234, help="init / data-order seed (the synthetic shard stays the same)")
    args = ap.parse_args(argv)
    out = open(args.out, "w") if args.out else sys.stdout
    finals, tails = {}, {}
    for be in args.backends.split(","):
        # "backend[:dtype]", e.g. torch:float32 = stock ops in fp32 (the numerics ground truth)
        name, _, dt = be.partition(":")
        curve, wall = train_curve(name, args.model, args.steps, args.batch, args.seq, args.lr,
                                  overrides={"dtype": dt} if dt else None, seed=args.seed)
        for step, tl, vl in curve:
            out.write(json.dumps({"backend": be, "model": args.model, "step": step, "train_loss": round(tl, 5),
                                  "val_loss": None if vl != vl else round(vl, 5)}) + "\n")
        finals[be] = curve[-1][1]
        tail = [tl for step, tl, _ in curve if step > args.steps - args.tail]  # the last `tail` steps' logged losses
        tails[be] = sum(tail) / max(1, len(tail))
        print(f"[convergence] backend={be} final train loss {curve[-1][1]:.4f} ({wall:.1f} s)", file=sys.stderr)
    if len(finals) >= 2:
        a, b = list(finals.values())[:2]
        gap = (a - b) / b  # signed: > 0 when the first backend ends higher
        ta, tb = list(tails.values())[:2]
        out.write(json.dumps({"summary": True, "final_loss": finals, "rel_gap": round(gap, 5),
                              "tail_mean": {k: round(v, 5) for k, v in tails.items()}, "tail_steps": args.tail,
                              "tail_rel_gap": round((ta - tb) / tb, 5), "seed": args.seed,
                              "steps": args.steps, "batch": args.batch, "seq": args.seq}) + "\n")
        print(f"[convergence] final-loss relative gap (first - second) / second {100 * gap:+.2f} %", file=sys.stderr)
    if out is not sys.stdout:
        out.close()


if __name__ == "__main__":
    main()

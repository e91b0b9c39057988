"""KV-cache generation throughput on one MI355X (serving path).

GPT-2 small (random init, bf16): prefill a ``--prompt``-token prompt for ``B`` sequences, then
decode ``--new`` tokens greedily, eager (one launch per kernel) vs one hipGraph replay per
token (``DecodeGraph``).  Also times the decode-attention kernel alone against the flash
forward kernel run with a single query row (what decode used before the split-KV kernel).
Prints one JSON line per configuration.

usage: python bench/decode_bench.py [--batches 1,16,64] [--prompt 128] [--new 256]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, iters=50, warmup=5):
    import torch
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--batches", default="1,16,64")
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--new", type=int, default=256)
    args = ap.parse_args()
    import torch
    from pretraining_llm_amd import ops
    from pretraining_llm_amd.models import GPT, get_preset
    ops._lib.require()
    dev = torch.device("cuda:0")

    # kernel-level: split-KV decode vs flash forward with one query row
    for B, S in ((1, 1024), (16, 1024), (64, 1024), (8, 4096)):
        H, D = 12, 64
        q = torch.randn(B, 1, H, D, device=dev, dtype=torch.bfloat16)
        k = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16)
        v = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16)
        sc = 1.0 / math.sqrt(D)
        t_dec = timeit(lambda: torch.ops.pllm.attn_decode(q, k, v, sc, None), iters=200)
        t_fa = timeit(lambda: torch.ops.pllm.attn_fwd(q, k, v, True, sc), iters=200)
        kv_bytes = 2 * B * S * H * D * 2
        print(json.dumps({"kernel": "attn_decode", "B": B, "S": S, "H": H, "D": D, "decode_us": round(t_dec * 1e6, 2),
                          "flash_fwd_1row_us": round(t_fa * 1e6, 2),
                          "decode_kv_GBps": round(kv_bytes / t_dec / 1e9, 1)}), flush=True)

    torch.manual_seed(0)
    cfg = get_preset(args.model)
    model = GPT(cfg).to(dev, torch.bfloat16).eval()
    for B in (int(b) for b in args.batches.split(",")):
        idx = torch.randint(0, cfg.vocab_size, (B, args.prompt), device=dev)
        res = {"model": args.model, "batch": B, "prompt": args.prompt, "new_tokens": args.new}
        for mode in ("eager", "graph"):
            g = mode == "graph"
            model.generate(idx, 4, temperature=0.0, cuda_graph=g)  # warm-up (library init, graph pools)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = model.generate(idx, args.new, temperature=0.0, cuda_graph=g)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            res[f"{mode}_s"] = round(dt, 4)
            res[f"{mode}_tok_per_s"] = round(B * args.new / dt, 1)
            res[f"{mode}_ms_per_token_step"] = round(1000 * dt / args.new, 3)
            assert out.shape == (B, args.prompt + args.new)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

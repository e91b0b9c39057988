#!/usr/bin/env python
"""Build the reference-parity fixture ``tests/fixtures/ref_tiny.safetensors``.

Runs the REFERENCE's own model code (Flink-ddd/pretraining-llm ``src/models/transformer.py``,
read from ``--ref`` / $PLLM_REFERENCE, default /root/reference; nothing is copied) on CPU:
``Transformer(n_head=4, n_embed=64, context_length=16, vocab_size=128, N_BLOCKS=2)`` with
torch.manual_seed(0) default init, then records
* its ``state_dict`` (per-head key/query/value weights, ``tril`` and ``pos_idxs`` buffers),
* logits and loss of ``forward(idx, targets)`` on a fixed batch,
* greedy continuations (argmax of the reference forward, with its context crop) and
* multinomial ``generate`` output under a fixed seed.
tests/test_ref_parity.py loads the fixture strictly into this framework's model and checks all of it.

The reference imports ``src.models...`` from its repo root; this script runs it in a child
process whose sys.path starts at the reference root (this repo has a ``src`` package too).
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys

CHILD = r'''
import sys, torch
sys.path.insert(0, REF)
from src.models.transformer import Transformer
from safetensors.torch import save_file
torch.manual_seed(0)
m = Transformer(n_head=NH, n_embed=C, context_length=CTX, vocab_size=V, N_BLOCKS=L)
m.eval()
g = torch.Generator().manual_seed(1)
idx = torch.randint(0, V, (3, CTX), generator=g)
tgt = torch.randint(0, V, (3, CTX), generator=g)
with torch.no_grad():
    logits, loss = m(idx, tgt)
    out = {f"sd.{k}": v.contiguous() for k, v in m.state_dict().items()}
    out.update(idx=idx, tgt=tgt, logits=logits.contiguous(), loss=loss.reshape(1))
    # greedy continuation through the reference forward (context crop to the last 16 tokens)
    start = idx[:, :5]
    seq = start
    for _ in range(20):
        lg, _ = m(seq[:, -CTX:])
        seq = torch.cat([seq, lg[:, -1].argmax(-1, keepdim=True)], 1)
    out["greedy"] = seq
    torch.manual_seed(123)
    out["sampled"] = m.generate(start, 20)
save_file(out, OUT)
print("wrote", OUT, len(out), "tensors")
'''


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default=os.environ.get("PLLM_REFERENCE", "/root/reference"))
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "tests", "fixtures", "ref_tiny.safetensors"))
    # dims of the reference Transformer (defaults: the ref_tiny fixture, head dim 16).  The GPU
    # fixture ref_hd32.safetensors uses --n-head 2 --n-embed 64 --ctx 32 --vocab 256 (head dim
    # 32: the HIP flash-attention kernels' smallest head dim)
    ap.add_argument("--n-head", type=int, default=4)
    ap.add_argument("--n-embed", type=int, default=64)
    ap.add_argument("--ctx", type=int, default=16)
    ap.add_argument("--vocab", type=int, default=128)
    ap.add_argument("--n-blocks", type=int, default=2)
    args = ap.parse_args(argv)
    code = (f"REF = {args.ref!r}\nOUT = {os.path.abspath(args.out)!r}\nNH = {args.n_head}\nC = {args.n_embed}\n"
            f"CTX = {args.ctx}\nV = {args.vocab}\nL = {args.n_blocks}\n" + CHILD)
    r = subprocess.run([sys.executable, "-c", code], cwd="/tmp", capture_output=True, text=True)
    sys.stdout.write(r.stdout)
    sys.stderr.write(r.stderr[-3000:])
    return r.returncode


if __name__ == "__main__":
    sys.exit(main())

"""Time the REFERENCE's training algorithm on MI355X at the headline shape (GPT-2-small dims, T=1024).

The reference's model math, re-expressed here in plain PyTorch (nothing imported or copied from the
reference tree, which does not exist on the GPU box): per-head key / query / value ``nn.Linear``
modules without bias, a materialised T x T score matrix per head (``q @ k^T / sqrt(hd)``,
``masked_fill`` against a ``tril`` buffer, softmax, ``@ v``), the heads concatenated with no output
projection (/root/reference/src/models/attention.py:47-57,95), a ReLU MLP 4C wide
(src/models/mlp.py:24-26), pre-LN blocks with residuals (src/models/transformer_block.py:28-47),
learned positions and an untied biased LM head (src/models/transformer.py:34-38), fp32 parameters
under bf16 autocast, F.cross_entropy, ``torch.optim.AdamW`` (scripts/train_transformer.py:66,126).
``--compile`` wraps the model in torch.compile as the reference's trainer does by default
(TORCH_COMPILE=1, scripts/train_transformer.py:33,118-120).

One JSON line: tokens/s of full training steps (forward, backward, AdamW step, zero_grad) with
synthetic tokens and random init.  This is the reference-algorithm baseline of BASELINE.md; the
headline bench (bench.py) runs GPT-2 small proper (W_o, GELU, tied head) on this framework."""
import argparse
import json
import math
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class RefHead(nn.Module):
    def __init__(self, hd, C, T):
        super().__init__()
        self.key = nn.Linear(C, hd, bias=False)
        self.query = nn.Linear(C, hd, bias=False)
        self.value = nn.Linear(C, hd, bias=False)
        self.register_buffer("tril", torch.tril(torch.ones(T, T)))

    def forward(self, x):
        T = x.shape[1]
        k, q = self.key(x), self.query(x)
        w = q @ k.transpose(-2, -1) * (1.0 / math.sqrt(k.shape[-1]))
        w = F.softmax(w.masked_fill(self.tril[:T, :T] == 0, float("-inf")), dim=-1)
        return w @ self.value(x)


class RefBlock(nn.Module):
    def __init__(self, H, C, T):
        super().__init__()
        self.ln1, self.ln2 = nn.LayerNorm(C), nn.LayerNorm(C)
        self.heads = nn.ModuleList(RefHead(C // H, C, T) for _ in range(H))
        self.hidden, self.proj = nn.Linear(C, 4 * C), nn.Linear(4 * C, C)

    def forward(self, x):
        h = self.ln1(x)
        x = x + torch.cat([hd(h) for hd in self.heads], dim=-1)
        return x + self.proj(F.relu(self.hidden(self.ln2(x))))


class RefLM(nn.Module):
    def __init__(self, V, T, C, H, L):
        super().__init__()
        self.tok, self.pos = nn.Embedding(V, C), nn.Embedding(T, C)
        self.blocks = nn.ModuleList(RefBlock(H, C, T) for _ in range(L))
        self.ln = nn.LayerNorm(C)
        self.head = nn.Linear(C, V)
        self.register_buffer("pos_idx", torch.arange(T))

    def forward(self, idx, tgt):
        T = idx.shape[1]
        x = self.tok(idx) + self.pos(self.pos_idx[:T])
        for b in self.blocks:
            x = b(x)
        logits = self.head(self.ln(x))
        return F.cross_entropy(logits.view(-1, logits.shape[-1]), tgt.view(-1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--compile", action="store_true")
    args = ap.parse_args()
    V, C, H, L, T, B = 50304, 768, 12, 12, args.seq, args.batch
    torch.manual_seed(0)
    model = RefLM(V, T, C, H, L).cuda()
    opt = torch.optim.AdamW(model.parameters(), lr=3e-4)
    step_model = torch.compile(model) if args.compile else model
    idx = torch.randint(0, V, (B, T), device="cuda")
    tgt = torch.randint(0, V, (B, T), device="cuda")

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = step_model(idx, tgt)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    t0 = time.perf_counter()
    for _ in range(args.warmup):
        loss = step()
    torch.cuda.synchronize()
    warm_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    n_params = sum(p.numel() for p in model.parameters())
    print(json.dumps({"metric": "tokens/sec, reference algorithm (materialised per-head attention, no W_o, ReLU)",
                      "value": round(B * T / dt, 1), "ms_per_step": round(dt * 1e3, 2), "batch": B, "seq": T,
                      "compile": args.compile, "params": n_params, "loss": round(float(loss), 4),
                      "warmup_s": round(warm_s, 1), "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2 ** 30, 1),
                      "dtype": "bf16 autocast, fp32 params, torch AdamW", "data": "synthetic"}), flush=True)


if __name__ == "__main__":
    main()

"""Autoregressive generation with a KV cache.

Reference behaviour (src/models/transformer.py:96-114): loop ``max_new_tokens``
times, crop the context to the last ``context_length`` tokens, run a FULL forward
(no KV cache), softmax the last position and ``torch.multinomial`` one token.

Here the prompt is prefilled once through the flash-attention kernel and every
new token is a single-position step that appends its K/V to a preallocated
cache (O(T) per token instead of O(T^2 * L)).  When the running sequence would
exceed ``context_length`` with learned absolute positions, the reference's crop
semantics are reproduced exactly by re-prefilling the cropped window.
``temperature``/``top_k`` extend the reference's plain multinomial sampling
(temperature 1, no top-k == reference).
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import ops


class KVCache:
    """Per-layer K/V buffers [B, S_max, Hkv, D] in the model's compute dtype."""

    def __init__(self, n_layers: int, batch: int, max_len: int, n_kv_head: int, head_dim: int, dtype, device):
        shape = (batch, max_len, n_kv_head, head_dim)
        self.k = [torch.empty(shape, dtype=dtype, device=device) for _ in range(n_layers)]
        self.v = [torch.empty(shape, dtype=dtype, device=device) for _ in range(n_layers)]
        self.max_len = max_len

    def update(self, layer: int, k: torch.Tensor, v: torch.Tensor, pos: int):
        T = k.shape[1]
        if pos + T > self.max_len:
            raise ValueError(f"KV cache overflow: {pos + T} > {self.max_len}")
        self.k[layer][:, pos:pos + T].copy_(k)
        self.v[layer][:, pos:pos + T].copy_(v)
        return self.k[layer][:, :pos + T], self.v[layer][:, :pos + T]


@torch.no_grad()
def forward_cached(model, idx: torch.Tensor, cache: KVCache, pos: int,
                   last: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Run tokens ``idx`` [B, T] at absolute positions pos..pos+T-1; returns logits of the last position
    (or, with ``last`` [B] int64, of row b's position last[b]: right-padded prompts of different
    lengths in one batch -- causal attention keeps every real token blind to the padding after it)."""
    cfg = model.config
    wpe = model.position_embed.weight if model.position_embed is not None else None
    x = ops.embedding(idx, model.token_embed.weight, wpe, pos_offset=pos)
    rope = model.rope_tables(idx.device, pos + idx.shape[1])
    res = None
    for i, blk in enumerate(model.attn_blocks):
        x, res = blk.forward_cached(x, res, cache, i, pos, rope)
    # only the last position's logits are needed: norm + head on that row alone
    if last is not None:
        rows = torch.arange(x.shape[0], device=x.device)
        xl = x[rows, last].unsqueeze(1)
        rl = res[rows, last].unsqueeze(1) if res is not None else None
    else:
        xl, rl = x[:, -1:], (res[:, -1:] if res is not None else None)
    logits, _ = model.layer_norm.linear(xl, rl, model.head_weight, model.head_bias)
    return logits[:, -1, :].float()


@torch.no_grad()
def forward_decode(model, tok: torch.Tensor, cache: KVCache, pos_t: torch.Tensor, len_t: torch.Tensor) -> torch.Tensor:
    """One decode step for tokens ``tok`` [B, 1] at the device position ``pos_t`` (int64 [1], or
    [B]: one position per sequence, continuous batching); ``len_t`` = pos_t + 1 as int32.  Every op is position-agnostic on the host (indexing by
    device tensors, decode kernel reading the key count from ``len_t``), so the whole step
    is hipGraph-capturable.  Returns fp32 logits [B, V]."""
    cfg = model.config
    x = model.token_embed.weight.index_select(0, tok.view(-1)).view(tok.shape[0], 1, -1)
    if model.position_embed is not None:  # pos_t: one position, or one per sequence
        x = x + model.position_embed.weight.index_select(0, pos_t).view(pos_t.numel(), 1, -1)
    rope = model.rope_tables(tok.device, cache.max_len) if cfg.pos == "rope" else None
    res = None
    for i, blk in enumerate(model.attn_blocks):
        x, res = blk.forward_decode(x, res, cache, i, pos_t, len_t, rope)
    logits, _ = model.layer_norm.linear(x, res, model.head_weight, model.head_bias)
    return logits[:, -1, :].float()


class DecodeGraph:
    """A decode step captured once as a hipGraph and replayed per token.

    A GPT-2-small step is ~130 small kernels (12 x {norm, 3 GEMMs, decode attention,
    activation, ...}); at serving batch sizes each is a few microseconds, so eager decode
    is launch-bound.  Replaying one graph removes the per-kernel host overhead.  Inputs
    live in static buffers (token ids, device position); outputs in a static logits buffer."""

    def __init__(self, model, cache: KVCache, batch: int, device, warmup: int = 2, per_row: bool = False):
        """``per_row``: one position per sequence (continuous batching: slots at different
        positions); ``__call__`` then takes a [batch] position tensor."""
        self.model, self.cache = model, cache
        n = batch if per_row else 1
        self.tok = torch.zeros(batch, 1, dtype=torch.long, device=device)
        self.pos_t = torch.zeros(n, dtype=torch.long, device=device)
        self.len_t = torch.ones(n, dtype=torch.int32, device=device)
        side = torch.cuda.Stream(device)
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(side):  # warm up (allocator pools, lazy library init) off-graph
            for _ in range(warmup):
                forward_decode(model, self.tok, cache, self.pos_t, self.len_t)
        torch.cuda.current_stream(device).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.logits = forward_decode(model, self.tok, cache, self.pos_t, self.len_t)

    def __call__(self, tok: torch.Tensor, pos) -> torch.Tensor:
        self.tok.copy_(tok)
        if isinstance(pos, torch.Tensor):
            self.pos_t.copy_(pos)
            self.len_t.copy_(pos + 1)
        else:
            self.pos_t.fill_(pos)
            self.len_t.fill_(pos + 1)
        self.graph.replay()
        return self.logits


def sample_next(logits: torch.Tensor, temperature: float = 1.0, top_k: Optional[int] = None,
                generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """logits [B, V] (fp32) -> next token ids [B, 1]; temperature 0 = greedy.

    On the GPU the draw is one fused Gumbel-max kernel (csrc/sampling.hip: an exact sample
    of softmax(logits / T) in a single pass, seeded from ``generator``); on the CPU it is the
    reference's softmax + multinomial (transformer.py:111-112)."""
    if top_k is not None and top_k < logits.shape[-1] and temperature != 0.0:
        v, _ = torch.topk(logits, top_k)
        logits = logits.masked_fill(logits < v[:, [-1]], float("-inf"))
    if logits.is_cuda and ops.get_backend() == "auto":  # fp32 logits of any model dtype
        seed = 0
        if temperature != 0.0:
            gdev = generator.device if generator is not None else "cpu"
            seed = int(torch.randint(0, 2 ** 62, (1,), generator=generator, device=gdev).item())
        return ops._ops().sample(logits, float(temperature), seed)
    if temperature == 0.0:
        return logits.argmax(-1, keepdim=True)
    probs = torch.softmax(logits / temperature, dim=-1)
    return torch.multinomial(probs, num_samples=1, generator=generator)


@torch.no_grad()
def generate(model, idx: torch.Tensor, max_new_tokens: int, temperature: float = 1.0, top_k: Optional[int] = None,
             use_cache: bool = True, generator: Optional[torch.Generator] = None,
             cuda_graph: bool = False, decode_cache: Optional[dict] = None) -> torch.Tensor:
    """``cuda_graph``: replay each single-token step from one captured hipGraph (GPU only).
    ``decode_cache``: a dict owned by the caller (e.g. the generation service) that keeps the KV
    cache and the captured decode graph per (batch, cache length) across calls, so a repeated
    shape skips the allocation and the capture (the prefill overwrites the rows a call reads)."""
    was_training = model.training
    model.eval()
    cfg = model.config
    ctx_len = cfg.context_length
    learned = cfg.pos == "learned"
    try:
        if not use_cache:
            for _ in range(max_new_tokens):
                idx_cond = idx[:, -ctx_len:]
                logits, _ = model(idx_cond)
                nxt = sample_next(logits[:, -1, :].float(), temperature, top_k, generator)
                idx = torch.cat([idx, nxt], dim=1)
            return idx
        B = idx.shape[0]
        max_len = min(idx.shape[1] + max_new_tokens, ctx_len) if learned else idx.shape[1] + max_new_tokens
        dtype = model.token_embed.weight.dtype
        key = (B, max(max_len, 1), dtype, idx.device)
        cache, graph = decode_cache.get(key, (None, None)) if decode_cache is not None else (None, None)
        if cache is None:
            cache = KVCache(cfg.n_blocks, B, max(max_len, 1), cfg.n_kv_head, cfg.head_dim, dtype, idx.device)
        window = idx[:, -ctx_len:] if learned else idx
        if graph is None and cuda_graph and idx.is_cuda and max_new_tokens > 1:
            # captured before the prefill: its warm-up steps write cache row 0, which the prefill overwrites
            graph = DecodeGraph(model, cache, B, idx.device)
        if decode_cache is not None:
            decode_cache[key] = (cache, graph)
        if not cuda_graph:
            graph = None
        logits = forward_cached(model, window, cache, 0)
        pos = window.shape[1]
        for step in range(max_new_tokens):
            nxt = sample_next(logits, temperature, top_k, generator)
            idx = torch.cat([idx, nxt], dim=1)
            if step == max_new_tokens - 1:
                break
            if learned and pos >= ctx_len:
                # reference crop semantics: positions restart at 0 for the last ctx_len tokens
                window = idx[:, -ctx_len:]
                logits = forward_cached(model, window, cache, 0)
                pos = window.shape[1]
            elif graph is not None:
                logits = graph(nxt, pos)
                pos += 1
            else:
                logits = forward_cached(model, nxt, cache, pos)
                pos += 1
        return idx
    finally:
        model.train(was_training)

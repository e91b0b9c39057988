"""Reference-API compatibility layer (names, constructor signatures, checkpoint layout).

The reference exposes ``src.models.{MLP, Head, MultiHeadAttention, Block, Transformer}``
(`src/models/__init__.py:2-5`) with these signatures:

* ``Head(head_size, n_embed, context_length)``            -- `attention.py:19`
* ``MultiHeadAttention(n_head, n_embed, context_length)``  -- `attention.py:72`
* ``MLP(n_embed)``                                          -- `mlp.py:16`
* ``Block(n_head, n_embed, context_length)``                -- `transformer_block.py:18`
* ``Transformer(n_head, n_embed, context_length, vocab_size, N_BLOCKS)`` -- `transformer.py:20`

Its checkpoint stores per-head ``attn.heads.{h}.{key,query,value}.weight`` ([hd, C]) and a
persistent fp32 ``tril`` buffer per head (`attention.py:29-33`).  Our model keeps one packed
QKV weight per layer (one GEMM instead of 3*H); the hooks below translate both ways so a
reference checkpoint loads strictly and our checkpoints load into reference-layout code.
"""
from __future__ import annotations

import re
from typing import Optional

import torch
import torch.nn as nn

from .. import ops
from .config import ModelConfig, _ref
from . import gpt as _gpt

_QKV_RE = re.compile(r"^(.*attn_blocks\.\d+\.attn\.)qkv\.weight$")
_HEAD_RE = re.compile(r"^(.*attn_blocks\.\d+\.attn\.)heads\.(\d+)\.(key|query|value|tril)(\.weight)?$")

WRAPPER_PREFIXES = ("module.", "_orig_mod.")


def strip_wrapper_prefixes(sd: dict) -> dict:
    """Remove DDP ``module.`` / torch.compile ``_orig_mod.`` prefixes (reference defect D7)."""
    out = {}
    for k, v in sd.items():
        changed = True
        while changed:
            changed = False
            for p in WRAPPER_PREFIXES:
                if k.startswith(p):
                    k = k[len(p):]
                    changed = True
        out[k] = v
    return out


def _split_state(model, state_dict, prefix, local_metadata):
    cfg: ModelConfig = model.config
    pg = getattr(model, "parallel", None)
    if pg is not None and pg.tp > 1:
        return state_dict  # a tensor-parallel shard keeps its packed local layout
    H, D, T = cfg.n_head, cfg.head_dim, cfg.context_length
    tril = None
    for key in [k for k in list(state_dict.keys()) if k.startswith(prefix)]:
        m = _QKV_RE.match(key[len(prefix):])
        if not m:
            continue
        base = prefix + m.group(1)
        w = state_dict.pop(key)
        q, k, v = w[:H * D], w[H * D:2 * H * D], w[2 * H * D:]
        if tril is None:
            tril = torch.tril(torch.ones(T, T, dtype=torch.float32, device=w.device))
        for h in range(H):
            sl = slice(h * D, (h + 1) * D)
            # reference per-head registration order: key, query, value (attention.py:29-31), then tril
            state_dict[f"{base}heads.{h}.tril"] = tril
            state_dict[f"{base}heads.{h}.key.weight"] = k[sl].clone()
            state_dict[f"{base}heads.{h}.query.weight"] = q[sl].clone()
            state_dict[f"{base}heads.{h}.value.weight"] = v[sl].clone()
    return state_dict


def _fuse_state(model, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys, error_msgs):
    cfg: ModelConfig = model.config
    H = cfg.n_head
    groups = {}
    for key in [k for k in list(state_dict.keys()) if k.startswith(prefix)]:
        m = _HEAD_RE.match(key[len(prefix):])
        if not m:
            continue
        base, h, kind = prefix + m.group(1), int(m.group(2)), m.group(3)
        val = state_dict.pop(key)
        if kind == "tril":
            continue  # constant mask: recomputed implicitly by the causal kernel
        groups.setdefault(base, {}).setdefault(kind, {})[h] = val
    for base, kinds in groups.items():
        try:
            q = torch.cat([kinds["query"][h] for h in range(H)], 0)
            k = torch.cat([kinds["key"][h] for h in range(H)], 0)
            v = torch.cat([kinds["value"][h] for h in range(H)], 0)
        except KeyError as e:
            error_msgs.append(f"incomplete per-head attention weights under {base}: missing {e}")
            continue
        state_dict[f"{base}qkv.weight"] = torch.cat([q, k, v], 0)


def install_ref_state_dict_hooks(model: nn.Module):
    model._register_state_dict_hook(lambda mod, sd, prefix, lm: _split_state(mod, sd, prefix, lm))
    model._register_load_state_dict_pre_hook(
        lambda sd, prefix, lm, strict, mk, uk, em: _fuse_state(model, sd, prefix, lm, strict, mk, uk, em))


# ---------------------------------------------------------------------------
# reference-signature classes
# ---------------------------------------------------------------------------
class Transformer(_gpt.GPT):
    """``Transformer(n_head, n_embed, context_length, vocab_size, N_BLOCKS)`` with the reference
    architecture (`transformer.py:20-39`). Extra keyword ``n_blocks`` is accepted as an alias so
    the reference trainer's ``model_args`` dict works (defect D4)."""

    def __init__(self, n_head: int, n_embed: int, context_length: int, vocab_size: int,
                 N_BLOCKS: Optional[int] = None, n_blocks: Optional[int] = None, **kw):
        L = N_BLOCKS if N_BLOCKS is not None else n_blocks
        if L is None:
            raise TypeError("Transformer() missing N_BLOCKS")
        cfg = _ref(n_head=n_head, n_embed=n_embed, context_length=context_length,
                   vocab_size=vocab_size, n_blocks=L, **kw)
        super().__init__(cfg)


class Head(nn.Module):
    """One causal attention head (`attention.py:6-58`): bias-free key/query/value projections
    and a persistent ``tril`` buffer; the math runs through the fused attention op."""

    def __init__(self, head_size: int, n_embed: int, context_length: int) -> None:
        super().__init__()
        self.key = nn.Linear(n_embed, head_size, bias=False)
        self.query = nn.Linear(n_embed, head_size, bias=False)
        self.value = nn.Linear(n_embed, head_size, bias=False)
        self.register_buffer("tril", torch.tril(torch.ones(context_length, context_length)))

    def forward(self, x):
        B, T, _ = x.shape
        q = self.query(x).unsqueeze(2)
        k = self.key(x).unsqueeze(2)
        v = self.value(x).unsqueeze(2)
        qkv = torch.cat([q, k, v], 2).reshape(B, T, -1)
        return ops.attention_packed(qkv, 1, 1, causal=True)


class MultiHeadAttention(_gpt.Attention):
    """``MultiHeadAttention(n_head, n_embed, context_length)`` (`attention.py:60-96`): H heads
    concatenated, no output projection; packed into one QKV GEMM."""

    def __init__(self, n_head: int, n_embed: int, context_length: int) -> None:
        super().__init__(_ref(n_head=n_head, n_embed=n_embed, context_length=context_length,
                              vocab_size=1, n_blocks=1))


class MLP(_gpt.MLP):
    """``MLP(n_embed)`` (`mlp.py:5-67`): Linear(C,4C) -> ReLU -> Linear(4C,C), with
    ``forward_embedding`` / ``project_embedding`` split."""

    def __init__(self, n_embed: int) -> None:
        super().__init__(_ref(n_embed=n_embed, n_head=1, vocab_size=1, n_blocks=1, context_length=1))


class Block(_gpt.Block):
    """``Block(n_head, n_embed, context_length)`` (`transformer_block.py:6-61`):
    ``x + attn(ln1(x))`` then ``+ mlp(ln2(.))``. ``forward(x)`` returns the block output and
    ``forward_embedding(x)`` returns ``(relu(hidden(ln2(res))), res)`` as in the reference."""

    def __init__(self, n_head: int, n_embed: int, context_length: int) -> None:
        super().__init__(_ref(n_head=n_head, n_embed=n_embed, context_length=context_length,
                              vocab_size=1, n_blocks=1))

    def forward(self, x, residual=None, rope=None):
        m, res = super().forward(x, residual, rope)
        if residual is None:        # reference semantics: a single tensor out
            return m if res is None else m + res  # (None: the projections added the stream already)
        return m, res

    def forward_embedding(self, x, residual=None, rope=None):
        return super().forward_embedding(x, residual, rope)

"""Tensor / sequence / context-parallel building blocks on RCCL (torch.distributed).

The reference has data parallelism only; the north star asks for
tensor- and sequence-parallel *hooks*.  These are the Megatron-style conjugate
collectives as autograd functions plus layers built on them:

* ``ColumnParallelLinear``  W split by output rows; input replicated (identity fwd /
  all-reduce bwd), output sharded on the last dim (optionally all-gathered).
* ``RowParallelLinear``     W split by input columns; input sharded; output all-reduced
  (or reduce-scattered along the sequence for sequence parallelism).
* ``TensorParallelAttention`` / ``TensorParallelMLP``: heads / FFN columns sharded,
  the flash-attention kernel runs unchanged on the local heads.
* sequence parallelism: ``scatter_to_sequence`` / ``gather_from_sequence`` /
  ``reduce_scatter_to_sequence`` around the norm/residual regions.
* Ulysses context parallelism: ``seq_to_head_all_to_all`` / ``head_to_seq_all_to_all``
  re-shard [B, T/P, H, D] <-> [B, T, H/P, D] so attention sees the whole sequence
  for a subset of heads.

Degree choice on MI355X: every GPU has 7 point-to-point xGMI links (~153 GB/s each);
a TP all-reduce inside the node is per-link bound, so TP is for models whose
weights/activations do not fit one 288 GB HBM stack, not a default.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from .. import ops


def _ws(group) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def _rank(group) -> int:
    return dist.get_rank(group) if dist.is_initialized() else 0


def _all_gather_last(x, group):
    ws = _ws(group)
    if ws == 1:
        return x
    parts = [torch.empty_like(x) for _ in range(ws)]
    dist.all_gather(parts, x.contiguous(), group=group)
    return torch.cat(parts, dim=-1)


def _all_gather_dim(x, dim, group):
    ws = _ws(group)
    if ws == 1:
        return x
    parts = [torch.empty_like(x) for _ in range(ws)]
    dist.all_gather(parts, x.contiguous(), group=group)
    return torch.cat(parts, dim=dim)


def _split_dim(x, dim, group):
    ws = _ws(group)
    if ws == 1:
        return x
    return x.chunk(ws, dim=dim)[_rank(group)].contiguous()


def _reduce_scatter_dim(x, dim, group):
    ws = _ws(group)
    if ws == 1:
        return x
    if dist.get_backend(group) == "nccl" and dim == 0:
        out = torch.empty((x.shape[0] // ws,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.reduce_scatter_tensor(out, x.contiguous(), group=group)
        return out
    y = x.contiguous().clone()
    dist.all_reduce(y, group=group)
    return _split_dim(y, dim, group)


class _CopyToTP(torch.autograd.Function):
    """identity forward, all-reduce backward (input of a column-parallel layer)"""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):
        if _ws(ctx.group) > 1:
            g = g.contiguous().clone()
            dist.all_reduce(g, group=ctx.group)
        return g, None


class _ReduceFromTP(torch.autograd.Function):
    """all-reduce forward, identity backward (output of a row-parallel layer)"""

    @staticmethod
    def forward(ctx, x, group):
        if _ws(group) > 1:
            x = x.contiguous().clone()
            dist.all_reduce(x, group=group)
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None


class _GatherFromTP(torch.autograd.Function):
    """all-gather on the last dim forward, split backward"""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _all_gather_last(x, group)

    @staticmethod
    def backward(ctx, g):
        return _split_dim(g, -1, ctx.group), None


class _ScatterToSeq(torch.autograd.Function):
    """split the sequence dim (dim 1) forward, all-gather backward"""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _split_dim(x, 1, group)

    @staticmethod
    def backward(ctx, g):
        return _all_gather_dim(g, 1, ctx.group), None


class _GatherFromSeq(torch.autograd.Function):
    """all-gather the sequence dim forward, reduce-scatter backward (the consumer is a TP region)"""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _all_gather_dim(x, 1, group)

    @staticmethod
    def backward(ctx, g):
        return _reduce_scatter_dim(g, 1, ctx.group), None


class _ReduceScatterToSeq(torch.autograd.Function):
    """reduce-scatter along the sequence forward (row-parallel output under SP), all-gather backward"""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _reduce_scatter_dim(x, 1, group)

    @staticmethod
    def backward(ctx, g):
        return _all_gather_dim(g, 1, ctx.group), None


def copy_to_tensor_parallel(x, group=None):
    return _CopyToTP.apply(x, group)


def reduce_from_tensor_parallel(x, group=None):
    return _ReduceFromTP.apply(x, group)


def gather_from_tensor_parallel(x, group=None):
    return _GatherFromTP.apply(x, group)


def scatter_to_sequence(x, group=None):
    return _ScatterToSeq.apply(x, group)


def gather_from_sequence(x, group=None):
    return _GatherFromSeq.apply(x, group)


def reduce_scatter_to_sequence(x, group=None):
    return _ReduceScatterToSeq.apply(x, group)


# ---------------------------------------------------------------------------
# layers
# ---------------------------------------------------------------------------
class ColumnParallelLinear(nn.Module):
    def __init__(self, in_features: int, out_features: int, bias: bool = True, group=None,
                 gather_output: bool = False, sequence_parallel: bool = False):
        super().__init__()
        ws = _ws(group)
        assert out_features % ws == 0, "out_features must divide the TP degree"
        self.group, self.gather_output, self.sp = group, gather_output, sequence_parallel
        self.weight = nn.Parameter(torch.empty(out_features // ws, in_features))
        self.bias = nn.Parameter(torch.zeros(out_features // ws)) if bias else None
        nn.init.normal_(self.weight, std=0.02)

    @torch.no_grad()
    def load_from_dense(self, weight, bias=None):
        self.weight.copy_(_split_dim(weight, 0, self.group))
        if self.bias is not None and bias is not None:
            self.bias.copy_(_split_dim(bias, 0, self.group))

    def forward(self, x):
        x = gather_from_sequence(x, self.group) if self.sp else copy_to_tensor_parallel(x, self.group)
        y = ops.linear(x, self.weight, self.bias)
        return gather_from_tensor_parallel(y, self.group) if self.gather_output else y


class RowParallelLinear(nn.Module):
    def __init__(self, in_features: int, out_features: int, bias: bool = True, group=None,
                 input_is_parallel: bool = True, sequence_parallel: bool = False):
        super().__init__()
        ws = _ws(group)
        assert in_features % ws == 0, "in_features must divide the TP degree"
        self.group, self.input_is_parallel, self.sp = group, input_is_parallel, sequence_parallel
        self.weight = nn.Parameter(torch.empty(out_features, in_features // ws))
        self.bias = nn.Parameter(torch.zeros(out_features)) if bias else None
        nn.init.normal_(self.weight, std=0.02)

    @torch.no_grad()
    def load_from_dense(self, weight, bias=None):
        self.weight.copy_(_split_dim(weight, 1, self.group))
        if self.bias is not None and bias is not None:
            self.bias.copy_(bias)

    def forward(self, x):
        if not self.input_is_parallel:
            x = _split_dim(x, -1, self.group)
        y = ops.linear(x, self.weight, None)
        y = reduce_scatter_to_sequence(y, self.group) if self.sp else reduce_from_tensor_parallel(y, self.group)
        return y + self.bias if self.bias is not None else y


class TensorParallelMLP(nn.Module):
    """GELU MLP with the 4C hidden dimension sharded (column -> row parallel, one all-reduce)."""

    def __init__(self, n_embed: int, hidden: int, group=None, sequence_parallel: bool = False, bias: bool = True):
        super().__init__()
        self.fc = ColumnParallelLinear(n_embed, hidden, bias, group, sequence_parallel=sequence_parallel)
        self.proj = RowParallelLinear(hidden, n_embed, bias, group, sequence_parallel=sequence_parallel)

    def forward(self, x):
        return self.proj(ops.gelu(self.fc(x)))


class TensorParallelAttention(nn.Module):
    """Causal self-attention with heads sharded over the TP group; packed QKV per rank."""

    def __init__(self, n_embed: int, n_head: int, group=None, sequence_parallel: bool = False, bias: bool = True):
        super().__init__()
        ws = _ws(group)
        assert n_head % ws == 0, "n_head must divide the TP degree"
        self.group, self.n_head, self.local_heads = group, n_head, n_head // ws
        self.head_dim = n_embed // n_head
        self.qkv = ColumnParallelLinear(n_embed, 3 * n_embed, bias, group, sequence_parallel=sequence_parallel)
        self.proj = RowParallelLinear(n_embed, n_embed, bias, group, sequence_parallel=sequence_parallel)

    @torch.no_grad()
    def load_from_dense(self, qkv_w, qkv_b, proj_w, proj_b):
        """Shard a dense packed [q|k|v] weight so each rank gets its heads' q, k and v rows."""
        C, H, D, r = qkv_w.shape[1], self.n_head, self.head_dim, _rank(self.group)
        lh = self.local_heads
        sel = []
        for part in range(3):
            base = part * H * D
            sel.append(torch.arange(base + r * lh * D, base + (r + 1) * lh * D))
        idx = torch.cat(sel).to(qkv_w.device)
        self.qkv.weight.copy_(qkv_w[idx])
        if qkv_b is not None and self.qkv.bias is not None:
            self.qkv.bias.copy_(qkv_b[idx])
        self.proj.load_from_dense(proj_w, proj_b)

    def forward(self, x):
        qkv = self.qkv(x)
        y = ops.attention_packed(qkv, self.local_heads, self.local_heads, causal=True)
        return self.proj(y)


# ---------------------------------------------------------------------------
# Ulysses context parallelism (all-to-all between sequence and head sharding)
# ---------------------------------------------------------------------------
def _a2a(x, scatter_dim: int, gather_dim: int, group):
    ws = _ws(group)
    if ws == 1:
        return x
    inputs = [t.contiguous() for t in x.chunk(ws, dim=scatter_dim)]
    if dist.get_backend(group) == "gloo":  # gloo has no all-to-all: gather everything, keep our chunks
        full = [torch.empty_like(x.contiguous()) for _ in range(ws)]
        dist.all_gather(full, x.contiguous(), group=group)
        me = _rank(group)
        return torch.cat([f.chunk(ws, dim=scatter_dim)[me] for f in full], dim=gather_dim)
    outputs = [torch.empty_like(inputs[0]) for _ in range(ws)]
    dist.all_to_all(outputs, inputs, group=group)
    return torch.cat(outputs, dim=gather_dim)


class _SeqToHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):  # [B, T/P, H, D] -> [B, T, H/P, D]
        ctx.group = group
        return _a2a(x, 2, 1, group)

    @staticmethod
    def backward(ctx, g):
        return _a2a(g, 1, 2, ctx.group), None


class _HeadToSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):  # [B, T, H/P, D] -> [B, T/P, H, D]
        ctx.group = group
        return _a2a(x, 1, 2, group)

    @staticmethod
    def backward(ctx, g):
        return _a2a(g, 2, 1, ctx.group), None


def seq_to_head_all_to_all(x, group=None):
    return _SeqToHead.apply(x, group)


def head_to_seq_all_to_all(x, group=None):
    return _HeadToSeq.apply(x, group)


def ulysses_attention(qkv_local, n_head: int, group=None, causal: bool = True):
    """Attention for a sequence-sharded packed qkv [B, T/P, 3*H*D]: all-to-all to head sharding,
    full-sequence attention on H/P heads, all-to-all back. Returns [B, T/P, H*D]."""
    B, Tl, W = qkv_local.shape
    D = W // (3 * n_head)
    x = qkv_local.view(B, Tl, 3 * n_head, D)
    q, k, v = x[:, :, :n_head], x[:, :, n_head:2 * n_head], x[:, :, 2 * n_head:]
    qh, kh, vh = (seq_to_head_all_to_all(t.contiguous(), group) for t in (q, k, v))
    Hl = qh.shape[2]
    packed = torch.cat([qh, kh, vh], dim=2).reshape(B, qh.shape[1], 3 * Hl * D)
    o = ops.attention_packed(packed, Hl, Hl, causal=causal).view(B, qh.shape[1], Hl, D)
    return head_to_seq_all_to_all(o, group).reshape(B, Tl, n_head * D)

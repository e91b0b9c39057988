"""Tensor, sequence and context parallelism wired into the GPT model and the Trainer.

The reference trains with data parallelism only (``DDP(model)``,
scripts/train_transformer.py:122-123).  Here a job of ``world`` ranks is a
``dp x cp x tp`` mesh (tensor-parallel ranks innermost, so a TP group is a set of
neighbouring GPUs of one node: on MI355X every pair of GPUs has its own xGMI link, and TP's
per-layer all-reduces are the latency-critical traffic):

* **TP** (``tp_size``): attention heads (and GQA kv heads) and FFN columns are sharded,
  Megatron-style.  The packed QKV / up-projection weights become column-parallel (each rank
  keeps the q, k, v rows of ITS heads -- for SwiGLU the matching gate and up rows), the
  output / down projections row-parallel, with one all-reduce per sub-layer in forward and
  one in backward (``parallel/tensor.py`` conjugate autograd functions).  The flash-attention
  kernel (RoPE fused) runs unchanged on the local heads.  Embeddings, norms and the LM head
  stay replicated; with plain TP every rank computes identical gradients for them.
* **SP** (``sequence_parallel``, with TP): the norm / residual regions hold only T/tp tokens
  per rank; all-gather before each column-parallel GEMM, reduce-scatter after each
  row-parallel one, LM head + CE on the local tokens.  Replicated parameters then carry
  partial gradients, which ``sync_replicated_grads`` sums over the TP group.
* **TP x CP**: both at once -- each rank keeps its heads (TP) of its sequence shard (CP) and runs
  ring / Ulysses attention over the CP group on the local heads; the MLP is TP-sharded.
* **SP without W_o** (the reference architecture): the concatenated heads return to sequence
  shards by one all-to-all over the TP group instead of a W_o reduce-scatter.
* **CP** (``cp_size``): the sequence is sharded over the CP group.  ``cp_mode="ring"``:
  load-balanced zigzag layout, ring attention over RCCL point-to-point with the flash kernels'
  LSE merge (``parallel/context.py``); ``cp_mode="ulysses"``: contiguous shards, all-to-all to
  head sharding around full-sequence flash attention.  Position embeddings / RoPE tables are
  gathered at the shard's global positions; gradients are averaged over dp x cp.

The model is built dense on every rank (same seed), then ``parallelize_gpt`` slices each
sharded weight, so a TP / CP run starts from exactly the dense model's weights and its loss and
gradients match the dense model's (tests/test_model_parallel.py).
"""
from __future__ import annotations

import dataclasses
from typing import List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from .. import ops
from . import context as cpar
from . import tensor as tpar


@dataclasses.dataclass
class ParallelGroups:
    world: int = 1
    rank: int = 0
    tp: int = 1
    tp_rank: int = 0
    tp_group: object = None
    cp: int = 1
    cp_rank: int = 0
    cp_group: object = None
    dp: int = 1
    dp_rank: int = 0
    dp_group: object = None
    grad_group: object = None      # ranks that average gradients: dp x cp (same tp rank)
    sequence_parallel: bool = False
    cp_mode: str = "ring"          # "ring": zigzag shards + ring attention; "ulysses": contiguous + all-to-all

    @property
    def model_parallel(self) -> bool:
        return self.tp > 1 or self.cp > 1


def init_parallel_groups(tp: int = 1, cp: int = 1, sequence_parallel: bool = False,
                         cp_mode: str = "ring") -> ParallelGroups:
    """Create the dp / cp / tp / gradient process groups of a ``dp x cp x tp`` mesh (every rank
    must call this, in the same order).  rank = (dp_rank * cp + cp_rank) * tp + tp_rank."""
    if cp_mode not in ("ring", "ulysses"):
        raise ValueError(f"cp_mode={cp_mode!r}: expected 'ring' or 'ulysses'")
    init = dist.is_initialized()
    world = dist.get_world_size() if init else 1
    rank = dist.get_rank() if init else 0
    if tp < 1 or cp < 1 or world % (tp * cp):
        raise ValueError(f"world size {world} is not divisible by tp_size {tp} x cp_size {cp}")
    if sequence_parallel and tp == 1:
        raise ValueError("sequence_parallel needs tp_size > 1")
    dp = world // (tp * cp)
    tp_rank, cp_rank, dp_rank = rank % tp, (rank // tp) % cp, rank // (tp * cp)
    g = ParallelGroups(world, rank, tp, tp_rank, None, cp, cp_rank, None, dp, dp_rank, None, None, sequence_parallel,
                       cp_mode)
    if not init or world == 1:
        return g

    def rk(d, c, t):
        return (d * cp + c) * tp + t

    for d in range(dp):                      # TP groups: neighbouring ranks
        for c in range(cp):
            grp = dist.new_group([rk(d, c, t) for t in range(tp)])
            if d == dp_rank and c == cp_rank:
                g.tp_group = grp
    for d in range(dp):                      # CP groups
        for t in range(tp):
            grp = dist.new_group([rk(d, c, t) for c in range(cp)])
            if d == dp_rank and t == tp_rank:
                g.cp_group = grp
    for c in range(cp):                      # DP groups
        for t in range(tp):
            grp = dist.new_group([rk(d, c, t) for d in range(dp)])
            if c == cp_rank and t == tp_rank:
                g.dp_group = grp
    for t in range(tp):                      # gradient-averaging groups (dp x cp)
        grp = dist.new_group([rk(d, c, t) for d in range(dp) for c in range(cp)])
        if t == tp_rank:
            g.grad_group = grp
    return g


def _rows(lo: int, hi: int) -> slice:
    return slice(lo, hi)


def _mark_sharded(*params):
    for p in params:
        if p is not None:
            p._pllm_tp_sharded = True


class TPAttention(nn.Module):
    """Head-sharded attention (column-parallel packed QKV, row-parallel output projection).
    Parameter names follow ``models.gpt.Attention`` (``qkv``, ``proj``) on local shapes."""

    fused_bias_ok = False  # the row-parallel bias is added after the all-reduce, here

    def __init__(self, dense, cfg, pg: ParallelGroups):
        super().__init__()
        tp, r = pg.tp, pg.tp_rank
        H, Hkv, D, C = cfg.n_head, cfg.n_kv_head, cfg.head_dim, cfg.n_embed
        if H % tp or Hkv % tp:
            raise ValueError(f"n_head {H} and n_kv_head {Hkv} must be divisible by tp_size {tp}")
        self.pg, self.cfg = pg, cfg
        self.n_head, self.n_kv_head, self.head_dim = H // tp, Hkv // tp, D
        Hl, Hkl = self.n_head, self.n_kv_head
        idx = torch.cat([torch.arange(r * Hl * D, (r + 1) * Hl * D),
                         H * D + torch.arange(r * Hkl * D, (r + 1) * Hkl * D),
                         (H + Hkv) * D + torch.arange(r * Hkl * D, (r + 1) * Hkl * D)])
        w = dense.qkv.weight
        self.qkv = nn.Linear(C, idx.numel(), bias=dense.qkv.bias is not None, device=w.device, dtype=w.dtype)
        with torch.no_grad():
            self.qkv.weight.copy_(w[idx.to(w.device)])
            if dense.qkv.bias is not None:
                self.qkv.bias.copy_(dense.qkv.bias[idx.to(w.device)])
        _mark_sharded(self.qkv.weight, self.qkv.bias)
        self.proj = None
        if dense.proj is not None:
            pw = dense.proj.weight
            self.proj = nn.Linear(Hl * D, C, bias=dense.proj.bias is not None, device=pw.device, dtype=pw.dtype)
            with torch.no_grad():
                self.proj.weight.copy_(pw[:, r * Hl * D:(r + 1) * Hl * D])
                if dense.proj.bias is not None:
                    self.proj.bias.copy_(dense.proj.bias)
            _mark_sharded(self.proj.weight)  # the bias stays replicated

    def forward(self, x, rope=None, fuse_out_bias: bool = False):
        g = self.pg.tp_group
        x = tpar.gather_from_sequence(x, g) if self.pg.sequence_parallel else tpar.copy_to_tensor_parallel(x, g)
        qkv = ops.linear(x, self.qkv.weight, self.qkv.bias)
        if self.pg.cp > 1:
            # 2-D: this rank's heads (TP) of this rank's sequence shard (CP), attention over the CP
            # group -- ring or Ulysses on the local heads
            y = cp_attention(qkv, self.n_head, self.n_kv_head, self.head_dim, rope, self.pg)
        else:
            cos, sin = rope if rope is not None else (None, None)
            y = ops.attention_packed(qkv, self.n_head, self.n_kv_head, causal=True, rope_cos=cos, rope_sin=sin)
        if self.proj is None:  # reference architecture: no W_o -> the heads are concatenated
            if self.pg.sequence_parallel:
                # back to sequence shards with every head: one all-to-all (head -> sequence
                # re-sharding, the Ulysses primitive) instead of a W_o reduce-scatter
                B, T, _ = y.shape
                yh = y.view(B, T, self.n_head, self.head_dim)
                return tpar.head_to_seq_all_to_all(yh, g).reshape(B, T // self.pg.tp, -1)
            return tpar.gather_from_tensor_parallel(y, g)
        y = ops.linear(y, self.proj.weight, None)
        y = tpar.reduce_scatter_to_sequence(y, g) if self.pg.sequence_parallel else tpar.reduce_from_tensor_parallel(y, g)
        return y + self.proj.bias if self.proj.bias is not None else y


class TPMLP(nn.Module):
    """FFN-column-sharded MLP (column-parallel up / gate+up, row-parallel down projection)."""

    fused_bias_ok = False

    def __init__(self, dense, cfg, pg: ParallelGroups):
        super().__init__()
        tp, r = pg.tp, pg.tp_rank
        Fh, C = cfg.ffn_hidden, cfg.n_embed
        if Fh % tp:
            raise ValueError(f"ffn_hidden {Fh} must be divisible by tp_size {tp}")
        self.pg, self.kind = pg, dense.kind
        Fl = Fh // tp
        idx = torch.arange(r * Fl, (r + 1) * Fl)
        if self.kind == "swiglu":  # packed [gate | up]: keep the matching rows of both
            idx = torch.cat([idx, Fh + idx])
        w = dense.hidden.weight
        self.hidden = nn.Linear(C, idx.numel(), bias=dense.hidden.bias is not None, device=w.device, dtype=w.dtype)
        pw = dense.proj.weight
        self.proj = nn.Linear(Fl, C, bias=dense.proj.bias is not None, device=pw.device, dtype=pw.dtype)
        with torch.no_grad():
            self.hidden.weight.copy_(w[idx.to(w.device)])
            if dense.hidden.bias is not None:
                self.hidden.bias.copy_(dense.hidden.bias[idx.to(w.device)])
            self.proj.weight.copy_(pw[:, r * Fl:(r + 1) * Fl])
            if dense.proj.bias is not None:
                self.proj.bias.copy_(dense.proj.bias)
        _mark_sharded(self.hidden.weight, self.hidden.bias, self.proj.weight)

    def _act(self, h):
        if self.kind == "gelu":
            return ops.gelu(h)
        if self.kind == "swiglu":
            return ops.swiglu(h)
        return ops.relu(h)

    def forward_embedding(self, x):
        g = self.pg.tp_group
        x = tpar.gather_from_sequence(x, g) if self.pg.sequence_parallel else tpar.copy_to_tensor_parallel(x, g)
        return tpar.gather_from_tensor_parallel(self._act(ops.linear(x, self.hidden.weight, self.hidden.bias)), g)

    def forward(self, x, fuse_out_bias: bool = False):
        g = self.pg.tp_group
        x = tpar.gather_from_sequence(x, g) if self.pg.sequence_parallel else tpar.copy_to_tensor_parallel(x, g)
        a = self._act(ops.linear(x, self.hidden.weight, self.hidden.bias))
        y = ops.linear(a, self.proj.weight, None)
        y = tpar.reduce_scatter_to_sequence(y, g) if self.pg.sequence_parallel else tpar.reduce_from_tensor_parallel(y, g)
        return y + self.proj.bias if self.proj.bias is not None else y


def cp_attention(qkv, H: int, Hkv: int, D: int, rope, pg: ParallelGroups):
    """Causal attention of a context-parallel shard: ``qkv`` [B, T_l, (H + 2 Hkv) D] (packed, this
    rank's heads) -> [B, T_l, H D].  RoPE is applied on the shard with its own position tables
    first; then ring attention over the CP group (zigzag shards) or Ulysses (contiguous shards:
    all-to-all to head sharding, full-sequence flash attention, all-to-all back)."""
    g = pg.cp_group
    if rope is not None:
        qkv = ops.rope_packed(qkv, rope[0], rope[1], H, Hkv)
    B, Tl, _ = qkv.shape
    q, k, v = ops._split_qkv(qkv, H, Hkv, D)
    if pg.cp_mode == "ulysses":
        if H % pg.cp or Hkv % pg.cp:
            raise ValueError(f"Ulysses: local n_head {H} and n_kv_head {Hkv} must be divisible by cp_size {pg.cp}")
        qh, kh, vh = (tpar.seq_to_head_all_to_all(t.contiguous(), g) for t in (q, k, v))  # [B, T, h/cp, D]
        T, Hl, Hkl = qh.shape[1], qh.shape[2], kh.shape[2]
        packed = torch.cat([qh, kh, vh], dim=2).reshape(B, T, (Hl + 2 * Hkl) * D)
        o = ops.attention_packed(packed, Hl, Hkl, causal=True).view(B, T, Hl, D)
        return tpar.head_to_seq_all_to_all(o, g).reshape(B, Tl, H * D)
    y = cpar.ring_attention(q, k, v, g, causal=True, layout="zigzag")
    return y.reshape(B, Tl, H * D)


class CPAttention(nn.Module):
    """Attention of a zigzag sequence shard: dense projections, ring attention over the CP group
    (RoPE applied with the shard's own position tables before the ring)."""

    fused_bias_ok = True

    def __init__(self, dense, pg: ParallelGroups):
        super().__init__()
        self.pg = pg
        self.qkv, self.proj = dense.qkv, dense.proj
        self.n_head, self.n_kv_head, self.head_dim = dense.n_head, dense.n_kv_head, dense.head_dim

    def forward(self, x, rope=None, fuse_out_bias: bool = False):
        qkv = ops.linear(x, self.qkv.weight, self.qkv.bias)
        y = cp_attention(qkv, self.n_head, self.n_kv_head, self.head_dim, rope, self.pg)
        if self.proj is not None:
            y = ops.linear(y, self.proj.weight, self.proj.bias, bias_grad_external=fuse_out_bias)
        return y


class UlyssesAttention(nn.Module):
    """Attention of a contiguous sequence shard by Ulysses re-sharding: the projections run on
    the local T/cp tokens, one all-to-all turns q / k / v from sequence- to head-sharded (each
    rank then holds the WHOLE sequence for H/cp query heads and Hkv/cp kv heads), the flash
    kernels run causal attention over the full sequence, and one all-to-all turns the output
    back.  Two all-to-alls of the activations per direction instead of the ring's cp - 1 K/V
    hops; needs n_head and n_kv_head divisible by cp_size.  RoPE is applied on the shard with its
    own position tables before the exchange."""

    fused_bias_ok = True

    def __init__(self, dense, pg: ParallelGroups):
        super().__init__()
        if dense.n_head % pg.cp or dense.n_kv_head % pg.cp:
            raise ValueError(f"Ulysses: n_head {dense.n_head} and n_kv_head {dense.n_kv_head} must be divisible by "
                             f"cp_size {pg.cp}")
        self.pg = pg
        self.qkv, self.proj = dense.qkv, dense.proj
        self.n_head, self.n_kv_head, self.head_dim = dense.n_head, dense.n_kv_head, dense.head_dim

    def forward(self, x, rope=None, fuse_out_bias: bool = False):
        qkv = ops.linear(x, self.qkv.weight, self.qkv.bias)
        y = cp_attention(qkv, self.n_head, self.n_kv_head, self.head_dim, rope, self.pg)
        if self.proj is not None:
            y = ops.linear(y, self.proj.weight, self.proj.bias, bias_grad_external=fuse_out_bias)
        return y


def parallelize_gpt(model, pg: ParallelGroups):
    """Shard a dense ``GPT`` in place for ``pg`` (TP: heads / FFN columns; CP: ring attention)."""
    if pg.tp > 1 and pg.cp > 1 and pg.sequence_parallel:
        raise ValueError("sequence_parallel with context parallelism is not supported (use tp x cp without SP)")
    cfg = model.config
    for blk in model.attn_blocks:
        if pg.tp > 1:
            blk.attn = TPAttention(blk.attn, cfg, pg)
            blk.mlp = TPMLP(blk.mlp, cfg, pg)
        elif pg.cp > 1:
            blk.attn = UlyssesAttention(blk.attn, pg) if pg.cp_mode == "ulysses" else CPAttention(blk.attn, pg)
    model.parallel = pg
    return model


def sharded_params(model) -> List[nn.Parameter]:
    return [p for p in model.parameters() if getattr(p, "_pllm_tp_sharded", False)]


@torch.no_grad()
def sync_replicated_grads(optimizer, pg: ParallelGroups):
    """Sequence parallelism: replicated parameters (norms, embeddings, LM head, row-parallel
    biases) saw only this rank's tokens -- sum their gradients over the TP group."""
    if pg.tp == 1 or not pg.sequence_parallel:
        return
    # (the DP / ZeRO reduction already ran: a sum over TP commutes with it, so this works on
    # whichever buffer the optimizer step reads -- the flat gradient or the ZeRO shard)
    buf, ranges = optimizer.replicated_grad_ranges()
    views = [buf[a:b] for a, b in ranges]
    if views:
        flat = torch.cat(views)
        dist.all_reduce(flat, group=pg.tp_group)
        o = 0
        for v in views:
            v.copy_(flat[o:o + v.numel()])
            o += v.numel()


@torch.no_grad()
def gather_dense_state(model, dense_model, pg: ParallelGroups, masters: Optional[dict] = None):
    """COLLECTIVE over the TP group: assemble the dense weights of a TP-sharded ``model`` into
    ``dense_model`` (same config, built dense -- on any device, e.g. the CPU); ranks that only
    contribute their shards pass ``dense_model=None``.  ``masters`` maps local parameter -> fp32
    value to gather instead of the compute copy.  The gathers run one parameter at a time on the
    parameters' own device, so no rank holds more than one dense tensor on the GPU.  Returns
    ``dense_model``."""
    dst = dict(dense_model.named_parameters()) if dense_model is not None else None
    g = pg.tp_group

    def gather(t):
        parts = [torch.empty_like(t) for _ in range(pg.tp)]
        dist.all_gather(parts, t.contiguous(), group=g)
        return parts

    cfg = model.config
    for name, p in model.named_parameters():  # identical order on every TP rank
        v = (masters.get(id(p), p) if masters else p).to(device=p.device, dtype=torch.float32)
        if not getattr(p, "_pllm_tp_sharded", False):
            full = v
        elif name.endswith("attn.qkv.weight") or name.endswith("attn.qkv.bias"):
            H, Hkv, D = cfg.n_head, cfg.n_kv_head, cfg.head_dim
            Hl, Hkl = H // pg.tp, Hkv // pg.tp
            parts = gather(v)
            full = torch.cat([x[:Hl * D] for x in parts] + [x[Hl * D:(Hl + Hkl) * D] for x in parts] +
                             [x[(Hl + Hkl) * D:] for x in parts], 0)
        elif name.endswith("mlp.hidden.weight") or name.endswith("mlp.hidden.bias"):
            parts = gather(v)
            if cfg.mlp == "swiglu":
                Fl = cfg.ffn_hidden // pg.tp
                full = torch.cat([x[:Fl] for x in parts] + [x[Fl:] for x in parts], 0)
            else:
                full = torch.cat(parts, 0)
        elif name.endswith("proj.weight"):  # row-parallel: sharded along the input columns
            full = torch.cat(gather(v), 1)
        else:
            raise RuntimeError(f"no unsharding rule for {name}")
        if dst is not None:
            dst[name].copy_(full)
        del full
    return dense_model


def build_dense_shell(cfg, device="cpu"):
    """An uninitialised dense ``GPT`` of ``cfg`` on ``device`` (default: host memory) for a
    consolidated checkpoint: built on the meta device and materialised with ``to_empty``, so it
    draws nothing from any RNG stream (a saving rank's RNG stays in step with the others) and
    costs no GPU memory."""
    from ..models import GPT
    with torch.random.fork_rng(devices=[]):
        with torch.device("meta"):
            m = GPT(cfg)
    m = m.to_empty(device=device).float()
    if getattr(m, "pos_idxs", None) is not None:  # the one persistent buffer (reference layout)
        m.pos_idxs.copy_(torch.arange(m.pos_idxs.numel()))
    return m

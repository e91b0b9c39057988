"""Ring (context-parallel) attention over RCCL point-to-point, built on the flash kernels'
log-sum-exp merge.

The reference materialises every head's T x T score matrix on one device
(src/models/attention.py:47-57) and caps the sequence at ``context_length``
(config/config.py:5).  Here a sequence is sharded over the ranks of a
context-parallel group; every rank keeps its queries and the key/value shards travel
around the ring:

* forward: at ring step i, rank r holds the K/V of rank (r - i) mod W.  Each (query
  chunk, key chunk) pair is either fully visible, causal (the diagonal) or fully masked;
  visible pairs run the flash forward kernel and the partial outputs are merged with
  their LSEs:  lse = logaddexp(lse_a, lse_b),  o = o_a e^(lse_a-lse) + o_b e^(lse_b-lse).
* backward: the flash backward kernel is run per visible pair with the FINAL o and lse
  (so every pair's gradient is exact); dQ stays local, dK/dV accumulate in fp32
  buffers that travel one ring step behind the K/V and arrive back at their owner after W hops.
* forward and backward post the next K/V shard's send/recv before the current pair's kernels
  run, and the backward's accumulator hop is waited for only after the next step's kernels, so
  the transfers over xGMI overlap the attention compute (one peer per direction: a ring is
  exactly the per-link pattern xGMI's point-to-point links serve best).

Layouts:
* ``"contiguous"``: rank r holds positions [r T_l, (r+1) T_l).  Simple; causal work is
  unbalanced (rank W-1 does W times the work of rank 0).
* ``"zigzag"``: the sequence is cut into 2W chunks and rank r holds chunks r and
  2W-1-r, which balances causal work; ``zigzag_shard`` / ``zigzag_unshard`` convert.
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from .. import ops


def _ws(group) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def _rank(group) -> int:
    return dist.get_rank(group) if dist.is_initialized() else 0


def _global(group, r: int) -> int:
    return dist.get_global_rank(group, r) if group is not None else r


def _chunk_ids(rank: int, world: int, layout: str) -> List[int]:
    if layout == "contiguous":
        return [rank]
    if layout == "zigzag":
        return [rank, 2 * world - 1 - rank]
    raise ValueError(f"unknown context-parallel layout {layout!r}")


def _mode(qc: int, kc: int, causal: bool) -> str:
    if not causal or kc < qc:
        return "full"
    return "diag" if kc == qc else "skip"


def zigzag_shard(x: torch.Tensor, dim: int, group=None) -> torch.Tensor:
    """Full-sequence tensor -> this rank's zigzag shard (chunks r and 2W-1-r along ``dim``)."""
    W, r = _ws(group), _rank(group)
    ch = x.chunk(2 * W, dim=dim)
    return torch.cat([ch[r], ch[2 * W - 1 - r]], dim=dim)


def zigzag_unshard(x: torch.Tensor, dim: int, group=None) -> torch.Tensor:
    """All-gather zigzag shards back into the full sequence order."""
    W = _ws(group)
    if W == 1:
        return x
    parts = [torch.empty_like(x) for _ in range(W)]
    dist.all_gather(parts, x.contiguous(), group=group)
    chunks = [None] * (2 * W)
    for r, p in enumerate(parts):
        a, b = p.chunk(2, dim=dim)
        chunks[r], chunks[2 * W - 1 - r] = a, b
    return torch.cat(chunks, dim=dim)


def zigzag_positions(local_len: int, group=None, device=None) -> torch.Tensor:
    """Global token positions of this rank's zigzag shard (for position embeddings / RoPE)."""
    W, r = _ws(group), _rank(group)
    c = local_len // 2
    return torch.cat([torch.arange(r * c, (r + 1) * c), torch.arange((2 * W - 1 - r) * c, (2 * W - r) * c)]).to(device)


class _Ring:
    """Posts one send to the next rank and one receive from the previous rank."""

    def __init__(self, group):
        self.group = group
        W, r = _ws(group), _rank(group)
        self.nxt, self.prv = _global(group, (r + 1) % W), _global(group, (r - 1) % W)
        self.reqs = []

    def start(self, tensors: List[torch.Tensor]) -> List[torch.Tensor]:
        # gloo moves CPU tensors only: device blocks travel through pinned host copies there
        # (test / CPU-cluster path); on RCCL they go GPU to GPU over xGMI
        self.host = dist.get_backend(self.group) == "gloo" and tensors[0].is_cuda
        send = [t.contiguous() for t in tensors]
        if self.host:
            send = [t.cpu() for t in send]
        recv = [torch.empty_like(t) for t in send]
        p2p = []
        for t, rv in zip(send, recv):
            p2p.append(dist.P2POp(dist.isend, t, self.nxt, self.group))
            p2p.append(dist.P2POp(dist.irecv, rv, self.prv, self.group))
        self.reqs = dist.batch_isend_irecv(p2p)
        self.recv, self.dev = recv, tensors[0].device
        return recv

    def wait(self):
        for q in self.reqs:
            q.wait()
        self.reqs = []
        if self.host:
            # hand back device tensors in place of the host buffers start() returned
            for i, t in enumerate(self.recv):
                self.recv[i] = t.to(self.dev, non_blocking=False)
        return self.recv


def _split(x: torch.Tensor, n: int) -> List[torch.Tensor]:
    return list(x.chunk(n, dim=1)) if n > 1 else [x]


def _merge(o_acc, lse_acc, o, lse):
    """In-place LSE merge of a partial block result (o [B,T,H,D], lse [B,H,T]) into fp32 accumulators
    (the HIP path: one fused kernel, csrc/elementwise.hip lse_merge_kernel)."""
    from .. import ops
    if (ops._hip(o) and o.dtype == torch.bfloat16 and o.shape[-1] % 8 == 0 and o.shape[-1] <= 128
            and 64 % (o.shape[-1] // 8) == 0 and o.stride(-1) == 1 and o_acc.stride(-1) == 1):
        ops._ops().lse_merge_(o_acc, lse_acc, o, lse.float())
        return
    lse = lse.float()
    new = torch.logaddexp(lse_acc, lse)
    a = torch.exp(lse_acc - new).nan_to_num_(0.0).transpose(1, 2).unsqueeze(-1)
    b = torch.exp(lse - new).nan_to_num_(0.0).transpose(1, 2).unsqueeze(-1)
    o_acc.mul_(a).add_(o.float() * b)
    lse_acc.copy_(new)


class _RingAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, group, causal, scale, layout):
        W, r = _ws(group), _rank(group)
        qids = _chunk_ids(r, W, layout)
        nq = len(qids)
        B, T, H, D = q.shape
        o_acc = torch.zeros(B, T, H, D, dtype=torch.float32, device=q.device)
        lse_acc = torch.full((B, H, T), float("-inf"), dtype=torch.float32, device=q.device)
        o_parts, lse_parts = _split(o_acc, nq), list(lse_acc.chunk(nq, dim=2)) if nq > 1 else [lse_acc]
        ring = _Ring(group)
        kv = (k.contiguous(), v.contiguous())
        for step in range(W):
            src = (r - step) % W
            nxt = ring.start(list(kv)) if step + 1 < W else None
            kids = _chunk_ids(src, W, layout)
            ks, vs = _split(kv[0], len(kids)), _split(kv[1], len(kids))
            for qi, qc in enumerate(qids):
                qq = _split(q, nq)[qi]
                for ki, kc in enumerate(kids):
                    m = _mode(qc, kc, causal)
                    if m == "skip":
                        continue
                    o, lse = ops.attention(qq, ks[ki], vs[ki], causal=(m == "diag"), scale=scale, return_lse=True)
                    _merge(o_parts[qi], lse_parts[qi], o, lse)
            if nxt is not None:
                ring.wait()
                kv = tuple(nxt)
        out = o_acc.to(q.dtype)
        ctx.save_for_backward(q, k, v, out, lse_acc)
        ctx.cfg = (group, causal, scale, layout)
        return out

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        group, causal, scale, layout = ctx.cfg
        W, r = _ws(group), _rank(group)
        qids = _chunk_ids(r, W, layout)
        nq = len(qids)
        do = do.contiguous()
        dq = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
        dq_parts = _split(dq, nq)
        qs, dos, os_ = _split(q, nq), _split(do, nq), _split(o, nq)
        lses = [t.contiguous() for t in lse.chunk(nq, dim=2)] if nq > 1 else [lse]
        # Two rings.  K/V (read-only) hop before the pair kernels, as in the forward.  The fp32
        # dK/dV accumulators of the visiting block travel ONE STEP BEHIND: each step's kernels
        # add into fresh local buffers, and only after them does the rank wait for the
        # accumulator the previous rank sent (one add), then pass the sum on.  So neither
        # transfer sits between two steps' kernels: the K/V hop overlaps this step's compute and
        # the accumulator hop overlaps the next step's.  After W hops every accumulator is back
        # at its owner.
        kv = [k.contiguous(), v.contiguous()]
        kv_ring, acc_ring = _Ring(group), _Ring(group)
        acc_in = False
        for step in range(W):
            src = (r - step) % W
            nxt = kv_ring.start(kv) if step + 1 < W else None
            kids = _chunk_ids(src, W, layout)
            ks, vs = _split(kv[0], len(kids)), _split(kv[1], len(kids))
            dk = torch.zeros(k.shape, dtype=torch.float32, device=k.device)
            dv = torch.zeros(v.shape, dtype=torch.float32, device=v.device)
            dks, dvs = _split(dk, len(kids)), _split(dv, len(kids))
            for qi, qc in enumerate(qids):
                for ki, kc in enumerate(kids):
                    m = _mode(qc, kc, causal)
                    if m == "skip":
                        continue
                    gq, gk, gv = ops.attention_block_bwd(dos[qi], qs[qi], ks[ki], vs[ki], os_[qi], lses[qi],
                                                         causal=(m == "diag"), scale=scale)
                    dq_parts[qi].add_(gq.float())
                    dks[ki].add_(gk.float())
                    dvs[ki].add_(gv.float())
            if acc_in:  # the accumulator of this K/V block from the ranks it visited before
                pdk, pdv = acc_ring.wait()
                dk.add_(pdk)
                dv.add_(pdv)
            if W > 1:
                acc_ring.start([dk, dv])
                acc_in = True
            if nxt is not None:
                kv = kv_ring.wait()
        if W > 1:
            dk, dv = acc_ring.wait()  # this rank's own K/V gradient, summed over every rank
        return dq.to(q.dtype), dk.to(k.dtype), dv.to(v.dtype), None, None, None, None


def ring_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, group=None, causal: bool = True,
                   scale: Optional[float] = None, layout: str = "zigzag") -> torch.Tensor:
    """Context-parallel attention over the ranks of ``group``.

    q [B, T_l, H, D], k/v [B, T_l, Hkv, D] are this rank's shards of the sequence in the
    given ``layout`` (``zigzag``: T_l must be even).  Returns this rank's output shard."""
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if _ws(group) == 1 and layout == "zigzag":
        layout = "contiguous"  # one rank: the zigzag shard IS the whole sequence in order
    return _RingAttnFn.apply(q, k, v, group, causal, scale, layout)

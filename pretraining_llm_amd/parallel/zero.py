"""ZeRO-1: optimizer-state sharding on top of the flat parameter/gradient buffers.

Reference: ``torch.optim.AdamW`` state fully replicated on every DDP rank
(scripts/train_transformer.py:122-126; SURVEY.md §2.5 "FSDP / ZeRO: No").

With 288 GB of HBM per MI355X, replicated fp32 master weights + moments (12 B/param) fit
comfortably up to several billion parameters, so this is an option, not the default:
it pays off when the optimizer state would crowd out activations (multi-B models at long
sequence lengths) and it cuts the per-rank AdamW pass to 1/world.

Layout (MI355X-first, built for RCCL over point-to-point xGMI):
* the flat gradient buffer is cut into fixed-size buckets from its END (backward produces
  the last layers' gradients first) -- a small first bucket, then ``bucket_mb`` ones --
  every bucket a multiple of ``world * 64`` elements, so each splits into ``world`` equal,
  64-element-aligned parts and rank r owns part r of EVERY bucket.  Every rank therefore
  owns 1/world of every bucket (balanced ring traffic on every xGMI link) and the
  ownership is independent of parameter boundaries;
* backward: a bucket is reduce-scattered (RCCL, async, strictly in bucket order) as soon
  as all parameters overlapping it have their gradients -- the same readiness machinery
  as the all-reduce engine (``p._pllm_grad_ready`` from in-place kernels, post-accumulate
  hooks otherwise).  A reduce-scatter moves half the bytes of an all-reduce;
* step: per bucket, the fused AdamW kernel updates the owned part (fp32 master/moments
  exist only for owned parts: 12 B/param / world) and writes the bf16 weights, then an
  async all-gather of that bucket's bf16 weights is issued, so bucket b's all-gather
  runs under bucket b+1's AdamW; the compute stream waits on all of them (no host sync);
* gradient clipping: sum of squares of the owned reduced gradients, one scalar
  all-reduce, device-side clip coefficient;
* ``state_dict`` is COLLECTIVE: the shards are all-gathered one bucket at a time into host
  memory of the writing rank, so the checkpoint keeps FlatAdamW's (torch.optim.AdamW-shaped)
  single-file format without any rank materialising the full state on its GPU;
  ``load_state_dict`` copies each rank's owned parts straight out of the full file.
"""
from __future__ import annotations

import contextlib
from typing import List, Optional

import torch
import torch.distributed as dist

from .. import ops as _ops_mod
from ..ops import _lib
from ..train.optim import ALIGN, FlatAdamW, _round_up


def _world_rank(group):
    if dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


class ShardedFlatAdamW(FlatAdamW):
    """FlatAdamW whose fp32 master weights and moments are sharded over a process group."""

    collective_state = True  # state_dict / load_state_dict must be called on every rank

    def __init__(self, model, lr: float = 5e-4, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.01,
                 decay_filter=None, max_grad_norm: float = 0.0, process_group=None, bucket_mb: float = 64.0,
                 first_bucket_mb: float = 4.0, transposed_shadow: Optional[bool] = None):
        self.pg = process_group
        self.world, self.rank = _world_rank(process_group)
        unit = self.world * ALIGN
        # lazy gradient zeroing off: the reduce-scattered buckets are read by this class's own step
        super().__init__(model, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, decay_filter=decay_filter,
                         max_grad_norm=max_grad_norm, transposed_shadow=transposed_shadow, pad_multiple=unit,
                         lazy_zero=False)
        esz = self.flat_grad.element_size()
        # buckets from the end of the buffer, each a multiple of world*ALIGN elements
        buckets = []
        end = self.total
        cap = max(unit, _round_up(int(first_bucket_mb * 2 ** 20) // esz, unit))
        while end > 0:
            start = max(0, end - cap)
            buckets.append((start, end))
            end = start
            cap = max(unit, _round_up(int(bucket_mb * 2 ** 20) // esz, unit))
        self.buckets = buckets                       # launch order (last layers first)
        self.own = []                                # (flat_start, flat_end, shard_offset) per bucket
        so = 0
        for bs, be in buckets:
            part = (be - bs) // self.world
            self.own.append((bs + self.rank * part, bs + (self.rank + 1) * part, so))
            so += part
        self.shard_numel = so
        # replace the replicated fp32 state by the owned slices
        full_master = self.master
        self.master = torch.empty(so, dtype=torch.float32, device=full_master.device)
        for fs, fe, o in self.own:
            self.master[o:o + fe - fs].copy_(full_master[fs:fe])
        del full_master
        self.exp_avg = torch.zeros(so, dtype=torch.float32, device=self.master.device)
        self.exp_avg_sq = torch.zeros(so, dtype=torch.float32, device=self.master.device)
        # reduced (summed) owned gradient parts land here
        self.grad_shard = torch.zeros(so, dtype=self.grad_dtype, device=self.master.device)
        self._inplace_ag = dist.is_initialized() and dist.get_backend(process_group) == "nccl"

    # ------------------------------------------------------------------
    def replicated_grad_ranges(self):
        """The TP-replicated parameters' owned slices, in ``grad_shard`` coordinates."""
        ranges = [(o + max(a, fs) - fs, o + min(b, fe) - fs) for fs, fe, o in self.own
                  for a, b in self._rep_ranges if max(a, fs) < min(b, fe)]
        return self.grad_shard, ranges

    def grad_norm(self, grad_scale: float = 1.0) -> torch.Tensor:
        ss = self._sumsq(self.grad_shard)
        if getattr(self, "tp", 1) > 1:
            ss = self._tp_adjust(ss)
        if self.world > 1:
            dist.all_reduce(ss, op=dist.ReduceOp.SUM, group=self.pg)
        if getattr(self, "tp", 1) > 1:
            dist.all_reduce(ss, op=dist.ReduceOp.SUM, group=self.tp_group)
        return ss[0].sqrt() * grad_scale

    def _update_part(self, fs, fe, o, grad_scale, clip):
        n = fe - fs
        b1, b2 = self.betas
        p, mst = self.flat_param[fs:fe], self.master[o:o + n]
        m, v, g = self.exp_avg[o:o + n], self.exp_avg_sq[o:o + n], self.grad_shard[o:o + n]
        if self.use_hip and _ops_mod.get_backend() == "auto":
            wm = None if self.wd_mask is None else self.wd_mask[fs // ALIGN:fe // ALIGN]
            _lib.require().adamw_(p, mst, m, v, g, self.lr, b1, b2, self.eps, self.weight_decay, self.step_count,
                                  grad_scale, clip, wm, None)
            return
        g32 = g.float() * grad_scale
        if clip is not None:
            g32 = g32 * clip
        wd = self.weight_decay
        if not self.all_decay:
            mst.mul_(torch.where(self.wd_elem_mask[fs:fe], 1.0 - self.lr * wd, 1.0))
            wd = 0.0
        _ops_mod.ref.adamw_(p, g32, m, v, self.lr, b1, b2, self.eps, wd, self.step_count, master=mst)

    def step(self, grad_scale: float = 1.0, graph: bool = False):
        if graph:
            raise RuntimeError("ShardedFlatAdamW: graph-captured steps are not supported (collectives in the step)")
        self.wait_params()  # a previous step's gathers not yet consumed (e.g. no forward in between)
        self._sync_lr()
        self.step_count += 1
        clip = None
        if self.max_grad_norm and self.max_grad_norm > 0:
            norm = self.grad_norm(grad_scale)
            self.last_grad_norm = norm
            clip = torch.clamp(self.max_grad_norm / (norm + 1e-6), max=1.0).to(torch.float32).reshape(1)
        # buckets in FORWARD order (start of the buffer = embeddings and first blocks first): the
        # next forward needs them in that order, so the first gathers issued are the first waited
        # for, and the later ones keep running under the first blocks' forward
        self._gathers = {}
        for b in reversed(range(len(self.buckets))):
            bs, be = self.buckets[b]
            fs, fe, o = self.own[b]
            self._update_part(fs, fe, o, grad_scale, clip)
            if self.world > 1:
                src = self.flat_param[fs:fe] if self._inplace_ag else self.flat_param[fs:fe].clone()
                self._gathers[b] = dist.all_gather_into_tensor(self.flat_param[bs:be], src, group=self.pg,
                                                               async_op=True)
        self._shadows_stale = True
        if not self.lazy_gather:
            self.wait_params()

    # ------------------------------------------------------------------ lazy parameter all-gather
    lazy_gather = False  # set by install_lazy_gather

    def wait_params(self, params=None):
        """Make the compute stream wait for the all-gathers of the buckets holding ``params``
        (every pending bucket when None; then also refresh the transposed weight shadows, which
        read every parameter).  A wait on RCCL is a stream dependency, not a host block."""
        pend = getattr(self, "_gathers", None) or {}
        if params is None:
            for b in list(pend):
                pend.pop(b).wait()
            if getattr(self, "_shadows_stale", False):
                self._shadows_stale = False
                self.refresh_shadows()
            return
        for b in self._buckets_of(params):
            h = pend.pop(b, None)
            if h is not None:
                h.wait()

    def _buckets_of(self, params):
        key = tuple(id(p) for p in params)
        cache = self.__dict__.setdefault("_bucket_cache", {})
        if key not in cache:
            idx = {id(p): i for i, p in enumerate(self.params)}
            out = set()
            for p in params:
                i = idx.get(id(p))
                if i is None:
                    continue
                a, e = self.offsets[i], self.offsets[i] + p.numel()
                out.update(b for b, (bs, be) in enumerate(self.buckets) if bs < e and be > a)
            cache[key] = sorted(out, reverse=True)  # forward order
        return cache[key]

    def install_lazy_gather(self, model):
        """Wait for each bucket's parameter all-gather right before its first use in the next
        forward instead of at the end of ``step()``: forward pre-hooks on the model (embeddings)
        and on every transformer block and the final norm wait for the buckets holding their
        parameters; a forward hook on the model waits for the rest (LM head, tied embedding) and
        refreshes the weight shadows before any backward.  Returns the hook handles."""
        if not (hasattr(model, "token_embed") and hasattr(model, "attn_blocks")):
            return []  # not a GPT: keep the blanket wait in step()
        self.lazy_gather = True
        hooks = []
        first = [p for m in (model.token_embed, getattr(model, "position_embed", None)) if m is not None
                 for p in m.parameters()]
        hooks.append(model.register_forward_pre_hook(lambda _m, _a: self.wait_params(first)))
        head = [p for p in (getattr(model, "head_weight", None), getattr(model, "head_bias", None)) if p is not None]
        final_norm = getattr(model, "layer_norm", None)
        for blk in list(getattr(model, "attn_blocks", [])) + [final_norm]:
            if blk is None:
                continue
            ps = list(blk.parameters())
            if blk is final_norm:
                # the LM head (+ fused CE, which also produces the head's gradient) runs INSIDE
                # GPT.forward right after the final norm, before the model's forward hook fires:
                # its buckets (the buffer's tail, gathered last) must be waited for here
                ps = ps + head
            hooks.append(blk.register_forward_pre_hook(lambda _m, _a, ps=ps: self.wait_params(ps)))
        if final_norm is None and head:
            hooks.append(model.register_forward_pre_hook(lambda _m, _a: self.wait_params(head)))
        hooks.append(model.register_forward_hook(lambda _m, _a, _o: self.wait_params()))
        return hooks

    # ------------------------------------------------------------------
    def _gather_full_cpu(self, shard: torch.Tensor, keep: bool) -> Optional[torch.Tensor]:
        """All-gather a sharded fp32 state vector ONE BUCKET AT A TIME through a bucket-sized
        device buffer into host memory (only on the rank that keeps it): no rank ever holds the
        full unsharded state on its GPU, which is what ZeRO-1 exists to avoid."""
        full = torch.zeros(self.total, dtype=shard.dtype) if keep else None
        for (bs, be), (fs, fe, o) in zip(self.buckets, self.own):
            n = fe - fs
            if self.world > 1:
                tmp = torch.empty(be - bs, dtype=shard.dtype, device=shard.device)
                dist.all_gather_into_tensor(tmp, shard[o:o + n].contiguous(), group=self.pg)
            else:
                tmp = shard[o:o + n]
            if keep:
                full[bs:be].copy_(tmp)
        return full

    def state_dict(self, writer_rank: int = 0) -> dict:
        """COLLECTIVE: every rank must call it.  Returns the full (unsharded) AdamW-format state
        on ``writer_rank`` (in host memory) and ``{}`` elsewhere."""
        self.wait_params()
        keep = self.rank == writer_rank
        full = [self._gather_full_cpu(t, keep) for t in (self.master, self.exp_avg, self.exp_avg_sq)]
        if not keep:
            return {}
        saved = (self.master, self.exp_avg, self.exp_avg_sq)
        self.master, self.exp_avg, self.exp_avg_sq = full
        try:
            return super().state_dict()
        finally:
            self.master, self.exp_avg, self.exp_avg_sq = saved

    @torch.no_grad()
    def load_state_dict(self, sd: dict):
        """Every rank reads the same full state and copies only the parts it owns (no collective,
        no unsharded device copy)."""
        self.wait_params()
        st = sd["state"]
        steps = []
        for i, p in enumerate(self.params):
            if i not in st and str(i) not in st:
                continue
            e = st[i] if i in st else st[str(i)]
            o, n = self.offsets[i], p.numel()
            src = {k: e[k].reshape(-1).to(self.master.device, torch.float32)
                   for k in ("exp_avg", "exp_avg_sq", "master") if k in e}
            if "master" not in src:
                src["master"] = self.flat_param[o:o + n].float()
            for fs, fe, so in self.own:
                lo, hi = max(o, fs), min(o + n, fe)
                if lo >= hi:
                    continue
                for name, dst in (("master", self.master), ("exp_avg", self.exp_avg),
                                  ("exp_avg_sq", self.exp_avg_sq)):
                    dst[so + lo - fs:so + hi - fs].copy_(src[name][lo - o:hi - o])
            self.flat_param[o:o + n].copy_(src["master"].to(self.flat_param.dtype))
            steps.append(float(e["step"]))
        if steps:
            self.step_count = int(max(steps))
        if sd.get("param_groups"):
            self.param_groups[0]["lr"] = sd["param_groups"][0].get("lr", self.lr)
            self._sync_lr()
        self.refresh_shadows()

    @torch.no_grad()
    def sync_master_from_params(self):
        self.wait_params()
        for fs, fe, o in self.own:
            self.master[o:o + fe - fs].copy_(self.flat_param[fs:fe].float())
        self.refresh_shadows()


class ZeroDataParallelEngine:
    """Gradient reduce-scatter engine for ``ShardedFlatAdamW`` (same surface as
    ``DataParallelEngine``: ``no_sync()``, ``finish_grad_sync() -> grad scale``)."""

    def __init__(self, optimizer: ShardedFlatAdamW, broadcast_params: bool = True, overlap: bool = True,
                 timing: bool = False, lazy_gather: bool = True):
        from .dp import CommTimer
        self.timer = CommTimer(timing and optimizer.flat_grad.is_cuda)
        if lazy_gather:
            self.hooks_lazy = optimizer.install_lazy_gather(optimizer.model)
        self.opt = optimizer
        self.pg = optimizer.pg
        self.world = optimizer.world
        self.enabled = True
        self._handles = []
        self._hooks = []
        opt = optimizer
        params = opt.params
        # parameters overlapping each bucket
        self.bucket_params: List[List[int]] = []
        self.param_buckets: List[List[int]] = [[] for _ in params]
        for b, (bs, be) in enumerate(opt.buckets):
            ids = [i for i, p in enumerate(params) if opt.offsets[i] < be and opt.offsets[i] + p.numel() > bs]
            self.bucket_params.append(ids)
            for i in ids:
                self.param_buckets[i].append(b)
        self._expected: Optional[List[int]] = None
        self._events = [0] * len(params)
        self._reset_counters()
        if broadcast_params and self.world > 1:
            src = dist.get_global_rank(self.pg, 0) if self.pg is not None else 0
            dist.broadcast(opt.flat_param, src=src, group=self.pg)
            opt.sync_master_from_params()
        if self.world > 1 and overlap:
            for i, p in enumerate(params):
                h = self._make_hook(i)
                self._hooks.append(p.register_post_accumulate_grad_hook(lambda _p, h=h: h()))
                p._pllm_grad_ready = h

    def _reset_counters(self):
        if self._expected is None:
            self._pending = [len(ids) for ids in self.bucket_params]
        else:
            self._pending = [sum(1 for i in ids if self._expected[i] > 0) for ids in self.bucket_params]
        self._events = [0] * len(self._events)
        self._next_launch = 0
        self._handles = []

    def _make_hook(self, i):
        def hook():
            if not self.enabled:
                return
            self._events[i] += 1
            if self._expected is None or self._events[i] != self._expected[i]:
                return
            for b in self.param_buckets[i]:
                self._pending[b] -= 1
            self._launch_ready()
        return hook

    def _launch(self, b):
        opt = self.opt
        bs, be = opt.buckets[b]
        fs, fe, o = opt.own[b]
        out = opt.grad_shard[o:o + fe - fs]
        self.timer.launch(b)
        self._handles.append(dist.reduce_scatter_tensor(out, opt.flat_grad[bs:be], op=dist.ReduceOp.SUM,
                                                        group=self.pg, async_op=True))

    def _launch_ready(self):
        while self._next_launch < len(self.opt.buckets) and self._pending[self._next_launch] <= 0:
            self._launch(self._next_launch)
            self._next_launch += 1

    @contextlib.contextmanager
    def no_sync(self):
        old = self.enabled
        self.enabled = False
        try:
            yield
        finally:
            self.enabled = old

    def finish_grad_sync(self):
        self.timer.backward_end()
        opt = self.opt
        if self.world > 1:
            while self._next_launch < len(opt.buckets):
                self._launch(self._next_launch)
                self._next_launch += 1
            for h in self._handles:
                h.wait()
            if self._expected is None and self.enabled and any(self._events):
                self._expected = list(self._events)
        else:
            for fs, fe, o in opt.own:
                opt.grad_shard[o:o + fe - fs].copy_(opt.flat_grad[fs:fe])
        self.timer.sync_end()
        self._reset_counters()
        return 1.0 / self.world

    def bucket_sizes_mb(self):
        esz = self.opt.flat_grad.element_size()
        return [(be - bs) * esz / 2 ** 20 for bs, be in self.opt.buckets]

    def remove_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []

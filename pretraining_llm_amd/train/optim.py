"""Flat-buffer mixed-precision AdamW.

Reference: ``torch.optim.AdamW(model.parameters(), lr=t_lr)`` with fp32
params under bf16 autocast (scripts/train_transformer.py:66,126): every forward
casts every weight to bf16 and the optimizer runs ~5 foreach kernels over each
of thousands of tensors.

MI355X-first layout instead:
* all parameters live in ONE contiguous buffer in the compute dtype (bf16 on
  the GPU); each ``nn.Parameter`` becomes a view into it, every segment 16-byte
  aligned;
* all gradients live in ONE contiguous buffer, fp32 by default (``grad_dtype``),
  so the data-parallel engine reduces contiguous buckets with no packing copies and
  zero_grad is one memset.  Like the reference (fp32 params under bf16 autocast ->
  fp32 ``.grad``, fp32 DDP all-reduce: scripts/train_transformer.py:66-69,122-126),
  micro-step accumulation, the tied embedding's two gradient pieces and the DP sum
  are all kept in fp32.  The backward kernels add straight into that buffer
  (``p._pllm_gradbuf``, see ops._acc_target); where grad and param dtypes agree it is
  also ``p.grad``, otherwise (bf16 params, fp32 grads -- torch forbids a ``.grad``
  of another dtype) any gradient autograd still produces is folded into the buffer
  by a post-accumulate hook and released;
* fp32 master weights and the two moments are flat fp32 buffers; one HIP
  kernel per param group (``torch.ops.pllm.adamw_``) reads the gradient,
  updates master/m/v and writes the bf16 compute weights in the same pass;
* gradient clipping uses one fused sum-of-squares reduction and a device-side
  clip coefficient (no host sync).

``state_dict()`` follows ``torch.optim.AdamW``'s format (``state[i]`` with
``step``/``exp_avg``/``exp_avg_sq`` per parameter index, ``param_groups`` with
the usual keys) plus an fp32 ``master`` entry per parameter for exact resume.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch
import torch.nn as nn

from .. import ops as _ops_mod
from ..ops import _lib
from ..ab import ab as _ab

ALIGN = 64  # elements; keeps every segment 16 B aligned for bf16 and fp32


def _round_up(n: int, a: int) -> int:
    return (n + a - 1) // a * a


class FlatAdamW:
    def __init__(self, model: nn.Module, lr: float = 5e-4, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.01, decay_filter=None, grad_dtype: Optional[torch.dtype] = None,
                 max_grad_norm: float = 0.0, transposed_shadow: Optional[bool] = None, pad_multiple: int = ALIGN,
                 lazy_zero: Optional[bool] = None):
        self.model = model
        self.lr = lr
        self.betas = betas
        self.eps = eps
        self.weight_decay = weight_decay
        self.max_grad_norm = max_grad_norm
        self.step_count = 0
        # unique params in registration order (tied weights appear once)
        params: List[nn.Parameter] = []
        names: List[str] = []
        seen = set()
        for n, p in model.named_parameters():
            if id(p) in seen or not p.requires_grad:
                continue
            seen.add(id(p))
            params.append(p)
            names.append(n)
        self.params, self.names = params, names
        decay = [True] * len(params)
        if decay_filter is not None:
            decay = [bool(decay_filter(n, p)) for n, p in zip(names, params)]
        # layout: registration order (backward produces gradients roughly in reverse of it,
        # which is what the DP engine's bucketing relies on); each segment 64-element aligned.
        # Weight decay is selected per 64-element block by a byte mask, so ONE launch covers
        # every parameter whatever its group.
        self.offsets: Dict[int, int] = {}
        off = 0
        for i, p in enumerate(params):
            self.offsets[i] = off
            off += _round_up(p.numel(), ALIGN)
        total = _round_up(off, pad_multiple)  # ZeRO pads to world * ALIGN (parallel/zero.py)
        self.decay = decay
        self.total = total
        dev = params[0].device
        pdtype = params[0].dtype
        self.param_dtype = pdtype
        self.grad_dtype = grad_dtype or torch.float32
        self.flat_param = torch.zeros(total, dtype=pdtype, device=dev)
        self.flat_grad = torch.zeros(total, dtype=self.grad_dtype, device=dev)
        self.grad_is_param_grad = self.grad_dtype == pdtype
        self._fold_hooks = []
        for i, p in enumerate(params):
            o = self.offsets[i]
            seg = self.flat_param[o:o + p.numel()].view_as(p)
            seg.copy_(p.data)
            p.data = seg
            p._pllm_gradbuf = self.flat_grad[o:o + p.numel()].view_as(p)
            p._pllm_flat_grad = True  # backward kernels add straight into p._pllm_gradbuf (ops._acc_target)
            if self.grad_is_param_grad:
                p.grad = p._pllm_gradbuf
            else:
                p.grad = None
                self._fold_hooks.append(p.register_post_accumulate_grad_hook(_fold_grad))
        self.master = self.flat_param.float() if pdtype != torch.float32 else self.flat_param.clone()
        self.exp_avg = torch.zeros(total, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(total, dtype=torch.float32, device=dev)
        self.use_hip = dev.type == "cuda" and pdtype == torch.bfloat16
        mask = torch.zeros(total // ALIGN, dtype=torch.uint8)
        elem_mask = torch.zeros(total, dtype=torch.bool)
        for i, p in enumerate(params):
            if decay[i]:
                o = self.offsets[i]
                mask[o // ALIGN:(o + _round_up(p.numel(), ALIGN)) // ALIGN] = 1
                elem_mask[o:o + p.numel()] = True
        self.all_decay = all(decay)
        self.wd_mask = None if self.all_decay else mask.to(dev)
        self.wd_elem_mask = None if self.all_decay else elem_mask.to(dev)
        self.last_grad_norm: Optional[torch.Tensor] = None
        # torch.optim-like surface for LR schedulers / logging
        self.param_groups = [{"lr": lr, "betas": betas, "eps": eps, "weight_decay": weight_decay}]
        # transposed bf16 shadows of the 2-D weights, rewritten after every step: the backward
        # data-gradient GEMMs read W^T contiguously (ops._dgrad), the layout hipBLASLt serves
        # faster.  One extra bf16 copy of the matrices (~250 MB for GPT-2 small).
        if transposed_shadow is None:
            transposed_shadow = self.use_hip and _ab("wt_shadow", True)
        self.shadowed = [p for p in params if transposed_shadow and p.dim() == 2
                         and not getattr(p, "_pllm_no_shadow", False)]
        sh_off, o = [], 0
        for p in self.shadowed:
            sh_off.append(o)
            o += _round_up(p.numel(), ALIGN)
        self.flat_shadow = torch.empty(o, dtype=pdtype, device=dev) if self.shadowed else None
        for p, so in zip(self.shadowed, sh_off):
            p._pllm_wT = self.flat_shadow[so:so + p.numel()].view(p.shape[1], p.shape[0])
        # one batched-transpose launch refreshes every shadow (csrc/transpose.hip) when all
        # dims are multiples of 8; otherwise per-matrix torch copies
        self._tp_desc, self._tp_tiles = None, 0
        if self.shadowed and self.use_hip and all(p.shape[0] % 8 == 0 and p.shape[1] % 8 == 0
                                                  for p in self.shadowed):
            self._tp_desc = _lib.require().transpose_plan([p.data for p in self.shadowed],
                                                          [p._pllm_wT for p in self.shadowed])
            self._tp_tiles = sum(((p.shape[0] + 63) // 64) * ((p.shape[1] + 63) // 64) for p in self.shadowed)
        self.refresh_shadows()
        # Lazy zeroing (HIP path): zero_grad clears only the slots that accumulating writers fill (norms,
        # biases, embedding tables) in one launch, and marks the weight-GEMM slots "fresh": their first
        # writer of the step -- the weight-gradient GEMM, which produces the whole gradient at once --
        # stores instead of adding (ops._set_target), so those slots are never zero-filled nor read back
        # as zeros.  Any other writer zeroes a fresh slot before adding (ops._acc_target); a slot no
        # writer touched is zeroed before the step reads it (_clear_unwritten).
        if lazy_zero is None:
            lazy_zero = _ab("lazy_zero", True)
        # (fp32 gradients of bf16 params only: with grad dtype == param dtype autograd may accumulate
        # into p.grad, which aliases the slot)
        self.lazy_zero = bool(lazy_zero) and self.use_hip and not self.grad_is_param_grad
        self._fresh_params = [p for p in params if p.dim() == 2 and not getattr(p, "_pllm_no_shadow", False)]
        if self.lazy_zero:
            runs = accumulate_only_runs(params, self.offsets, total, {id(p) for p in self._fresh_params})
            self._zero_runs = torch.tensor(runs if runs else [[0, 0]], dtype=torch.int64, device=dev)
            self._zero_len = sum(b - a for a, b in runs)
            # the buffer starts zeroed, so the first step may store too -- and must: a step captured
            # into a hipGraph before any zero_grad would otherwise bake the accumulating form, and its
            # replays would add onto the slots the partial zero_grad leaves alone
            for p in self._fresh_params:
                p._pllm_grad_fresh = True

    def _clear_unwritten(self, idx=None):
        """Fresh slots no writer touched this step (an unused weight) hold last step's gradient: zero them.
        ``idx``: only these parameter indices (a DP bucket about to be all-reduced: a stale slot must be
        zeroed BEFORE it enters the sum, or a weight unused on some ranks only would add last step's
        gradient into every replica -- parallel/dp.py DataParallel._launch)."""
        if self.lazy_zero:
            params = self._fresh_params if idx is None else [self.params[i] for i in idx]
            for p in params:
                if getattr(p, "_pllm_grad_fresh", False):
                    p._pllm_grad_fresh = False
                    p._pllm_gradbuf.zero_()

    @torch.no_grad()
    def refresh_shadows(self):
        if not self.shadowed:
            return
        if self._tp_desc is not None:
            _lib.require().transpose_run(self._tp_desc, self._tp_tiles)
        else:
            for p in self.shadowed:
                p._pllm_wT.copy_(p.t())
        for p in self.shadowed:
            p._pllm_wT_ver = p._version

    # ------------------------------------------------------------------
    def grad_view(self, i: int) -> torch.Tensor:
        o = self.offsets[i]
        return self.flat_grad[o:o + self.params[i].numel()]

    def zero_grad(self, set_to_none: bool = False):
        # set_to_none is ignored on purpose: grads are views into the flat buffer
        if self.lazy_zero:
            _lib.require().zero_ranges_(self.flat_grad, self._zero_runs, self._zero_len)
            for p in self._fresh_params:
                p._pllm_grad_fresh = True
        else:
            self.flat_grad.zero_()
        for i, p in enumerate(self.params):
            if self.grad_is_param_grad:
                if p.grad is None or p.grad.data_ptr() != self.grad_view(i).data_ptr():
                    p.grad = self.grad_view(i).view_as(p)
            else:
                p.grad = None

    def _sync_lr(self):
        self.lr = self.param_groups[0]["lr"]

    def _sumsq(self, buf: torch.Tensor) -> torch.Tensor:
        if self.use_hip and _ops_mod.get_backend() == "auto":
            return _lib.require().sumsq(buf).reshape(1).float()
        return buf.float().pow(2).sum().reshape(1)

    def set_tensor_parallel(self, group, tp: int):
        """Tensor parallelism (parallel/model_parallel.py): the global gradient norm sums the
        sharded parameters over the TP group and counts the replicated ones (norms, embeddings,
        LM head, row-parallel biases -- identical on every TP rank) once."""
        self.tp_group, self.tp = group, tp
        # replicated segments rounded up to ALIGN (the padding of the flat gradient is always
        # zero) and merged where adjacent: every range starts and ends on a 64-element boundary
        # (the HIP sum of squares needs numel % 8 == 0) and there are few of them
        runs = []
        for i, p in enumerate(self.params):
            if getattr(p, "_pllm_tp_sharded", False):
                continue
            a, b = self.offsets[i], self.offsets[i] + _round_up(p.numel(), ALIGN)
            if runs and runs[-1][1] == a:
                runs[-1][1] = b
            else:
                runs.append([a, b])
        self._rep_ranges = [(a, b) for a, b in runs]

    def replicated_grad_ranges(self):
        """(buffer the optimizer step reads, [(start, end)] of the TP-replicated parameters in it)."""
        return self.flat_grad, self._rep_ranges

    def _tp_adjust(self, ss: torch.Tensor) -> torch.Tensor:
        """ss (this rank's local sum of squares of its gradient buffer) -> this rank's share of the
        global one: replicated ranges weighted 1/tp, so a SUM over the TP group counts them once."""
        buf, ranges = self.replicated_grad_ranges()
        if ranges:
            # one reduction per contiguous run, no concatenated copy of the replicated gradients
            rep = torch.stack([self._sumsq(buf[a:b]) for a, b in ranges]).sum(0)
            ss = ss - rep * (1.0 - 1.0 / self.tp)
        return ss

    def grad_norm(self, grad_scale: float = 1.0) -> torch.Tensor:
        self._clear_unwritten()
        ss = self._sumsq(self.flat_grad)
        if getattr(self, "tp", 1) > 1:
            import torch.distributed as dist
            ss = self._tp_adjust(ss)
            dist.all_reduce(ss, op=dist.ReduceOp.SUM, group=self.tp_group)
        return ss[0].sqrt() * grad_scale

    @torch.no_grad()
    def prepare_graph_step(self, lr: float):
        """Host half of a graph-captured step: advance the step counter and write
        [lr, 1/bc1, 1/sqrt(bc2)] into the device buffer the captured AdamW launch reads."""
        self.param_groups[0]["lr"] = lr
        self._sync_lr()
        self.step_count += 1
        b1, b2 = self.betas
        bc1 = 1.0 - b1 ** self.step_count
        bc2 = 1.0 - b2 ** self.step_count
        if getattr(self, "hyper", None) is None:
            self.hyper = torch.zeros(4, dtype=torch.float32, device=self.flat_param.device)
            # a ring of pinned staging buffers, each guarded by the event of the H2D copy that
            # last read it: the host may run several steps ahead of the GPU (graph replays are
            # asynchronous) and must never overwrite a buffer whose copy is still queued
            self._hyper_ring = [torch.zeros(4, dtype=torch.float32).pin_memory() for _ in range(4)]
            self._hyper_ev = [None] * 4
            self._hyper_i = 0
        i = self._hyper_i
        self._hyper_i = (i + 1) % len(self._hyper_ring)
        if self._hyper_ev[i] is not None:
            self._hyper_ev[i].synchronize()
        host = self._hyper_ring[i]
        host.copy_(torch.tensor([lr, 1.0 / bc1, 1.0 / math.sqrt(bc2), 0.0]))
        self.hyper.copy_(host, non_blocking=True)
        if self.hyper.is_cuda:
            ev = torch.cuda.Event()
            ev.record()
            self._hyper_ev[i] = ev

    def step(self, grad_scale: float = 1.0, graph: bool = False):
        """One AdamW step. ``grad_scale`` multiplies the raw flat gradient (e.g. 1/world for a
        summed all-reduce, 1/accum_steps for accumulation).  ``graph=True``: the scalars come
        from the device buffer written by ``prepare_graph_step`` (hipGraph-capturable)."""
        if not graph:
            self._sync_lr()
            self.step_count += 1
        self._clear_unwritten()
        clip = None
        if self.max_grad_norm and self.max_grad_norm > 0:
            if (self.use_hip and _ops_mod.get_backend() == "auto" and getattr(self, "tp", 1) <= 1
                    and self.flat_grad.numel() % 8 == 0):
                # norm and clip coefficient in two launches (partial sums of squares + one finishing block)
                nc = _lib.require().grad_norm_clip(self.flat_grad, float(grad_scale), float(self.max_grad_norm))
                self.last_grad_norm = nc[0]
                clip = nc[1:2]
            else:
                norm = self.grad_norm(grad_scale)
                self.last_grad_norm = norm
                clip = torch.clamp(self.max_grad_norm / (norm + 1e-6), max=1.0).to(torch.float32).reshape(1)
        b1, b2 = self.betas
        if self.use_hip and _ops_mod.get_backend() == "auto":
            _lib.require().adamw_(self.flat_param, self.master, self.exp_avg, self.exp_avg_sq, self.flat_grad,
                                  self.lr, b1, b2, self.eps, self.weight_decay, self.step_count, grad_scale, clip,
                                  self.wd_mask, self.hyper if graph else None)
            self.refresh_shadows()
            return
        if graph:
            raise RuntimeError("graph-captured optimizer steps need the HIP AdamW kernel (bf16 params on GPU)")
        g32 = self.flat_grad.float() * grad_scale
        if clip is not None:
            g32 = g32 * clip
        if self.all_decay:
            _ops_mod.ref.adamw_(self.flat_param, g32, self.exp_avg, self.exp_avg_sq, self.lr, b1, b2, self.eps,
                                self.weight_decay, self.step_count, master=self.master)
        else:
            # decoupled decay applied only where the mask says so, then a wd=0 update everywhere
            self.master.mul_(torch.where(self.wd_elem_mask, 1.0 - self.lr * self.weight_decay, 1.0))
            _ops_mod.ref.adamw_(self.flat_param, g32, self.exp_avg, self.exp_avg_sq, self.lr, b1, b2, self.eps,
                                0.0, self.step_count, master=self.master)
        self.refresh_shadows()

    def wait_params(self, params=None):
        """Parameters are always current here (ZeRO-1's optimizer overrides this: its weights
        arrive by all-gathers that the next forward waits for lazily)."""

    # ------------------------------------------------------------------
    def state_dict(self) -> dict:
        state = {}
        for i, p in enumerate(self.params):
            o, n = self.offsets[i], p.numel()
            state[i] = {
                "step": torch.tensor(float(self.step_count)),
                "exp_avg": self.exp_avg[o:o + n].view(p.shape).clone(),
                "exp_avg_sq": self.exp_avg_sq[o:o + n].view(p.shape).clone(),
                "master": self.master[o:o + n].view(p.shape).clone(),
            }
        groups = []
        for decay_flag in (True, False):
            idx = [i for i in range(len(self.params)) if self.decay[i] == decay_flag]
            if not idx:
                continue
            groups.append({"lr": self.lr, "betas": self.betas, "eps": self.eps,
                           "weight_decay": self.weight_decay if decay_flag else 0.0, "amsgrad": False,
                           "maximize": False, "foreach": None, "capturable": False, "differentiable": False,
                           "fused": None, "decoupled_weight_decay": True, "params": idx})
        return {"state": state, "param_groups": groups}

    @torch.no_grad()
    def load_state_dict(self, sd: dict):
        st = sd["state"]
        steps = []
        for i, p in enumerate(self.params):
            if i not in st and str(i) not in st:
                continue
            e = st[i] if i in st else st[str(i)]
            o, n = self.offsets[i], p.numel()
            self.exp_avg[o:o + n].copy_(e["exp_avg"].reshape(-1))
            self.exp_avg_sq[o:o + n].copy_(e["exp_avg_sq"].reshape(-1))
            if "master" in e:
                self.master[o:o + n].copy_(e["master"].reshape(-1))
            else:
                self.master[o:o + n].copy_(self.flat_param[o:o + n].float())
            steps.append(float(e["step"]))
        if steps:
            self.step_count = int(max(steps))
        if sd.get("param_groups"):
            self.param_groups[0]["lr"] = sd["param_groups"][0].get("lr", self.lr)
            self._sync_lr()
        self.flat_param.copy_(self.master.to(self.flat_param.dtype))
        self.refresh_shadows()

    @torch.no_grad()
    def sync_master_from_params(self):
        """Call after loading model weights directly into the params."""
        self.master.copy_(self.flat_param.float())
        self.refresh_shadows()


def accumulate_only_runs(params, offsets, total: int, fresh_ids) -> list:
    """[start, end) element ranges of the flat gradient buffer NOT owned by a lazily zeroed (fresh) slot:
    the accumulate-only parameters, the alignment padding between slots and the tail padding, merged
    where adjacent (every bound a multiple of ALIGN)."""
    runs, pos = [], 0
    for i, p in enumerate(params):
        o = offsets[i]
        if id(p) in fresh_ids:
            if o > pos:
                runs.append((pos, o))
            pos = o + _round_up(p.numel(), ALIGN)
    if total > pos:
        runs.append((pos, total))
    return runs


def _fold_grad(p):
    """Post-accumulate hook (grad dtype != param dtype): add the gradient autograd produced
    for ``p`` into its slot of the flat gradient buffer and release it."""
    if p.grad is not None:
        if getattr(p, "_pllm_grad_fresh", False):  # lazily zeroed slot: this is its first write
            p._pllm_grad_fresh = False
            p._pllm_gradbuf.copy_(p.grad)
        else:
            p._pllm_gradbuf.add_(p.grad)
        p.grad = None


def no_decay_1d(name: str, p: torch.Tensor) -> bool:
    """GPT-2/nanoGPT convention: decay only >=2-D weights (matrices, embeddings)."""
    return p.dim() >= 2

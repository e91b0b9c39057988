"""hipGraph capture of a whole training step (forward, backward, bucketed RCCL
all-reduce, clipping, AdamW, zero_grad).

The reference relies on ``torch.compile`` (scripts/train_transformer.py:31-33,118-120)
to cut framework overhead.  Here the hot ops are already hand-written kernels, so
what is left is per-launch host cost (~400 launches per GPT-2-small step); a captured
step replays them with one ``hipGraphLaunch``.  Everything a step needs from the host
is moved into device buffers first: the batch is copied into static input tensors,
the AdamW scalars (lr, bias corrections) into ``FlatAdamW.hyper``, the gradient-clip
coefficient and CE normaliser are computed on device, and the data-parallel engine's
bucket order is learned in eager warmup steps before capture.

Gradient accumulation (``accum`` > 1) is captured too: the graph holds every micro-step's
forward and backward -- all but the last under the DP engine's ``no_sync`` (no collective),
the last one launching the bucketed all-reduces from the backward hooks -- then one optimizer
step over the fp32 accumulated gradient scaled by 1/accum.  The static inputs are
``[accum, B, T]``.
"""
from __future__ import annotations

import contextlib
import os
from typing import Optional, Tuple

import torch


def graph_step_policy(*, cuda: bool, world: int, dist_backend: Optional[str], zero: bool = False,
                      model_parallel: bool = False, loss_scaling: bool = False, bf16: bool = True,
                      hip_ops: bool = True, graph_collectives: bool = False) -> Tuple[bool, Optional[str]]:
    """THE decision whether a training step is replayed as one captured hipGraph, shared by
    ``Trainer`` (TORCH_COMPILE default) and ``bench.py`` (``--cuda-graph auto``) so the path the
    driver's multi-GPU bench measures is the path ``torchrun scripts/train_transformer.py`` runs.

    Returns ``(use_graph, reason_if_not)``.  With more than one rank the step is EAGER: the bucketed
    RCCL all-reduces are launched from the backward hooks on RCCL's own stream and overlap the rest of
    the backward.  ``graph_collectives=True`` (capture those collectives inside the graph) is refused:
    rehearsed over a one-rank RCCL communicator (PLLM_AB dp_world1=1, profiles/r6_graph_collectives_abort.log)
    the capture aborts the process -- ProcessGroupNCCL's watchdog queries an event recorded in the capturing
    stream (hipErrorCapturedEvent) -- so the option falls back to the eager step with that reason."""
    if not cuda:
        return False, "not a GPU run"
    if zero:
        return False, "ZeRO-1 (collectives inside the optimizer step)"
    if model_parallel:
        return False, "tensor / context parallelism"
    if loss_scaling:
        return False, "loss scaling (host-side skip decision)"
    if not bf16:
        return False, "non-bf16 dtype (the graphed step runs the bf16 HIP kernels)"
    if not hip_ops:
        return False, "stock torch ops backend (PLLM_TORCH_OPS / set_backend)"
    if world > 1 or graph_collectives:
        if world > 1 and dist_backend != "nccl":
            return False, f"dist backend {dist_backend} (collectives cannot be captured)"
        if graph_collectives:
            return False, ("graph_collectives: capturing RCCL collectives aborts in ProcessGroupNCCL's watchdog "
                           "(hipErrorCapturedEvent, profiles/r6_graph_collectives_abort.log); eager step")
        return False, "world > 1: eager step with hook-launched RCCL buckets (the bench's multi-GPU path)"
    return True, None


def gemm_persistent_policy(world: int, setting="auto") -> bool:
    """Whether the ping-pong GEMM / weight-gradient kernels use persistent grids (one workgroup per CU
    walking a tile list) -- shared by ``Trainer`` (config ``gemm_persistent``) and ``bench.py``
    (``--gemm-persistent``).  ``auto``: persistent at world 1 (0.6 % faster than one workgroup per
    tile, profiles/r4_gemm_persistent_ab.txt); at world > 1 one workgroup per tile, because the
    RCCL kernels of the overlapped all-reduces occupy CUs, and a persistent workgroup that cannot
    start there would hold its whole tile list back (a workgroup of these kernels fills a CU's
    registers, so nothing shares the CU with it)."""
    if setting in (None, "auto"):
        from ..ab import ab
        env = ab("gemm_persistent", -1)  # A/B override of the automatic choice (ab.py)
        if env >= 0:
            return env == 1
        return world <= 1
    if isinstance(setting, str):
        return setting.lower() in ("1", "true", "yes", "on")
    return bool(setting)


class GraphedTrainStep:
    def __init__(self, model, optimizer, engine, batch: int, seq: int, device, warmup: int = 2, accum: int = 1):
        self.model, self.opt, self.engine = model, optimizer, engine
        self.accum = int(accum)
        self.xs = torch.zeros(self.accum, batch, seq, dtype=torch.int64, device=device)
        self.ys = torch.zeros(self.accum, batch, seq, dtype=torch.int64, device=device)
        self.x, self.y = self.xs[0], self.ys[0]  # accum == 1 views (bench.py)
        self.warmup = warmup
        self.graph = None
        self.loss = None

    def _body(self):
        total = None
        for m in range(self.accum):
            ctx = self.engine.no_sync() if m < self.accum - 1 else contextlib.nullcontext()
            with ctx:
                _, loss = self.model(self.xs[m], self.ys[m], return_logits=False)
                loss.backward()
            total = loss.detach().float() if total is None else total + loss.detach().float()
        scale = self.engine.finish_grad_sync()
        self.opt.step(grad_scale=scale / self.accum, graph=True)
        self.opt.zero_grad()
        return total / self.accum

    def _load(self, x, y, non_blocking=False):
        # x, y: one micro-batch [B, T] (accum == 1) or all of them [accum, B, T]
        self.xs.copy_(x.view(self.xs.shape), non_blocking=non_blocking)
        self.ys.copy_(y.view(self.ys.shape), non_blocking=non_blocking)

    def capture(self, x, y, lr: float):
        """Run ``warmup`` eager steps on (x, y) (real optimizer steps) on a side stream, then capture.
        The loss of the last warmup step is kept in ``warmup_loss``."""
        self._load(x, y)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(self.warmup):
                self.opt.prepare_graph_step(lr)
                self.warmup_loss = self._body().clone()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        # the capture itself performs no optimizer step: undo the counter advance it needs
        self.opt.prepare_graph_step(lr)
        with torch.cuda.graph(self.graph):
            self.loss = self._body()
        self.opt.step_count -= 1
        return self

    def __call__(self, x, y, lr: float):
        if self.graph is None:
            raise RuntimeError("call capture() first")
        self._load(x, y, non_blocking=True)
        self.opt.prepare_graph_step(lr)
        self.graph.replay()
        return self.loss

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
"""
from __future__ import annotations

import torch


class GraphedTrainStep:
    def __init__(self, model, optimizer, engine, batch: int, seq: int, device, warmup: int = 2):
        self.model, self.opt, self.engine = model, optimizer, engine
        self.x = torch.zeros(batch, seq, dtype=torch.int64, device=device)
        self.y = torch.zeros(batch, seq, dtype=torch.int64, device=device)
        self.warmup = warmup
        self.graph = None
        self.loss = None

    def _body(self):
        _, loss = self.model(self.x, self.y, return_logits=False)
        loss.backward()
        scale = self.engine.finish_grad_sync()
        self.opt.step(grad_scale=scale, graph=True)
        self.opt.zero_grad()
        return loss.detach()

    def capture(self, x, y, lr: float):
        """Run ``warmup`` eager steps on (x, y) (real optimizer steps) on a side stream, then capture.
        The loss of the last warmup step is kept in ``warmup_loss``."""
        self.x.copy_(x)
        self.y.copy_(y)
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
        self.x.copy_(x, non_blocking=True)
        self.y.copy_(y, non_blocking=True)
        self.opt.prepare_graph_step(lr)
        self.graph.replay()
        return self.loss

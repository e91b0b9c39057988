"""Rank body of tests/test_dist_gloo.py::test_trainer_and_bench_take_the_same_step_path (launched by
torch.distributed.run, 2 gloo ranks on the CPU).

The step-path policy (train/graph.py graph_step_policy) is stubbed to the RCCL branch -- a GPU run on
the nccl backend with the HIP ops -- and GraphedTrainStep is replaced by a stand-in that records its
construction and runs the same step eagerly (no hipGraph on the CPU).  Then the Trainer trains two
steps and bench.py runs (--gpus 2 --device cpu); each rank prints one JSON line with the step mode
each path actually TOOK (a capture object built and stepped, or not)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from pretraining_llm_amd.train import graph as g  # noqa: E402

GC = sys.argv[1] == "graph_collectives"
_orig = g.graph_step_policy


def _stub(**kw):
    kw["cuda"] = True
    kw["hip_ops"] = True
    kw["bf16"] = True  # the CPU run is fp32; a GPU run computes in bf16
    if kw.get("dist_backend") == "gloo":
        kw["dist_backend"] = "nccl"
    return _orig(**kw)


class _EagerStandIn:
    built = []

    def __init__(self, model, opt, engine, batch, seq, device, warmup=2, accum=1):
        self.model, self.opt, self.engine, self.accum, self.steps = model, opt, engine, int(accum), 0
        _EagerStandIn.built.append(self)

    def _step(self, x, y, lr):
        import contextlib
        x, y = x.reshape(self.accum, -1, x.shape[-1]), y.reshape(self.accum, -1, y.shape[-1])
        self.opt.param_groups[0]["lr"] = lr
        tot = None
        for m in range(self.accum):
            ctx = self.engine.no_sync() if m < self.accum - 1 else contextlib.nullcontext()
            with ctx:
                _, loss = self.model(x[m], y[m], return_logits=False)
                loss.backward()
            tot = loss.detach() if tot is None else tot + loss.detach()
        scale = self.engine.finish_grad_sync()
        self.opt.step(grad_scale=scale / self.accum)
        self.opt.zero_grad()
        self.steps += 1
        return tot / self.accum

    def capture(self, x, y, lr):
        self.warmup_loss = self._step(x, y, lr)
        return self

    def __call__(self, x, y, lr):
        return self._step(x, y, lr)


g.graph_step_policy = _stub
g.GraphedTrainStep = _EagerStandIn

from config.config import PRESET_RUNS, default_config  # noqa: E402
from pretraining_llm_amd.train.trainer import Trainer  # noqa: E402

cfg = dict(default_config)
cfg.update(PRESET_RUNS["gpt2-tiny-cpu"])
tmp = sys.argv[2]  # shared by the ranks (rank 0 writes the synthetic shard)
cfg.update(t_train_steps=2, t_eval_steps=100, log_interval=1, eval_at_start=False, t_out_path=None,
           synthetic_dir=tmp, synthetic_tokens=60_000, t_batch_size=2, seq_len=64, compile=True,
           ddp_backend="gloo", graph_collectives=GC)
tr = Trainer(cfg, log=lambda *_: None)
tr.train()
trainer_rec = {"step_mode": tr.step_mode, "capture_objects": len(_EagerStandIn.built),
               "captured_steps": sum(o.steps for o in _EagerStandIn.built)}
_EagerStandIn.built.clear()

import io  # noqa: E402
import contextlib  # noqa: E402
import bench  # noqa: E402

buf = io.StringIO()
argv = ["--gpus", "2", "--device", "cpu", "--model", "gpt2-tiny", "--steps", "2", "--warmup", "1", "--batch", "2",
        "--seq", "64"] + (["--graph-collectives"] if GC else [])
rank = int(os.environ.get("RANK", "0"))
with contextlib.redirect_stdout(buf):
    rc = bench.main(argv)
bench_rec = None
for line in buf.getvalue().splitlines():
    if line.startswith("{"):
        bench_rec = json.loads(line)
out = {"rank": rank, "trainer": trainer_rec,
       "bench": {"rc": rc, "capture_objects": len(_EagerStandIn.built),
                 "captured_steps": sum(o.steps for o in _EagerStandIn.built),
                 "step_mode": bench_rec["config"]["step_mode"] if bench_rec else None}}
print("PROBE " + json.dumps(out), flush=True)

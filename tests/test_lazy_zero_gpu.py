"""Lazy gradient zeroing (train/optim.py FlatAdamW(lazy_zero=True), ops._set_target / _acc_target): zero_grad
clears only the accumulate-only slots and the weight-gradient GEMMs overwrite their slots on the first write of
a step.  The training trajectory must be bit-identical to full zeroing, with gradient accumulation, in the
captured (hipGraph) step and eagerly, and a weight no writer touched must read as a zero gradient."""
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _ext():
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    yield


@pytest.mark.parametrize("preset", ["gpt2-tiny", "llama-tiny"])
@pytest.mark.parametrize("compile_", [None, False])
def test_lazy_zero_matches_full_zero(preset, compile_, tmp_path, monkeypatch):
    from pretraining_llm_amd.train.trainer import Trainer
    from config.config import default_config
    monkeypatch.delenv("TORCH_COMPILE", raising=False)
    base = dict(default_config)
    base.update(model_preset=preset, t_batch_size=4, seq_len=128, t_train_steps=6, t_lr=1e-3, warmup_steps=2,
                log_interval=1, t_eval_steps=1000, eval_at_start=False, t_out_path=None, synthetic_data=True,
                synthetic_tokens=200_000, synthetic_dir=str(tmp_path), max_grad_norm=1.0, device="cuda",
                grad_accum_steps=2, compile=compile_)
    out = {}
    for lazy in ("0", "1"):
        monkeypatch.setenv("PLLM_AB", f"lazy_zero={lazy}")
        recs = []
        tr = Trainer(dict(base), log=lambda *_: None)
        assert tr.opt.lazy_zero == (lazy == "1")
        tr.metrics.log = recs.append
        tr.train()
        out[lazy] = ([r["train_loss"] for r in recs], tr.opt.master.clone())
    # the same sums in the same order (a store where the other adds onto zero): equal to rounding noise at
    # most; a stale or doubled gradient slot would be off by orders of magnitude more
    for a, b in zip(out["0"][0], out["1"][0]):
        assert abs(a - b) <= 1e-5 * max(1.0, abs(b)), (out["0"][0], out["1"][0])
    rel = ((out["0"][1] - out["1"][1]).norm() / out["0"][1].norm()).item()
    assert rel < 1e-6, rel


def test_lazy_zero_unwritten_weight_reads_zero():
    """A weight used in one step and not in the next: its slot must not keep the old gradient."""
    from pretraining_llm_amd import ops
    from pretraining_llm_amd.train.optim import FlatAdamW

    class Two(nn.Module):
        def __init__(self):
            super().__init__()
            self.a = nn.Linear(128, 128, bias=False)
            self.b = nn.Linear(128, 128, bias=False)

    torch.manual_seed(0)
    m = Two().to(DEV, torch.bfloat16)
    opt = FlatAdamW(m, lr=1e-3, max_grad_norm=1.0, lazy_zero=True)
    assert opt.lazy_zero
    x = torch.randn(64, 128, device=DEV).bfloat16()
    opt.zero_grad()
    ops.linear(ops.linear(x, m.a.weight), m.b.weight).float().square().mean().backward()
    gb = m.b.weight._pllm_gradbuf.clone()
    assert gb.abs().sum() > 0
    opt.step()
    opt.zero_grad()
    ops.linear(x, m.a.weight).float().square().mean().backward()  # b unused this step
    assert getattr(m.b.weight, "_pllm_grad_fresh", False)
    opt.grad_norm()
    assert not getattr(m.b.weight, "_pllm_grad_fresh", True)
    assert (m.b.weight._pllm_gradbuf == 0).all()
    assert (m.a.weight._pllm_gradbuf != 0).any()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_zero_ranges_kernel(dtype):
    """torch.ops.pllm.zero_ranges_: exactly the listed 16-B aligned ranges become zero, nothing else moves."""
    torch.manual_seed(2)
    n = 1 << 20
    buf = torch.randn(n, device=DEV).to(dtype) + 3
    ranges = [(0, 64), (128, 4096), (8192, 8192 + 64), (100000 // 64 * 64, 300000 // 64 * 64), (n - 640, n)]
    before = buf.clone()
    r = torch.tensor(ranges, dtype=torch.int64, device=DEV)
    torch.ops.pllm.zero_ranges_(buf, r, sum(b - a for a, b in ranges))
    mask = torch.zeros(n, dtype=torch.bool, device=DEV)
    for a, b in ranges:
        mask[a:b] = True
    assert (buf[mask] == 0).all()
    assert torch.equal(buf[~mask], before[~mask])

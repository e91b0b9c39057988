"""Precision modes and dynamic loss scaling (reference: GradScaler(enabled=dtype == 'float16'),
scripts/train_transformer.py:41,69,92-93)."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_scaler_update_semantics():
    from pretraining_llm_amd.train.amp import DynamicLossScaler
    s = DynamicLossScaler(init_scale=1024.0, growth_interval=3)
    s.update(True)
    assert s.scale == 512.0 and s.skipped_steps == 1
    for _ in range(2):
        s.update(False)
    assert s.scale == 512.0
    s.update(False)
    assert s.scale == 1024.0 and s.growth_tracker == 0
    s.update(False)
    sd = s.state_dict()
    assert set(sd) == {"scale", "growth_factor", "backoff_factor", "growth_interval", "_growth_tracker"}
    t = DynamicLossScaler()
    t.load_state_dict(sd)
    assert (t.scale, t.growth_tracker, t.growth_interval) == (1024.0, 1, 3)
    off = DynamicLossScaler(enabled=False)
    x = torch.tensor(3.0)
    assert off.scale_loss(x) is x
    off.update(True)
    assert off.scale == 2.0 ** 16


def test_precision_modes():
    from pretraining_llm_amd.train.amp import precision_mode
    cuda, cpu = torch.device("cuda", 0), torch.device("cpu")
    assert precision_mode("bfloat16", cuda) == (torch.bfloat16, None)
    assert precision_mode("float16", cuda) == (torch.bfloat16, None)  # the reference's bf16 + GradScaler
    assert precision_mode("float16_autocast", cuda) == (torch.float32, torch.float16)
    assert precision_mode("float32", cuda) == (torch.float32, None)
    assert precision_mode("bfloat16", cpu) == (torch.float32, None)
    assert precision_mode("bfloat16", cpu, cpu_bf16=True) == (torch.bfloat16, None)
    with pytest.raises(ValueError):
        precision_mode("float8", cuda)


@pytest.mark.gpu
def test_hip_dispatch_is_bf16_only():
    """fp32 / fp16 CUDA tensors (dtype float32 / float16 training modes) take the torch path;
    bf16 and integer-only CUDA operands take the HIP kernels."""
    from pretraining_llm_amd.ops import _lib
    dev = "cuda"
    assert _lib.use_hip(torch.zeros(1, device=dev, dtype=torch.bfloat16))
    assert not _lib.use_hip(torch.zeros(1, device=dev, dtype=torch.float32))
    assert not _lib.use_hip(torch.zeros(1, device=dev, dtype=torch.float16))
    assert _lib.use_hip(torch.zeros(1, device=dev, dtype=torch.long))
    assert _lib.use_hip(torch.zeros(1, device=dev, dtype=torch.long), torch.zeros(1, device=dev, dtype=torch.bfloat16))
    assert not _lib.use_hip(torch.zeros(1, dtype=torch.bfloat16))


def _cfg(tmp_path, **kw):
    sys.path.insert(0, ROOT)
    from config.config import PRESET_RUNS, default_config
    cfg = dict(default_config)
    cfg.update(PRESET_RUNS["gpt2-tiny-cpu"])
    cfg.update(dict(t_out_path=str(tmp_path / "m.pt"), synthetic_dir=str(tmp_path / "syn"), t_train_steps=12,
                    t_eval_steps=6, log_interval=6, t_eval_iters=1, t_batch_size=2, seq_len=64,
                    synthetic_tokens=50_000, device="cpu"))
    cfg.update(kw)
    return cfg


def test_loss_scaling_is_exact_in_fp32(tmp_path):
    """Power-of-two loss scaling changes nothing in fp32: the unscale folded into the optimizer's
    grad_scale restores the gradient exactly."""
    from pretraining_llm_amd.train import Trainer
    a = Trainer(_cfg(tmp_path), log=lambda *_: None).train()
    b = Trainer(_cfg(tmp_path, loss_scaling=True, t_out_path=str(tmp_path / "b.pt")), log=lambda *_: None).train()
    assert b.scaler.enabled and not a.scaler.enabled and b.scaler.skipped_steps == 0
    for p, q in zip(a.model.parameters(), b.model.parameters()):
        assert torch.allclose(p, q, atol=1e-6, rtol=1e-5)
    ck = torch.load(tmp_path / "b.pt", weights_only=True)
    assert ck["scaler_state_dict"]["scale"] == b.scaler.scale


def test_overflow_skips_step_and_backs_off(tmp_path):
    """A scale that overflows the gradient skips the optimizer step (weights untouched), halves
    the scale, and training proceeds once the scale fits (GradScaler semantics)."""
    from pretraining_llm_amd.train import Trainer
    tr = Trainer(_cfg(tmp_path, loss_scaling=True, loss_scale_init=2.0 ** 140, t_train_steps=1, t_out_path=None),
                 log=lambda *_: None)
    before = [p.detach().clone() for p in tr.model.parameters()]
    tr.train_step()
    assert tr.scaler.skipped_steps == 1 and tr.scaler.scale == 2.0 ** 139 and tr.step == 1
    for p, q in zip(before, tr.model.parameters()):
        assert torch.equal(p, q)
    for _ in range(80):  # back off until the scaled gradient fits in fp32
        n = tr.scaler.skipped_steps
        tr.train_step()
        if tr.scaler.skipped_steps == n:
            break
    assert tr.scaler.skipped_steps == n and 2.0 ** 60 < tr.scaler.scale < 2.0 ** 139
    assert any(not torch.equal(p, q) for p, q in zip(before, tr.model.parameters()))


@pytest.mark.gpu
def test_fp16_and_fp32_modes_train_on_gpu(tmp_path):
    """dtype float16 (the reference's: bf16 HIP path + dynamic loss scaling), float16_autocast (fp32
    weights, fp16 autocast, loss scaling) and float32 train the GPT-2 tiny config on the GPU and
    track the bf16 HIP-kernel run."""
    import json
    from pretraining_llm_amd.train import Trainer
    finals = {}
    for dt in ("bfloat16", "float16", "float16_autocast", "float32"):
        d = tmp_path / dt
        tr = Trainer(_cfg(d, device="cuda", dtype=dt, t_train_steps=60, t_eval_steps=30, log_interval=10,
                          t_batch_size=8, seq_len=128, metrics_path=str(d / "m.jsonl"), t_out_path=None),
                     log=lambda *_: None)
        assert tr.scaler.enabled == dt.startswith("float16")
        assert next(tr.model.parameters()).dtype == (torch.bfloat16 if dt in ("bfloat16", "float16") else torch.float32)
        tr.train()
        recs = [json.loads(l) for l in open(d / "m.jsonl")]
        assert recs[-1]["train_loss"] < recs[0]["train_loss"] - 1.0, (dt, recs[0], recs[-1])
        finals[dt] = recs[-1]["train_loss"]
        if dt.startswith("float16"):
            assert tr.scaler.scale >= 1.0
    for dt in ("float16", "float16_autocast"):
        assert abs(finals[dt] - finals["float32"]) < 0.05 * finals["float32"], finals
    assert abs(finals["bfloat16"] - finals["float32"]) < 0.05 * finals["float32"], finals

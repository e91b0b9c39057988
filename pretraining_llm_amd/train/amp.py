"""Mixed-precision modes and dynamic loss scaling over the flat gradient buffer.

Reference (scripts/train_transformer.py:41,69,92-93): ``torch.cuda.amp.GradScaler(enabled=
dtype == 'float16')``; ``scaler.scale(loss).backward()``, ``scaler.step(opt)``,
``scaler.update()``.  The reference wraps every forward in bf16 autocast whatever ``dtype``
says, so its ``float16`` mode is bf16 compute WITH loss scaling.

Here (``Trainer``):

* ``dtype='bfloat16'`` (default): bf16 weights on the hand-written HIP kernels, fp32 master
  weights and gradients (train/optim.py).  No loss scaling (bf16 has fp32's exponent range).
* ``dtype='float16'``: what the reference's ``float16`` setting does -- bf16 compute (here the
  bf16 HIP path, as ``'bfloat16'``) WITH dynamic loss scaling.
* ``dtype='float16_autocast'`` (explicit opt-in, no reference counterpart): true fp16 numerics,
  fp32 weights, forward under ``torch.autocast(float16)`` (fp16 GEMMs on hipBLASLt through torch;
  the hand-written kernels are bf16-only, so this mode is much slower) and dynamic loss scaling.
* ``dtype='float32'``: fp32 weights and compute through torch.
* ``loss_scaling`` (None = on iff ``dtype`` is ``'float16'`` or ``'float16_autocast'``) switches
  the scaler on or off explicitly.

``DynamicLossScaler`` has ``GradScaler``'s semantics (scale 2^16, x2 after 2000 clean steps,
x0.5 and a skipped optimizer step on an inf/nan gradient) but works on the optimizer's flat
gradient: the unscale is folded into the AdamW kernel's ``grad_scale`` (no extra pass), and
the inf check is one reduction over the buffer the optimizer reads, MAX-reduced over all
ranks so every rank skips the same steps.
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist


class DynamicLossScaler:
    def __init__(self, init_scale: float = 2.0 ** 16, growth_factor: float = 2.0, backoff_factor: float = 0.5,
                 growth_interval: int = 2000, enabled: bool = True):
        self.scale = float(init_scale)
        self.growth_factor = float(growth_factor)
        self.backoff_factor = float(backoff_factor)
        self.growth_interval = int(growth_interval)
        self.enabled = bool(enabled)
        self.growth_tracker = 0
        self.skipped_steps = 0

    def scale_loss(self, loss: torch.Tensor) -> torch.Tensor:
        return loss * self.scale if self.enabled else loss

    @torch.no_grad()
    def found_inf(self, optimizer) -> bool:
        """True when the gradient the optimizer step would read holds an inf / nan on ANY rank."""
        buf = getattr(optimizer, "grad_shard", None)
        if buf is None:
            buf = optimizer.flat_grad
        bad = (~torch.isfinite(buf).all()).float().reshape(1)
        if dist.is_initialized() and dist.get_world_size() > 1:
            if dist.get_backend() == "gloo" and bad.is_cuda:
                host = bad.cpu()
                dist.all_reduce(host, op=dist.ReduceOp.MAX)
                bad = host
            else:
                dist.all_reduce(bad, op=dist.ReduceOp.MAX)
        return bool(bad.item())

    def update(self, found_inf: bool):
        if not self.enabled:
            return
        if found_inf:
            self.scale *= self.backoff_factor
            self.growth_tracker = 0
            self.skipped_steps += 1
        else:
            self.growth_tracker += 1
            if self.growth_tracker == self.growth_interval:
                self.scale *= self.growth_factor
                self.growth_tracker = 0

    def state_dict(self) -> dict:
        # the keys of torch.amp.GradScaler.state_dict()
        return {"scale": self.scale, "growth_factor": self.growth_factor, "backoff_factor": self.backoff_factor,
                "growth_interval": self.growth_interval, "_growth_tracker": self.growth_tracker}

    def load_state_dict(self, sd: dict):
        self.scale = float(sd.get("scale", self.scale))
        self.growth_factor = float(sd.get("growth_factor", self.growth_factor))
        self.backoff_factor = float(sd.get("backoff_factor", self.backoff_factor))
        self.growth_interval = int(sd.get("growth_interval", self.growth_interval))
        self.growth_tracker = int(sd.get("_growth_tracker", self.growth_tracker))


DTYPES = ("bfloat16", "float16", "float16_autocast", "float32")


def loss_scaling_default(dtype_name: str) -> bool:
    """The reference's ``GradScaler(enabled=dtype == 'float16')`` (train_transformer.py:41)."""
    return dtype_name in ("float16", "float16_autocast")


def precision_mode(dtype_name: str, device: torch.device, cpu_bf16: bool = False):
    """-> (parameter dtype, autocast dtype or None) for a training ``dtype`` setting."""
    if dtype_name not in DTYPES:
        raise ValueError(f"dtype={dtype_name!r}: expected one of {DTYPES}")
    if device.type == "cpu":
        # CPU runs are the fp32 numerics reference (cpu_bf16 for bf16 plumbing checks)
        return (torch.bfloat16 if cpu_bf16 and dtype_name in ("bfloat16", "float16") else torch.float32), None
    if dtype_name in ("bfloat16", "float16"):  # float16 = the reference's bf16 compute + GradScaler
        return torch.bfloat16, None
    if dtype_name == "float16_autocast":
        return torch.float32, torch.float16
    return torch.float32, None


def autocast_ctx(device: torch.device, dtype):
    if dtype is None:
        return contextlib.nullcontext()
    return torch.autocast(device_type=device.type, dtype=dtype)

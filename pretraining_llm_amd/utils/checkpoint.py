"""Checkpoint save/load in the reference format.

Reference: at the end of training rank 0 does
``torch.save({'model_state_dict': model.state_dict(), 'optimizer_state_dict':
optimizer.state_dict()}, t_out_path)`` (scripts/train_transformer.py:104-109) and
``generate_text.py`` loads ``ckpt['model_state_dict']`` strictly (:21,31).

Kept: the two top-level keys and plain ``state_dict`` contents (weights-only
loadable).  Fixed: keys are always unwrapped (no ``module.``/``_orig_mod.``,
D7), the parent directory is created (D8), writes are atomic (tmp + rename),
and extra resume keys are stored -- ``step``, ``config``, ``model_config``,
``data_state``, ``rng`` -- all plain dicts/ints/strings/tensors so
``torch.load(weights_only=True)`` still works.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from ..models.compat import strip_wrapper_prefixes


def unwrap(model):
    while hasattr(model, "module"):
        model = model.module
    return getattr(model, "_orig_mod", model)


def rng_state() -> dict:
    st = {"torch": torch.get_rng_state()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def save_checkpoint(path: str, model, optimizer=None, step: Optional[int] = None, config: Optional[dict] = None,
                    data_state: Optional[dict] = None, extra: Optional[dict] = None,
                    optimizer_state: Optional[dict] = None) -> str:
    m = unwrap(model)
    sd = {k: v.detach().cpu() if torch.is_tensor(v) else v for k, v in m.state_dict().items()}
    ckpt = {"model_state_dict": strip_wrapper_prefixes(sd)}
    if optimizer is not None:
        optimizer_state = optimizer.state_dict()
    if optimizer_state is not None:
        ckpt["optimizer_state_dict"] = _to_cpu(optimizer_state)
    if step is not None:
        ckpt["step"] = int(step)
    if config is not None:
        ckpt["config"] = _plain(config)
    if hasattr(m, "config") and hasattr(m.config, "to_dict"):
        ckpt["model_config"] = _plain(m.config.to_dict())
    if data_state is not None:
        ckpt["data_state"] = _plain(data_state)
    ckpt["rng"] = rng_state()
    if extra:
        ckpt.update(extra)
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = f"{path}.tmp{os.getpid()}"
    torch.save(ckpt, tmp)
    os.replace(tmp, path)
    return path


def load_checkpoint(path: str, map_location="cpu") -> dict:
    ckpt = torch.load(path, map_location=map_location, weights_only=True)
    if "model_state_dict" in ckpt:
        ckpt["model_state_dict"] = strip_wrapper_prefixes(ckpt["model_state_dict"])
    return ckpt


def _to_cpu(obj):
    if torch.is_tensor(obj):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj


def _plain(obj):
    """Reduce to weights-only-safe builtins."""
    if isinstance(obj, dict):
        return {str(k): _plain(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [_plain(v) for v in obj]
    if isinstance(obj, (int, float, str, bool)) or obj is None:
        return obj
    if torch.is_tensor(obj):
        return obj.detach().cpu()
    return str(obj)

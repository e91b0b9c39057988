"""Checkpoint save/load in the reference format.

Reference: at the end of training rank 0 does
``torch.save({'model_state_dict': model.state_dict(), 'optimizer_state_dict':
optimizer.state_dict()}, t_out_path)`` (scripts/train_transformer.py:104-109) and
``generate_text.py`` loads ``ckpt['model_state_dict']`` strictly (:21,31).

Kept: the two top-level keys and plain ``state_dict`` contents (weights-only
loadable).  ``model_state_dict`` holds fp32 weights like the reference's (its model
lives in fp32 under autocast): they are taken from the optimizer's fp32 master copy,
not the bf16 compute weights, so a bf16 model loads them back bit-exactly and an fp32
consumer gets full precision.  Fixed: keys are always unwrapped (no ``module.``/``_orig_mod.``,
D7), the parent directory is created (D8), writes are atomic (tmp + rename),
and extra resume keys are stored -- ``step``, ``config``, ``model_config``,
``data_state``, ``rng`` -- all plain dicts/ints/strings/tensors so
``torch.load(weights_only=True)`` still works.
"""
from __future__ import annotations

import contextlib
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


@contextlib.contextmanager
def master_weights(params, optimizer_state: Optional[dict]):
    """Temporarily point each parameter's ``.data`` at its fp32 master value from an
    AdamW-format optimizer state (``state[i]['master']``, i = position in ``params``), so
    ``model.state_dict()`` -- including the reference-layout hooks that split the packed QKV
    weight -- emits fp32 weights.  No-op when the state carries no masters."""
    st = (optimizer_state or {}).get("state", {})
    saved = []
    try:
        for i, p in enumerate(params or []):
            e = st.get(i, st.get(str(i)))
            if e is None or "master" not in e or p.dtype == torch.float32:
                continue
            saved.append((p, p.data))
            p.data = e["master"].detach().reshape(p.shape).cpu().float()
        yield
    finally:
        for p, d in saved:
            p.data = d


def save_checkpoint(path: str, model, optimizer=None, step: Optional[int] = None, config: Optional[dict] = None,
                    data_state: Optional[dict] = None, extra: Optional[dict] = None,
                    optimizer_state: Optional[dict] = None, params=None) -> str:
    """``params``: the optimizer's parameter list (index i of ``optimizer_state['state']``);
    taken from ``optimizer.params`` when an optimizer is given."""
    m = unwrap(model)
    if optimizer is not None:
        optimizer_state = optimizer.state_dict()
        params = getattr(optimizer, "params", params)
    with master_weights(params, optimizer_state):
        sd = {k: v.detach().cpu() if torch.is_tensor(v) else v for k, v in m.state_dict().items()}
    ckpt = {"model_state_dict": strip_wrapper_prefixes(sd)}
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

"""Workspace budgets derived from the HBM actually free on the device.

Two transient workspaces scale with the problem rather than with the model: the LM-head +
cross-entropy logits chunk (``ops._LMHeadCEFn``: rows x vocab bf16) and the attention
backward's dQ partial slabs (``attn_bwd``: key blocks x B x H x T x D bf16).  Fixed budgets
(8 GiB / 4 GiB) were sized on one box; with tensor / context-parallel shards, larger
vocabularies or a fuller HBM they either waste memory or run the device out of it.  Here each
budget is ``fraction`` of what the device can still give -- free HBM (``hipMemGetInfo``) plus
what the caching allocator holds reserved but unused -- clamped to [floor, cap].  The cap keeps
the measured single-chunk / single-pass behaviour of the shipped configs (bigger chunks buy
nothing); the floor keeps the chunking from degenerating.  Environment overrides
(``PLLM_CE_WORKSPACE_MB``, ``PLLM_ATTN_BWD_WS_MB``) still win.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

MiB = 2 ** 20


def free_hbm_bytes(device: torch.device) -> int:
    """Bytes a new allocation on ``device`` can get: free device memory plus the caching
    allocator's reserved-but-unallocated pool."""
    if device.type != "cuda" or not torch.cuda.is_available():
        return 1 << 62  # CPU, or fake CUDA tensors traced on a host without a GPU
    idx = device.index if device.index is not None else torch.cuda.current_device()
    free, _total = torch.cuda.mem_get_info(idx)
    slack = torch.cuda.memory_reserved(idx) - torch.cuda.memory_allocated(idx)
    return int(free + max(0, slack))


# Budget policy.  The chunking a budget selects changes the fp32 grouping of some sums (e.g. the
# LM-head weight gradient accumulates per CE chunk), so a budget re-read from the free HBM on every
# call makes same-seed runs depend on the memory state.  ``freeze_budgets()`` (the Trainer calls
# it) computes each budget once, at its first use, and keeps it; ``freeze_budgets(pin_caps=True)``
# (``deterministic=True``) pins every budget to its cap, independent of the device's state.
_policy = {"mode": "live"}   # live | frozen | caps
_frozen: dict = {}


def freeze_budgets(pin_caps: bool = False) -> None:
    _policy["mode"] = "caps" if pin_caps else "frozen"
    _frozen.clear()


def live_budgets() -> None:
    _policy["mode"] = "live"
    _frozen.clear()


def workspace_budget(device: torch.device, cap_bytes: int, fraction: float, floor_bytes: int,
                     free_fn: Optional[Callable[[torch.device], int]] = None) -> int:
    """``fraction`` x free HBM, clamped to [floor_bytes, cap_bytes] (CPU: the cap); see the policy
    above for the frozen / pinned modes."""
    mode = _policy["mode"]
    if mode == "caps" or (device.type != "cuda" and free_fn is None):
        return int(cap_bytes)
    key = (str(device), int(cap_bytes), float(fraction), int(floor_bytes))
    if mode == "frozen" and key in _frozen:
        return _frozen[key]
    free = (free_fn or free_hbm_bytes)(device)
    b = int(max(floor_bytes, min(cap_bytes, fraction * free)))
    if mode == "frozen":
        _frozen[key] = b
    return b


# defaults: caps = the budgets measured to keep every shipped config in one chunk / pass
CE_CAP = 8192 * MiB
CE_FRACTION = 0.25
CE_FLOOR = 256 * MiB
ATTN_WS_CAP = 4096 * MiB
ATTN_WS_FRACTION = 0.25
ATTN_WS_FLOOR = 64 * MiB

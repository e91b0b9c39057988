"""Token-shard data pipeline.

Reference API kept: ``get_batch_iterator(data_path, batch_size, context_length,
device='cpu', ddp=False, ddp_rank=0, ddp_world_size=1)`` yields int64 ``(x, y)``
with ``y`` = ``x`` shifted by one (data_loader/data_loader.py:7-52).

Differences (deliberate):
* the window gather runs in the native loader (``csrc/host/token_loader.cpp``)
  on a producer thread, contiguous per-rank shards, seeded counter RNG;
* batches land in pinned host buffers and are copied H2D on a dedicated side
  stream with an event the consumer's stream waits on (for any ``cuda:N``);
* a missing file can be replaced by a synthetic shard (``synthetic=True``).
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Iterator, Optional, Tuple

import numpy as np
import torch

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_HOST_SO = os.path.join(_HERE, "_host.so")
_lib = None
_lib_lock = threading.Lock()


def _host_lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lib_lock:
        if _lib is None:
            if not os.path.exists(_HOST_SO):
                from ..build import build_host
                build_host()
            lib = ctypes.CDLL(_HOST_SO)
            lib.pllm_loader_create.restype = ctypes.c_void_p
            lib.pllm_loader_create.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int]
            lib.pllm_loader_next.restype = ctypes.c_int64
            lib.pllm_loader_next.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
            lib.pllm_loader_batch_at.restype = None
            lib.pllm_loader_batch_at.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
            lib.pllm_loader_shard_tokens.restype = ctypes.c_int64
            lib.pllm_loader_shard_tokens.argtypes = [ctypes.c_void_p]
            lib.pllm_loader_destroy.restype = None
            lib.pllm_loader_destroy.argtypes = [ctypes.c_void_p]
            _lib = lib
    return _lib


class TokenLoader:
    """Random contiguous windows from a flat uint16 token file, one shard per rank."""

    def __init__(self, path: str, batch_size: int, context_length: int, rank: int = 0, world_size: int = 1,
                 seed: int = 1337, start_batch: int = 0, prefetch: int = 4, device: Optional[torch.device] = None):
        self.path = path
        self.B, self.T = int(batch_size), int(context_length)
        self.rank, self.world = int(rank), int(world_size)
        self.seed = int(seed)
        lib = _host_lib()
        self._h = lib.pllm_loader_create(path.encode(), self.rank, self.world, self.B, self.T,
                                         ctypes.c_uint64(self.seed & (2 ** 64 - 1)), int(start_batch), int(prefetch))
        if not self._h:
            raise FileNotFoundError(f"cannot open token shard {path!r} (missing or shorter than context_length+2 "
                                    f"tokens per rank)")
        self.batches_consumed = int(start_batch)
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        pin = self.device.type == "cuda"
        nbuf = 2
        self._hx = [torch.empty(self.B, self.T, dtype=torch.int64, pin_memory=pin) for _ in range(nbuf)]
        self._hy = [torch.empty(self.B, self.T, dtype=torch.int64, pin_memory=pin) for _ in range(nbuf)]
        self._slot = 0
        self._copy_stream = torch.cuda.Stream(device=self.device) if pin else None
        self._events = [None] * nbuf

    def shard_tokens(self) -> int:
        return int(_host_lib().pllm_loader_shard_tokens(self._h))

    def batch_at(self, index: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """Deterministic regeneration of batch ``index`` on the host (tests, debugging)."""
        x = torch.empty(self.B, self.T, dtype=torch.int64)
        y = torch.empty(self.B, self.T, dtype=torch.int64)
        _host_lib().pllm_loader_batch_at(self._h, int(index), x.data_ptr(), y.data_ptr())
        return x, y

    def next(self) -> Tuple[torch.Tensor, torch.Tensor]:
        s = self._slot
        self._slot = (s + 1) % len(self._hx)
        hx, hy = self._hx[s], self._hy[s]
        if self._events[s] is not None:
            self._events[s].synchronize()  # the H2D copy that last read this pinned slot is done
        _host_lib().pllm_loader_next(self._h, hx.data_ptr(), hy.data_ptr())
        self.batches_consumed += 1
        if self._copy_stream is None:
            if self.device.type == "cpu":
                return hx.clone(), hy.clone()
            return hx.to(self.device), hy.to(self.device)
        cur = torch.cuda.current_stream(self.device)
        with torch.cuda.stream(self._copy_stream):
            x = hx.to(self.device, non_blocking=True)
            y = hy.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._copy_stream)
        cur.wait_event(ev)
        x.record_stream(cur)
        y.record_stream(cur)
        self._events[s] = ev
        return x, y

    def __iter__(self):
        return self

    def __next__(self):
        return self.next()

    def state_dict(self) -> dict:
        return {"path": self.path, "seed": self.seed, "batches_consumed": self.batches_consumed,
                "rank": self.rank, "world_size": self.world}

    def close(self):
        if getattr(self, "_h", None):
            _host_lib().pllm_loader_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def get_batch_iterator(data_path: str, batch_size: int, context_length: int, device: str = "cpu",
                       ddp: bool = False, ddp_rank: int = 0, ddp_world_size: int = 1, seed: int = 1337,
                       start_batch: int = 0) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
    """Reference-compatible infinite ``(x, y)`` generator (data_loader/data_loader.py:7)."""
    rank, world = (ddp_rank, ddp_world_size) if ddp else (0, 1)
    loader = TokenLoader(data_path, batch_size, context_length, rank, world, seed=seed, start_batch=start_batch,
                         device=torch.device(device))
    try:
        while True:
            yield loader.next()
    finally:
        loader.close()

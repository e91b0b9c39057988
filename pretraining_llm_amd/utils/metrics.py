"""Throughput / MFU accounting and structured logging.

The reference prints one line per 1000 steps with wall time that includes the
evaluation (scripts/train_transformer.py:97-102) and no tokens/s.  Here step
time is measured with device events, tokens/s is whole-job, MFU uses
6*N_matmul + 12*L*T*C FLOPs/token against the MI355X dense bf16
peak, and each log record can be appended to a JSONL file.
"""
from __future__ import annotations

import json
import os
import time
from typing import Optional

import torch

MI355X_BF16_DENSE_PEAK = 2.5e15  # FLOP/s per GPU (vendor dense figure; no sparsity)


class StepTimer:
    """Wall-clock timer around a span of GPU work (syncs the device at both ends)."""

    def __init__(self, device: torch.device):
        self.device = device

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def __enter__(self):
        self._sync()
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        self._sync()
        self.elapsed = time.perf_counter() - self.t0


def mfu(tokens_per_s_per_gpu: float, flops_per_token: float, peak: float = MI355X_BF16_DENSE_PEAK) -> float:
    return tokens_per_s_per_gpu * flops_per_token / peak


class MetricsLogger:
    def __init__(self, jsonl_path: Optional[str] = None, enabled: bool = True):
        self.enabled = enabled
        self.path = jsonl_path
        if enabled and jsonl_path:
            os.makedirs(os.path.dirname(os.path.abspath(jsonl_path)), exist_ok=True)

    def log(self, record: dict):
        if not self.enabled:
            return
        if self.path:
            with open(self.path, "a") as f:
                f.write(json.dumps(record) + "\n")


def peak_memory_gb(device: torch.device) -> float:
    if device.type == "cuda":
        return torch.cuda.max_memory_allocated(device) / 1e9
    return 0.0

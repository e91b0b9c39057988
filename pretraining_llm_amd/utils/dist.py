"""Process-group bootstrap: one process per GPU, env:// rendezvous (torchrun).

Reference: scripts/train_transformer.py:14-29 (``RANK`` in env -> DDP,
``init_process_group(backend=config['ddp_backend'])`` -- a KeyError as shipped,
SURVEY.md D1).  Here the backend defaults to ``"nccl"`` (= RCCL on ROCm) on GPUs
and ``"gloo"`` on CPU, a timeout is always set, and the device is bound before
the first collective so RCCL picks the right xGMI endpoints.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    enabled: bool
    rank: int
    local_rank: int
    world_size: int
    device: torch.device
    backend: str

    @property
    def is_master(self) -> bool:
        return self.rank == 0


def init_distributed(backend: str = "auto", device: str = "auto", timeout_s: int = 1800) -> DistInfo:
    env_dist = int(os.environ.get("RANK", -1)) != -1 and int(os.environ.get("WORLD_SIZE", 1)) >= 1
    rank = int(os.environ.get("RANK", 0))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    if device == "auto":
        device = "cuda" if torch.cuda.is_available() else "cpu"
    # Rehearsal switches for a multi-rank launch on a ONE-GPU box (functional only, never a
    # measurement): PLLM_DIST_BACKEND=gloo overrides the backend, PLLM_DIST_ONE_DEVICE=1 puts
    # every local rank on device 0 (RCCL itself refuses two ranks on one GPU).
    one_device = os.environ.get("PLLM_DIST_ONE_DEVICE", "0") == "1"
    backend = os.environ.get("PLLM_DIST_BACKEND", backend)
    if device.startswith("cuda"):
        idx = 0 if one_device else local_rank if env_dist else (torch.device(device).index or 0)
        dev = torch.device("cuda", idx)
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    if backend == "auto":
        backend = "nccl" if dev.type == "cuda" else "gloo"
    if env_dist and not dist.is_initialized():
        kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
        if dev.type == "cuda" and backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(**kw)
    return DistInfo(enabled=env_dist and world > 1, rank=rank, local_rank=local_rank, world_size=world,
                    device=dev, backend=backend)


def barrier():
    if dist.is_initialized():
        dist.barrier()


def destroy():
    if dist.is_initialized():
        dist.destroy_process_group()

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


# RCCL settings worth recording with every multi-GPU measurement (what ran, not what was meant)
_COMM_ENV_PREFIXES = ("NCCL_", "RCCL_", "TORCH_NCCL_", "HSA_NO_SCRATCH_RECLAIM", "HSA_ENABLE_IPC_MODE_LEGACY",
                      "GPU_MAX_HW_QUEUES")


def apply_rccl_env(channels=None, extra=None, overwrite: bool = True) -> dict:
    """Set RCCL's environment BEFORE the process group (communicator) is created.

    ``channels``: pin RCCL's channel count (``NCCL_MIN_NCHANNELS`` = ``NCCL_MAX_NCHANNELS``).  On
    MI355X every GPU has 7 point-to-point xGMI links (~153 GB/s each) to its 7 peers; one ring
    uses one outgoing link per GPU, so a large all-reduce needs several channels (rings) in flight
    to aggregate the links, while each channel's kernel occupies CUs that the overlapped backward
    wants.  ``None`` keeps RCCL's own choice (its topology tuner); scripts/gpu/rccl_sweep.sh sweeps
    it on an 8-GPU node.  ``extra``: any other ``NCCL_*`` / ``RCCL_*`` / ``TORCH_NCCL_*`` settings
    (e.g. ``{"TORCH_NCCL_HIGH_PRIORITY": "1"}``: RCCL's stream at high priority, so bucket
    all-reduces are dispatched ahead of queued backward kernels).  Returns the settings made."""
    made = {}
    if channels:
        made["NCCL_MIN_NCHANNELS"] = made["NCCL_MAX_NCHANNELS"] = str(int(channels))
    for k, v in (extra or {}).items():
        made[str(k)] = str(v)
    for k, v in made.items():
        if overwrite or k not in os.environ:
            os.environ[k] = v
    return made


def comm_env() -> dict:
    """The RCCL-relevant environment of this process (recorded in bench / metrics output)."""
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith(_COMM_ENV_PREFIXES)}


def parse_env_list(spec) -> dict:
    """``"A=1,B=2"`` (CLI) or a dict (config) -> dict."""
    if not spec:
        return {}
    if isinstance(spec, dict):
        return {str(k): str(v) for k, v in spec.items()}
    out = {}
    for item in str(spec).split(","):
        if item.strip():
            k, _, v = item.partition("=")
            out[k.strip()] = v.strip()
    return out


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

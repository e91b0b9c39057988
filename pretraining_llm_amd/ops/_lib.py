"""Loader for the in-tree gfx950 HIP extension (``pretraining_llm_amd/_C.so``).

The extension is built by ``pretraining_llm_amd/build.py`` with ``hipcc
--offload-arch=gfx950`` directly (no hipify, no cpp_extension JIT) and
registers its ops under ``torch.ops.pllm``.

Policy (no silent fallback on a GPU):
* bf16 CUDA(HIP) tensors always go to the HIP kernels (the hand-written kernels
  are bf16: the training compute dtype).  If the extension is missing when a GPU
  op is requested, ``require()`` raises.
* fp32 / fp16 CUDA tensors -- only the explicitly selected ``dtype='float32'`` and
  ``dtype='float16'`` (fp16 autocast + dynamic loss scaling) training modes make
  them -- run the PyTorch implementation of the op (hipBLASLt GEMMs through torch).
* CPU tensors use the pure-PyTorch reference implementation of the same op
  (which is also the numerics oracle for the tests).
"""
from __future__ import annotations

import os
import threading

import torch

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO_PATH = os.environ.get("PLLM_SO") or os.path.join(_HERE, "_C.so")  # PLLM_SO: A/B builds

_lock = threading.Lock()
_loaded = False
_err: str | None = None


def load(raise_on_error: bool = False) -> bool:
    global _loaded, _err
    if _loaded:
        return True
    with _lock:
        if _loaded:
            return True
        if not os.path.exists(SO_PATH):
            _err = f"HIP extension not built: {SO_PATH} missing (run `python -m pretraining_llm_amd.build`)"
        else:
            try:
                torch.ops.load_library(SO_PATH)
                from . import fake  # meta implementations for FakeTensor tracing (torch.compile)
                fake.register()
                from ..ab import ab
                # A/B (ab.py): weight-gradient kernel variant (csrc/gemm_wgrad.hip) and the hybrid
                # whole-tile + sliced-last-round split (csrc/wgrad_pp.hip) against uniform split-K slices
                if ab("wgrad_variant", -1) >= 0:
                    torch.ops.pllm.wgrad_set_mfma(ab("wgrad_variant", -1))
                if ab("wgrad_hy", -1) >= 0:
                    torch.ops.pllm.wgrad_set_hy(ab("wgrad_hy", -1))
                # PLLM_GEMM_RESERVE_CUS=n: CUs the persistent GEMM grids leave to concurrent RCCL kernels
                res = os.environ.get("PLLM_GEMM_RESERVE_CUS")
                per = ab("gemm_persistent", -1)  # 0|1: persistent GEMM grids
                if res or per >= 0:
                    torch.ops.pllm.gemm_set_config(0, 0, -1, int(res) if res else -1, per)
                _loaded = True
                _err = None
            except Exception as e:  # pragma: no cover - depends on the box
                _err = f"failed to load {SO_PATH}: {e}"
        if not _loaded and raise_on_error:
            raise RuntimeError(_err)
        return _loaded


def available() -> bool:
    return load(False)


def require():
    """Return the op namespace, raising loudly if the extension is unavailable."""
    if not _loaded:
        load(raise_on_error=True)
    return torch.ops.pllm


def use_hip(*tensors) -> bool:
    """True when the op must run on the HIP kernels: a CUDA/HIP tensor whose first
    floating-point CUDA operand is bf16 (integer-only operands: any CUDA tensor)."""
    cuda = False
    for t in tensors:
        if isinstance(t, torch.Tensor) and t.is_cuda:
            if t.is_floating_point():
                return t.dtype == torch.bfloat16
            cuda = True
    return cuda


def error() -> str | None:
    load(False)
    return _err

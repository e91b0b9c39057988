"""Fused ops with autograd: HIP (gfx950) kernels on GPU, PyTorch reference on CPU.

Every op here is a ``torch.autograd.Function`` whose forward/backward call
``torch.ops.pllm.*`` (hand-written HIP kernels in ``pretraining_llm_amd/csrc``)
when its inputs live on the GPU, and the reference in ``reference.py``
otherwise.  There is no third path: a GPU tensor with a missing extension
raises (see ``_lib.require``).

``set_backend("torch")`` forces stock PyTorch ops everywhere (SDPA attention,
F.layer_norm, F.cross_entropy in fp32 like the reference's autocast); it exists
only to measure the stock-PyTorch baseline on the same model and
is never selected implicitly.
"""
from __future__ import annotations

import contextlib
import math
import os
from typing import Optional

import torch
import torch.nn.functional as F

from . import _lib
from . import reference as ref

_BACKEND = "auto"   # auto -> HIP for GPU tensors, reference for CPU tensors; "torch" -> stock torch always


def set_backend(name: str):
    global _BACKEND
    assert name in ("auto", "torch"), name
    _BACKEND = name


def get_backend() -> str:
    return _BACKEND


@contextlib.contextmanager
def backend(name: str):
    old = _BACKEND
    set_backend(name)
    try:
        yield
    finally:
        set_backend(old)


def _hip(*ts) -> bool:
    return _BACKEND == "auto" and _lib.use_hip(*ts)


# Numerics bisection (diagnostic): PLLM_TORCH_OPS=attn,norm,act,ce,embed,linear runs the named op
# families through stock PyTorch ops while everything else stays on the HIP kernels
# (scripts/convergence.py compares the resulting loss curves against fp32).
_TORCH_OPS = frozenset(x for x in os.environ.get("PLLM_TORCH_OPS", "").split(",") if x)


def _hip_op(name: str, *ts) -> bool:
    return name not in _TORCH_OPS and _hip(*ts)


def _stock(name: str) -> bool:
    """True when op family ``name`` runs on stock torch ops (torch backend, or bisected out)."""
    return _BACKEND == "torch" or name in _TORCH_OPS


def _ops():
    return _lib.require()


# ---------------------------------------------------------------------------
# Direct gradient accumulation.  When the optimizer owns a flat gradient
# buffer (train/optim.py FlatAdamW marks its params ``_pllm_flat_grad``), the
# backward kernels/GEMMs ADD their weight gradients straight into
# ``p._pllm_gradbuf`` (a view of that buffer, fp32 by default: in-kernel
# read-add-write epilogues) instead of returning a fresh tensor that autograd's
# AccumulateGrad would then add in a separate pass.  ``_notify`` tells the
# data-parallel engine that a contribution landed (it replaces the
# post-accumulate-grad hook for these).
# ---------------------------------------------------------------------------
def _acc_target(p):
    """The flat-gradient slot a writer ADDS into.  A slot the optimizer left uncleared (lazy zeroing,
    ``FlatAdamW(lazy_zero=True)``: it expects an overwriting first write, see ``_set_target``) is
    zeroed here first, so every accumulating writer stays correct whatever runs first."""
    if p is None or not getattr(p, "_pllm_flat_grad", False):
        return None
    buf = getattr(p, "_pllm_gradbuf", None)
    if buf is not None and getattr(p, "_pllm_grad_fresh", False):
        p._pllm_grad_fresh = False
        buf.zero_()
    return buf


def _set_target(p):
    """(slot, overwrite) for a writer that produces a weight's whole gradient at once (the weight-
    gradient GEMMs): when the optimizer left the slot uncleared this step, the writer stores instead of
    adding -- no zero fill and no read of zeros (train/optim.py lazy zeroing)."""
    if p is None or not getattr(p, "_pllm_flat_grad", False):
        return None, False
    buf = getattr(p, "_pllm_gradbuf", None)
    fresh = buf is not None and getattr(p, "_pllm_grad_fresh", False)
    if fresh:
        p._pllm_grad_fresh = False
    return buf, fresh


def _notify(p):
    cb = getattr(p, "_pllm_grad_ready", None)
    if cb is not None:
        cb()


class _LinearFn(torch.autograd.Function):
    """y = x W^T + b on hipBLASLt; backward accumulates dW (beta=1 GEMM) and db in place.

    ``bias_grad_external``: the bias gradient is produced by the consumer's backward kernel
    (the next norm's dx column sums, or the activation backward), so this function leaves it
    alone instead of re-reading dy."""

    @staticmethod
    def forward(ctx, x, weight, bias, bias_grad_external, res=None):
        ctx.save_for_backward(x, weight)
        ctx.w, ctx.b = weight, bias
        ctx.bias_ext = bias_grad_external
        ctx.has_res = res is not None
        if res is not None:  # + the residual stream, added by the GEMM (resid_gemm_ok)
            N = weight.shape[0]
            # (gemm_lt takes contiguous operands only; reshape of a strided view can stay strided)
            return _ops().gemm_lt(x.reshape(-1, x.shape[-1]).contiguous(), weight, bias, 0,
                                  not torch.are_deterministic_algorithms_enabled(),
                                  res.reshape(-1, N))[0].view(*x.shape[:-1], N)
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = _dgrad(dy, weight)
        dy2 = dy.reshape(-1, dy.shape[-1])
        # the bias gradient rides along the weight-gradient GEMM when both go into flat targets
        btgt = None
        if (ctx.b is not None and ctx.needs_input_grad[2] and not ctx.bias_ext and ctx.needs_input_grad[1]
                and FUSED_WGRAD_BIAS):
            btgt = _acc_target(ctx.b)
        if ctx.needs_input_grad[1]:
            x2 = x.reshape(-1, x.shape[-1])
            tgt, fresh = _set_target(ctx.w)
            if tgt is None:
                btgt = None
            dw = _weight_grad(dy2, x2, tgt, btgt, overwrite=fresh)
            if tgt is not None:
                _notify(ctx.w)
        if btgt is not None:
            _notify(ctx.b)
        elif ctx.b is not None and ctx.needs_input_grad[2] and not ctx.bias_ext:
            tgt = _acc_target(ctx.b)
            if tgt is not None:
                _ops().bias_grad(dy2.contiguous(), tgt)
                _notify(ctx.b)
            else:
                db = _ops().bias_grad(dy2.contiguous())
        ctx.w = ctx.b = None
        return dx, dw, db, None, (dy if ctx.has_res else None)


import os as _os

from ..ab import ab as _ab

# weight-gradient GEMM engine: "hip" = hand-written split-K MFMA kernel (csrc/gemm_wgrad.hip),
# default: 824-1114 TFLOP/s at M=65536 vs 432-1003 for hipBLASLt's token-major "NT" kernels
# (bench/gemm_bench.py, profiles/r1_wgrad_v2_gemm_bench.jsonl); "blas" = hipBLASLt/rocBLAS
# through torch (beta=1 addmm into the flat gradient)
WGRAD_ENGINE = _os.environ.get("PLLM_WGRAD", "hip")
# (tokens M, P, Q) weight-gradient shapes where hipBLASLt measured faster than the hand-written
# kernel on MI355X (bench/gemm_bench.py --shapes llama --M 16384, profiles/r1_wgrad_plan_ab.jsonl):
# llama-1.3B at 8 x 2048 tokens -- QKV, MLP down projection and LM head
WGRAD_BLAS_SHAPES = {(16384, 6144, 2048), (16384, 2048, 5504), (16384, 50304, 2048)}


# (Weight gradients on a side HIP stream were measured and removed: +1.5 % on one box, -0.8 % on
# another, sporadic 2.5-3x slower runs; profiles/r1_wgrad_side_stream_ab.txt.)
# A linear layer's bias gradient computed inside its weight-gradient GEMM (csrc/gemm_wgrad.hip: MFMAs
# against an all-ones operand by the first Q-tile's workgroups) instead of a separate column-sum pass
# over dy (the GPT-2 QKV projection); PLLM_AB=wgrad_bias=0 for the separate pass
FUSED_WGRAD_BIAS = _ab("wgrad_bias", True)


def _dgrad(dy, weight):
    """dx = dy @ weight.  When the optimizer keeps a transposed shadow of the weight
    (FlatAdamW ``transposed_shadow``), the product runs as dy @ (W^T)^T: hipBLASLt's
    kernels for that operand layout are 10-15% faster at these shapes than for
    dy @ W (bench/gemm_fwd_bench.py: dgrad_nt vs dgrad_nn)."""
    wt = getattr(weight, "_pllm_wT", None)
    if wt is not None and getattr(weight, "_pllm_wT_ver", None) == weight._version:
        return dy @ wt.t()
    return dy @ weight


def _weight_grad(dy2, x2, tgt, btgt=None, overwrite: bool = False):
    """dW = dy2^T @ x2, added into ``tgt`` (bf16 or fp32) when given (returns None) else returned;
    ``overwrite``: stored into ``tgt`` instead (its first write of the step, ``_set_target``).
    ``btgt`` (with ``tgt``): the bias gradient (column sums of dy2) is added into it as well -- on the
    hand-written kernel inside the GEMM (its all-ones MFMAs), else by the bias_grad kernels."""
    hip_ok = dy2.shape[1] % 8 == 0 and x2.shape[1] % 8 == 0 and dy2.shape[0] % 64 == 0
    f32_tgt = tgt is not None and tgt.dtype == torch.float32 and dy2.dtype != torch.float32
    # an fp32 gradient target always takes the hand-written kernel (fp32 read-add-write epilogue)
    use_hip = hip_ok and (f32_tgt or (WGRAD_ENGINE == "hip" and
                                      (dy2.shape[0], dy2.shape[1], x2.shape[1]) not in WGRAD_BLAS_SHAPES))
    if use_hip:
        dy2, x2 = dy2.contiguous(), x2.contiguous()
        if tgt is not None:
            _ops().wgrad(dy2, x2, tgt.view(dy2.shape[1], x2.shape[1]), btgt, overwrite)
            return None
        return _ops().wgrad(dy2, x2)
    if btgt is not None:
        _ops().bias_grad(dy2.contiguous(), btgt)
    if tgt is not None:
        if f32_tgt:
            dw = (torch.mm(dy2.t(), x2, out_dtype=torch.float32) if dy2.is_cuda
                  else dy2.t().float() @ x2.float())
            tgt.copy_(dw.view_as(tgt)) if overwrite else tgt.add_(dw.view_as(tgt))
        elif overwrite:
            torch.mm(dy2.t(), x2, out=tgt.view(dy2.shape[1], x2.shape[1]))
        else:
            tgt.addmm_(dy2.t(), x2)
        return None
    return dy2.t() @ x2


def linear(x, weight, bias=None, bias_grad_external: bool = False, residual=None):
    """``residual`` (only when resid_gemm_ok holds -- the caller checks): x W^T + b + residual."""
    if _hip_op("linear", x) and torch.is_grad_enabled() and weight.requires_grad:
        # a bias gradient is left to the consumer's kernel only while that consumer (norm / act)
        # runs on the HIP kernels
        ext = bias_grad_external and bias is not None and not (_TORCH_OPS & {"norm", "act"})
        return _LinearFn.apply(x, weight, bias, ext, residual)
    if residual is not None:
        return F.linear(x, weight, bias) + residual
    if _hip(x) and not (torch.is_grad_enabled() and x.requires_grad):
        # decode-sized inference projections (<= 8 token rows): weight-streaming skinny GEMM
        # (csrc/gemv.hip) instead of the training-sized library tiles
        K = x.shape[-1]
        rows = x.numel() // K if K else 0
        if 0 < rows <= 8 and K % 8 == 0 and weight.is_contiguous() and _aligned16(weight):
            y = _ops().gemv(x.reshape(rows, K).contiguous(), weight, bias)[0]
            return y.view(*x.shape[:-1], weight.shape[0])
    return F.linear(x, weight, bias)


# ---------------------------------------------------------------------------
# MLP with the activation in the GEMM epilogues (csrc/gemm.hip)
# ---------------------------------------------------------------------------
def gemm_config(reserve_cus: Optional[int] = None, persistent: Optional[bool] = None) -> bool:
    """Configure the hand-written fused-epilogue TN GEMM (``torch.ops.pllm.gemm_tn``: the ping-pong main loop of
    csrc/gemm_pp.hip; shapes it does not take -- K < 128, the delta epilogue with T % 16 != 0 -- fall back to the
    round-3 persistent loop of csrc/gemm.hip): ``reserve_cus``: CUs its persistent grid leaves free (RCCL
    kernels run beside the backward at world > 1); ``persistent`` False: the ping-pong GEMM and weight-gradient
    kernels launch one workgroup per tile / work item instead of one per CU, so a CU held by a concurrent RCCL
    kernel delays no tile list (the hardware deals the tiles to the free CUs).  None keeps the current
    setting; returns False without the extension (CPU)."""
    if not _lib.available():
        return False
    torch.ops.pllm.gemm_set_config(0, 0, -1, -1 if reserve_cus is None else int(reserve_cus),
                                   -1 if persistent is None else int(bool(persistent)))
    return True


# PLLM_FUSED_MLP: "bwd" (default) = forward on hipBLASLt + the activation kernel, backward through
# the fused data-gradient epilogue (act' + b1's gradient: 476-480 vs 512 us per GPT-2 layer, bench/
# gemm_tn_bench.py); "all" = the forward activation in the GEMM epilogue too (its main loop is
# still slower than hipBLASLt's: 423-440 vs 408 us with the separate GELU pass); "0" = neither
_FM = _os.environ.get("PLLM_FUSED_MLP", "bwd")
FUSED_MLP = _FM in ("1", "all", "bwd")
FUSED_MLP_FWD = _FM in ("1", "all")
# PLLM_AB fused_swiglu_fwd=1|0: the llama up-projection with its SwiGLU in the GEMM epilogue (epilogue 7)
FUSED_SWIGLU_FWD = _ab("fused_swiglu_fwd", True)
# PLLM_AB lt_relu=1|0: the ReLU MLP's up-projection (reference architecture) with bias + ReLU in hipBLASLt's
# epilogue (csrc/blaslt.cpp) instead of the library GEMM + act_fwd pass (bench/gelu_epi_bench.py:
# 394 vs 494 us at the ref-3b shape).  GELU has no such path: the library build that ships with torch has
# no GELU epilogue with the pre-activation output the backward needs (HIPBLASLT_EPILOGUE_GELU_AUX*)
LT_RELU_FWD = _ab("lt_relu", True)


def fused_mlp_ok(x, w1, b1, w2, act: str) -> bool:
    """The fused path: GELU / ReLU MLPs with an up-projection bias on the HIP training path."""
    if not FUSED_MLP or act not in ("gelu", "relu") or b1 is None or not torch.is_grad_enabled():
        return False
    if not (_hip_op("linear", x) and _hip_op("act", x) and w1.requires_grad):
        return False
    C, Fh = x.shape[-1], w1.shape[0]
    return (C % 64 == 0 and Fh % 64 == 0 and x.numel() > 0 and tuple(w1.shape) == (Fh, C)
            and tuple(w2.shape) == (C, Fh) and w1.is_contiguous() and w2.is_contiguous()
            and _aligned16(w1) and _aligned16(w2) and b1.is_contiguous())


class _FusedMLPFn(torch.autograd.Function):
    """y = proj(act(hidden(x))) with the activation fused into the GEMM epilogues:

    forward   [pre,] a = act(x W1^T + b1)    one gemm_tn launch (GELU keeps the pre-activation);
                                             PLLM_FUSED_MLP=bwd: hipBLASLt + the activation kernel
              y = a W2^T + b2                hipBLASLt
    backward  dW2 += dy^T a, db2             (b2 skipped when the next norm emits it)
              da_pre = (dy W2) * act'(.)     one gemm_tn launch through W2's transposed shadow,
                                             + b1's gradient from the epilogue's column sums
              dx = da_pre W1, dW1 += da_pre^T x
    Gradient-ready notifications keep the unfused order (W2, b2, b1, W1) for the DP buckets.
    Reference: the MLP of /root/reference/src/models/mlp.py:24-26,39-41."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, gelu, out_bias_ext, res=None):
        C = x.shape[-1]
        x2 = x.reshape(-1, C)
        if not FUSED_MLP_FWD and not gelu and LT_RELU_FWD:
            # ReLU in hipBLASLt's own bias epilogue: one pass writes the activation (the
            # backward needs only its sign); relu commutes with the bf16 rounding, so the result
            # equals the separate pass
            a = _ops().gemm_lt(x2.contiguous(), w1, b1, 2, not torch.are_deterministic_algorithms_enabled())[0]
            ctx.save_for_backward(x2, a)
        elif not FUSED_MLP_FWD:
            pre = F.linear(x2, w1, b1)
            a = _ops().act_fwd(pre, 1 if gelu else 0)
            if gelu:
                ctx.save_for_backward(x2, a, pre)
            else:
                ctx.save_for_backward(x2, a)
        elif gelu:
            a, pre = _ops().gemm_tn(x2, w1, b1, 1)
            ctx.save_for_backward(x2, a, pre)
        else:
            a, _ = _ops().gemm_tn(x2, w1, b1, 2)
            ctx.save_for_backward(x2, a)
        ctx.gelu, ctx.ext = gelu, out_bias_ext
        ctx.params = (w1, b1, w2, b2)
        ctx.xshape = x.shape
        ctx.has_res = res is not None
        if res is not None:  # the block's residual stream added in the GEMM (one rounding, see resid_gemm_ok)
            return _ops().gemm_lt(a, w2, b2, 0, not torch.are_deterministic_algorithms_enabled(),
                                  res.reshape(-1, C))[0].view(*x.shape[:-1], C)
        return F.linear(a, w2, b2).view(*x.shape[:-1], C)

    @staticmethod
    def backward(ctx, dy):
        if ctx.gelu:
            x2, a, pre = ctx.saved_tensors
        else:
            x2, a = ctx.saved_tensors
            pre = a
        w1, b1, w2, b2 = ctx.params
        ctx.params = None
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        dw1 = db1 = dw2 = db2 = None
        # down projection: weight and bias gradients
        tgt, fresh = _set_target(w2)
        dw2 = _weight_grad(dy2, a, tgt, overwrite=fresh)
        if tgt is not None:
            _notify(w2)
        if b2 is not None and not ctx.ext:
            tgt = _acc_target(b2)
            if tgt is not None:
                _ops().bias_grad(dy2, tgt)
                _notify(b2)
            else:
                db2 = _ops().bias_grad(dy2)
        # its data gradient fused with the activation backward and b1's gradient
        w2t = getattr(w2, "_pllm_wT", None)
        if w2t is None or getattr(w2, "_pllm_wT_ver", None) != w2._version:
            w2t = w2.t().contiguous()
        tgt = _acc_target(b1)
        bacc = tgt if tgt is not None else torch.zeros(b1.shape[0], device=dy2.device, dtype=torch.float32)
        dpre = _ops().gemm_tn(dy2, w2t, None, 3 if ctx.gelu else 4, pre, bacc)[0]
        if tgt is not None:
            _notify(b1)
        else:
            db1 = bacc.to(b1.dtype)
        # up projection
        dx = _dgrad(dpre, w1) if ctx.needs_input_grad[0] else None
        tgt, fresh = _set_target(w1)
        dw1 = _weight_grad(dpre, x2, tgt, overwrite=fresh)
        if tgt is not None:
            _notify(w1)
        if dx is not None:
            dx = dx.view(ctx.xshape)
        return dx, dw1, db1, dw2, db2, None, None, (dy if ctx.has_res else None)


def fused_mlp(x, w1, b1, w2, b2, act: str, out_bias_ext: bool = False, residual=None):
    """``residual``: y + residual is returned (added by the down projection's GEMM, resid_gemm_ok)."""
    ext = bool(out_bias_ext and b2 is not None and not (_TORCH_OPS & {"norm", "act"}))
    return _FusedMLPFn.apply(x, w1, b1, w2, b2, act == "gelu", ext, residual)


# PLLM_AB resid_gemm=1|0: a block's residual add (reference: x = x + attn(ln1(x)); x = x + mlp(ln2(x)),
# /root/reference/src/models/transformer_block.py:44,46) done by its output projection's GEMM (hipBLASLt beta = 1,
# s = residual + x W^T + b in one rounding, csrc/blaslt.cpp gemm_lt) instead of by the next norm, which
# then reads one stream instead of two and writes one instead of two.  Round-4 measurement
# (profiles/r4_residual_in_gemm_negative.md): -3.9 / -15.9 us per GPT-2 layer (attention out / MLP down),
# -14.5 us at llama's attention output projection, but +105 us at its down projection (2048 x 5504: no fast
# beta = 1 solution among hipBLASLt's candidates), so weights of at most RESID_GEMM_MAX_W elements only.
# The size rule is a heuristic fitted to the measured shapes: its bound (4,194,304 = 2048 x 2048 = 1024 x 4096)
# admits exactly the measured-good ones among the presets -- GPT-2 small (768 x 768, 768 x 3072) and medium
# (1024 x 1024, 1024 x 4096) projections, llama's W_o (2048 x 2048) -- and none of the MLP downs of llama / ref-3b
# (2048 x 5504, 2048 x 8192) nor unmeasured mid-size ones (1024 x 5504, 1536 x 4096).  A new preset with a
# projection under the bound should have its beta = 1 GEMM re-measured (bench/residual_gemm_bench.py).
RESID_GEMM = _ab("resid_gemm", True)
RESID_GEMM_MAX_W = 2048 * 2048


def resid_gemm_ok(res, w) -> bool:
    return (RESID_GEMM and res is not None and torch.is_grad_enabled() and _hip(res) and not _TORCH_OPS
            and res.dtype == torch.bfloat16 and res.is_contiguous() and w.numel() <= RESID_GEMM_MAX_W
            and res.shape[-1] == w.shape[0] and w.shape[1] % 8 == 0)


def fused_swiglu_ok(x, w1, b1, w2, b2) -> bool:
    """The fused SwiGLU (llama) MLP: no biases, on the HIP training path (PLLM_FUSED_MLP != 0)."""
    if not FUSED_MLP or b1 is not None or b2 is not None or not torch.is_grad_enabled():
        return False
    if not (_hip_op("linear", x) and _hip_op("act", x) and w1.requires_grad):
        return False
    C, F2 = x.shape[-1], w1.shape[0]
    return (C % 64 == 0 and F2 % 16 == 0 and x.numel() > 0 and tuple(w1.shape) == (F2, C)
            and tuple(w2.shape) == (C, F2 // 2) and w1.is_contiguous() and w2.is_contiguous()
            and _aligned16(w1) and _aligned16(w2))


class _FusedSwiGLUMLPFn(torch.autograd.Function):
    """y = (silu(g) * u) W2^T with [g | u] = x W1^T (the llama MLP), the SwiGLU backward fused into
    the down-projection's data-gradient GEMM:

    forward   gu = x W1^T (hipBLASLt), a = swiglu(gu) (swiglu_fwd_kernel), y = a W2^T (hipBLASLt)
    backward  dW2 += dy^T a
              [dg | du] = swiglu'(gu, dy W2)   one gemm_tn launch (epilogue 5) through W2's
                                               transposed shadow: no swiglu_bwd pass over the
                                               [tokens, 2F] activations
              dx = [dg | du] W1, dW1 += [dg | du]^T x
    Same roundings as the unfused path (dy W2 rounded to bf16 before the SwiGLU backward).
    Reference MLP: /root/reference/src/models/mlp.py:24-26 (the llama preset's SwiGLU variant)."""

    @staticmethod
    def forward(ctx, x, w1, w2):
        C = x.shape[-1]
        x2 = x.reshape(-1, C)
        if FUSED_SWIGLU_FWD and _ops().gemm_uses_pp(C, 7):
            # the SwiGLU in the up-projection's epilogue (gemm_tn epilogue 7, ping-pong kernel):
            # no swiglu_fwd pass re-reading the [tokens, 2F] pre-activations
            a, gu = _ops().gemm_tn(x2, w1, None, 7)
        else:
            gu = F.linear(x2, w1)
            a = _ops().swiglu_fwd(gu)
        ctx.save_for_backward(x2, gu, a)
        ctx.params = (w1, w2)
        ctx.xshape = x.shape
        return F.linear(a, w2).view(*x.shape[:-1], C)

    @staticmethod
    def backward(ctx, dy):
        x2, gu, a = ctx.saved_tensors
        w1, w2 = ctx.params
        ctx.params = None
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        tgt, fresh = _set_target(w2)
        dw2 = _weight_grad(dy2, a, tgt, overwrite=fresh)
        if tgt is not None:
            _notify(w2)
        w2t = getattr(w2, "_pllm_wT", None)
        if w2t is None or getattr(w2, "_pllm_wT_ver", None) != w2._version:
            w2t = w2.t().contiguous()
        dgu = _ops().gemm_tn(dy2, w2t, None, 5, gu, None)[0]
        dx = _dgrad(dgu, w1) if ctx.needs_input_grad[0] else None
        tgt, fresh = _set_target(w1)
        dw1 = _weight_grad(dgu, x2, tgt, overwrite=fresh)
        if tgt is not None:
            _notify(w1)
        if dx is not None:
            dx = dx.view(ctx.xshape)
        return dx, dw1, dw2


def fused_swiglu_mlp(x, w1, w2):
    return _FusedSwiGLUMLPFn.apply(x, w1, w2)


_ACT_IDS = {None: 0, "gelu": 1, "relu": 2}


def _aligned16(t) -> bool:
    """16-byte alignment of a view, from its storage offset (allocations are 256-B aligned);
    unlike data_ptr() this is well-defined on FakeTensors (torch.compile tracing)."""
    return (t.storage_offset() * t.element_size()) % 16 == 0


def _gemv_ok(x, weight):
    K = x.shape[-1]
    rows = x.numel() // K if K else 0
    return (_hip(x) and not torch.is_grad_enabled() and 0 < rows <= 8 and K % 8 == 0
            and weight.is_contiguous() and _aligned16(weight))


def norm_linear(x, residual, norm_weight, norm_bias, eps: float, rms: bool, weight, bias=None,
                act: Optional[str] = None, kv=None):
    """Inference-only ``(act(norm(x + residual) @ weight^T + bias), x + residual)``.

    For decode-sized inputs (<= 8 token rows) on the HIP path this is ONE launch of the
    skinny-GEMM kernel with the norm as its prologue and the activation as its epilogue
    (csrc/gemv.hip): a decode block then runs no separate norm or activation kernels.
    Otherwise it is the unfused norm -> linear -> activation sequence.

    ``kv = (k_cache, v_cache, pos_t, q_cols)`` (decode QKV projection, caches [B, S_max, Hkv, D],
    ``pos_t`` int64 [1] on the device): output columns q_cols.. are also appended to the caches
    at position ``pos_t`` -- by the kernel's epilogue on the fused path."""
    if _gemv_ok(x, weight) and norm_weight.dtype == x.dtype:
        K = x.shape[-1]
        rows = x.numel() // K
        x2 = x.reshape(rows, K).contiguous()
        r2 = residual.reshape(rows, K).contiguous() if residual is not None else None
        kc = vc = pos = None
        q_cols = 0
        if kv is not None:
            kc, vc, pos, q_cols = kv
        out = _ops().gemv(x2, weight, bias, r2, norm_weight, None if rms else norm_bias, eps, int(rms),
                          _ACT_IDS[act], kc, vc, pos, q_cols)
        y = out[0].view(*x.shape[:-1], weight.shape[0])
        s = out[1].view(x.shape) if residual is not None else x
        return y, s
    if rms:
        h, s = rms_norm(x, norm_weight, eps, residual)
    else:
        h, s = layer_norm(x, norm_weight, norm_bias, eps, residual)
    y = linear(h, weight, bias)
    if act == "gelu":
        y = gelu(y)
    elif act == "relu":
        y = relu(y)
    if kv is not None:
        kc, vc, pos, q_cols = kv
        B, kvc = kc.shape[0], kc[0, 0].numel()
        y2 = y.reshape(B, -1)
        if pos.numel() > 1:  # one position per sequence (continuous batching)
            rows = torch.arange(B, device=pos.device)
            kc.index_put_((rows, pos), y2[:, q_cols:q_cols + kvc].reshape(B, *kc.shape[2:]))
            vc.index_put_((rows, pos), y2[:, q_cols + kvc:].reshape(B, *vc.shape[2:]))
        else:
            kc.index_copy_(1, pos, y2[:, q_cols:q_cols + kvc].reshape(B, 1, *kc.shape[2:]))
            vc.index_copy_(1, pos, y2[:, q_cols + kvc:].reshape(B, 1, *vc.shape[2:]))
    return y, s


# ---------------------------------------------------------------------------
# LayerNorm / RMSNorm with optional fused residual add
#   s = x + residual (if residual given);  y = norm(s) * w (+ b)
#   returns (y, s).  The backward adds the residual-stream gradient (ds from
#   the next layer) into dx in the same kernel.
# ---------------------------------------------------------------------------
class _NormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, eps, rms, x_bias):
        shp = x.shape
        C = shp[-1]
        x2 = x.reshape(-1, C)
        r2 = residual.reshape(-1, C) if residual is not None else None
        y, s, mean, rstd = _ops().norm_fwd(x2, r2, weight, bias, eps, rms)
        if residual is None:
            s = x2  # the op returns an empty s: the normalised stream is x itself
        ctx.save_for_backward(s, weight, mean, rstd)
        ctx.w, ctx.b, ctx.xb = weight, bias, x_bias
        ctx.has_bias = bias is not None
        ctx.has_res = residual is not None
        ctx.rms = rms
        ctx.shp = shp
        if residual is None:
            return y.view(shp), x  # s is x itself: hand the caller's tensor back
        return y.view(shp), s.view(shp)

    @staticmethod
    def backward(ctx, dy, ds):
        s, weight, mean, rstd = ctx.saved_tensors
        C = ctx.shp[-1]
        dy2 = dy.reshape(-1, C).contiguous()
        ds2 = ds.reshape(-1, C).contiguous() if ds is not None else None
        tw = _acc_target(ctx.w)
        tb = _acc_target(ctx.b) if ctx.has_bias else None
        txb = _acc_target(ctx.xb) if ctx.xb is not None else None
        direct = tw is not None and (not ctx.has_bias or tb is not None)
        dxb = None
        if direct:
            outs = (_ops().norm_bwd_acc(dy2, s, weight, mean, rstd, ds2, ctx.has_bias, ctx.rms, tw, tb, txb),)
            dw = db = None
            _notify(ctx.w)
            if ctx.has_bias:
                _notify(ctx.b)
            if txb is not None:
                _notify(ctx.xb)
        else:
            outs = _ops().norm_bwd(dy2, s, weight, mean, rstd, ds2, ctx.has_bias, ctx.rms)
            dw = outs[1]
            db = outs[2] if ctx.has_bias else None
            if txb is not None:
                _ops().bias_grad(outs[0], txb)
                _notify(ctx.xb)
        if ctx.xb is not None and txb is None:
            dxb = _ops().bias_grad(outs[0])
        ctx.w = ctx.b = ctx.xb = None
        dx = outs[0].view(ctx.shp)
        return dx, (dx if ctx.has_res else None), dw, db, None, None, dxb


def _norm_ref(x, residual, weight, bias, eps, rms):
    s = x if residual is None else x + residual
    if _stock("norm"):
        if rms:
            y = F.rms_norm(s, (s.shape[-1],), weight, eps)
        else:
            y = F.layer_norm(s, (s.shape[-1],), weight, bias, eps)
        return y, s
    if rms:
        y = ref.rms_norm(s, weight, eps)
    else:
        y = ref.layer_norm(s, weight, bias, eps)
    return y, s


def layer_norm(x, weight, bias, eps: float = 1e-5, residual: Optional[torch.Tensor] = None,
               x_bias: Optional[torch.Tensor] = None):
    """(LayerNorm(x + residual), x + residual).  ``x_bias``: the bias of the linear layer that
    produced ``x`` (created with ``bias_grad_external=True``); its gradient is the column sum of
    dx and is produced by this norm's backward kernel (HIP path)."""
    if _hip_op("norm", x):
        return _NormFn.apply(x.contiguous(), residual.contiguous() if residual is not None else None,
                             weight, bias, eps, False, x_bias)
    return _norm_ref(x, residual, weight, bias, eps, False)


def rms_norm(x, weight, eps: float = 1e-5, residual: Optional[torch.Tensor] = None,
             x_bias: Optional[torch.Tensor] = None):
    if _hip_op("norm", x):
        return _NormFn.apply(x.contiguous(), residual.contiguous() if residual is not None else None,
                             weight, None, eps, True, x_bias)
    return _norm_ref(x, residual, weight, None, eps, True)


# ---------------------------------------------------------------------------
# Flash attention on a packed QKV projection output.
#   qkv: [B, T, (H + 2*Hkv) * D]   ->  out [B, T, H*D]
# The HIP kernels read Q/K/V straight out of the packed GEMM output (strided
# views) and write dQ/dK/dV straight into a packed gradient buffer, so no
# split/cat copies exist on either side of the attention.
# ---------------------------------------------------------------------------
def _split_qkv(qkv, H, Hkv, D):
    B, T, _ = qkv.shape
    q = qkv[..., : H * D].view(B, T, H, D)
    k = qkv[..., H * D: (H + Hkv) * D].view(B, T, Hkv, D)
    v = qkv[..., (H + Hkv) * D:].view(B, T, Hkv, D)
    return q, k, v


class _FlashAttnPacked(torch.autograd.Function):
    """Attention over the packed QKV projection.  With ``cos``/``sin`` (RoPE) one pre-pass
    writes the rotated q and k heads to a [B, T, (H + Hkv) D] buffer that both the forward and
    the backward kernels read (kept for the backward: 2/3 of qkv for MHA); the backward kernels
    rotate dq / dk back while storing them, so the gradient comes back for the unrotated packed
    tensor.  Rotating inside the tile loops instead (rope_pre=False: tables read per tile)
    measured +22 % forward / +25 % backward at the llama shape (profiles/r2_rope_prepass_ab.txt)."""

    @staticmethod
    def forward(ctx, qkv, H, Hkv, causal, scale, cos, sin):
        B, T, W = qkv.shape
        D = W // (H + 2 * Hkv)
        q, k, v = _split_qkv(qkv, H, Hkv, D)
        qk = None
        if cos is not None and _ROPE_PREPASS:
            qk = _ops().rope_qk(qkv, cos, sin, H + 2 * Hkv, H + Hkv, T)
            q = qk[..., : H * D].view(B, T, H, D)
            k = qk[..., H * D:].view(B, T, Hkv, D)
            o, lse = _ops().attn_fwd(q, k, v, causal, scale)
        else:
            o, lse = _ops().attn_fwd(q, k, v, causal, scale, cos, sin)
        ctx.save_for_backward(qkv, qk, o, lse, cos, sin)
        ctx.cfg = (H, Hkv, D, causal, scale)
        return o.view(B, T, H * D)

    @staticmethod
    def backward(ctx, do):
        qkv, qk, o, lse, cos, sin = ctx.saved_tensors
        H, Hkv, D, causal, scale = ctx.cfg
        B, T, _ = qkv.shape
        q, k, v = _split_qkv(qkv, H, Hkv, D)
        if qk is not None:
            q = qk[..., : H * D].view(B, T, H, D)
            k = qk[..., H * D:].view(B, T, Hkv, D)
        dqkv = torch.empty_like(qkv)
        dq, dk, dv = _split_qkv(dqkv, H, Hkv, D)
        _attn_ws(qkv.device)
        _ops().attn_bwd(do.contiguous().view(B, T, H, D), q, k, v, o, lse, dq, dk, dv, causal, scale, cos, sin,
                        qk is None)
        return dqkv, None, None, None, None, None, None


class _AttnProjFn(torch.autograd.Function):
    """``attention_packed`` followed by the output projection y = O W_o^T (+ b_o).  The backward runs
    the projection's data gradient through the fused-epilogue GEMM (csrc/gemm.hip epilogue 6), which
    also emits the attention backward's row constants delta = rowsum(dO * O) per (batch, head,
    query) while dO is in registers, so the attn_bwd_pre_kernel pass over dO and O is gone.  Head
    dim 64 (a wave's 64 output columns are one head).  Same math as _FlashAttnPacked + _LinearFn."""

    @staticmethod
    def forward(ctx, qkv, H, Hkv, causal, scale, cos, sin, w, b, bias_ext, res=None):
        B, T, W = qkv.shape
        D = W // (H + 2 * Hkv)
        q, k, v = _split_qkv(qkv, H, Hkv, D)
        qk = None
        if cos is not None and _ROPE_PREPASS:
            qk = _ops().rope_qk(qkv, cos, sin, H + 2 * Hkv, H + Hkv, T)
            q = qk[..., : H * D].view(B, T, H, D)
            k = qk[..., H * D:].view(B, T, Hkv, D)
            o, lse = _ops().attn_fwd(q, k, v, causal, scale)
        else:
            o, lse = _ops().attn_fwd(q, k, v, causal, scale, cos, sin)
        ctx.save_for_backward(qkv, qk, o, lse, cos, sin)
        ctx.cfg = (H, Hkv, D, causal, scale)
        ctx.w, ctx.b, ctx.bias_ext = w, b, bias_ext
        ctx.has_res = res is not None
        if res is not None:  # the block's residual stream added in the GEMM (resid_gemm_ok)
            C = w.shape[0]
            return _ops().gemm_lt(o.view(B * T, H * D), w, b, 0, not torch.are_deterministic_algorithms_enabled(),
                                  res.reshape(-1, C))[0].view(B, T, C)
        return F.linear(o.view(B, T, H * D), w, b)

    @staticmethod
    def backward(ctx, dy):
        qkv, qk, o, lse, cos, sin = ctx.saved_tensors
        H, Hkv, D, causal, scale = ctx.cfg
        w, b = ctx.w, ctx.b
        ctx.w = ctx.b = None
        B, T, _ = qkv.shape
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        o2 = o.view(B * T, H * D)
        # projection weight / bias gradients (as _LinearFn.backward)
        dw = db = None
        need_b = b is not None and ctx.needs_input_grad[8] and not ctx.bias_ext
        if ctx.needs_input_grad[7]:
            tgt, fresh = _set_target(w)
            btgt = _acc_target(b) if (need_b and tgt is not None and FUSED_WGRAD_BIAS) else None
            dw = _weight_grad(dy2, o2, tgt, btgt, overwrite=fresh)
            if tgt is not None:
                _notify(w)
            if btgt is not None:
                _notify(b)
                need_b = False
        if need_b:
            bt = _acc_target(b)
            if bt is not None:
                _ops().bias_grad(dy2, bt)
                _notify(b)
            else:
                db = _ops().bias_grad(dy2)
        # dO and delta from one GEMM through W_o's transposed shadow
        wt = getattr(w, "_pllm_wT", None)
        if wt is None or getattr(w, "_pllm_wT_ver", None) != w._version:
            wt = w.t().contiguous()
        do2, delta = _ops().gemm_tn(dy2, wt, None, 6, o2, None, T)
        q, k, v = _split_qkv(qkv, H, Hkv, D)
        if qk is not None:
            q = qk[..., : H * D].view(B, T, H, D)
            k = qk[..., H * D:].view(B, T, Hkv, D)
        dqkv = torch.empty_like(qkv)
        dq, dk, dv = _split_qkv(dqkv, H, Hkv, D)
        _attn_ws(qkv.device)
        _ops().attn_bwd(do2.view(B, T, H, D), q, k, v, o, lse, dq, dk, dv, causal, scale, cos, sin, qk is None,
                        delta)
        return dqkv, None, None, None, None, None, None, dw, db, None, (dy if ctx.has_res else None)


# PLLM_AB attn_proj_fused=0: the output projection's backward on hipBLASLt + the attention's delta pre-pass
FUSED_ATTN_PROJ = _ab("attn_proj_fused", True)
# head dims served by it: 64.  (D = 128 -- two 64-column delta halves per head -- measured 0.5 % slower on
# llama-1.3B, profiles/r4_attn_experiments.md, and was removed: the D = 128 backward, csrc/attn_bwd_ks.hip,
# forms delta itself)
ATTN_PROJ_HEAD_DIMS = (64,)


def attn_proj_ok(qkv, n_head: int, n_kv_head: int, w, b) -> bool:
    """The fused attention + output projection path (_AttnProjFn): HIP training path, head dim 64."""
    if not FUSED_ATTN_PROJ or not torch.is_grad_enabled() or not (_hip_op("attn", qkv) and _hip_op("linear", qkv)):
        return False
    B, T, W = qkv.shape
    D = W // (n_head + 2 * n_kv_head)
    C_out = w.shape[0]
    return (D in ATTN_PROJ_HEAD_DIMS and B * T > 0 and tuple(w.shape) == (C_out, n_head * D) and C_out % 64 == 0
            and w.is_contiguous() and _aligned16(w) and (b is None or b.is_contiguous()))


def attention_proj(qkv, n_head: int, n_kv_head: int, w, b, causal: bool = True, scale: Optional[float] = None,
                   rope_cos=None, rope_sin=None, bias_grad_external: bool = False, residual=None):
    """``linear(attention_packed(qkv, ...), w, b)`` (+ ``residual``, added by the GEMM) with the fused
    backward (see _AttnProjFn)."""
    D = qkv.shape[-1] // (n_head + 2 * n_kv_head)
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    ext = bool(bias_grad_external and b is not None and not (_TORCH_OPS & {"norm", "act"}))
    return _AttnProjFn.apply(qkv, n_head, n_kv_head, causal, scale, rope_cos, rope_sin, w, b, ext, residual)


_ATTN_WS_MB = [None]


def _attn_ws(device):
    """Attention-backward dQ slab budget from the HBM still free (utils/memory.py: a quarter of
    it, capped at the 4 GiB that keeps every shipped config in one pass, floored at 64 MiB),
    quantised to 256 MiB steps so it is re-sent to the extension only when it moves;
    PLLM_ATTN_BWD_WS_MB fixes it instead."""
    if "PLLM_ATTN_BWD_WS_MB" in os.environ:
        return
    from ..utils import memory as _mem
    b = _mem.workspace_budget(device, _mem.ATTN_WS_CAP, _mem.ATTN_WS_FRACTION, _mem.ATTN_WS_FLOOR)
    mb = max(64.0, float(b // (256 * _mem.MiB) * 256))
    if mb != _ATTN_WS_MB[0]:
        _ops().attn_bwd_set_workspace_mb(mb)
        _ATTN_WS_MB[0] = mb


# RoPE for the HIP attention: pre-pass rotation (default) or rotation inside the kernels' tile loops
_ROPE_PREPASS = _ab("rope_prepass", True)


class _RopePackedFn(torch.autograd.Function):
    """Rotate the q and k heads of a packed qkv tensor (rotate-half convention)."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, H, Hkv):
        B, T, W = qkv.shape
        out = _ops().rope(qkv.contiguous(), cos, sin, H + 2 * Hkv, H + Hkv, T, 0, False)
        ctx.save_for_backward(cos, sin)
        ctx.cfg = (H, Hkv, T)
        return out

    @staticmethod
    def backward(ctx, dout):
        cos, sin = ctx.saved_tensors
        H, Hkv, T = ctx.cfg
        d = _ops().rope(dout.contiguous(), cos, sin, H + 2 * Hkv, H + Hkv, T, 0, True)
        return d, None, None, None, None


def rope_packed(qkv, cos, sin, n_head: int, n_kv_head: int):
    if _hip(qkv):
        return _RopePackedFn.apply(qkv, cos, sin, n_head, n_kv_head)
    B, T, W = qkv.shape
    D = W // (n_head + 2 * n_kv_head)
    q, k, v = _split_qkv(qkv, n_head, n_kv_head, D)
    q = ref.rope(q, cos[:T], sin[:T])
    k = ref.rope(k, cos[:T], sin[:T])
    return torch.cat([q.reshape(B, T, -1), k.reshape(B, T, -1), v.reshape(B, T, -1)], -1)


def attention_packed(qkv, n_head: int, n_kv_head: int, causal: bool = True, scale: Optional[float] = None,
                     rope_cos: Optional[torch.Tensor] = None, rope_sin: Optional[torch.Tensor] = None):
    """Causal self-attention over a packed qkv tensor. RoPE (if cos/sin given) is
    applied to the q and k heads first (rotate-half convention)."""
    B, T, W = qkv.shape
    D = W // (n_head + 2 * n_kv_head)
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if _hip_op("attn", qkv):
        # RoPE fused into the attention kernels (q/k rotated while staged, dq/dk rotated back)
        return _FlashAttnPacked.apply(qkv, n_head, n_kv_head, causal, scale, rope_cos, rope_sin)
    if rope_cos is not None:
        qkv = rope_packed(qkv, rope_cos, rope_sin, n_head, n_kv_head)
    q, k, v = _split_qkv(qkv, n_head, n_kv_head, D)
    if _stock("attn") and qkv.is_cuda:
        # stock-PyTorch baseline path (SDPA), used only by the explicit torch backend
        qh, kh, vh = (t.transpose(1, 2) for t in (q, k, v))
        o = F.scaled_dot_product_attention(qh, kh, vh, is_causal=causal, scale=scale,
                                           enable_gqa=(n_kv_head != n_head))
        return o.transpose(1, 2).reshape(B, T, n_head * D)
    o, _ = ref.attention(q, k, v, causal=causal, scale=scale)
    return o.reshape(B, T, n_head * D)


def attention(q, k, v, causal: bool = True, scale: Optional[float] = None, return_lse: bool = False):
    """Unpacked attention q [B,T,H,D], k/v [B,S,Hkv,D] (forward only; used by the
    KV-cache decode and context-parallel paths).  Queries are aligned to the end
    of the key sequence."""
    D = q.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if _hip(q) and q.shape[1] == 1 and not return_lse and q.shape[2] // k.shape[2] in (1, 2, 4, 8):
        # one query per sequence (KV-cache decode): split-KV streaming kernel (csrc/attn_decode.hip)
        return _ops().attn_decode(q, k, v, scale)
    if _hip(q):
        o, lse = _ops().attn_fwd(q, k, v, causal, scale)
    else:
        o, lse = ref.attention(q, k, v, causal=causal, scale=scale)
    return (o, lse) if return_lse else o


def attention_decode(q, k, v, seqlen: Optional[torch.Tensor] = None, scale: Optional[float] = None):
    """Single-query attention q [B,1,H,D] over cached k/v [B,S,Hkv,D]; ``seqlen`` (int32 [1]
    device tensor) optionally limits the keys to the first ``seqlen`` rows, read on the
    device so a captured decode step (hipGraph) replays at every position."""
    D = q.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if _hip(q):
        return _ops().attn_decode(q, k, v, scale, seqlen)
    if seqlen is not None and seqlen.numel() > 1:  # one key count per sequence
        return torch.cat([ref.attention(q[b:b + 1], k[b:b + 1, :int(n)], v[b:b + 1, :int(n)], causal=False,
                                        scale=scale)[0] for b, n in enumerate(seqlen.tolist())])
    if seqlen is not None:
        n = int(seqlen.item())
        k, v = k[:, :n], v[:, :n]
    o, _ = ref.attention(q, k, v, causal=False, scale=scale)
    return o


def attention_block_bwd(do, q, k, v, o, lse, causal: bool = True, scale: Optional[float] = None):
    """Backward of one (query block, key block) attention product given the final output
    ``o`` and the log-sum-exp ``lse`` [B,H,T] of the WHOLE softmax row (context-parallel
    building block).  Returns (dq, dk, dv) in the dtype of q (HIP) or fp32 (CPU oracle)."""
    D = q.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if _hip(q):
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        _attn_ws(q.device)
        _ops().attn_bwd(do, q, k, v, o, lse.contiguous(), dq, dk, dv, causal, scale)
        return dq, dk, dv
    return ref.attention_bwd(do, q, k, v, o, lse, causal=causal, scale=scale)


# ---------------------------------------------------------------------------
# activations (op ids of the HIP act kernels: 0 relu, 1 gelu-tanh)
# ---------------------------------------------------------------------------
class _GeluFn(torch.autograd.Function):
    """GELU(tanh); with ``bias`` (the producing linear's bias, created with
    bias_grad_external=True) the backward kernel also emits that bias's gradient."""

    @staticmethod
    def forward(ctx, x, bias):
        ctx.save_for_backward(x)
        ctx.b = bias
        return _ops().act_fwd(x, 1)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = dy.contiguous()
        b, ctx.b = ctx.b, None
        if b is None:
            return _ops().act_bwd(dy, x, 1), None
        tgt = _acc_target(b)
        if tgt is not None:
            dx = _ops().act_bwd_bias(dy, x, 1, tgt)
            _notify(b)
            return dx, None
        dx = _ops().act_bwd(dy, x, 1)
        return dx, _ops().bias_grad(dx)


class _ReluFn(torch.autograd.Function):
    """ReLU (reference MLP activation); optional fused bias gradient like _GeluFn."""

    @staticmethod
    def forward(ctx, x, bias):
        y = _ops().act_fwd(x, 0)
        ctx.save_for_backward(y)
        ctx.b = bias
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dy = dy.contiguous()
        b, ctx.b = ctx.b, None
        if b is None:
            return _ops().act_bwd(dy, y, 0), None
        tgt = _acc_target(b)
        if tgt is not None:
            dx = _ops().act_bwd_bias(dy, y, 0, tgt)
            _notify(b)
            return dx, None
        dx = _ops().act_bwd(dy, y, 0)
        return dx, _ops().bias_grad(dx)


class _SwigluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        ctx.save_for_backward(gu)
        return _ops().swiglu_fwd(gu)

    @staticmethod
    def backward(ctx, dy):
        (gu,) = ctx.saved_tensors
        return _ops().swiglu_bwd(dy.contiguous(), gu)


def gelu(x, bias: Optional[torch.Tensor] = None):
    if _hip_op("act", x):
        return _GeluFn.apply(x.contiguous(), bias)
    if _stock("act"):
        return F.gelu(x, approximate="tanh")
    return ref.gelu_tanh(x)


def swiglu(gate_up):
    if _hip_op("act", gate_up):
        return _SwigluFn.apply(gate_up.contiguous())
    return ref.swiglu(gate_up)


def relu(x, bias: Optional[torch.Tensor] = None):
    if _hip_op("act", x):
        return _ReluFn.apply(x.contiguous(), bias)
    return ref.relu(x)


# ---------------------------------------------------------------------------
# Embedding (token + optional learned position), deterministic backward
# ---------------------------------------------------------------------------
class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, wte, wpe):
        x = _ops().embedding_fwd(idx, wte, wpe, 0)
        ctx.save_for_backward(idx)
        ctx.V = wte.shape[0]
        ctx.n_pos = 0 if wpe is None else wpe.shape[0]
        ctx.wte, ctx.wpe = wte, wpe
        return x

    @staticmethod
    def backward(ctx, dx):
        (idx,) = ctx.saved_tensors
        has_pos = ctx.n_pos > 0
        tt = _acc_target(ctx.wte)
        tp = _acc_target(ctx.wpe) if has_pos else None
        if tt is not None and (not has_pos or tp is not None):
            _ops().embedding_bwd_acc(dx.contiguous(), idx, ctx.V, ctx.n_pos, has_pos, tt, tp)
            _notify(ctx.wte)
            if has_pos:
                _notify(ctx.wpe)
            ctx.wte = ctx.wpe = None
            return None, None, None
        ctx.wte = ctx.wpe = None
        outs = _ops().embedding_bwd(dx.contiguous(), idx, ctx.V, ctx.n_pos, has_pos)
        return None, outs[0], (outs[1] if has_pos else None)


def embedding(idx, wte, wpe=None, pos_offset: int = 0):
    if _hip_op("embed", wte):
        if pos_offset:
            return _ops().embedding_fwd(idx.contiguous(), wte, wpe, pos_offset)
        return _EmbeddingFn.apply(idx.contiguous(), wte, wpe)
    return ref.embedding(idx, wte, wpe, pos_offset)


# ---------------------------------------------------------------------------
# LM head + fused cross entropy, chunked over rows.
# The reference materialises [B*T, V] fp32 logits and a softmax (transformer.py:71-77:
# 3+ GiB at its own config).  Here the rows are processed in chunks of CE_CHUNK_ROWS:
# per chunk the LM-head GEMM writes bf16 logits into ONE reused [rows, V] workspace, the
# HIP CE kernel turns them in place into dlogits (never storing probabilities), and the
# two backward GEMMs (dh = dlogits W, dW += dlogits^T h) plus the head-bias column sums
# run right away on the same workspace while it is hot.  Nothing logits-sized outlives a
# chunk; the backward only scales the saved dh / fp32 dW / db by the upstream gradient.
# ---------------------------------------------------------------------------
# Chunk size: the fewest equal chunks (multiples of 64 rows) whose bf16 logits workspace fits
# CE_WORKSPACE_MB, or exactly CE_CHUNK_ROWS rows when that is set.  Measured on MI355X
# (GPT-2 small, 65,536 rows x 50,304, profiles/r2_ce_chunk_sweep.jsonl): 63.4 ms/step unchunked
# (29.9 GB peak) vs 64.5 / 65.3 / 70.6 / 73.8 ms at 16K / 8K / 4K / 2K rows (24.8-23.1 GB): the
# backward GEMMs lose efficiency at small M, so the default budget (8 GiB) keeps every shipped
# config in one chunk and only bounds the workspace when batch x vocab grows past it.  Also
# measured slower: sub-chunks of 1K / 2K / 4K rows for GEMM -> CE -> dgrad (logits kept in the
# Infinity Cache between them) with one weight-gradient GEMM over the whole dlogits afterwards:
# 75.7 / 68.5 / 66.6 ms vs 60.5 ms per step (scripts/gpu/r2_cesub.sh, profiles/r2_ce_subchunk_negative.txt).
# The workspace budget is a quarter of the HBM the device can still give (utils/memory.py),
# capped at those 8 GiB and floored at 256 MiB; PLLM_CE_WORKSPACE_MB fixes it instead.
CE_CHUNK_ROWS = _ab("ce_chunk_rows", 0)
CE_WORKSPACE_MB = float(_os.environ["PLLM_CE_WORKSPACE_MB"]) if "PLLM_CE_WORKSPACE_MB" in _os.environ else None


def _ce_budget_bytes(device) -> int:
    if CE_WORKSPACE_MB is not None:
        return int(CE_WORKSPACE_MB * 2 ** 20)
    from ..utils import memory as _mem
    return _mem.workspace_budget(device, _mem.CE_CAP, _mem.CE_FRACTION, _mem.CE_FLOOR)


def _ce_chunk_rows(N: int, V: int = 50304, budget_bytes: Optional[int] = None) -> int:
    if CE_CHUNK_ROWS > 0:
        r = max(64, CE_CHUNK_ROWS // 64 * 64)
        return N if N <= r else r
    per_row = 2 * V
    budget = budget_bytes if budget_bytes is not None else 8192 * 2 ** 20
    n_chunks = max(1, math.ceil(N * per_row / budget))
    if n_chunks == 1:
        return N
    return max(64, (math.ceil(N / n_chunks) + 63) // 64 * 64)


class _LMHeadCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, weight, bias, targets, ignore_index):
        N, C = h.shape
        V = weight.shape[0]
        n_valid = (targets != ignore_index).sum().clamp_min(1)
        inv_n = n_valid.to(torch.float32).reciprocal().reshape(1)
        need_h = ctx.needs_input_grad[0]
        need_w = ctx.needs_input_grad[1]
        need_b = bias is not None and ctx.needs_input_grad[2]
        R = _ce_chunk_rows(N, V, _ce_budget_bytes(h.device))
        ws = torch.empty(R, V, dtype=h.dtype, device=h.device)
        dh = torch.empty_like(h) if need_h else None
        # the first chunk's weight gradient stores into dw (no zero fill, no read of zeros), later ones add.
        # When the weight's flat-gradient slot is untouched this step (lazy zeroing: the first writer
        # overwrites) the chunks write straight into that slot and the backward only scales it in place by
        # the upstream gradient -- a no-op launch when that is 1 -- instead of a 154 MB fp32 buffer copied and
        # scaled into the slot (GPT-2 small: ~55 us per step).  A slot already holding gradient (accumulation
        # micro-steps) keeps the separate buffer: the scale applies to this micro-step's part only.
        direct = None
        if need_w:
            tgt, fresh = _set_target(weight)
            if tgt is not None and fresh and tgt.dtype == torch.float32 and tgt.is_contiguous():
                direct = tgt
        dw = (direct.view(V, C) if direct is not None else
              torch.empty(V, C, dtype=torch.float32, device=h.device)) if need_w else None
        db = torch.zeros(V, dtype=torch.float32, device=h.device) if need_b else None
        rows = torch.empty(N, dtype=torch.float32, device=h.device)
        wt = getattr(weight, "_pllm_wT", None)
        wt = wt if wt is not None and getattr(weight, "_pllm_wT_ver", None) == weight._version else None
        for r0 in range(0, N, R):
            r1 = min(N, r0 + R)
            hc, lg = h[r0:r1], ws[:r1 - r0]
            if bias is not None:
                torch.addmm(bias, hc, weight.t(), out=lg)
            else:
                torch.mm(hc, weight.t(), out=lg)
            rows[r0:r1] = _ops().cross_entropy(lg, targets[r0:r1], lg, ignore_index, inv_n)
            if need_h:  # dh = dlogits @ W (through the W^T shadow when present, see _dgrad)
                torch.mm(lg, wt.t() if wt is not None else weight, out=dh[r0:r1])
            if need_w:
                _weight_grad(lg, hc, dw, overwrite=r0 == 0)
            if need_b:
                _ops().bias_grad(lg, db)
        ctx.direct = direct is not None
        ctx.save_for_backward(dh, None if ctx.direct else dw, db)
        ctx.w, ctx.b = weight, bias
        ctx.wdtype = weight.dtype
        return rows.sum() * inv_n[0]

    @staticmethod
    def backward(ctx, dloss):
        dh, dw, db = ctx.saved_tensors
        g = dloss.to(torch.float32).reshape(())
        gh = None
        if dh is not None:
            if dh.is_cuda and dh.numel() % 8 == 0 and _lib.available():
                _ops().scale_(dh, g.reshape(1))  # (no pass when g == 1)
                gh = dh
            else:
                gh = dh.mul_(g.to(dh.dtype))
        gw = gb = None
        if ctx.direct:  # the weight gradient is already in its flat slot: scale it there (no-op when g == 1)
            slot = getattr(ctx.w, "_pllm_gradbuf")
            _ops().scale_(slot.view(-1), g.reshape(1))
            _notify(ctx.w)
        elif dw is not None:
            tgt, fresh = _set_target(ctx.w)
            if tgt is not None:
                if fresh:
                    torch.mul(dw.view(-1), g, out=tgt.view(-1))
                else:
                    tgt.view(-1).addcmul_(dw.view(-1), g)
                _notify(ctx.w)
            else:
                gw = dw.mul_(g).to(ctx.wdtype)
        if db is not None:
            tgt = _acc_target(ctx.b)
            if tgt is not None:
                tgt.addcmul_(db, g)
                _notify(ctx.b)
            else:
                gb = db.mul_(g).to(ctx.wdtype)
        ctx.w = ctx.b = None
        return gh, gw, gb, None, None


def lm_head_cross_entropy(h, weight, bias, targets, ignore_index: int = -100):
    """mean CE of ``h @ weight^T + bias`` against ``targets`` without returning logits
    (chunked over rows on the HIP path: no [N, V] buffer in training or evaluation)."""
    targets = targets.reshape(-1)
    h = h.reshape(-1, h.shape[-1])
    if _hip_op("ce", h) and torch.is_grad_enabled() and (h.requires_grad or weight.requires_grad):
        return _LMHeadCEFn.apply(h, weight, bias, targets, ignore_index)
    if _hip_op("ce", h):
        N, V = h.shape[0], weight.shape[0]
        R = _ce_chunk_rows(N, V, _ce_budget_bytes(h.device))
        ws = torch.empty(R, V, dtype=h.dtype, device=h.device)
        rows = torch.empty(N, dtype=torch.float32, device=h.device)
        for r0 in range(0, N, R):
            r1 = min(N, r0 + R)
            lg = ws[:r1 - r0]
            if bias is not None:
                torch.addmm(bias, h[r0:r1], weight.t(), out=lg)
            else:
                torch.mm(h[r0:r1], weight.t(), out=lg)
            rows[r0:r1] = _ops().cross_entropy(lg, targets[r0:r1], None, ignore_index)
        return rows.sum() / (targets != ignore_index).sum().clamp_min(1)
    logits = F.linear(h, weight, bias)
    return cross_entropy(logits, targets, ignore_index)


def cross_entropy(logits, targets, ignore_index: int = -100):
    """Mean token cross-entropy over ``logits [N, V]`` (no in-place tricks)."""
    targets = targets.reshape(-1)
    if _hip(logits) and not (torch.is_grad_enabled() and logits.requires_grad):
        rows = _ops().cross_entropy(logits.contiguous(), targets, None, ignore_index)
        return rows.sum() / (targets != ignore_index).sum().clamp_min(1)
    return ref.cross_entropy(logits, targets, ignore_index)


# ---------------------------------------------------------------------------
# misc
# ---------------------------------------------------------------------------
def rope_cache(seq_len: int, head_dim: int, theta: float, device):
    cos, sin = ref.rope_cos_sin(seq_len, head_dim, theta, device=device)
    return cos.contiguous(), sin.contiguous()


def apply_rope(x, cos, sin, pos_offset: int = 0):
    """x [B,T,H,D] -> rotated copy (no autograd; used by decode). cos/sin index from pos_offset."""
    if _hip(x):
        B, T, H, D = x.shape
        y = _ops().rope(x.contiguous().view(B, T, H * D), cos, sin, H, H, T, pos_offset, False)
        return y.view(B, T, H, D)
    T = x.shape[1]
    return ref.rope(x, cos[pos_offset:pos_offset + T], sin[pos_offset:pos_offset + T])

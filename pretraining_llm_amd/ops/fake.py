"""Fake (meta) implementations of every ``torch.ops.pllm`` op.

They describe each HIP kernel's outputs (shape, dtype, device) without running it, which is
what FakeTensor tracing -- ``torch.compile`` / ``torch.export`` / AOTAutograd, the reference's
``TORCH_COMPILE`` path (scripts/train_transformer.py:31-33,118-120) -- needs to trace a model
built on these ops.  Ops that only mutate their ``(a!)`` arguments
return nothing or fresh tensors: no op output aliases an input (bindings.cpp), so
functionalization can reason about them.  Registered once, right after the extension loads
(``_lib.load``); ``torch.library.opcheck`` cross-checks them against the real kernels on the
GPU (tests/test_compile_gpu.py).
"""
from __future__ import annotations

import torch

_REGISTERED = False


def _reg(name):
    return torch.library.register_fake(f"pllm::{name}")


def register() -> None:
    global _REGISTERED
    if _REGISTERED:
        return
    _REGISTERED = True
    f32 = torch.float32

    @_reg("norm_fwd")
    def _(x, residual, weight, bias, eps, rms):
        N = x.shape[0]
        s = torch.empty_like(x) if residual is not None else x.new_empty((0,))
        return [torch.empty_like(x), s, x.new_empty((N,), dtype=f32), x.new_empty((N,), dtype=f32)]

    @_reg("norm_bwd")
    def _(dy, s, weight, mean, rstd, ds, has_bias, rms):
        C = dy.shape[1]
        return (torch.empty_like(dy), weight.new_empty((C,)), weight.new_empty((C,) if has_bias else (0,)))

    @_reg("norm_bwd_acc")
    def _(dy, s, weight, mean, rstd, ds, has_bias, rms, dw_acc, db_acc=None, xb_acc=None):
        return torch.empty_like(dy)

    @_reg("bias_grad")
    def _(dy, out_acc=None):
        if out_acc is not None:
            return dy.new_empty((0,))
        return dy.new_empty((dy.shape[-1],))

    @_reg("wgrad")
    def _(dy, x, out_acc=None, bias_acc=None, overwrite=False):
        if out_acc is not None:
            return dy.new_empty((0,))
        return dy.new_empty((dy.shape[1], x.shape[1]))

    @_reg("zero_ranges_")
    def _(buf, ranges, total_len):
        return None

    @_reg("gemm_lt")
    def _(x, w, bias, epi, tune=True, residual=None):
        M, N = x.shape[0], w.shape[0]
        return x.new_empty((M, N)), x.new_empty((M, N) if epi == 1 else (0,))

    @_reg("gemm_lt_out")
    def _(x, w, bias, out, tune=True):
        return None

    @_reg("gemm_tn")
    def _(a, b, bias, epi, aux=None, bias_acc=None, T=0):
        M, N = a.shape[0], b.shape[0]
        if epi == 6:  # dO and delta [M / T, N / 64, T] fp32
            return a.new_empty((M, N)), a.new_empty((M // T, N // 64, T), dtype=torch.float32)
        if epi == 7:  # SwiGLU forward: silu(gate) * up [M, F] and [gate | up] [M, 2F], b = [2F, K]
            return a.new_empty((M, N // 2)), a.new_empty((M, N))
        return a.new_empty((M, 2 * N if epi == 5 else N)), a.new_empty((M if epi == 1 else 0, N))

    @_reg("act_fwd")
    def _(x, op):
        return torch.empty_like(x)

    @_reg("act_bwd")
    def _(dy, x, op):
        return torch.empty_like(dy)

    @_reg("act_bwd_bias")
    def _(dy, x, op, bias_acc):
        return torch.empty_like(dy)

    @_reg("swiglu_fwd")
    def _(gu):
        return gu.new_empty((*gu.shape[:-1], gu.shape[-1] // 2))

    @_reg("swiglu_bwd")
    def _(dy, gu):
        return torch.empty_like(gu)

    @_reg("rope")
    def _(x, cos, sin, n_heads_total, n_rot, T, pos_offset, inverse):
        return torch.empty_like(x)

    @_reg("rope_qk")
    def _(x, cos, sin, n_heads_total, n_rot, T):
        return x.new_empty((*x.shape[:-1], x.shape[-1] // n_heads_total * n_rot))

    @_reg("scale_")
    def _(x, s):
        return None

    @_reg("lse_merge_")
    def _(o_acc, lse_acc, o, lse):
        return None

    @_reg("cross_entropy")
    def _(logits, targets, dlogits, ignore_index, inv_n=None):
        return logits.new_empty((logits.shape[0],), dtype=f32)

    @_reg("adamw_")
    def _(param, master, m, v, grad, lr, b1, b2, eps, wd, step, grad_scale, scale, wd_mask, hyper=None):
        return None

    @_reg("sumsq")
    def _(x):
        return x.new_empty((), dtype=f32)

    @_reg("grad_norm_clip")
    def _(x, grad_scale, max_norm):
        return x.new_empty((2,), dtype=f32)

    @_reg("embedding_fwd")
    def _(idx, wte, wpe, pos_offset):
        return wte.new_empty((idx.shape[0], idx.shape[1], wte.shape[1]))

    @_reg("embedding_bwd")
    def _(dx, idx, V, n_pos, has_wpe):
        C = dx.shape[-1]
        return (dx.new_empty((V, C)), dx.new_empty((n_pos, C) if has_wpe else (0,)))

    @_reg("embedding_bwd_acc")
    def _(dx, idx, V, n_pos, has_wpe, dwte_acc, dwpe_acc=None):
        return None

    @_reg("transpose_plan")
    def _(src, dst):
        return src[0].new_empty((len(src), 6), dtype=torch.int64)

    @_reg("transpose_run")
    def _(desc, total_tiles):
        return None

    @_reg("sample")
    def _(logits, temperature, seed):
        return logits.new_empty((logits.shape[0], 1), dtype=torch.int64)

    @_reg("attn_fwd")
    def _(q, k, v, causal, scale, rope_cos=None, rope_sin=None):
        B, T, H, _ = q.shape
        return [q.new_empty(q.shape), q.new_empty((B, H, T), dtype=f32)]

    @_reg("attn_decode")
    def _(q, k, v, scale, seqlen=None):
        return q.new_empty(q.shape)

    @_reg("attn_bwd")
    def _(dout, q, k, v, o, lse, dq, dk, dv, causal, scale, rope_cos=None, rope_sin=None, rope_in=True, delta=None):
        return None

    @_reg("gemv")
    def _(x, w, bias, res=None, gamma=None, beta=None, eps=1e-5, rms=0, act=0, kc=None, vc=None, pos=None,
          q_cols=0):
        y = x.new_empty((x.shape[0], w.shape[0]))
        return (y, x.new_empty(x.shape if res is not None else (0,)))

"""Pure-PyTorch reference implementations of every fused op.

These are (a) the CPU execution path and (b) the fp32 numerics oracle that
the HIP-kernel tests compare against.  They are written for clarity, in fp32
internally, and mirror the math of the reference repo where one exists:

* attention: `src/models/attention.py:47-57` (q@k^T * hd^-1/2, causal
  masked_fill(-inf), softmax, @v) -- here batched over heads.
* layer norm: `transformer_block.py:28-31` (nn.LayerNorm, affine).
* cross entropy: `transformer.py:72-77` (F.cross_entropy, mean).
* AdamW: `train_transformer.py:126` (torch.optim.AdamW defaults).
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F


def layer_norm(x, weight, bias, eps: float):
    xf = x.float()
    mu = xf.mean(-1, keepdim=True)
    var = (xf - mu).pow(2).mean(-1, keepdim=True)
    y = (xf - mu) * torch.rsqrt(var + eps)
    if weight is not None:
        y = y * weight.float()
    if bias is not None:
        y = y + bias.float()
    return y.to(x.dtype)


def rms_norm(x, weight, eps: float):
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    if weight is not None:
        y = y * weight.float()
    return y.to(x.dtype)


def attention(q, k, v, causal: bool = True, scale: Optional[float] = None):
    """q: [B,T,H,D], k/v: [B,S,Hkv,D] -> out [B,T,H,D], lse [B,H,T] (natural log)."""
    B, T, H, D = q.shape
    S, Hkv = k.shape[1], k.shape[2]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    qf = q.float().transpose(1, 2)                      # B,H,T,D
    kf = k.float().transpose(1, 2)
    vf = v.float().transpose(1, 2)
    if Hkv != H:
        rep = H // Hkv
        kf = kf.repeat_interleave(rep, dim=1)
        vf = vf.repeat_interleave(rep, dim=1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale  # B,H,T,S
    if causal:
        # queries are aligned to the END of the key sequence (decode/KV-cache convention)
        off = S - T
        mask = torch.ones(T, S, dtype=torch.bool, device=q.device).tril(diagonal=off)
        s = s.masked_fill(~mask, float("-inf"))
    lse = torch.logsumexp(s, dim=-1)                    # B,H,T
    p = torch.exp(s - lse.unsqueeze(-1))
    o = torch.matmul(p, vf)                             # B,H,T,D
    return o.transpose(1, 2).to(q.dtype), lse


def attention_bwd(do, q, k, v, o, lse, causal: bool = True, scale: Optional[float] = None):
    """Flash-style backward of one attention block given the row statistics of the WHOLE
    softmax (``lse`` [B,H,T], natural log, and the final output ``o``), so partial key
    blocks (ring / context parallel) produce exact partial gradients.
    Returns fp32 (dq [B,T,H,D], dk [B,S,Hkv,D], dv [B,S,Hkv,D])."""
    B, T, H, D = q.shape
    S, Hkv = k.shape[1], k.shape[2]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    rep = H // Hkv
    qf, dof, of = (t.float().transpose(1, 2) for t in (q, do, o))            # B,H,T,D
    kf = k.float().transpose(1, 2).repeat_interleave(rep, dim=1)             # B,H,S,D
    vf = v.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        mask = torch.ones(T, S, dtype=torch.bool, device=q.device).tril(diagonal=S - T)
        s = s.masked_fill(~mask, float("-inf"))
    p = torch.exp(s - lse.float().unsqueeze(-1))
    dv = torch.matmul(p.transpose(-1, -2), dof)                              # B,H,S,D
    dp = torch.matmul(dof, vf.transpose(-1, -2))
    delta = (dof * of).sum(-1, keepdim=True)
    ds = p * (dp - delta)
    dq = torch.matmul(ds, kf) * scale
    dk = torch.matmul(ds.transpose(-1, -2), qf) * scale
    dk = dk.view(B, Hkv, rep, S, D).sum(2)
    dv = dv.view(B, Hkv, rep, S, D).sum(2)
    return dq.transpose(1, 2), dk.transpose(1, 2), dv.transpose(1, 2)


def gelu_tanh(x):
    return F.gelu(x.float(), approximate="tanh").to(x.dtype)


def swiglu(gate_up):
    """gate_up [..., 2F] laid out [gate | up] -> silu(gate) * up  [..., F]."""
    g, u = gate_up.float().chunk(2, dim=-1)
    return (F.silu(g) * u).to(gate_up.dtype)


def relu(x):
    return torch.relu(x)


def rope_cos_sin(seq_len: int, head_dim: int, theta: float = 10000.0, device=None, offset: int = 0):
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64, device=device) / head_dim))
    t = torch.arange(offset, offset + seq_len, dtype=torch.float64, device=device)
    freqs = torch.outer(t, inv)                         # T, D/2
    return freqs.cos().float(), freqs.sin().float()


def rope(x, cos, sin):
    """Rotate-half (GPT-NeoX / Llama HF) convention on x [B,T,H,D]; cos/sin [T, D/2]."""
    D = x.shape[-1]
    xf = x.float()
    x1, x2 = xf[..., : D // 2], xf[..., D // 2:]
    c = cos[None, :, None, :]
    s = sin[None, :, None, :]
    out = torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)
    return out.to(x.dtype)


def cross_entropy(logits, targets, ignore_index: int = -100):
    return F.cross_entropy(logits.float(), targets.long(), ignore_index=ignore_index)


def embedding(idx, wte, wpe=None, pos_offset: int = 0):
    x = F.embedding(idx, wte)
    if wpe is not None:
        T = idx.shape[1]
        x = x + wpe[pos_offset:pos_offset + T].unsqueeze(0)
    return x


@torch.no_grad()
def adamw_(param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, step,
           master: Optional[torch.Tensor] = None, grad_scale: float = 1.0):
    """In-place AdamW (torch.optim.AdamW semantics, decoupled weight decay)."""
    p = master if master is not None else param
    g = grad.float() * grad_scale
    p.mul_(1.0 - lr * weight_decay)
    exp_avg.lerp_(g, 1.0 - beta1)
    exp_avg_sq.mul_(beta2).addcmul_(g, g, value=1.0 - beta2)
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    denom = (exp_avg_sq.sqrt() / math.sqrt(bc2)).add_(eps)
    p.addcdiv_(exp_avg, denom, value=-lr / bc1)
    if master is not None:
        param.copy_(master.to(param.dtype))

"""The pure-PyTorch oracles (ops/reference.py) that every HIP kernel is tested against are
themselves checked here, on CPU in fp64 (finite-difference checks on tiny
oracle shapes):

* autograd.gradcheck through the reference attention (causal, GQA, queries aligned to
  the end of a longer key sequence), norms, activations and RoPE;
* the hand-derived flash-style backward ``attention_bwd`` (row statistics of the WHOLE
  softmax, used by ring attention's partial key blocks) equals autograd's gradient;
* the reference ops agree with torch.nn.functional where an equivalent exists.

The oracles compute in fp32 whatever the input dtype (they model the kernels' fp32
accumulation), so finite differences use eps = 1e-3 and fp32-level tolerances.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from pretraining_llm_amd.ops import reference as ref

D64 = torch.float64
GC = dict(eps=1e-3, atol=2e-3, rtol=2e-3)  # finite differences through fp32 internals


def gradcheck(fn, inputs):
    return torch.autograd.gradcheck(fn, inputs, **GC)


@pytest.mark.parametrize("causal,H,Hkv,T,S", [(True, 2, 2, 5, 5), (True, 4, 2, 3, 7), (False, 2, 1, 4, 6)])
def test_attention_reference_gradcheck(causal, H, Hkv, T, S):
    torch.manual_seed(0)
    q = torch.randn(1, T, H, 4, dtype=D64, requires_grad=True)
    k = torch.randn(1, S, Hkv, 4, dtype=D64, requires_grad=True)
    v = torch.randn(1, S, Hkv, 4, dtype=D64, requires_grad=True)
    assert gradcheck(lambda a, b, c: ref.attention(a, b, c, causal=causal)[0], (q, k, v))


@pytest.mark.parametrize("causal,H,Hkv,T,S", [(True, 4, 2, 6, 6), (True, 2, 2, 3, 9), (False, 4, 1, 5, 7)])
def test_attention_flash_backward_matches_autograd(causal, H, Hkv, T, S):
    torch.manual_seed(1)
    D = 8
    q = torch.randn(2, T, H, D, dtype=D64, requires_grad=True)
    k = torch.randn(2, S, Hkv, D, dtype=D64, requires_grad=True)
    v = torch.randn(2, S, Hkv, D, dtype=D64, requires_grad=True)
    o, lse = ref.attention(q, k, v, causal=causal)
    do = torch.randn_like(o)
    gq, gk, gv = torch.autograd.grad(o, (q, k, v), do)
    dq, dk, dv = ref.attention_bwd(do, q.detach(), k.detach(), v.detach(), o.detach(), lse.detach(), causal=causal)
    for a, b in ((dq, gq), (dk, gk), (dv, gv)):
        assert torch.allclose(a.to(D64), b, atol=1e-5, rtol=1e-4)
    # and the forward agrees with SDPA (expanded GQA heads, end-aligned causal mask)
    rep = H // Hkv
    mask = torch.ones(T, S, dtype=torch.bool).tril(S - T) if causal else None
    sd = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2).repeat_interleave(rep, 1),
                                        v.transpose(1, 2).repeat_interleave(rep, 1), attn_mask=mask)
    assert torch.allclose(o, sd.transpose(1, 2), atol=1e-5)


def test_norm_reference_gradcheck_and_functional():
    torch.manual_seed(2)
    x = torch.randn(3, 6, dtype=D64, requires_grad=True)
    w = torch.randn(6, dtype=D64, requires_grad=True)
    b = torch.randn(6, dtype=D64, requires_grad=True)
    assert gradcheck(lambda a, c, d: ref.layer_norm(a, c, d, 1e-5), (x, w, b))
    assert gradcheck(lambda a, c: ref.rms_norm(a, c, 1e-5), (x, w))
    assert torch.allclose(ref.layer_norm(x, w, b, 1e-5), F.layer_norm(x, (6,), w, b, 1e-5), atol=1e-5)
    rms = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * w
    assert torch.allclose(ref.rms_norm(x, w, 1e-5), rms, atol=1e-5)


def test_activation_references():
    torch.manual_seed(3)
    x = torch.randn(4, 10, dtype=D64, requires_grad=True)
    assert torch.allclose(ref.gelu_tanh(x), F.gelu(x, approximate="tanh"), atol=1e-5)
    assert gradcheck(ref.gelu_tanh, (x,))
    assert gradcheck(ref.swiglu, (x,))
    g, u = x.chunk(2, -1)
    assert torch.allclose(ref.swiglu(x), F.silu(g) * u, atol=1e-5)


def test_rope_reference_is_a_rotation():
    torch.manual_seed(4)
    T, D = 7, 8
    x = torch.randn(2, T, 3, D, dtype=D64, requires_grad=True)
    cos, sin = ref.rope_cos_sin(T, D, 10000.0)
    y = ref.rope(x, cos.to(D64), sin.to(D64))
    # norm-preserving per (token, head) and invertible with the negated angle
    assert torch.allclose(y.norm(dim=-1), x.norm(dim=-1), atol=1e-6)
    back = ref.rope(y, cos.to(D64), -sin.to(D64))
    assert torch.allclose(back, x, atol=1e-6)
    assert gradcheck(lambda a: ref.rope(a, cos.to(D64), sin.to(D64)), (x,))
    # relative-position property: <R_m q, R_n k> depends only on m - n
    q = torch.randn(D, dtype=D64)
    k = torch.randn(D, dtype=D64)
    cs, sn = ref.rope_cos_sin(12, D, 10000.0)
    rot = lambda vec, p: ref.rope(vec.view(1, 1, 1, D).expand(1, 12, 1, D), cs.to(D64), sn.to(D64))[0, p, 0]  # noqa: E731
    assert abs(torch.dot(rot(q, 5), rot(k, 2)) - torch.dot(rot(q, 9), rot(k, 6))) < 1e-5  # fp32 internals


def test_cross_entropy_and_embedding_references():
    torch.manual_seed(5)
    logits = torch.randn(6, 11, dtype=D64, requires_grad=True)
    t = torch.tensor([1, 2, -100, 4, 10, 0])
    assert torch.allclose(ref.cross_entropy(logits, t).double(), F.cross_entropy(logits, t, ignore_index=-100), atol=1e-5)
    assert gradcheck(lambda a: ref.cross_entropy(a, t).double(), (logits,))
    wte = torch.randn(20, 4, dtype=D64)
    wpe = torch.randn(8, 4, dtype=D64)
    idx = torch.randint(0, 20, (2, 5))
    e = ref.embedding(idx, wte, wpe, pos_offset=2)
    assert torch.allclose(e, wte[idx] + wpe[2:7], atol=1e-5)


def test_adamw_reference_matches_torch_optim():
    # fp32 master / moments, as the framework keeps them
    torch.manual_seed(6)
    p0 = torch.randn(50)
    pt = p0.clone().requires_grad_()
    opt = torch.optim.AdamW([pt], lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=0.05)
    p, m, v = p0.clone(), torch.zeros(50), torch.zeros(50)
    for step in range(1, 5):
        g = torch.randn(50)
        pt.grad = g.clone()
        opt.step()
        ref.adamw_(p, g, m, v, 1e-2, 0.9, 0.99, 1e-8, 0.05, step)
    assert torch.allclose(p, pt.detach(), atol=1e-6)
    assert math.isfinite(float(p.sum()))

"""Numerics of the fused-epilogue TN GEMM (csrc/gemm.hip) against fp32 PyTorch math.

C = epi(A B^T): plain (+bias), bias+GELU (pre-activation kept), bias+ReLU, and the data
gradient fused with the GELU / ReLU backward plus the bias-gradient column sums."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _ext():
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    yield


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _gelu(x):
    return torch.nn.functional.gelu(x, approximate="tanh")


def _gelu_df(x):
    k, c = 0.7978845608028654, 0.044715
    u = k * (x + c * x ** 3)
    t = torch.tanh(u)
    return 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * k * (1 + 3 * c * x * x)


SHAPES = [(512, 768, 768), (300, 520, 128), (1024, 3072, 768), (777, 264, 192), (8448, 2056, 64),
          (16640, 1032, 320)]


# phased 4 = the ping-pong kernel (csrc/gemm_pp.hip; its MFMA shape is fixed, mf is ignored),
# the default (csrc/gemm.hip g_gemm_phased); 0 / 2 = the round-3 kernel kept for A/B
DEFAULT_KERNEL = 4
KERNELS = [(16, 0), (32, 0), (16, 2), (32, 2), (16, 4)]


@pytest.mark.parametrize("mf,phased", KERNELS)
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm_tn_forward_epilogues(M, N, K, mf, phased):
    torch.manual_seed(3)
    big = torch.randn(M, K + 64, device=DEV).bfloat16()
    a = big[:, 32:32 + K]  # row-strided A
    b = (torch.randn(N, K, device=DEV) / K ** 0.5).bfloat16()
    bias = (0.5 * torch.randn(N, device=DEV)).bfloat16()
    ref = a.float() @ b.float().t()
    torch.ops.pllm.gemm_set_config(mf, 4, phased)
    try:
        out, _ = torch.ops.pllm.gemm_tn(a, b, None, 0)
        assert out.shape == (M, N)
        assert _rel(out, ref) < 5e-3, _rel(out, ref)
        out, _ = torch.ops.pllm.gemm_tn(a, b, bias, 0)
        pre_ref = ref + bias.float()
        assert _rel(out, pre_ref) < 5e-3
        act, pre = torch.ops.pllm.gemm_tn(a, b, bias, 1)
        assert _rel(pre, pre_ref) < 5e-3
        # the activation is computed from the bf16-rounded pre-activation, like the unfused path
        assert _rel(act, _gelu(pre.float())) < 5e-3, _rel(act, _gelu(pre.float()))
        assert _rel(act, _gelu(pre_ref)) < 1e-2
        y, _ = torch.ops.pllm.gemm_tn(a, b, bias, 2)
        assert _rel(y, torch.relu(pre_ref)) < 5e-3
        assert torch.equal(torch.ops.pllm.gemm_tn(a, b, bias, 1)[0], act)  # deterministic
    finally:
        torch.ops.pllm.gemm_set_config(16, 4, DEFAULT_KERNEL)


@pytest.mark.parametrize("mf,phased", KERNELS)
@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("f32_bias_grad", [True, False])
def test_gemm_tn_backward_epilogues(M, N, K, mf, f32_bias_grad, phased):
    torch.manual_seed(5)
    dy = (0.3 * torch.randn(M, K, device=DEV)).bfloat16()
    wt = (torch.randn(N, K, device=DEV) / K ** 0.5).bfloat16()
    pre = torch.randn(M, N, device=DEV).bfloat16()
    da = (dy.float() @ wt.float().t()).bfloat16().float()  # the unfused path's bf16 data gradient
    torch.ops.pllm.gemm_set_config(mf, 4, phased)
    try:
        for epi, aux, ref in ((3, pre, da * _gelu_df(pre.float())),
                              (4, torch.relu(pre), da * (pre.float() > 0))):
            acc = torch.randn(N, device=DEV)
            acc = acc if f32_bias_grad else acc.bfloat16()
            acc0 = acc.clone()
            out, _ = torch.ops.pllm.gemm_tn(dy, wt, None, epi, aux, acc)
            assert _rel(out, ref) < 1e-2, (epi, _rel(out, ref))
            db_ref = acc0.double() + out.double().sum(0)  # column sums of the bf16 output
            tol = 1e-5 if f32_bias_grad else 1e-2
            assert _rel(acc.double(), db_ref) < tol, (epi, _rel(acc.double(), db_ref))
            out2, _ = torch.ops.pllm.gemm_tn(dy, wt, None, epi, aux)
            assert torch.equal(out, out2)
    finally:
        torch.ops.pllm.gemm_set_config(16, 4, DEFAULT_KERNEL)


def test_gemm_tn_contract_checks():
    a = torch.randn(64, 100, device=DEV).bfloat16()
    b = torch.randn(64, 100, device=DEV).bfloat16()
    with pytest.raises(RuntimeError):
        torch.ops.pllm.gemm_tn(a, b, None, 0)  # K % 64
    a = torch.randn(64, 128, device=DEV).bfloat16()
    b = torch.randn(60, 128, device=DEV).bfloat16()
    with pytest.raises(RuntimeError):
        torch.ops.pllm.gemm_tn(a, b, None, 0)  # N % 8
    b = torch.randn(64, 128, device=DEV).bfloat16()
    with pytest.raises(RuntimeError):
        torch.ops.pllm.gemm_tn(a, b, None, 3)  # epi 3 without aux


@pytest.mark.parametrize("kind", ["gelu", "relu"])
@pytest.mark.parametrize("ext", [False, True])
@pytest.mark.parametrize("fwd", [False, True])
def test_fused_mlp_matches_unfused(kind, ext, fwd, monkeypatch):
    """ops.fused_mlp (activation in the GEMM epilogues; fwd=False: backward only) vs hipBLASLt
    GEMMs + activation kernels."""
    from pretraining_llm_amd import ops
    monkeypatch.setattr(ops, "FUSED_MLP_FWD", fwd)
    torch.manual_seed(11)
    C, Fh = 256, 1024
    x0 = torch.randn(4, 128, C, device=DEV).bfloat16()
    w1 = (torch.randn(Fh, C, device=DEV) / C ** 0.5).bfloat16()
    b1 = (0.1 * torch.randn(Fh, device=DEV)).bfloat16()
    w2 = (torch.randn(C, Fh, device=DEV) / Fh ** 0.5).bfloat16()
    b2 = (0.1 * torch.randn(C, device=DEV)).bfloat16()
    dy = torch.randn(4, 128, C, device=DEV).bfloat16()

    def run(fused):
        ps = [t.clone().requires_grad_() for t in (x0, w1, b1, w2, b2)]
        x, W1, B1, W2, B2 = ps
        with torch.enable_grad():
            if fused:
                assert ops.fused_mlp_ok(x, W1, B1, W2, kind)
                y = ops.fused_mlp(x, W1, B1, W2, B2, kind, out_bias_ext=ext)
            else:
                h = ops.linear(x, W1, B1)
                a = ops.gelu(h) if kind == "gelu" else ops.relu(h)
                y = ops.linear(a, W2, B2)
            y.backward(dy)
        return y.detach(), [p.grad for p in ps]

    yf, gf = run(True)
    yu, gu = run(False)
    assert _rel(yf, yu) < 1e-2
    names = ["x", "w1", "b1", "w2", "b2"]
    for n, a, b in zip(names, gf, gu):
        if n == "b2" and ext:
            assert a is None  # left to the next norm's backward
            continue
        assert a is not None, n
        assert _rel(a, b) < 2e-2, (n, _rel(a, b))


def _silu(x):
    return x * torch.sigmoid(x)


@pytest.mark.parametrize("mf,phased", [(32, 0), (16, 0), (16, 4)])
@pytest.mark.parametrize("M,N,K", [(512, 768, 768), (300, 520, 128), (777, 264, 192), (4160, 1376, 256)])
def test_gemm_tn_swiglu_backward_epilogue(M, N, K, mf, phased):
    """epi 5: [dgate | dup] = swiglu'([gate | up], dy W2) in the data-gradient GEMM's epilogue
    vs fp32 math on the bf16-rounded data gradient (what swiglu_bwd_kernel reads)."""
    torch.manual_seed(7)
    dy = (0.3 * torch.randn(M, K, device=DEV)).bfloat16()
    wt = (torch.randn(N, K, device=DEV) / K ** 0.5).bfloat16()
    gu = torch.randn(M, 2 * N, device=DEV).bfloat16()
    d = (dy.float() @ wt.float().t()).bfloat16().float()
    g, u = gu.float()[:, :N], gu.float()[:, N:]
    sg = torch.sigmoid(g)
    ref = torch.cat([d * u * sg * (1 + g * (1 - sg)), d * _silu(g)], dim=1)
    torch.ops.pllm.gemm_set_config(mf, 4, phased)
    try:
        out, aux = torch.ops.pllm.gemm_tn(dy, wt, None, 5, gu)
        assert out.shape == (M, 2 * N) and aux.numel() == 0
        assert _rel(out[:, :N], ref[:, :N]) < 1e-2, _rel(out[:, :N], ref[:, :N])
        assert _rel(out[:, N:], ref[:, N:]) < 1e-2, _rel(out[:, N:], ref[:, N:])
        # bit-identical to the unfused kernel pair it replaces (same bf16 roundings)
        unfused = torch.ops.pllm.swiglu_bwd(torch.ops.pllm.gemm_tn(dy, wt, None, 0)[0], gu)
        assert (out.float() - unfused.float()).abs().max().item() <= 2 ** -6 * unfused.float().abs().max().item()
        assert torch.equal(torch.ops.pllm.gemm_tn(dy, wt, None, 5, gu)[0], out)  # deterministic
    finally:
        torch.ops.pllm.gemm_set_config(16, 4, DEFAULT_KERNEL)


def test_fused_swiglu_mlp_matches_unfused():
    """ops.fused_swiglu_mlp (SwiGLU backward in the down-projection's data-gradient epilogue) vs
    hipBLASLt GEMMs + the swiglu kernels."""
    from pretraining_llm_amd import ops
    torch.manual_seed(13)
    C, Fh = 256, 704
    x0 = torch.randn(4, 128, C, device=DEV).bfloat16()
    w1 = (torch.randn(2 * Fh, C, device=DEV) / C ** 0.5).bfloat16()
    w2 = (torch.randn(C, Fh, device=DEV) / Fh ** 0.5).bfloat16()
    dy = torch.randn(4, 128, C, device=DEV).bfloat16()

    def run(fused):
        ps = [t.clone().requires_grad_() for t in (x0, w1, w2)]
        x, W1, W2 = ps
        with torch.enable_grad():
            if fused:
                assert ops.fused_swiglu_ok(x, W1, None, W2, None)
                y = ops.fused_swiglu_mlp(x, W1, W2)
            else:
                y = ops.linear(ops.swiglu(ops.linear(x, W1)), W2)
            y.backward(dy)
        return y.detach(), [p.grad for p in ps]

    yf, gf = run(True)
    yu, gu = run(False)
    # forward: the SwiGLU in the up-projection's epilogue (epilogue 7) vs hipBLASLt + swiglu_fwd:
    # the same math, different fp32 summation order in the GEMM
    assert _rel(yf, yu) < 1e-2, _rel(yf, yu)
    for n, a, b in zip(["x", "w1", "w2"], gf, gu):
        assert a is not None, n
        assert _rel(a, b) < 1e-2, (n, _rel(a, b))


@pytest.mark.parametrize("phased", [0, 4])
@pytest.mark.parametrize("B,T,H", [(2, 256, 12), (3, 200, 4), (1, 1024, 16)])
def test_gemm_tn_attn_delta_epilogue(B, T, H, phased):
    """epi 6: dO = dy W_o (as epi 0, bitwise) plus delta[b, h, t] = sum_d dO * O per 64-wide head,
    against fp64 math on the bf16 dO (what attn_bwd_pre_kernel reads)."""
    torch.manual_seed(19)
    C = H * 64
    M = B * T
    dy = (0.5 * torch.randn(M, C, device=DEV)).bfloat16()
    wt = (torch.randn(C, C, device=DEV) / C ** 0.5).bfloat16()  # W_o^T shadow [H*D, C_out]
    o = torch.randn(M, C, device=DEV).bfloat16()
    torch.ops.pllm.gemm_set_config(16, 4, phased)
    try:
        do, delta = torch.ops.pllm.gemm_tn(dy, wt, None, 6, o, None, T)
        assert delta.shape == (B, H, T) and delta.dtype == torch.float32
        assert torch.equal(do, torch.ops.pllm.gemm_tn(dy, wt, None, 0)[0])
        ref = (do.double() * o.double()).view(B, T, H, 64).sum(-1).permute(0, 2, 1)
        assert _rel(delta.double(), ref) < 1e-6, _rel(delta.double(), ref)
        assert torch.equal(torch.ops.pllm.gemm_tn(dy, wt, None, 6, o, None, T)[1], delta)  # deterministic
    finally:
        torch.ops.pllm.gemm_set_config(16, 4, DEFAULT_KERNEL)


@pytest.mark.parametrize("bias", [True, False])
@pytest.mark.parametrize("ext", [False, True])
@pytest.mark.parametrize("D,Hkv", [(64, 4), (64, 2)])
def test_attn_proj_fused_matches_unfused(bias, ext, D, Hkv):
    """ops.attention_proj (projection dgrad + delta in one GEMM, attention backward without its
    delta pass; GQA too) vs attention_packed + linear."""
    from pretraining_llm_amd import ops
    torch.manual_seed(23)
    B, T, H = 2, 256, 4
    C = H * D
    qkv0 = (0.5 * torch.randn(B, T, (H + 2 * Hkv) * D, device=DEV)).bfloat16()
    w0 = (torch.randn(C, C, device=DEV) / C ** 0.5).bfloat16()
    b0 = (0.1 * torch.randn(C, device=DEV)).bfloat16() if bias else None
    dy = torch.randn(B, T, C, device=DEV).bfloat16()

    def run(fused):
        ps = [t.clone().requires_grad_() if t is not None else None for t in (qkv0, w0, b0)]
        qkv, w, b = ps
        with torch.enable_grad():
            if fused:
                assert ops.attn_proj_ok(qkv, H, Hkv, w, b)
                y = ops.attention_proj(qkv, H, Hkv, w, b, bias_grad_external=ext)
            else:
                y = ops.linear(ops.attention_packed(qkv, H, Hkv), w, b, bias_grad_external=ext)
            y.backward(dy)
        return y.detach(), [p.grad if p is not None else None for p in ps]

    yf, gf = run(True)
    yu, gu = run(False)
    assert torch.equal(yf, yu)
    for n, a, c in zip(["qkv", "w", "b"], gf, gu):
        if c is None:
            assert a is None, n
            continue
        assert a is not None, n
        assert _rel(a, c) < 1e-2, (n, _rel(a, c))


@pytest.mark.parametrize("preset", ["gpt2-small", "llama-1.3b"])
def test_resid_gemm_block_matches_norm_side_add(preset, monkeypatch):
    """A block's residual add done by the output projections' GEMMs (ops.resid_gemm_ok: hipBLASLt
    beta = 1 in attention_proj / fused_mlp / linear) vs by the next norm.  GPT-2: both projections take
    it and the block hands the stream on with residual None; llama: its attention output projection takes
    it (the SwiGLU MLP does not), so the block still returns a residual.  A two-block model's loss and every
    parameter gradient match the norm-side form (one bf16 rounding of the stream instead of two)."""
    from pretraining_llm_amd import ops
    from pretraining_llm_amd.models import GPT, get_preset
    torch.manual_seed(31)
    cfg = get_preset(preset).replace(n_blocks=2)
    model = GPT(cfg).to(device=DEV, dtype=torch.bfloat16)
    T = 256
    idx = torch.randint(0, cfg.vocab_size, (2, T), device=DEV)
    tgt = torch.randint(0, cfg.vocab_size, (2, T), device=DEV)
    blk = model.attn_blocks[0]
    rope = model.rope_tables(DEV, T)
    x0 = torch.randn(2, T, cfg.n_embed, device=DEV).bfloat16()
    r0 = torch.randn(2, T, cfg.n_embed, device=DEV).bfloat16()
    gpt2 = preset.startswith("gpt2")

    def run(on):
        monkeypatch.setattr(ops, "RESID_GEMM", on)
        assert ops.resid_gemm_ok(r0, blk.attn.proj.weight) == on
        model.zero_grad(set_to_none=True)
        with torch.enable_grad():
            m, r = blk(x0.clone().requires_grad_(), r0.clone(), rope, None, True)
            if gpt2:
                assert (r is None) == on, "the residual-in-GEMM path did not run" if on else "unexpected fusion"
            s = m.float() if r is None else m.float() + r.float()
            _, loss = model(idx, tgt)
            loss.backward()
        return s.detach(), loss.detach().float(), [p.grad.detach().float().clone() for p in model.parameters()]

    s1, l1, g1 = run(True)
    s0, l0, g0 = run(False)
    assert _rel(s1, s0) < 1e-2, _rel(s1, s0)
    assert abs(l1.item() - l0.item()) < 1e-2 * abs(l0.item())
    for i, (a, b) in enumerate(zip(g1, g0)):
        assert _rel(a, b) < 3e-2, (i, _rel(a, b))
    # and against fp32 math on stock torch ops (the same weights in fp32, ops backend "torch")
    import copy
    m32 = copy.deepcopy(model).float()
    m32.zero_grad(set_to_none=True)
    with ops.backend("torch"), torch.enable_grad():
        m, r = m32.attn_blocks[0](x0.float(), r0.float(), rope, None, True)
        s32 = m if r is None else m + r
        _, l32 = m32(idx, tgt)
        l32.backward()
    assert _rel(s1, s32) < 1.5e-2, _rel(s1, s32)
    assert abs(l1.item() - l32.item()) < 1e-2 * abs(l32.item()), (l1.item(), l32.item())
    for i, (a, p32) in enumerate(zip(g1, m32.parameters())):
        assert _rel(a, p32.grad) < 5e-2, (i, _rel(a, p32.grad))


def test_resid_gemm_under_activation_checkpointing():
    """The residual-in-GEMM blocks recomputed under activation checkpointing (every block checkpointed) give
    the loss and gradients of the stored-activation run (same kernels, same cached GEMM plans)."""
    from pretraining_llm_amd import ops
    from pretraining_llm_amd.models import GPT, get_preset
    assert ops.RESID_GEMM
    torch.manual_seed(37)
    cfg = get_preset("gpt2-small").replace(n_blocks=2)
    m1 = GPT(cfg).to(device=DEV, dtype=torch.bfloat16)
    m2 = GPT(cfg.replace(activation_checkpointing=True)).to(device=DEV, dtype=torch.bfloat16)
    m2.load_state_dict(m1.state_dict())
    idx = torch.randint(0, cfg.vocab_size, (2, 256), device=DEV)
    tgt = torch.randint(0, cfg.vocab_size, (2, 256), device=DEV)
    assert m2.checkpointed_blocks(idx) == 2 and m1.checkpointed_blocks(idx) == 0
    losses = []
    with torch.enable_grad():
        for m in (m1, m2):
            _, loss = m(idx, tgt)
            loss.backward()
            losses.append(loss.item())
    assert abs(losses[0] - losses[1]) < 1e-3 * abs(losses[0])
    for (n, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        assert _rel(p2.grad.float(), p1.grad.float()) < 1e-2, (n, _rel(p2.grad.float(), p1.grad.float()))


@pytest.mark.parametrize("phased", [0, 4])
@pytest.mark.parametrize("reserve", [0, 32, 240])
def test_gemm_tn_reserved_cus(phased, reserve):
    """reserve_cus caps the persistent grid (CUs left to RCCL kernels during an overlapped backward):
    more tiles per workgroup, the same result bit for bit."""
    torch.manual_seed(29)
    M, N, K = 4096, 2304, 768
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) / K ** 0.5).bfloat16()
    bias = torch.randn(N, device=DEV).bfloat16()
    torch.ops.pllm.gemm_set_config(16, 4, phased, 0)
    try:
        ref = torch.ops.pllm.gemm_tn(a, b, bias, 1)
        torch.ops.pllm.gemm_set_config(16, 4, phased, reserve)
        out = torch.ops.pllm.gemm_tn(a, b, bias, 1)
        assert torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1])
        assert _rel(out[1], a.float() @ b.float().t() + bias.float()) < 5e-3
    finally:
        torch.ops.pllm.gemm_set_config(16, 4, DEFAULT_KERNEL, 0)


@pytest.mark.parametrize("M,N,K", [(65536, 768, 768), (65536, 3072, 768), (8192, 2304, 3072)])
def test_gemm_pp_large_shapes(M, N, K):
    """The ping-pong kernel at training shapes (many tiles per workgroup) vs fp32 math and vs the
    round-3 kernel (same bf16 rounding: identical up to fp32 summation order)."""
    torch.manual_seed(31)
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) / K ** 0.5).bfloat16()
    try:
        torch.ops.pllm.gemm_set_config(16, 4, 4)
        out = torch.ops.pllm.gemm_tn(a, b, None, 0)[0]
        torch.ops.pllm.gemm_set_config(16, 4, 0)
        old = torch.ops.pllm.gemm_tn(a, b, None, 0)[0]
    finally:
        torch.ops.pllm.gemm_set_config(16, 4, DEFAULT_KERNEL)
    rows = torch.randint(0, M, (512,), device=DEV)
    ref = a[rows].float() @ b.float().t()
    assert _rel(out[rows], ref) < 5e-3
    assert (out.float() - old.float()).abs().max().item() <= 2 ** -6 * old.float().abs().max().item()


@pytest.mark.parametrize("M,F,K", [(512, 704, 256), (300, 520, 128), (4160, 1376, 2048), (777, 264, 192)])
def test_gemm_tn_swiglu_forward_epilogue(M, F, K):
    """epi 7: a = silu(gate) * up with [gate | up] = x W1^T in one launch (ping-pong kernel), the
    [gate | up] pre-activations kept in bf16; vs fp32 math and vs the unfused pair."""
    torch.manual_seed(37)
    x = torch.randn(M, K, device=DEV).bfloat16()
    w1 = (torch.randn(2 * F, K, device=DEV) / K ** 0.5).bfloat16()
    gu_ref = x.float() @ w1.float().t()
    a, gu = torch.ops.pllm.gemm_tn(x, w1, None, 7)
    assert a.shape == (M, F) and gu.shape == (M, 2 * F)
    assert _rel(gu, gu_ref) < 5e-3, _rel(gu, gu_ref)
    g, u = gu.float()[:, :F], gu.float()[:, F:]
    assert _rel(a, _silu(g) * u) < 5e-3  # from the bf16-rounded pre-activations
    unf = torch.ops.pllm.swiglu_fwd(gu)
    assert (a.float() - unf.float()).abs().max().item() <= 2 ** -7 * unf.float().abs().max().item()
    assert torch.equal(torch.ops.pllm.gemm_tn(x, w1, None, 7)[0], a)  # deterministic


def test_gemm_non_persistent_grids():
    """gemm_config(persistent=False): one workgroup per tile / work item (the hardware deals them to
    free CUs, e.g. beside RCCL kernels) -- the same results bit for bit as the persistent grids, for the
    fused-epilogue GEMM and the weight-gradient kernel, with several tiles / items per CU."""
    from pretraining_llm_amd import ops
    torch.manual_seed(43)
    M, N, K = 16384, 3072, 768
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) / K ** 0.5).bfloat16()
    bias = torch.randn(N, device=DEV).bfloat16()
    dy = (0.3 * torch.randn(M, 2304, device=DEV)).bfloat16()
    w0 = torch.randn(2304, K, device=DEV)
    outs = []
    try:
        for pers in (True, False):
            ops.gemm_config(persistent=pers)
            g = torch.ops.pllm.gemm_tn(a, b, bias, 1)
            acc = w0.clone()
            torch.ops.pllm.wgrad(dy, a, acc)
            outs.append((g, acc))
    finally:
        ops.gemm_config(persistent=True)
    (g1, w1), (g2, w2) = outs
    assert torch.equal(g1[0], g2[0]) and torch.equal(g1[1], g2[1])
    assert torch.equal(w1, w2)
    assert _rel(w1.double(), w0.double() + dy.double().t() @ a.double()) < 1e-5


@pytest.mark.parametrize("M,N,K", [(512, 768, 768), (300, 520, 128), (4096, 3072, 768), (777, 264, 192)])
@pytest.mark.parametrize("bias", [False, True])
def test_gemm_lt_epilogues(M, N, K, bias):
    """torch.ops.pllm.gemm_lt (hipBLASLt called directly, csrc/blaslt.cpp): plain / bias and bias + ReLU
    epilogues vs fp32 math; the ``out`` variant writes into a caller's buffer; ReLU equals ReLU of the
    plain product bit for bit (ReLU commutes with the bf16 rounding)."""
    torch.manual_seed(5)
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).bfloat16()
    b = (0.1 * torch.randn(N, device=DEV)).bfloat16() if bias else None
    ref = x.float() @ w.float().t() + (b.float() if bias else 0)
    y, pre = torch.ops.pllm.gemm_lt(x, w, b, 0)
    assert y.shape == (M, N) and pre.numel() == 0
    assert _rel(y, ref) < 1e-2
    r, _ = torch.ops.pllm.gemm_lt(x, w, b, 2)
    assert _rel(r, ref.relu()) < 1e-2
    assert torch.equal(r, y.relu())
    res = torch.randn(M, N, device=DEV).bfloat16()
    s_, _ = torch.ops.pllm.gemm_lt(x, w, b, 0, True, res)  # residual addend (beta = 1)
    assert _rel(s_, ref + res.float()) < 1e-2
    out = torch.full((M + 3, N), 7.0, device=DEV).bfloat16()
    torch.ops.pllm.gemm_lt_out(x, w, b, out[1:M + 1])
    assert torch.equal(out[1:M + 1], y)
    assert (out[0] == 7).all() and (out[M + 1:] == 7).all()
    plans = torch.ops.pllm.gemm_lt_plans()
    assert len(plans) % 7 == 0 and plans


def test_gemm_lt_contract_checks():
    x = torch.randn(64, 128, device=DEV).bfloat16()
    w = torch.randn(96, 128, device=DEV).bfloat16()
    with pytest.raises(RuntimeError):
        torch.ops.pllm.gemm_lt(x, w[:, :64].contiguous(), None, 0)  # K mismatch
    with pytest.raises(RuntimeError):
        torch.ops.pllm.gemm_lt(x.float(), w, None, 0)  # dtype
    with pytest.raises(RuntimeError):
        torch.ops.pllm.gemm_lt(x, w, torch.zeros(95, device=DEV).bfloat16(), 0)  # bias length
    with pytest.raises(RuntimeError):
        torch.ops.pllm.gemm_lt_out(x, w, None, torch.empty(64, 95, device=DEV).bfloat16())


@pytest.mark.parametrize("lt", [False, True])
def test_relu_mlp_lt_forward(lt, monkeypatch):
    """The reference architecture's ReLU MLP with bias + ReLU in hipBLASLt's epilogue vs the library GEMM +
    act_fwd pass: same forward and gradients."""
    from pretraining_llm_amd import ops
    monkeypatch.setattr(ops, "FUSED_MLP_FWD", False)
    torch.manual_seed(3)
    C, Fh = 256, 1024
    x0 = torch.randn(2, 256, C, device=DEV).bfloat16()
    w1 = (torch.randn(Fh, C, device=DEV) / C ** 0.5).bfloat16()
    b1 = (0.1 * torch.randn(Fh, device=DEV)).bfloat16()
    w2 = (torch.randn(C, Fh, device=DEV) / Fh ** 0.5).bfloat16()
    b2 = (0.1 * torch.randn(C, device=DEV)).bfloat16()
    dy = torch.randn(2, 256, C, device=DEV).bfloat16()

    def run(use_lt):
        monkeypatch.setattr(ops, "LT_RELU_FWD", use_lt)
        ps = [t.clone().requires_grad_() for t in (x0, w1, b1, w2, b2)]
        with torch.enable_grad():
            y = ops.fused_mlp(*ps, "relu")
            y.backward(dy)
        return y.detach(), [p.grad for p in ps]

    y0, g0 = run(False)
    y1, g1 = run(lt)
    assert _rel(y1, y0) < 2e-3
    for a, b in zip(g1, g0):
        assert _rel(a, b) < 2e-3

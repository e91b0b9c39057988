"""Model / module tests on CPU (reference test strategy: SURVEY.md §4, §7.4)."""
import math

import pytest
import torch

from pretraining_llm_amd.models import GPT, get_preset
from pretraining_llm_amd.models.compat import Block, Head, MLP, MultiHeadAttention, Transformer


def _tiny(**kw):
    return get_preset("gpt2-tiny").replace(vocab_size=512, context_length=64, **kw)


@pytest.mark.parametrize("preset", ["gpt2-tiny", "llama-tiny"])
def test_forward_shapes_and_init_loss(preset):
    torch.manual_seed(0)
    cfg = get_preset(preset).replace(vocab_size=512, context_length=64)
    m = GPT(cfg)
    x = torch.randint(0, 512, (2, 64))
    y = torch.randint(0, 512, (2, 64))
    logits, loss = m(x, y)
    assert logits.shape == (2, 64, 512)
    assert abs(loss.item() - math.log(512)) < 0.5  # ~ln(V) at init
    _, loss2 = m(x, y, return_logits=False)
    assert torch.allclose(loss, loss2)


def test_param_count_matches_formula():
    for name in ["gpt2-small", "llama-tiny", "ref-small"]:
        cfg = get_preset(name)
        if cfg.n_blocks > 12:
            continue
        m = GPT(cfg)
        assert sum(p.numel() for p in m.parameters()) == cfg.num_params(), name


def test_gpt2_small_is_124m():
    cfg = get_preset("gpt2-small")
    assert abs(cfg.num_params() - 124.5e6) < 0.5e6


def test_reference_api_shapes():
    """The reference's module smoke mains (attention.py:98-111, mlp.py:69-80,
    transformer_block.py:63-76, transformer.py:116-136) as assertions."""
    torch.manual_seed(0)
    mha = MultiHeadAttention(n_head=4, n_embed=32, context_length=5)
    x = torch.randn(2, 5, 32)
    assert mha(x).shape == (2, 5, 32)
    assert MLP(16)(torch.randn(2, 3, 16)).shape == (2, 3, 16)
    assert Block(4, 32, 5)(x).shape == (2, 5, 32)
    h = Head(8, 32, 5)
    assert h(x).shape == (2, 5, 8)
    t = Transformer(4, 32, 5, 100, 2)
    idx = torch.randint(0, 100, (2, 5))
    logits, loss = t(idx, idx)
    assert logits.shape == (2, 5, 100) and loss.ndim == 0
    out = t.generate(idx[:, :2], 5)
    assert out.shape == (2, 7)
    # the reference ctor kwarg name from the trainer's model_args works too (defect D4)
    t2 = Transformer(n_head=4, n_embed=32, context_length=5, vocab_size=100, n_blocks=2)
    assert len(t2.attn_blocks) == 2


def test_reference_state_dict_layout():
    """arch=ref checkpoints use the reference key set: per-head key/query/value + tril."""
    t = Transformer(4, 32, 8, 100, 2)
    sd = t.state_dict()
    assert "pos_idxs" in sd and "token_embed.weight" in sd and "position_embed.weight" in sd
    for i in range(2):
        for h in range(4):
            for k in ("key", "query", "value"):
                assert sd[f"attn_blocks.{i}.attn.heads.{h}.{k}.weight"].shape == (8, 32)
            assert sd[f"attn_blocks.{i}.attn.heads.{h}.tril"].shape == (8, 8)
        assert sd[f"attn_blocks.{i}.mlp.hidden.weight"].shape == (128, 32)
        assert sd[f"attn_blocks.{i}.mlp.proj.weight"].shape == (32, 128)
        assert f"attn_blocks.{i}.ln1.weight" in sd and f"attn_blocks.{i}.ln2.bias" in sd
    assert sd["lm_head.weight"].shape == (100, 32) and sd["lm_head.bias"].shape == (100,)
    assert not any(k.endswith("qkv.weight") for k in sd)
    # round trip: load into a fresh model strictly
    t2 = Transformer(4, 32, 8, 100, 2)
    t2.load_state_dict(sd, strict=True)
    idx = torch.randint(0, 100, (2, 8))
    assert torch.allclose(t(idx)[0], t2(idx)[0])


def test_reference_math_equivalence():
    """Our fused ref-arch model computes exactly the reference's per-head math."""
    torch.manual_seed(1)
    t = Transformer(2, 16, 6, 50, 1)
    idx = torch.randint(0, 50, (2, 6))
    sd = t.state_dict()
    x = t.token_embed(idx) + t.position_embed(torch.arange(6))
    blk = t.attn_blocks[0]
    h = torch.nn.functional.layer_norm(x, (16,), blk.ln1.weight, blk.ln1.bias, 1e-5)
    heads = []
    for hh in range(2):
        k = h @ sd[f"attn_blocks.0.attn.heads.{hh}.key.weight"].t()
        q = h @ sd[f"attn_blocks.0.attn.heads.{hh}.query.weight"].t()
        v = h @ sd[f"attn_blocks.0.attn.heads.{hh}.value.weight"].t()
        w = q @ k.transpose(-2, -1) * 8 ** -0.5
        w = w.masked_fill(torch.tril(torch.ones(6, 6)) == 0, float("-inf")).softmax(-1)
        heads.append(w @ v)
    x = x + torch.cat(heads, -1)
    h2 = torch.nn.functional.layer_norm(x, (16,), blk.ln2.weight, blk.ln2.bias, 1e-5)
    x = x + blk.mlp.proj(torch.relu(blk.mlp.hidden(h2)))
    x = torch.nn.functional.layer_norm(x, (16,), t.layer_norm.weight, t.layer_norm.bias, 1e-5)
    ref_logits = t.lm_head(x)
    ours, _ = t(idx)
    assert torch.allclose(ours, ref_logits, atol=1e-5)


def test_forward_embedding_multi_block():
    """Reference Transformer.forward_embedding crashes for N_BLOCKS>1 (D9); ours is defined."""
    t = Transformer(4, 32, 8, 100, 3)
    idx = torch.randint(0, 100, (2, 8))
    hidden, res = t.forward_embedding(idx)
    assert hidden.shape == (2, 8, 128) and res.shape == (2, 8, 32)
    t1 = Transformer(4, 32, 8, 100, 1)
    h1, r1 = t1.forward_embedding(idx)
    assert h1.shape == (2, 8, 128) and r1.shape == (2, 8, 32)


@pytest.mark.parametrize("preset", ["gpt2-tiny", "llama-tiny"])
def test_kv_cache_generation_matches_recompute(preset):
    torch.manual_seed(3)
    cfg = get_preset(preset).replace(vocab_size=256, context_length=32)
    m = GPT(cfg).eval()
    idx = torch.randint(0, 256, (2, 5))
    a = m.generate(idx, 20, temperature=0.0, use_cache=True)
    b = m.generate(idx, 20, temperature=0.0, use_cache=False)
    assert torch.equal(a, b)


@pytest.mark.parametrize("preset", ["gpt2-tiny", "llama-tiny"])
def test_device_position_decode_step_matches_cached(preset):
    """forward_decode (position as a device tensor -- the hipGraph-capturable step) gives the
    same logits as the host-position KV-cache step."""
    from pretraining_llm_amd.inference.generate import KVCache, forward_cached, forward_decode
    torch.manual_seed(6)
    cfg = get_preset(preset).replace(vocab_size=256, context_length=32)
    m = GPT(cfg).eval()
    idx = torch.randint(0, 256, (2, 7))
    mk = lambda: KVCache(cfg.n_blocks, 2, 32, cfg.n_kv_head, cfg.head_dim, torch.float32, "cpu")  # noqa: E731
    c1, c2 = mk(), mk()
    forward_cached(m, idx[:, :6], c1, 0)
    forward_cached(m, idx[:, :6], c2, 0)
    a = forward_cached(m, idx[:, 6:], c1, 6)
    b = forward_decode(m, idx[:, 6:], c2, torch.tensor([6]), torch.tensor([7], dtype=torch.int32))
    assert torch.allclose(a, b, atol=1e-5, rtol=1e-4)
    assert torch.equal(c1.k[1][:, :7], c2.k[1][:, :7])


def test_generation_context_crop_beyond_context_length():
    torch.manual_seed(4)
    cfg = _tiny().replace(context_length=16)
    m = GPT(cfg).eval()
    idx = torch.randint(0, 512, (1, 10))
    a = m.generate(idx, 20, temperature=0.0, use_cache=True)
    b = m.generate(idx, 20, temperature=0.0, use_cache=False)
    assert a.shape == (1, 30)
    assert torch.equal(a, b)


def test_activation_checkpointing_same_grads():
    torch.manual_seed(5)
    cfg = _tiny()
    m1 = GPT(cfg)
    m2 = GPT(cfg.replace(activation_checkpointing=True))
    m2.load_state_dict(m1.state_dict())
    x = torch.randint(0, 512, (2, 64))
    l1 = m1(x, x)[1]
    l1.backward()
    l2 = m2(x, x)[1]
    l2.backward()
    assert torch.allclose(l1, l2)
    for (n, p1), (_, p2) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.allclose(p1.grad, p2.grad, atol=1e-6), n


def test_gqa_llama_forward_backward():
    torch.manual_seed(6)
    cfg = get_preset("llama-tiny")
    m = GPT(cfg)
    x = torch.randint(0, cfg.vocab_size, (2, 32))
    _, loss = m(x, x)
    loss.backward()
    assert all(p.grad is not None for p in m.parameters())


def test_activation_checkpointing_auto_policy():
    """'auto' checkpoints only when the activation estimate exceeds half the free HBM: never
    on CPU tensors; the estimate is 2 B x (6C + 2F) per token and layer."""
    cfg = get_preset("gpt2-medium").replace(vocab_size=256, context_length=64, activation_checkpointing="auto")
    m = GPT(cfg)
    assert m.activation_bytes(32768) == 2 * (6 * 1024 + 2 * 4096) * 32768 * 24
    assert m.use_checkpointing(torch.zeros(2, 8, dtype=torch.long)) is False
    assert GPT(_tiny().replace(activation_checkpointing=True)).use_checkpointing(torch.zeros(1, 4, dtype=torch.long))
    # partial: only as many blocks as it takes to fit the budget
    full = m.activation_bytes(32768)
    assert m.auto_checkpoint_blocks(32768, 2 * full) == 0
    saved = full / 24 - 4 * 1024 * 32768
    assert m.auto_checkpoint_blocks(32768, full - 5.5 * saved) == 6
    assert m.auto_checkpoint_blocks(32768, 0) == 24
    assert GPT(_tiny().replace(activation_checkpointing=0.5)).checkpointed_blocks(torch.zeros(1, 4)) == 1


def test_partial_activation_checkpointing_same_grads():
    """Checkpointing a fraction of the blocks leaves loss and gradients unchanged."""
    cfg = _tiny().replace(n_blocks=3)
    torch.manual_seed(0)
    m1 = GPT(cfg)
    m2 = GPT(cfg.replace(activation_checkpointing=0.5))
    m2.load_state_dict(m1.state_dict())
    assert m2.checkpointed_blocks(torch.zeros(1, 4)) == 2
    x = torch.randint(0, cfg.vocab_size, (2, 16))
    losses = []
    for m in (m1, m2):
        _, loss = m(x, x)
        loss.backward()
        losses.append(loss.item())
    assert abs(losses[0] - losses[1]) < 1e-6
    for (n, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        torch.testing.assert_close(p1.grad, p2.grad, rtol=1e-5, atol=1e-6, msg=n)


@pytest.mark.parametrize("mod", ["attention", "mlp", "transformer_block", "transformer"])
def test_reference_module_demos_run(mod):
    """The src.models.* modules keep the reference's runnable shape demos."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-m", f"src.models.{mod}"], cwd=root, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "->" in r.stdout or "loss" in r.stdout

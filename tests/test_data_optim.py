"""Data pipeline and optimizer tests (CPU)."""
import numpy as np
import pytest
import torch

from pretraining_llm_amd.data import TokenLoader, ensure_synthetic_shard, get_batch_iterator, write_tokens
from pretraining_llm_amd.train.optim import FlatAdamW, no_decay_1d


@pytest.fixture()
def shard(tmp_path):
    toks = np.arange(20000) % 60000
    return write_tokens(str(tmp_path / "tok.bin"), toks)


def test_loader_windows_are_contiguous_and_shifted(shard):
    L = TokenLoader(shard, 4, 32, seed=1)
    x, y = L.next()
    assert x.dtype == torch.int64 and x.shape == (4, 32)
    assert torch.equal(x[:, 1:], y[:, :-1])
    # the source is arange, so a window must be consecutive integers
    assert torch.all(x[:, 1:] - x[:, :-1] == 1)


def test_loader_rank_shards_are_contiguous_and_disjoint(shard):
    """Contiguous per-rank shards (the reference strided data[rank::world])."""
    seen = []
    for r in range(4):
        L = TokenLoader(shard, 8, 16, rank=r, world_size=4, seed=2)
        assert L.shard_tokens() == 5000
        lo, hi = r * 5000, (r + 1) * 5000
        for _ in range(5):
            x, y = L.next()
            assert x.min() >= lo and y.max() < hi
            assert torch.all(x[:, 1:] - x[:, :-1] == 1)
        seen.append(L)


def test_loader_deterministic_and_resumable(shard):
    a = TokenLoader(shard, 2, 16, seed=7)
    batches = [a.next() for _ in range(5)]
    b = TokenLoader(shard, 2, 16, seed=7, start_batch=3)
    x3, y3 = b.next()
    assert torch.equal(x3, batches[3][0]) and torch.equal(y3, batches[3][1])
    x2, _ = a.batch_at(2)
    assert torch.equal(x2, batches[2][0])
    c = TokenLoader(shard, 2, 16, seed=8)
    assert not torch.equal(c.next()[0], batches[0][0])


def test_reference_batch_iterator_signature(shard):
    it = get_batch_iterator(shard, 3, 8, "cpu", ddp=True, ddp_rank=1, ddp_world_size=2)
    x, y = next(it)
    assert x.shape == (3, 8) and y.shape == (3, 8)
    assert x.min() >= 10000


def test_missing_file_raises(tmp_path):
    with pytest.raises(FileNotFoundError):
        TokenLoader(str(tmp_path / "nope.bin"), 2, 8)


def test_synthetic_shard_is_uint16_and_reproducible(tmp_path):
    p1 = ensure_synthetic_shard(str(tmp_path / "a.bin"), 5000, 50304, seed=3)
    p2 = ensure_synthetic_shard(str(tmp_path / "b.bin"), 5000, 50304, seed=3)
    a = np.memmap(p1, dtype=np.uint16, mode="r")
    b = np.memmap(p2, dtype=np.uint16, mode="r")
    assert a.size == 5000 and np.array_equal(a, b)
    assert a.max() < 50304


def _model():
    from pretraining_llm_amd.models import GPT, get_preset
    torch.manual_seed(0)
    return GPT(get_preset("gpt2-tiny").replace(vocab_size=128, context_length=16, n_embed=32, n_head=2))


@pytest.mark.parametrize("decay_all", [True, False])
def test_flat_adamw_matches_torch_adamw(decay_all):
    m1, m2 = _model(), _model()
    m2.load_state_dict(m1.state_dict())
    params = list(m2.parameters())
    if decay_all:
        ref = torch.optim.AdamW(params, lr=1e-2, weight_decay=0.1)
    else:
        ref = torch.optim.AdamW([{"params": [p for p in params if p.dim() >= 2], "weight_decay": 0.1},
                                 {"params": [p for p in params if p.dim() < 2], "weight_decay": 0.0}], lr=1e-2)
    opt = FlatAdamW(m1, lr=1e-2, weight_decay=0.1, decay_filter=None if decay_all else no_decay_1d)
    x = torch.randint(0, 128, (2, 16))
    for _ in range(3):
        for m in (m1, m2):
            _, loss = m(x, x.roll(1, 1))
            loss.backward()
        opt.step()
        opt.zero_grad()
        ref.step()
        ref.zero_grad()
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        assert torch.allclose(a, b, atol=1e-6, rtol=1e-5), n


def test_flat_adamw_params_are_views_and_state_dict_roundtrip():
    m = _model()
    opt = FlatAdamW(m, lr=1e-3)
    for p in m.parameters():
        assert p.data_ptr() >= opt.flat_param.data_ptr()
        assert p.grad is not None and p.grad.data_ptr() >= opt.flat_grad.data_ptr()
    x = torch.randint(0, 128, (2, 16))
    _, loss = m(x, x)
    loss.backward()
    opt.step()
    sd = opt.state_dict()
    assert set(sd["state"][0]) >= {"step", "exp_avg", "exp_avg_sq"}
    assert sd["param_groups"][0]["betas"] == (0.9, 0.999)
    m2 = _model()
    m2.load_state_dict(m.state_dict())
    opt2 = FlatAdamW(m2, lr=1e-3)
    opt2.load_state_dict(sd)
    assert opt2.step_count == 1
    assert torch.equal(opt2.exp_avg, opt.exp_avg) and torch.equal(opt2.master, opt.master)


def test_grad_clipping():
    m = _model()
    opt = FlatAdamW(m, lr=1e-3, max_grad_norm=1e-3)
    x = torch.randint(0, 128, (2, 16))
    _, loss = m(x, x)
    loss.backward()
    n = opt.grad_norm()
    ref = torch.sqrt(sum(p.grad.float().pow(2).sum() for p in m.parameters()))
    assert torch.allclose(n, ref, rtol=1e-5)
    opt.step()
    assert opt.last_grad_norm is not None


def test_workspace_budgets_follow_free_hbm():
    """LM-head/CE chunk and attention-backward slab budgets: a quarter of the free HBM, clamped to
    [floor, cap] (utils/memory.py); a small budget splits the CE rows into 64-aligned chunks."""
    from pretraining_llm_amd.ops import _ce_chunk_rows
    from pretraining_llm_amd.utils import memory as M
    dev = torch.device("cuda", 0)
    GiB = 2 ** 30
    M.live_budgets()  # a Trainer built by an earlier test froze them
    assert M.workspace_budget(dev, M.CE_CAP, M.CE_FRACTION, M.CE_FLOOR, free_fn=lambda d: 200 * GiB) == M.CE_CAP
    assert M.workspace_budget(dev, M.CE_CAP, M.CE_FRACTION, M.CE_FLOOR, free_fn=lambda d: 8 * GiB) == 2 * GiB
    assert M.workspace_budget(dev, M.CE_CAP, M.CE_FRACTION, M.CE_FLOOR, free_fn=lambda d: 0) == M.CE_FLOOR
    assert M.workspace_budget(torch.device("cpu"), 5, 0.25, 1) == 5
    N, V = 65536, 50304  # GPT-2 small B64 x T1024
    assert _ce_chunk_rows(N, V, M.CE_CAP) == N                     # one chunk with a roomy device
    r = _ce_chunk_rows(N, V, 2 * GiB)                               # a fuller device: 4 chunks
    assert r % 64 == 0 and -(-N // r) == 4 and r * V * 2 <= 2 * GiB + 64 * V * 2
    # frozen at first use (the Trainer's default) / pinned to the cap (deterministic=True)
    try:
        M.freeze_budgets()
        first = M.workspace_budget(dev, M.CE_CAP, M.CE_FRACTION, M.CE_FLOOR, free_fn=lambda d: 8 * GiB)
        later = M.workspace_budget(dev, M.CE_CAP, M.CE_FRACTION, M.CE_FLOOR, free_fn=lambda d: 1 * GiB)
        assert first == later == 2 * GiB
        M.freeze_budgets(pin_caps=True)
        assert M.workspace_budget(dev, M.CE_CAP, M.CE_FRACTION, M.CE_FLOOR, free_fn=lambda d: 1 * GiB) == M.CE_CAP
    finally:
        M.live_budgets()


def test_lazy_zero_accumulate_only_runs():
    """train/optim.accumulate_only_runs: the ranges lazy zeroing clears cover every slot except the fresh
    (weight-GEMM) ones, padding included, merged and ALIGN-aligned."""
    import torch.nn as nn
    from pretraining_llm_amd.train.optim import ALIGN, _round_up, accumulate_only_runs
    ps = [nn.Parameter(torch.zeros(n)) for n in (10, 64 * 3, 70, 5, 128, 1)]
    offs, o = {}, 0
    for i, p in enumerate(ps):
        offs[i] = o
        o += _round_up(p.numel(), ALIGN)
    total = _round_up(o, 4 * ALIGN)
    fresh = {id(ps[1]), id(ps[4])}
    runs = accumulate_only_runs(ps, offs, total, fresh)
    covered = torch.zeros(total, dtype=torch.bool)
    for a, b in runs:
        assert a % ALIGN == 0 and b % ALIGN == 0 and a < b
        covered[a:b] = True
    for i, p in enumerate(ps):
        seg = covered[offs[i]:offs[i] + p.numel()]
        assert (not seg.any()) if id(p) in fresh else seg.all()
    assert covered[o:].all()  # tail padding
    assert all(runs[k][1] < runs[k + 1][0] for k in range(len(runs) - 1))  # merged, ordered

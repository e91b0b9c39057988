"""Numerics at scale on the GPU: >= 100 optimizer steps of a small GPT-2 on the learnable Markov
synthetic stream through the hand-written HIP kernels track the same run on stock PyTorch ops
(scripts/convergence.py; the full GPT-2-small curves are in profiles/r2_convergence_*.jsonl)."""
import pytest

pytestmark = pytest.mark.gpu


def test_hip_training_tracks_stock_torch(tmp_path):
    from scripts.convergence import train_curve
    kw = dict(model="gpt2-tiny", steps=120, batch=8, seq=256, lr=1e-3, log_every=10, tokens=600_000,
              data_dir=str(tmp_path))
    hip, _ = train_curve("auto", **kw)
    ref, _ = train_curve("torch", **kw)
    first, last = hip[0][1], hip[-1][1]
    assert last < first - 2.0, hip          # it learns (from ~ln V = 10.8)
    gap = abs(last - ref[-1][1]) / ref[-1][1]
    assert gap < 0.02, (hip[-1], ref[-1])  # and tracks the stock-op run
    # the whole curve, not just the end point
    for (s1, a, _), (s2, b, _) in zip(hip, ref):
        assert s1 == s2 and abs(a - b) / b < 0.03, (s1, a, b)

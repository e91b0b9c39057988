"""Batched generation service (pretraining_llm_amd/inference/server.py) on CPU: concurrent requests
with one prompt length share a decode batch, greedy outputs equal single-request generate(), the
HTTP layer (FastAPI TestClient) round-trips tokens and text, bad requests are rejected."""
import threading

import pytest
import torch

from pretraining_llm_amd.inference.server import GenerationServer, GenRequest, create_app
from pretraining_llm_amd.models import GPT, get_preset


@pytest.fixture(scope="module")
def model():
    torch.manual_seed(0)
    return GPT(get_preset("gpt2-tiny").replace(context_length=64)).eval()


def test_batches_concurrent_requests_and_matches_generate(model):
    srv = GenerationServer(model, max_batch=8, max_wait_ms=200.0)
    try:
        prompts = [[5, 9, 13, 2], [7, 7, 1, 3], [100, 4, 8, 15], [42, 42, 42, 42], [1, 2, 3]]
        futs = [srv.submit(GenRequest(p, max_new_tokens=6, temperature=0.0)) for p in prompts]
        res = [f.result(timeout=120) for f in futs]
        assert [r.batch_size for r in res[:4]] == [4, 4, 4, 4] and res[4].batch_size == 1
        for p, r in zip(prompts, res):
            ref = model.generate(torch.tensor([p]), max_new_tokens=6, temperature=0.0)[0].tolist()
            assert r.tokens == ref and r.new_tokens == ref[len(p):]
        assert srv.stats["requests"] == 5 and srv.stats["batches"] == 2 and srv.stats["max_batch_seen"] == 4
        with pytest.raises(ValueError):
            srv.submit(GenRequest([], max_new_tokens=3))
        with pytest.raises(ValueError):
            srv.submit(GenRequest([model.config.vocab_size], max_new_tokens=3))
    finally:
        srv.close()


def test_http_app(model):
    pytest.importorskip("httpx")
    from fastapi.testclient import TestClient

    from pretraining_llm_amd.data.tokenizer import ByteTokenizer
    srv = GenerationServer(model, max_batch=4, max_wait_ms=100.0)
    try:
        client = TestClient(create_app(srv, ByteTokenizer()))
        h = client.get("/health").json()
        assert h["status"] == "ok" and h["n_blocks"] == 2
        out = {}

        def call(i):
            out[i] = client.post("/generate", json={"tokens": [3, 1, 4, 1 + i], "max_new_tokens": 5,
                                                    "temperature": 0.0}).json()
        ts = [threading.Thread(target=call, args=(i,)) for i in range(3)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert all(len(out[i]["tokens"]) == 5 and out[i]["prompt_tokens"] == 4 for i in range(3))
        assert max(out[i]["batch_size"] for i in range(3)) >= 2
        r = client.post("/generate", json={"prompt": "hi", "max_new_tokens": 3, "temperature": 0.0}).json()
        assert r["text"].startswith("hi") and len(r["tokens"]) == 3
        assert client.post("/generate", json={"max_new_tokens": 3}).status_code == 400
        assert client.get("/stats").json()["requests"] >= 4
    finally:
        srv.close()


@pytest.mark.parametrize("preset", ["gpt2-tiny", "llama-tiny"])
def test_continuous_batching_matches_single_requests(preset):
    """Mixed prompt lengths share the decode slots (per-sequence positions); slots recycle as
    requests finish; greedy outputs equal single-request generate(), including a learned-position
    sequence that runs past context_length (crop semantics) and a one-token request."""
    from pretraining_llm_amd.inference.server import ContinuousGenerationServer
    torch.manual_seed(1)
    cfg = get_preset(preset).replace(context_length=64)
    m = GPT(cfg).eval()
    V = cfg.vocab_size
    g = torch.Generator().manual_seed(3)
    reqs = [(torch.randint(0, V, (n,), generator=g).tolist(), k)
            for n, k in [(5, 7), (11, 3), (2, 9), (17, 1), (8, 6), (30, 5)]]
    if cfg.pos == "learned":
        reqs.append((torch.randint(0, V, (60,), generator=g).tolist(), 10))  # crosses the 64-token context
    srv = ContinuousGenerationServer(m, max_batch=3, max_len=80)
    try:
        futs = [srv.submit(GenRequest(p, max_new_tokens=k, temperature=0.0)) for p, k in reqs]
        res = [f.result(timeout=300) for f in futs]
    finally:
        srv.close()
    for (p, k), r in zip(reqs, res):
        ref = m.generate(torch.tensor([p]), max_new_tokens=k, temperature=0.0)[0].tolist()
        assert r.tokens == ref, (len(p), k)
    assert srv.stats["requests"] == len(reqs) and srv.stats["max_active_slots"] == 3
    assert max(r.batch_size for r in res) == 3


def test_continuous_batching_rejects_and_closes():
    from pretraining_llm_amd.inference.server import ContinuousGenerationServer
    m = GPT(get_preset("llama-tiny").replace(context_length=32)).eval()
    srv = ContinuousGenerationServer(m, max_batch=2, max_len=40)
    try:
        with pytest.raises(ValueError):
            srv.submit(GenRequest([1, 2, 3], max_new_tokens=38))  # beyond the cache length
        assert len(srv.submit(GenRequest([1, 2, 3], max_new_tokens=4, temperature=0.7, seed=5)).result(60).new_tokens) == 4
    finally:
        srv.close()
    with pytest.raises(RuntimeError):
        srv.submit(GenRequest([1], max_new_tokens=1))


def test_http_app_continuous(model):
    pytest.importorskip("httpx")
    from fastapi.testclient import TestClient

    from pretraining_llm_amd.data.tokenizer import ByteTokenizer
    from pretraining_llm_amd.inference.server import ContinuousGenerationServer
    srv = ContinuousGenerationServer(model, max_batch=4)
    try:
        client = TestClient(create_app(srv, ByteTokenizer()))
        outs = {}

        def call(i):
            outs[i] = client.post("/generate", json={"tokens": list(range(1, 3 + i)), "max_new_tokens": 4 + i,
                                                     "temperature": 0.0}).json()
        ts = [threading.Thread(target=call, args=(i,)) for i in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        for i in range(4):
            ref = model.generate(torch.tensor([list(range(1, 3 + i))]), max_new_tokens=4 + i, temperature=0.0)
            assert outs[i]["tokens"] == ref[0, 2 + i:].tolist()
        assert client.get("/stats").json()["requests"] == 4
    finally:
        srv.close()


def _latency_matches_observed(srv, reqs):
    """Submit ``reqs`` at once; every result's latency_ms must sit within 10 % of the wall time the
    caller observes between its submit and the future completing (stamped after the host read-back,
    never at enqueue time)."""
    import time
    done_at = {}
    futs = []
    for i, r in enumerate(reqs):
        f = srv.submit(r)
        f.add_done_callback(lambda _f, i=i: done_at.__setitem__(i, time.perf_counter()))
        futs.append(f)
    res = [f.result(timeout=300) for f in futs]
    for i, (r, out) in enumerate(zip(reqs, res)):
        observed = 1e3 * (done_at[i] - r.t_submit)
        assert out.latency_ms <= observed + 1e-3 and out.latency_ms >= 0.9 * observed - 1.0, (i, out.latency_ms, observed)
    return res


@pytest.mark.parametrize("continuous", [False, True])
def test_latency_is_wall_time(model, continuous):
    from pretraining_llm_amd.inference.server import ContinuousGenerationServer
    srv = ContinuousGenerationServer(model, max_batch=4) if continuous else GenerationServer(model, max_batch=8,
                                                                                               max_wait_ms=50.0)
    try:
        _latency_matches_observed(srv, [GenRequest([3, 1, 4, 1 + i], max_new_tokens=6, temperature=0.0)
                                        for i in range(6)])
    finally:
        srv.close()


def test_seeded_requests_reproducible_regardless_of_batch(model):
    """Two concurrent requests with the same seed get the same tokens as a single-request
    generate() with that seed: seeded requests are never batched together."""
    srv = GenerationServer(model, max_batch=8, max_wait_ms=100.0)
    try:
        p = [5, 9, 13, 2]
        futs = [srv.submit(GenRequest(p, max_new_tokens=8, temperature=0.9, seed=11)) for _ in range(2)]
        res = [f.result(timeout=120) for f in futs]
    finally:
        srv.close()
    g = torch.Generator().manual_seed(11)
    ref = model.generate(torch.tensor([p]), max_new_tokens=8, temperature=0.9, generator=g)[0].tolist()
    assert res[0].tokens == ref and res[1].tokens == ref
    assert all(r.batch_size == 1 for r in res)


def test_submit_after_close_fails_fast(model):
    srv = GenerationServer(model, max_batch=2)
    srv.close()
    with pytest.raises(RuntimeError):
        srv.submit(GenRequest([1, 2], max_new_tokens=2))

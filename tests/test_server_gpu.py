"""Batched generation service on the GPU: the HIP decode path (hipGraph-replayed steps) serves a
batch of concurrent requests; each request's tokens equal a direct batched generate() of the same
prompts (the service only groups and dispatches)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_server_gpu_batch_matches_generate():
    from pretraining_llm_amd.inference.server import GenerationServer, GenRequest
    from pretraining_llm_amd.models import GPT, get_preset
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    model = GPT(get_preset("gpt2-tiny").replace(context_length=128)).to(device=dev, dtype=torch.bfloat16).eval()
    prompts = [[(7 * i + j) % 500 for j in range(12)] for i in range(6)]
    srv = GenerationServer(model, max_batch=8, max_wait_ms=300.0)
    try:
        futs = [srv.submit(GenRequest(p, max_new_tokens=10, temperature=0.0)) for p in prompts]
        res = [f.result(timeout=120) for f in futs]
    finally:
        srv.close()
    assert all(r.batch_size == 6 for r in res)
    ref = model.generate(torch.tensor(prompts, device=dev), max_new_tokens=10, temperature=0.0,
                         cuda_graph=True).tolist()
    assert [r.tokens for r in res] == ref


def test_decode_kernels_per_row_positions():
    """attn_decode with one key count per sequence and the skinny GEMM's KV-cache append at one
    position per row equal the per-sequence calls."""
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    torch.manual_seed(2)
    dev = torch.device("cuda", 0)
    B, S, H, Hkv, D = 5, 96, 8, 4, 64
    q = torch.randn(B, 1, H, D, device=dev).bfloat16()
    k = torch.randn(B, S, Hkv, D, device=dev).bfloat16()
    v = torch.randn(B, S, Hkv, D, device=dev).bfloat16()
    lens = torch.tensor([1, 17, 96, 40, 63], dtype=torch.int32, device=dev)
    o = torch.ops.pllm.attn_decode(q, k, v, 0.125, lens)
    for b in range(B):
        ob = torch.ops.pllm.attn_decode(q[b:b + 1], k[b:b + 1], v[b:b + 1], 0.125, lens[b:b + 1])
        assert torch.equal(o[b:b + 1], ob), b
    # KV append at per-row positions from the decode QKV projection epilogue
    M, K = 3, 256
    kvc = Hkv * D
    N = H * D + 2 * kvc
    x = torch.randn(M, K, device=dev).bfloat16()
    w = torch.randn(N, K, device=dev).bfloat16() * 0.05
    kc = torch.zeros(M, S, Hkv, D, device=dev).bfloat16()
    vc = torch.zeros_like(kc)
    pos = torch.tensor([0, 7, 95], dtype=torch.long, device=dev)
    y = torch.ops.pllm.gemv(x, w, None, None, None, None, 1e-5, 0, 0, kc, vc, pos, H * D)[0]
    for m, p in enumerate(pos.tolist()):
        assert torch.equal(kc[m, p].reshape(-1), y[m, H * D:H * D + kvc])
        assert torch.equal(vc[m, p].reshape(-1), y[m, H * D + kvc:])
        assert kc[m].reshape(S, -1).abs().sum(-1).nonzero().view(-1).tolist() == [p]


@pytest.mark.parametrize("preset", ["gpt2-tiny", "llama-tiny"])
def test_continuous_batching_gpu_matches_single_requests(preset):
    from pretraining_llm_amd.inference.server import ContinuousGenerationServer, GenRequest
    from pretraining_llm_amd.models import GPT, get_preset
    torch.manual_seed(4)
    dev = torch.device("cuda", 0)
    cfg = get_preset(preset).replace(context_length=128)
    model = GPT(cfg).to(device=dev, dtype=torch.bfloat16).eval()
    g = torch.Generator().manual_seed(5)
    reqs = [(torch.randint(0, cfg.vocab_size, (n,), generator=g).tolist(), k)
            for n, k in [(9, 12), (33, 5), (3, 20), (64, 8), (17, 1), (40, 16)]]
    srv = ContinuousGenerationServer(model, max_batch=4, max_len=160)
    try:
        res = [f.result(timeout=120) for f in [srv.submit(GenRequest(p, max_new_tokens=k, temperature=0.0))
                                                for p, k in reqs]]
    finally:
        srv.close()
    for (p, k), r in zip(reqs, res):
        ref = model.generate(torch.tensor([p], device=dev), max_new_tokens=k, temperature=0.0,
                             cuda_graph=True)[0].tolist()
        assert r.tokens == ref, (len(p), k)
    assert srv.stats["max_active_slots"] == 4


@pytest.mark.parametrize("continuous", [False, True])
def test_server_gpu_latency_is_wall_time(continuous):
    """Decode is asynchronous on the GPU: latency_ms must include the device work (stamped after the
    host read-back), i.e. match the caller's own submit -> completion time within 10 %."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_server import _latency_matches_observed

    from pretraining_llm_amd.inference.server import ContinuousGenerationServer, GenerationServer, GenRequest
    from pretraining_llm_amd.models import GPT, get_preset
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    model = GPT(get_preset("gpt2-small").replace(context_length=256)).to(device=dev, dtype=torch.bfloat16).eval()
    srv = ContinuousGenerationServer(model, max_batch=16, max_len=200) if continuous else \
        GenerationServer(model, max_batch=16, max_wait_ms=50.0)
    try:
        srv.submit(GenRequest([1, 2, 3], max_new_tokens=4, temperature=0.0)).result(timeout=120)  # warm-up
        _latency_matches_observed(srv, [GenRequest([(5 * i + j) % 1000 for j in range(16)], max_new_tokens=64,
                                                   temperature=0.8) for i in range(16)])
    finally:
        srv.close()

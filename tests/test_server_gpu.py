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

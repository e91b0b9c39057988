"""Serving throughput of the batched generation service (pretraining_llm_amd/inference/server.py):
N concurrent requests (same prompt length / sampling) vs the same requests one at a time, GPT-2
small (random init, bf16) on one MI355X.  Prints one JSON line per mode."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--requests", type=int, default=64)
    ap.add_argument("--prompt", type=int, default=32)
    ap.add_argument("--new", type=int, default=128)
    ap.add_argument("--sequential", type=int, default=8, help="requests timed one at a time (batch 1)")
    a = ap.parse_args()
    from pretraining_llm_amd.inference.server import GenerationServer, GenRequest
    from pretraining_llm_amd.models import GPT, get_preset
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    model = GPT(get_preset(a.model)).to(device=dev, dtype=torch.bfloat16).eval()
    V = model.config.vocab_size
    g = torch.Generator().manual_seed(1)
    prompts = torch.randint(0, V, (a.requests, a.prompt), generator=g).tolist()
    srv = GenerationServer(model, max_batch=a.requests, max_wait_ms=50.0)
    try:
        srv.submit(GenRequest(prompts[0], max_new_tokens=4, temperature=0.8)).result()  # warm-up
        t0 = time.perf_counter()
        futs = [srv.submit(GenRequest(p, max_new_tokens=a.new, temperature=0.8)) for p in prompts]
        res = [f.result() for f in futs]
        dt = time.perf_counter() - t0
        print(json.dumps({"mode": "batched", "requests": a.requests, "new_tokens": a.new, "wall_s": round(dt, 3),
                          "tokens_per_s": round(a.requests * a.new / dt, 1),
                          "batch_sizes": sorted({r.batch_size for r in res}),
                          "p50_latency_ms": sorted(r.latency_ms for r in res)[len(res) // 2]}), flush=True)
        t0 = time.perf_counter()
        for p in prompts[:a.sequential]:
            srv.submit(GenRequest(p, max_new_tokens=a.new, temperature=0.8)).result()
        dt = time.perf_counter() - t0
        print(json.dumps({"mode": "one_at_a_time", "requests": a.sequential, "new_tokens": a.new,
                          "wall_s": round(dt, 3), "tokens_per_s": round(a.sequential * a.new / dt, 1)}), flush=True)
    finally:
        srv.close()


if __name__ == "__main__":
    main()

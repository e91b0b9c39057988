"""Serving throughput of the generation services (pretraining_llm_amd/inference/server.py), GPT-2
small (random init, bf16) on one MI355X: N concurrent requests of one prompt length through the
lockstep server, N requests of MIXED prompt lengths through the continuous-batching server and
through the lockstep server, and a few requests one at a time.  Prints one JSON line per mode."""
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
    from pretraining_llm_amd.inference.server import ContinuousGenerationServer, GenerationServer, GenRequest
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
        # mixed prompt lengths: lockstep can only batch equal lengths
        mixed = [torch.randint(0, V, (int(n),), generator=g).tolist()
                 for n in torch.randint(8, 2 * a.prompt, (a.requests,), generator=g)]
        t0 = time.perf_counter()
        res = [f.result() for f in [srv.submit(GenRequest(p, max_new_tokens=a.new, temperature=0.8)) for p in mixed]]
        dt = time.perf_counter() - t0
        print(json.dumps({"mode": "lockstep_mixed_lengths", "requests": a.requests, "new_tokens": a.new,
                          "wall_s": round(dt, 3), "tokens_per_s": round(a.requests * a.new / dt, 1),
                          "max_batch": max(r.batch_size for r in res)}), flush=True)
    finally:
        srv.close()
    cs = ContinuousGenerationServer(model, max_batch=a.requests, max_len=2 * a.prompt + a.new + 8)
    try:
        cs.submit(GenRequest(mixed[0], max_new_tokens=4, temperature=0.8)).result()  # warm-up
        t0 = time.perf_counter()
        res = [f.result() for f in [cs.submit(GenRequest(p, max_new_tokens=a.new, temperature=0.8)) for p in mixed]]
        dt = time.perf_counter() - t0
        assert all(len(r.new_tokens) == a.new for r in res)
        lat = sorted(r.latency_ms for r in res)
        print(json.dumps({"mode": "continuous_mixed_lengths", "requests": a.requests, "new_tokens": a.new,
                          "latency_ms_min_max": [round(lat[0], 1), round(lat[-1], 1)],
                          "wall_s": round(dt, 3), "tokens_per_s": round(a.requests * a.new / dt, 1),
                          "max_active_slots": cs.stats["max_active_slots"], "decode_steps": cs.stats["decode_steps"],
                          "p50_latency_ms": round(sorted(r.latency_ms for r in res)[len(res) // 2], 1)}), flush=True)
    finally:
        cs.close()


if __name__ == "__main__":
    main()

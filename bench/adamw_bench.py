"""Fused flat AdamW (+ the grad-norm sum of squares) alone at the GPT-2-small and llama-1.3B parameter counts:
fp32 gradient / master / moments, bf16 params.  Median us per call and TB/s of the bytes moved (AdamW: 4 fp32
reads + 3 fp32 writes + 1 bf16 write per parameter; sumsq: 1 fp32 read).  Select an A/B build with PLLM_SO."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timeit(fn, reps=5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    P = torch.ops.pllm
    for name, n in (("gpt2-small", 124_475_904), ("llama-1.3b", 1_423_000_000)):
        n = n // 64 * 64
        g = torch.randn(n, device="cuda") * 1e-3
        master = torch.randn(n, device="cuda")
        m = torch.zeros(n, device="cuda")
        v = torch.zeros(n, device="cuda")
        p = master.bfloat16()
        step = [0]

        def adam():
            step[0] += 1
            P.adamw_(p, master, m, v, g, 1e-4, 0.9, 0.95, 1e-8, 0.1, step[0], 1.0, None, None, None)

        def ss():
            P.sumsq(g)
        for _ in range(3):
            adam()
            ss()
        ta = statistics.median(timeit(adam) for _ in range(5))
        ts = statistics.median(timeit(ss) for _ in range(5))
        print(json.dumps({"model": name, "n": n, "adamw_us": round(ta, 1), "adamw_tbs": round(n * 30 / ta / 1e6, 2),
                          "sumsq_us": round(ts, 1), "sumsq_tbs": round(n * 4 / ts / 1e6, 2),
                          "so": os.environ.get("PLLM_SO", "in-tree")}), flush=True)
        del g, master, m, v, p
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

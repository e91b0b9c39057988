"""Probe: the GPT-2 forward projection GEMMs (bias epilogue) under the shipped TunableOp table vs the
library heuristics, same process / timing; inputs like the step's (LayerNorm output, GPT-2 init)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def timeit(fn, iters=20, rounds=5):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(rounds):
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / iters)
    return round(best * 1e6, 1)


def main():
    tuned = len(sys.argv) > 1 and sys.argv[1] == "tuned"
    if tuned:
        from pretraining_llm_amd.utils.gemm_tuning import enable_tuned_gemms
        enable_tuned_gemms(0)
    M = 65536
    for N, K in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
        torch.manual_seed(0)
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
        b = (torch.randn(N, device="cuda") * 0.02).bfloat16()
        r = {"N": N, "K": K, "tuned": tuned}
        for rep in range(2):
            r[f"linear_bias_us_{rep}"] = timeit(lambda: F.linear(x, w, b))
            r[f"linear_nobias_us_{rep}"] = timeit(lambda: F.linear(x, w))
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()

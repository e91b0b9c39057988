"""Split-K slice-count sweep of the weight-gradient kernel (csrc/gemm_wgrad.hip) on the GPT-2-small /
llama-1.3B training shapes: the cost-model choice (wgrad_plan) against forced counts, fp32 target,
kernel + slab reduce timed together (min over rounds).  One JSON line per shape."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timeit(fn, iters=10, rounds=3):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(rounds):
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / iters)
    return best * 1e6


def main():
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    P_ = torch.ops.pllm
    shapes = [(65536, 2304, 768), (65536, 768, 768), (65536, 3072, 768), (65536, 768, 3072), (65536, 50304, 768),
              (32768, 6144, 2048), (32768, 2048, 2048), (32768, 11008, 2048), (32768, 2048, 5504),
              (32768, 32000, 2048)]
    for M, P, Q in shapes:
        dy = (torch.randn(M, P, device="cuda") * 0.1).bfloat16()
        x = torch.randn(M, Q, device="cuda").bfloat16()
        tgt = torch.zeros(P, Q, device="cuda")
        res = {"M": M, "P": P, "Q": Q}
        P_.wgrad_force_slices(0)
        res["auto_us"] = round(timeit(lambda: P_.wgrad(dy, x, tgt)), 1)
        best = (res["auto_us"], 0)
        for s in (1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48):
            if M // 64 // s < 8:
                break
            P_.wgrad_force_slices(s)
            t = round(timeit(lambda: P_.wgrad(dy, x, tgt)), 1)
            res[f"s{s}_us"] = t
            best = min(best, (t, s))
        P_.wgrad_force_slices(0)
        res["best_s"], res["best_us"] = best[1], best[0]
        res["gain_pct"] = round(100 * (res["auto_us"] - best[0]) / res["auto_us"], 1)
        print(json.dumps(res), flush=True)
        del dy, x, tgt


if __name__ == "__main__":
    main()

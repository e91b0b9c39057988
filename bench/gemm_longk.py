"""Main-loop ceiling at long K: the ping-pong TN GEMM (gemm_tn epi 0) vs hipBLASLt (F.linear) vs the
weight-gradient kernel on the same FLOPs in token-major form (dW[P,Q] = dY[M,P]^T X[M,Q] with
M = K) -- does a ping-pong main loop with transposed fragment reads have room over wgrad_kernel?
Interleaved rounds, median microseconds.  usage: python bench/gemm_longk.py [--rounds 5]"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

# (rows, cols, K): TN rows x cols over K; the wgrad form has P = rows, Q = cols, M = K tokens
SHAPES = [(50304, 768, 65536), (65536, 768, 50304), (3072, 768, 65536), (11008, 2048, 32768), (6144, 2048, 32768)]


def once(fn, reps=3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    P_ = torch.ops.pllm
    P_.gemm_set_config(16, 4, 4)
    for R, C, K in SHAPES:
        a = torch.empty(R, K, device="cuda").uniform_(-1, 1).bfloat16()
        b = (torch.empty(C, K, device="cuda").uniform_(-1, 1) / K ** 0.5).bfloat16()
        var = {"pp": lambda: P_.gemm_tn(a, b, None, 0), "blas": lambda: F.linear(a, b)}
        if R != 65536:
            dy = a.t().contiguous()  # [M = K, P = R] token-major
            x = b.t().contiguous()   # [M, Q = C]
            tgt = torch.zeros(R, C, device="cuda")
            var["wgrad"] = lambda: P_.wgrad(dy, x, tgt)
        for fn in var.values():
            fn()
        ts = {k: [] for k in var}
        for _ in range(args.rounds):
            for k, fn in var.items():
                ts[k].append(once(fn))
        fl = 2 * R * C * K
        rec = {"rows": R, "cols": C, "K": K}
        for k, v in ts.items():
            med = statistics.median(v)
            rec[k + "_us"] = round(med, 1)
            rec[k + "_tflops"] = round(fl / med / 1e6, 1)
        print(json.dumps(rec), flush=True)
        del a, b, var
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

"""Microbenchmark: the GPT-2-small forward / dgrad GEMM shapes through hipBLASLt in every
operand layout the model could use (M = tokens per step), with the shipped TunableOp
selections on or off.  Used to pick the weight layout and the bias path of ops.linear.

  fwd_addmm  : F.linear(x, W, b)        (W [N,K] row-major -> "NT", bias epilogue)
  fwd_mm     : F.linear(x, W)           (no bias)
  fwd_nn     : x @ Wt, Wt = W^T stored [K,N] contiguous
  dgrad_nn   : dy @ W                   (the backward data-gradient of fwd_*)
  dgrad_nt   : dy @ Wt^T
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=65536)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--no-tuned", action="store_true")
    ap.add_argument("--shapes", default="2304x768,768x768,3072x768,768x3072,50304x768")
    args = ap.parse_args()
    if not args.no_tuned:
        from pretraining_llm_amd.utils.gemm_tuning import enable_tuned_gemms
        enable_tuned_gemms(0)
    dev = torch.device("cuda")
    M = args.M
    for s in args.shapes.split(","):
        N, K = (int(v) for v in s.split("x"))
        torch.manual_seed(0)
        x = torch.randn(M, K, device=dev).bfloat16()
        W = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
        b = torch.randn(N, device=dev).bfloat16()
        Wt = W.t().contiguous()
        dy = torch.randn(M, N, device=dev).bfloat16()
        fl = 2.0 * M * N * K
        cases = {
            "fwd_addmm": lambda: F.linear(x, W, b),
            "fwd_mm": lambda: F.linear(x, W),
            "fwd_nn": lambda: x @ Wt,
            "dgrad_nn": lambda: dy @ W,
            "dgrad_nt": lambda: dy @ Wt.t(),
        }
        res = {"N": N, "K": K, "M": M, "tuned": not args.no_tuned}
        for name, fn in cases.items():
            t = min(timeit(fn) for _ in range(args.rounds))
            res[name + "_us"] = round(1e6 * t, 1)
            res[name + "_tflops"] = round(fl / t / 1e12, 1)
        print(json.dumps(res), flush=True)
        del x, W, b, Wt, dy


if __name__ == "__main__":
    main()

"""Microbenchmark: hand-written NT GEMM with fused MLP epilogues (csrc/gemm_nt.hip) vs
hipBLASLt (+ the separate activation kernels) at the GPT-2-small shapes, M = 65,536 tokens,
random bf16 operands.  Interleaved rounds in one process; prints one JSON line per case.

  plain   : gemm_nt epi 0 (pipe 0 / 1) vs F.linear (hipBLASLt, bias epilogue)
  mlp_up  : gemm_nt epi 1 (h and gelu(h) in one pass) vs F.linear + act_fwd
  mlp_dgrad: gemm_nt epi 2 ((dy W) * gelu'(h), bias grad) vs dy @ W + act_bwd_bias
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


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm()).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=65536)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    from pretraining_llm_amd.ops import _lib
    ops = _lib.require()
    dev = torch.device("cuda")
    M = args.M
    torch.manual_seed(0)
    for N, K in ((3072, 768), (2304, 768), (768, 768), (768, 3072)):
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * K ** -0.5
        b = torch.randn(N, device=dev, dtype=torch.bfloat16) * 0.1
        ref = (x[:2048].float() @ w.float().t() + b.float())
        res = {"case": "plain", "M": M, "N": N, "K": K}
        for p in (0, 1):
            ops.gemm_nt_set_pipe(p)
            res[f"rel_err_pipe{p}"] = rel(ops.gemm_nt(x[:2048], w, b, 0)[0], ref)
        fl = 2.0 * M * N * K
        for _ in range(args.rounds):
            for p in (0, 1):
                ops.gemm_nt_set_pipe(p)
                res.setdefault(f"pipe{p}_us", []).append(1e6 * timeit(lambda: ops.gemm_nt(x, w, b, 0)))
            res.setdefault("blas_us", []).append(1e6 * timeit(lambda: F.linear(x, w, b)))
        for k in ("pipe0", "pipe1", "blas"):
            res[f"{k}_tflops"] = round(fl / (min(res[f"{k}_us"]) * 1e-6) / 1e12, 1)
        print(json.dumps(res), flush=True)
        del x, w, b

    # fused MLP epilogues at the up/down projection shapes (C=768, F=3072)
    C, Fh = 768, 3072
    x = torch.randn(M, C, device=dev, dtype=torch.bfloat16)
    w1 = torch.randn(Fh, C, device=dev, dtype=torch.bfloat16) * C ** -0.5
    b1 = torch.randn(Fh, device=dev, dtype=torch.bfloat16) * 0.1
    dy = torch.randn(M, C, device=dev, dtype=torch.bfloat16)
    wpT = torch.randn(Fh, C, device=dev, dtype=torch.bfloat16) * Fh ** -0.5   # W_p^T [F, C]
    h = F.linear(x, w1, b1)
    bg = torch.zeros(Fh, device=dev, dtype=torch.bfloat16)
    for p in (0, 1):
        ops.gemm_nt_set_pipe(p)
        g1, h1 = ops.gemm_nt(x, w1, b1, 1)
        bg.zero_()
        (dh1,) = ops.gemm_nt(dy, wpT, None, 2, h, bg)
        dref = ops.act_bwd(dy @ wpT.t(), h, 1)
        res = {"case": "fused_check", "pipe": p, "h_rel": rel(h1, h), "g_rel": rel(g1, ops.act_fwd(h, 1)),
               "dh_rel": rel(dh1, dref), "db_rel": rel(bg, dref.float().sum(0))}
        print(json.dumps(res), flush=True)
    fl = 2.0 * M * C * Fh
    res = {"case": "mlp_up", "M": M, "N": Fh, "K": C}
    res2 = {"case": "mlp_dgrad", "M": M, "N": Fh, "K": C}
    bgb = torch.zeros(Fh, device=dev, dtype=torch.bfloat16)
    for _ in range(args.rounds):
        for p in (0, 1):
            ops.gemm_nt_set_pipe(p)
            res.setdefault(f"fused_pipe{p}_us", []).append(1e6 * timeit(lambda: ops.gemm_nt(x, w1, b1, 1)))
            res2.setdefault(f"fused_pipe{p}_us", []).append(
                1e6 * timeit(lambda: ops.gemm_nt(dy, wpT, None, 2, h, bg)))
        res.setdefault("blas_plus_act_us", []).append(
            1e6 * timeit(lambda: ops.act_fwd(F.linear(x, w1, b1), 1)))
        res2.setdefault("blas_plus_act_us", []).append(
            1e6 * timeit(lambda: ops.act_bwd_bias(dy @ wpT.t(), h, 1, bgb)))
    for r in (res, res2):
        for k in list(r):
            if k.endswith("_us"):
                r[k.replace("_us", "_best_us")] = round(min(r[k]), 1)
                r[k.replace("_us", "_tflops")] = round(fl / (min(r[k]) * 1e-6) / 1e12, 1)
        print(json.dumps(r), flush=True)
    ops.gemm_nt_set_pipe(0)


if __name__ == "__main__":
    main()

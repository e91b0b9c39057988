"""Microbenchmark: weight-gradient GEMM dW[P,Q] += dY[M,P]^T X[M,Q] on MI355X,
hand-written gfx950 kernel (torch.ops.pllm.wgrad) vs hipBLASLt/rocBLAS (torch addmm_,
with the shipped TunableOp selections).  Interleaved rounds in one process."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shapes", default="gpt2", choices=["gpt2", "llama"])
    ap.add_argument("--f32", action="store_true", help="fp32 gradient target (the training default)")
    ap.add_argument("--variants", default="32,16", help="wgrad_set_mfma values to compare (32: 32x32x16 tiles, 16: 16x16x32 tiles)")
    args = ap.parse_args()
    from pretraining_llm_amd.ops import _lib
    from pretraining_llm_amd.utils.gemm_tuning import enable_tuned_gemms
    _lib.require()
    enable_tuned_gemms(0)
    dev = torch.device("cuda")
    M = args.M
    shapes = {"gpt2": [(2304, 768), (768, 768), (3072, 768), (768, 3072), (50304, 768)],
              "llama": [(6144, 2048), (2048, 2048), (11008, 2048), (2048, 5504), (50304, 2048)]}[args.shapes]
    out = []
    for P, Q in shapes:
        torch.manual_seed(0)
        dy = (torch.randn(M, P, device=dev) * 0.1).bfloat16()
        x = torch.randn(M, Q, device=dev).bfloat16()
        tgt = torch.zeros(P, Q, device=dev, dtype=torch.float32 if args.f32 else torch.bfloat16)
        # correctness on the first 4096 rows
        r = torch.ops.pllm.wgrad(dy[:4096], x[:4096])
        ref = dy[:4096].float().t() @ x[:4096].float()
        rel = ((r.float() - ref).norm() / ref.norm()).item()
        flops = 2.0 * M * P * Q
        res = {"P": P, "Q": Q, "M": M, "rel_err": rel}
        variants = [int(v) for v in args.variants.split(",")]
        for mf in variants:
            torch.ops.pllm.wgrad_set_mfma(mf)
            r = torch.ops.pllm.wgrad(dy[:4096], x[:4096])
            res[f"rel_err{mf}"] = ((r.float() - ref).norm() / ref.norm()).item()
        for _ in range(args.rounds):
            for mf in variants:
                torch.ops.pllm.wgrad_set_mfma(mf)
                res.setdefault(f"hip{mf}_us", []).append(1e6 * timeit(lambda: torch.ops.pllm.wgrad(dy, x, tgt)))
            if not args.f32:
                res.setdefault("blas_us", []).append(1e6 * timeit(lambda: tgt.addmm_(dy.t(), x)))
        torch.ops.pllm.wgrad_set_mfma(32)
        for k in [f"hip{v}" for v in variants] + ([] if args.f32 else ["blas"]):
            res[f"{k}_tflops"] = flops / (min(res[f"{k}_us"]) * 1e-6) / 1e12
        print(json.dumps(res), flush=True)
        out.append(res)
        del dy, x, tgt


if __name__ == "__main__":
    main()

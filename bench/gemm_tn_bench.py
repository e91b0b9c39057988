"""Time the hand-written fused-epilogue TN GEMM (torch.ops.pllm.gemm_tn) against hipBLASLt
(torch F.linear / mm) on the GPT-2 / Llama training shapes, and the fused MLP epilogues against
the unfused GEMM + activation pair.  One JSON line per case (min over rounds).

usage: python bench/gemm_tn_bench.py [--mf 32|16] [--group 4]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

# (M, N, K): forward projections (N = out features) of GPT-2 small B64 and llama-1.3B B16
SHAPES = [(65536, 3072, 768), (65536, 768, 3072), (65536, 2304, 768), (65536, 768, 768),
          (32768, 11008, 2048), (32768, 2048, 5504), (32768, 6144, 2048), (32768, 2048, 2048)]


def timeit(fn, rounds=5, reps=5):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(rounds):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) / reps)
    return min(ts) * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mf", type=int, default=16)
    ap.add_argument("--group", type=int, default=4)
    ap.add_argument("--fused", action="store_true", help="also time the fused MLP epilogues")
    ap.add_argument("--phased", type=int, default=0)
    ap.add_argument("--swiglu", action="store_true",
                    help="only the llama SwiGLU backward: gemm_tn epilogue 5 vs hipBLASLt + swiglu_bwd")
    args = ap.parse_args()
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    P = torch.ops.pllm
    P.gemm_set_config(args.mf, args.group, args.phased)
    if args.swiglu:
        # llama-1.3B B16 T2048 (C 2048, F 5504) and B8: dA[M, F] = dy[M, C] @ W_down[C, F] -> [dg | du]
        for M, F_, C in ((32768, 5504, 2048), (16384, 5504, 2048)):
            dy = torch.randn(M, C, device="cuda").bfloat16()
            wdt = (torch.randn(F_, C, device="cuda") / C ** 0.5).bfloat16()  # W_down^T shadow [F, C]
            gu = torch.randn(M, 2 * F_, device="cuda").bfloat16()
            fused = timeit(lambda: P.gemm_tn(dy, wdt, None, 5, gu))
            P.gemm_set_config(args.mf, args.group, 4)
            fused_pp = timeit(lambda: P.gemm_tn(dy, wdt, None, 5, gu))
            P.gemm_set_config(args.mf, args.group, args.phased)
            unf = timeit(lambda: P.swiglu_bwd(dy @ wdt.t(), gu))
            dg = timeit(lambda: dy @ wdt.t())
            print(json.dumps({"M": M, "F": F_, "C": C, "mf": args.mf, "fused_swiglu_bwd_us": round(fused, 1), "pp_fused_swiglu_bwd_us": round(fused_pp, 1),
                              "blas_plus_swiglu_bwd_us": round(unf, 1), "blas_dgrad_us": round(dg, 1)}), flush=True)
            del dy, wdt, gu
        return
    for M, N, K in SHAPES:
        a = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
        b = torch.randn(N, device="cuda").bfloat16()
        fl = 2 * M * N * K
        ours = timeit(lambda: P.gemm_tn(a, w, b, 0))
        lib = timeit(lambda: F.linear(a, w, b))
        rec = {"M": M, "N": N, "K": K, "mf": args.mf, "group": args.group, "phased": args.phased, "ours_us": round(ours, 1),
               "ours_tflops": round(fl / ours / 1e6, 1), "blas_us": round(lib, 1),
               "blas_tflops": round(fl / lib / 1e6, 1)}
        if args.fused and N > K:
            rec["fused_gelu_us"] = round(timeit(lambda: P.gemm_tn(a, w, b, 1)), 1)
            rec["blas_plus_gelu_us"] = round(timeit(lambda: P.act_fwd(F.linear(a, w, b), 1)), 1)
            # MLP down-projection data gradient: dA[M, N] = dy[M, K] @ W_down[K, N], fused with the
            # GELU backward + bias-gradient column sums; B operand = W_down^T [N, K] (the shadow)
            pre = torch.randn(M, N, device="cuda").bfloat16()
            dy = torch.randn(M, K, device="cuda").bfloat16()
            wdown = (torch.randn(K, N, device="cuda") / N ** 0.5).bfloat16()
            wdt = wdown.t().contiguous()
            acc = torch.zeros(N, device="cuda")
            rec["fused_dgelu_us"] = round(timeit(lambda: P.gemm_tn(dy, wdt, None, 3, pre, acc)), 1)
            rec["blas_plus_dgelu_us"] = round(timeit(lambda: P.act_bwd_bias(dy @ wdt.t(), pre, 1, acc)), 1)
            del pre, dy, wdown, wdt, acc
        print(json.dumps(rec), flush=True)
        del a, w, b


if __name__ == "__main__":
    main()

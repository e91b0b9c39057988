"""One-wave-per-SIMD TN GEMM (csrc/gemm_1w.hip) vs the ping-pong kernel (gemm_tn, csrc/gemm_pp.hip) vs hipBLASLt
(F.linear) on the GPT-2 / llama training shapes, with bias, random data, interleaved rounds in one process.
One JSON line per shape: median / min microseconds and TF/s.

usage: python bench/gemm_1w_bench.py [--rounds 7] [--shapes gpt2|llama|all]"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

GPT2 = [(65536, 3072, 768), (65536, 768, 3072), (65536, 2304, 768), (65536, 768, 768), (65536, 768, 2304),
        (65536, 50304, 768)]
LLAMA = [(32768, 11008, 2048), (32768, 2048, 5504), (32768, 6144, 2048), (32768, 2048, 2048)]


def once(fn, reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--shapes", default="all", choices=["gpt2", "llama", "all"])
    args = ap.parse_args()
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    P = torch.ops.pllm
    shapes = (GPT2 if args.shapes != "llama" else []) + (LLAMA if args.shapes != "gpt2" else [])
    for M, N, K in shapes:
        g = torch.Generator(device="cuda").manual_seed(M + N + K)
        a = torch.empty(M, K, device="cuda").uniform_(-1, 1, generator=g).bfloat16()
        w = (torch.empty(N, K, device="cuda").uniform_(-1, 1, generator=g) / K ** 0.5).bfloat16()
        b = torch.empty(N, device="cuda").uniform_(-1, 1, generator=g).bfloat16()
        var = {"w1": lambda: P.gemm_1w(a, w, b), "pp": lambda: P.gemm_tn(a, w, b, 0), "blas": lambda: F.linear(a, w, b)}
        ref = F.linear(a, w, b).float()
        err = ((P.gemm_1w(a, w, b).float() - ref).norm() / ref.norm()).item()
        for fn in var.values():
            for _ in range(3):
                fn()
        ts = {k: [] for k in var}
        for _ in range(args.rounds):
            for k, fn in var.items():
                ts[k].append(once(fn, args.reps))
        fl = 2 * M * N * K
        rec = {"M": M, "N": N, "K": K, "w1_rel_err": round(err, 6)}
        for k, v in ts.items():
            med = statistics.median(v)
            rec[k + "_us"] = round(med, 1)
            rec[k + "_min_us"] = round(min(v), 1)
            rec[k + "_tflops"] = round(fl / med / 1e6, 1)
        rec["w1_vs_blas"] = round(rec["blas_us"] / rec["w1_us"], 3)
        rec["w1_vs_pp"] = round(rec["pp_us"] / rec["w1_us"], 3)
        print(json.dumps(rec), flush=True)
        del a, w, b
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

"""Ping-pong TN GEMM (csrc/gemm_pp.hip, gemm_set_config phased=4) vs the round-3 persistent kernel
(phased=0) vs hipBLASLt (F.linear, TunableOp off here) on the GPT-2 / llama training shapes, random
data, the variants INTERLEAVED round by round in one process (cdna_hip_programming.md §5.4 rule 24).
One JSON line per shape: median and min microseconds per variant, TF/s of the medians.

Variants: pp (ping-pong kernel, the default), r3, blas.

usage: python bench/gemm_pp_bench.py [--rounds 7] [--fused] [--shapes gpt2|llama|all] [--no-r3]"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

GPT2 = [(65536, 3072, 768), (65536, 768, 3072), (65536, 2304, 768), (65536, 768, 768)]
LLAMA = [(32768, 11008, 2048), (32768, 2048, 5504), (32768, 6144, 2048), (32768, 2048, 2048)]
HEAD = [(65536, 50304, 768), (32768, 50304, 2048)]  # the LM-head forwards (no bias)


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
    ap.add_argument("--fused", action="store_true", help="also the fused MLP epilogues (GELU fwd / dGELU+colsum)")
    ap.add_argument("--shapes", default="all", choices=["gpt2", "llama", "all", "head"])
    ap.add_argument("--tuned", action="store_true", help="the shipped TunableOp GEMM selections on (as in bench.py)")
    ap.add_argument("--group", type=int, default=4)
    ap.add_argument("--no-r3", action="store_true", help="skip the round-3 kernel variants")
    args = ap.parse_args()
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    P = torch.ops.pllm
    shapes = HEAD if args.shapes == "head" else \
        (GPT2 if args.shapes != "llama" else []) + (LLAMA if args.shapes != "gpt2" else [])
    if args.tuned:
        from pretraining_llm_amd.utils.gemm_tuning import enable_tuned_gemms
        enable_tuned_gemms(0)

    def with_cfg(ph, fn):
        def run():
            P.gemm_set_config(16, args.group, ph, -1)
            fn()
        return run

    for M, N, K in shapes:
        g = torch.Generator(device="cuda").manual_seed(M + N + K)
        a = torch.empty(M, K, device="cuda").uniform_(-1, 1, generator=g).bfloat16()
        w = (torch.empty(N, K, device="cuda").uniform_(-1, 1, generator=g) / K ** 0.5).bfloat16()
        b = torch.empty(N, device="cuda").uniform_(-1, 1, generator=g).bfloat16()
        if args.shapes == "head":
            var = {"pp": with_cfg(4, lambda: P.gemm_tn(a, w, None, 0)),
                   "r3": with_cfg(0, lambda: P.gemm_tn(a, w, None, 0)),
                   "blas": lambda: torch.mm(a, w.t())}
        else:
            var = {"pp": with_cfg(4, lambda: P.gemm_tn(a, w, b, 0)),
                   "r3": with_cfg(0, lambda: P.gemm_tn(a, w, b, 0)),
                   "blas": lambda: F.linear(a, w, b)}
        extra = {}
        if args.fused and N > K:
            pre = torch.empty(M, N, device="cuda").uniform_(-2, 2, generator=g).bfloat16()
            dy = torch.empty(M, K, device="cuda").uniform_(-1, 1, generator=g).bfloat16()
            wdt = (torch.empty(N, K, device="cuda").uniform_(-1, 1, generator=g) / N ** 0.5).bfloat16()
            acc = torch.zeros(N, device="cuda")
            extra = {"pp_gelu": with_cfg(4, lambda: P.gemm_tn(a, w, b, 1)),
                     "r3_gelu": with_cfg(0, lambda: P.gemm_tn(a, w, b, 1)),
                     "blas_gelu": lambda: P.act_fwd(F.linear(a, w, b), 1),
                     "pp_dgelu": with_cfg(4, lambda: P.gemm_tn(dy, wdt, None, 3, pre, acc)),
                     "r3_dgelu": with_cfg(0, lambda: P.gemm_tn(dy, wdt, None, 3, pre, acc)),
                     "blas_dgelu": lambda: P.act_bwd_bias(dy @ wdt.t(), pre, 1, acc)}
        var.update(extra)
        if args.no_r3:
            var = {k: v for k, v in var.items() if not k.startswith("r3")}
        for fn in var.values():  # warm-up (TunableOp off: library heuristics)
            for _ in range(3):
                fn()
        ts = {k: [] for k in var}
        for _ in range(args.rounds):
            for k, fn in var.items():
                ts[k].append(once(fn, args.reps))
        P.gemm_set_config(16, 4, 4, -1)  # the default kernel
        fl = 2 * M * N * K
        rec = {"M": M, "N": N, "K": K}
        for k, v in ts.items():
            med = statistics.median(v)
            rec[k + "_us"] = round(med, 1)
            rec[k + "_min_us"] = round(min(v), 1)
            if k in ("pp", "r3", "blas"):
                rec[k + "_tflops"] = round(fl / med / 1e6, 1)
        rec["pp_vs_blas"] = round(rec["blas_us"] / rec["pp_us"], 3)
        print(json.dumps(rec), flush=True)
        del a, w, b
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

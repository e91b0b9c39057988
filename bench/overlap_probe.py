"""Does a memory-bound pass hide under a weight-gradient GEMM when the two run on different HIP streams?

Pairs from the GPT-2-small backward (M = 65536 tokens): a weight-gradient GEMM (wgrad_pp, fp32 target; the
work that only feeds the flat gradient and could move to a side stream) against a memory-bound kernel of the
data-gradient chain (LayerNorm backward with the residual-stream gradient; the GELU forward pass as a second
streaming shape).  For each pair: A alone, B alone, A then B on one stream, A || B on two streams (B launched
first on the main stream, A on the side stream, joined).  Microseconds per pair, medians over rounds.

usage: python bench/overlap_probe.py [--rounds 7] [--reps 10]"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


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
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    P = torch.ops.pllm
    M, C = 65536, 768
    main_s = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    # memory-bound kernels
    s = torch.randn(M, C, device="cuda").bfloat16()
    w = torch.randn(C, device="cuda").bfloat16()
    b = torch.randn(C, device="cuda").bfloat16()
    out = P.norm_fwd(s, None, w, b, 1e-5, False)
    mean, rstd = out[-2], out[-1]
    dyn = torch.randn(M, C, device="cuda").bfloat16()
    ds = torch.randn(M, C, device="cuda").bfloat16()
    pre = torch.randn(M, 4 * C, device="cuda").bfloat16()
    mem = {"norm_bwd": lambda: P.norm_bwd(dyn, s, w, mean, rstd, ds, True, False),
           "gelu_fwd": lambda: P.act_fwd(pre, 1)}
    # weight gradients (fp32 targets, overwrite = the first write of the step)
    g_fc1 = torch.randn(M, 4 * C, device="cuda").bfloat16()
    x = torch.randn(M, C, device="cuda").bfloat16()
    t_fc1 = torch.zeros(4 * C, C, device="cuda")
    g_ao = torch.randn(M, C, device="cuda").bfloat16()
    t_ao = torch.zeros(C, C, device="cuda")
    comp = {"wgrad_fc1": lambda: P.wgrad(g_fc1, x, t_fc1, None, True),
            "wgrad_attn_out": lambda: P.wgrad(g_ao, x, t_ao, None, True)}
    ev = torch.cuda.Event()

    def par(a, bfn):
        def run():
            bfn()  # the data-gradient chain's kernel on the main stream
            ev.record(main_s)
            with torch.cuda.stream(side):
                a()  # (independent data: no wait needed for the probe)
            main_s.wait_stream(side)
        return run

    for cn, cf in comp.items():
        for mn, mf in mem.items():
            var = {"A": cf, "B": mf, "seq": lambda cf=cf, mf=mf: (mf(), cf()), "par": par(cf, mf)}
            for fn in var.values():
                for _ in range(3):
                    fn()
            ts = {k: [] for k in var}
            for _ in range(args.rounds):
                for k, fn in var.items():
                    ts[k].append(once(fn, args.reps))
            rec = {"A": cn, "B": mn}
            for k, v in ts.items():
                rec[k + "_us"] = round(statistics.median(v), 1)
            rec["par_saves_us"] = round(rec["seq_us"] - rec["par_us"], 1)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()

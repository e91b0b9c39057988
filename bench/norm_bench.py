"""Norm forward / backward microbench at the training shapes: GPT-2 (65536 x 768, LayerNorm, with and without
the fused residual add) and llama (32768 x 2048, RMSNorm).  One JSON line per case: median us and TB/s of the
bytes each call must move.  usage: python bench/norm_bench.py [--rounds 7]"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timeit(fn, reps=20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    args = ap.parse_args()
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    P = torch.ops.pllm
    for N, C, rms, res in ((65536, 768, False, False), (65536, 768, False, True), (32768, 2048, True, False),
                           (16384, 1024, False, False), (32768, 1024, False, False), (32768, 2048, True, True)):
        x = torch.randn(N, C, device="cuda").bfloat16()
        r = torch.randn(N, C, device="cuda").bfloat16() if res else None
        w = torch.randn(C, device="cuda").bfloat16()
        b = None if rms else torch.randn(C, device="cuda").bfloat16()
        fn = lambda: P.norm_fwd(x, r, w, b, 1e-5, rms)  # noqa: E731
        out = fn()
        y = out[0]
        ref = (x.float() + (r.float() if res else 0))
        if rms:
            ref_y = ref * torch.rsqrt(ref.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
        else:
            ref_y = torch.nn.functional.layer_norm(ref, (C,), w.float(), b.float(), 1e-5)
        err = ((y.float() - ref_y).norm() / ref_y.norm()).item()
        for _ in range(3):
            fn()
        ts = [timeit(fn) for _ in range(args.rounds)]
        nbytes = N * C * 2 * (2 + (2 if res else 0))
        med = statistics.median(ts)
        rec = {"N": N, "C": C, "rms": rms, "res": res, "us": round(med, 1), "min_us": round(min(ts), 1),
               "tbs": round(nbytes / med / 1e6, 2), "rel_err": round(err, 5)}
        # backward: dy, s and the residual-stream gradient ds in, dx out (+ weight / bias column partials)
        mean, rstd = out[-2], out[-1]
        s_in = out[1] if res else x
        dy = torch.randn(N, C, device="cuda").bfloat16()
        ds = torch.randn(N, C, device="cuda").bfloat16()
        fb = lambda: P.norm_bwd(dy, s_in, w, mean, rstd, ds, not rms, rms)  # noqa: E731
        for _ in range(3):
            fb()
        tb = [timeit(fb) for _ in range(args.rounds)]
        medb = statistics.median(tb)
        rec.update({"bwd_us": round(medb, 1), "bwd_tbs": round(N * C * 2 * 4 / medb / 1e6, 2),
                    "so": os.environ.get("PLLM_SO", "in-tree")})
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()

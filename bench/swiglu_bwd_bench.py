"""The llama SwiGLU backward on the ping-pong kernel (gemm_tn epilogue 5: dA = dy W_down, then [dg | du] from the
saved [gate | up]) at the llama-1.3B shapes; median / min microseconds of --rounds timings of --reps calls.
For same-box A/B of extension builds (scripts/gpu/ab.sh)."""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    P = torch.ops.pllm
    for M, F_, C in ((32768, 5504, 2048), (16384, 5504, 2048)):
        g = torch.Generator(device="cuda").manual_seed(M)
        dy = torch.randn(M, C, device="cuda", generator=g).bfloat16()
        wdt = (torch.randn(F_, C, device="cuda", generator=g) / C ** 0.5).bfloat16()  # W_down^T shadow [F, C]
        gu = torch.randn(M, 2 * F_, device="cuda", generator=g).bfloat16()
        fn = lambda: P.gemm_tn(dy, wdt, None, 5, gu)  # noqa: E731
        out = fn()[0]
        ref = P.swiglu_bwd(dy @ wdt.t(), gu)
        ref = ref[0] if isinstance(ref, (tuple, list)) else ref
        err = ((out.float() - ref.float()).norm() / ref.float().norm()).item()
        for _ in range(3):
            fn()
        ts = []
        for _ in range(args.rounds):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.reps):
                fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) / args.reps * 1e6)
        print(json.dumps({"M": M, "F": F_, "C": C, "us": round(statistics.median(ts), 1), "min_us": round(min(ts), 1),
                          "rel_err_vs_unfused": round(err, 5), "so": os.environ.get("PLLM_SO", "in-tree")}), flush=True)
        del dy, wdt, gu


if __name__ == "__main__":
    main()

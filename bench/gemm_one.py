"""One GEMM shape, a few launches each of the hand-written TN GEMM (gemm_tn, epi 0) and hipBLASLt
(F.linear) -- a target for rocprofv3 kernel traces and counter passes."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=65536)
    ap.add_argument("--N", type=int, default=768)
    ap.add_argument("--K", type=int, default=3072)
    ap.add_argument("--mf", type=int, default=16)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--phased", type=int, default=0, help="gemm_set_config phased (4 = ping-pong kernel)")
    ap.add_argument("--no-blas", action="store_true")
    ap.add_argument("--time", action="store_true", help="print the median microseconds of the hand-written GEMM")
    args = ap.parse_args()
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    torch.ops.pllm.gemm_set_config(args.mf, 4, args.phased)
    a = torch.empty(args.M, args.K, device="cuda").uniform_(-1, 1).bfloat16()
    w = (torch.empty(args.N, args.K, device="cuda").uniform_(-1, 1) / args.K ** 0.5).bfloat16()
    b = torch.randn(args.N, device="cuda").bfloat16()
    for _ in range(args.reps):
        torch.ops.pllm.gemm_tn(a, w, b, 0)
        if not args.no_blas:
            F.linear(a, w, b)
    torch.cuda.synchronize()
    if args.time:
        import statistics
        import time
        ts = []
        for _ in range(15):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                torch.ops.pllm.gemm_tn(a, w, b, 0)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) / 5 * 1e6)
        print(f"M={args.M} N={args.N} K={args.K} phased={args.phased} so={os.environ.get('PLLM_SO', 'in-tree')} "
              f"median_us={statistics.median(ts):.1f} min_us={min(ts):.1f}", flush=True)


if __name__ == "__main__":
    main()

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
    args = ap.parse_args()
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    torch.ops.pllm.gemm_set_config(args.mf, 4, 0)
    a = torch.randn(args.M, args.K, device="cuda").bfloat16()
    w = (torch.randn(args.N, args.K, device="cuda") / args.K ** 0.5).bfloat16()
    b = torch.randn(args.N, device="cuda").bfloat16()
    for _ in range(args.reps):
        torch.ops.pllm.gemm_tn(a, w, b, 0)
        F.linear(a, w, b)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()

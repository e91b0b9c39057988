"""Does the GELU forward pass read its input from the Infinity Cache when the up-projection runs in row chunks?

GPT-2 small MLP up-projection (M 65536, C 768, 4C 3072): pre = x W1^T + b1 (hipBLASLt), a = gelu(pre) (act_fwd).
Whole: one GEMM writes the 403 MB pre-activation, then act_fwd reads it back from HBM.  Chunked: GEMM + act_fwd per
row chunk, so each chunk's pre-activation (<= 100 MB) is still in the 256 MiB Infinity Cache when act_fwd reads it.
Medians over interleaved rounds, microseconds per full MLP up-projection + activation.

usage: python bench/mlp_chunk_probe.py [--rounds 9]"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def once(fn, reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    from pretraining_llm_amd.ops import _lib
    from pretraining_llm_amd.utils.gemm_tuning import enable_tuned_gemms
    _lib.require()
    enable_tuned_gemms(0)
    P = torch.ops.pllm
    M, C = 65536, 768
    x = torch.randn(M, C, device="cuda").bfloat16()
    w1 = (torch.randn(4 * C, C, device="cuda") * 0.02).bfloat16()
    b1 = torch.randn(4 * C, device="cuda").bfloat16()
    pre = torch.empty(M, 4 * C, device="cuda", dtype=torch.bfloat16)

    def whole():
        p = F.linear(x, w1, b1)
        return P.act_fwd(p, 1)

    def whole_lt():
        P.gemm_lt_out(x, w1, b1, pre, True)
        return P.act_fwd(pre, 1)

    def chunked(n, lt):
        R = M // n

        def run():
            outs = []
            for i in range(n):
                xc, pc = x[i * R:(i + 1) * R], pre[i * R:(i + 1) * R]
                if lt:
                    P.gemm_lt_out(xc, w1, b1, pc, True)
                else:
                    torch.addmm(b1, xc, w1.t(), out=pc)
                outs.append(P.act_fwd(pc, 1))
            return outs
        return run

    var = {"whole": whole, "whole_lt": whole_lt, "gemm_only": lambda: F.linear(x, w1, b1),
           "act_only": lambda: P.act_fwd(pre, 1)}
    for n in (2, 4, 8):
        var[f"chunk{n}_lt"] = chunked(n, True)
        var[f"chunk{n}_torch"] = chunked(n, False)
    ref = whole()
    for k, fn in var.items():
        for _ in range(3):
            out = fn()
        if k.startswith("chunk"):
            got = torch.cat(out)
            assert torch.allclose(got.float(), ref.float(), atol=2e-2, rtol=2e-2), k
    ts = {k: [] for k in var}
    for _ in range(args.rounds):
        for k, fn in var.items():
            ts[k].append(once(fn, args.reps))
    print(json.dumps({k: round(statistics.median(v), 1) for k, v in ts.items()}), flush=True)


if __name__ == "__main__":
    main()

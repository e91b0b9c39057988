"""Time the hand-written wgrad kernel (torch.ops.pllm.wgrad, fp32 target accumulate) on the GPT-2 /
Llama training shapes; one JSON line per shape (min over rounds).  Select an A/B build with PLLM_SO,
or compare wgrad_set_mfma variants in one process, interleaved: --variants 0,100 (0 = the default:
the ping-pong kernel of csrc/wgrad_pp.hip; 100 = the one-barrier kernel of csrc/gemm_wgrad.hip)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

SHAPES = [(65536, 50304, 768), (65536, 2304, 768), (65536, 768, 768), (65536, 3072, 768), (65536, 768, 3072),
          (32768, 6144, 2048), (32768, 2048, 2048), (32768, 11008, 2048), (32768, 2048, 5504), (32768, 50304, 2048)]


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default=None, help="comma-separated wgrad_set_mfma codes, interleaved")
    args = ap.parse_args()
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    variants = [int(v) for v in args.variants.split(",")] if args.variants else [None]
    for M, P, Q in SHAPES:
        dy = (torch.randn(M, P, device="cuda") * 0.1).bfloat16()
        x = torch.randn(M, Q, device="cuda").bfloat16()
        tgt = torch.zeros(P, Q, device="cuda")
        ts = {v: [] for v in variants}
        for v in variants:
            if v is not None:
                torch.ops.pllm.wgrad_set_mfma(v)
            for _ in range(3):
                torch.ops.pllm.wgrad(dy, x, tgt)
        for _ in range(5):
            for v in variants:
                if v is not None:
                    torch.ops.pllm.wgrad_set_mfma(v)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(5):
                    torch.ops.pllm.wgrad(dy, x, tgt)
                torch.cuda.synchronize()
                ts[v].append((time.perf_counter() - t0) / 5)
        rec = {"M": M, "P": P, "Q": Q}
        for v in variants:
            us = min(ts[v]) * 1e6
            tag = "" if v is None else f"_v{v}"
            rec["us" + tag] = round(us, 1)
            rec["tflops" + tag] = round(2 * M * P * Q / us / 1e6, 1)
        print(json.dumps(rec), flush=True)
        del dy, x, tgt
    torch.ops.pllm.wgrad_set_mfma(0)


if __name__ == "__main__":
    main()

"""Time the hand-written wgrad kernel (torch.ops.pllm.wgrad, fp32 target accumulate) on the GPT-2 /
Llama training shapes; one JSON line per shape (min over rounds).  Select an A/B build with PLLM_SO."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

SHAPES = [(65536, 50304, 768), (65536, 2304, 768), (65536, 768, 768), (65536, 3072, 768), (65536, 768, 3072),
          (32768, 6144, 2048), (32768, 2048, 2048), (32768, 11008, 2048), (32768, 2048, 5504), (32768, 50304, 2048)]


def main():
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    for M, P, Q in SHAPES:
        dy = (torch.randn(M, P, device="cuda") * 0.1).bfloat16()
        x = torch.randn(M, Q, device="cuda").bfloat16()
        tgt = torch.zeros(P, Q, device="cuda")
        for _ in range(3):
            torch.ops.pllm.wgrad(dy, x, tgt)
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                torch.ops.pllm.wgrad(dy, x, tgt)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) / 5)
        us = min(ts) * 1e6
        print(json.dumps({"M": M, "P": P, "Q": Q, "us": round(us, 1), "tflops": round(2 * M * P * Q / us / 1e6, 1)}),
              flush=True)
        del dy, x, tgt


if __name__ == "__main__":
    main()

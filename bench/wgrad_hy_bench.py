"""Weight-gradient kernel: split-K slices (wgrad_plan) vs the hybrid last-round split (wgrad_set_hy(1)) on the GPT-2 / llama
training shapes, fp32 accumulate target, interleaved rounds; median microseconds and TFLOP/s."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

SHAPES = [(65536, 50304, 768), (32768, 11008, 2048), (32768, 50304, 2048), (16384, 50304, 2048), (65536, 3072, 768)]
from pretraining_llm_amd.ops import _lib  # noqa: E402
P = _lib.require()


def once(fn, reps=3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


for M, Pd, Q in SHAPES:
    dy = (torch.randn(M, Pd, device="cuda") * 0.1).bfloat16()
    x = torch.randn(M, Q, device="cuda").bfloat16()
    tgt = torch.zeros(Pd, Q, device="cuda")
    ts = {0: [], 1: [], 2: []}
    for r in range(7):
        for sk in (0, 1, 2):  # 2: the hybrid with its remainder as one round of slices (PLLM_AB wgrad_hy_cost=0)
            P.wgrad_set_hy(min(sk, 1))
            os.environ["PLLM_AB"] = "wgrad_hy_cost=0" if sk == 2 else ""
            f = lambda: P.wgrad(dy, x, tgt)
            f()
            ts[sk].append(once(f))
    os.environ["PLLM_AB"] = ""
    P.wgrad_set_hy(1)
    fl = 2 * M * Pd * Q
    med = {k: statistics.median(v) for k, v in ts.items()}
    print(json.dumps({"M": M, "P": Pd, "Q": Q, "slices_us": round(med[0], 1), "hy_us": round(med[1], 1),
                      "slices_tflops": round(fl / med[0] / 1e6, 1), "hy_tflops": round(fl / med[1] / 1e6, 1),
                      "speedup": round(med[0] / med[1], 3),
                      "hy_one_round_us": round(med[2], 1), "cost_vs_one_round": round(med[2] / med[1], 3)}), flush=True)
    del dy, x, tgt

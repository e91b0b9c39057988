"""Ping-pong TN GEMM with odd workgroups started n x 8128 cycles late (torch.ops.pllm.gemm_pp_set_stagger),
de-phasing the end-of-tile store bursts of neighbouring CUs; stagger values interleaved round by round,
median microseconds per (shape, epilogue)."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

CASES = [(65536, 3072, 768, 0), (65536, 2304, 768, 0), (65536, 3072, 768, 1), (65536, 768, 3072, 0),
         (32768, 11008, 2048, 0)]
STAG = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,4").split(",")]
from pretraining_llm_amd.ops import _lib  # noqa: E402
P = _lib.require()
P.gemm_set_config(0, 0, 4, -1, 0, 1)


def once(fn, reps=5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


for M, N, K, epi in CASES:
    a = torch.randn(M, K, device="cuda").bfloat16()
    b = (torch.randn(N, K, device="cuda") * K ** -0.5).bfloat16()
    bias = torch.randn(N, device="cuda").bfloat16()
    ts = {s: [] for s in STAG}
    ref = None
    for r in range(7):
        for s in STAG:
            P.gemm_pp_set_stagger(s)
            f = lambda: P.gemm_tn(a, b, bias, epi)
            f()
            ts[s].append(once(f))
            if r == 0:
                out = f()[0]
                if ref is None:
                    ref = out
                assert torch.equal(out, ref), "stagger changed the result"
    P.gemm_pp_set_stagger(0)
    print(json.dumps({"M": M, "N": N, "K": K, "epi": epi,
                      **{f"stagger{s}_us": round(statistics.median(v), 1) for s, v in ts.items()}}), flush=True)

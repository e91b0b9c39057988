"""Weight-gradient shapes dW[P, Q] = dY[M, P]^T X[M, Q] on hipBLASLt's token-major ("NT") kernels through torch
(torch.mm(dy.t(), x), bf16 out; --tune: TunableOp tunes each shape first) vs the hand-written ping-pong kernel
(torch.ops.pllm.wgrad into an fp32 gradient).  Median microseconds, interleaved rounds."""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

SHAPES = [(65536, 50304, 768), (65536, 2304, 768), (65536, 768, 768), (65536, 3072, 768), (65536, 768, 3072),
          (32768, 6144, 2048), (32768, 2048, 2048), (32768, 11008, 2048), (32768, 2048, 5504)]

ap = argparse.ArgumentParser()
ap.add_argument("--tune", action="store_true")
ap.add_argument("--rounds", type=int, default=5)
args = ap.parse_args()
if args.tune:
    os.environ["PYTORCH_TUNABLEOP_ENABLED"] = "1"
    os.environ["PYTORCH_TUNABLEOP_TUNING"] = "1"
    os.environ["PYTORCH_TUNABLEOP_FILENAME"] = "/tmp/wgrad_nt_tune%d.csv"
    os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS", "200")
from pretraining_llm_amd.ops import _lib  # noqa: E402
_lib.require()


def once(fn, reps=3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


for M, P, Q in SHAPES:
    dy = (torch.randn(M, P, device="cuda") * 0.1).bfloat16()
    x = torch.randn(M, Q, device="cuda").bfloat16()
    tgt = torch.zeros(P, Q, device="cuda")
    fns = {"blas_nt": lambda: torch.mm(dy.t(), x), "pp": lambda: torch.ops.pllm.wgrad(dy, x, tgt)}
    for f in fns.values():
        f(), f()
    ts = {k: [] for k in fns}
    for _ in range(args.rounds):
        for k, f in fns.items():
            ts[k].append(once(f))
    med = {k: statistics.median(v) for k, v in ts.items()}
    fl = 2 * M * P * Q
    print(json.dumps({"M": M, "P": P, "Q": Q, "tune": int(args.tune), **{f"{k}_us": round(v, 1) for k, v in med.items()},
                      **{f"{k}_tflops": round(fl / v / 1e6, 1) for k, v in med.items()}}), flush=True)
    del dy, x, tgt

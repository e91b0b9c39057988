"""The residual add of a block's output projections (attention out, MLP down) done by the projection GEMM
(hipBLASLt beta = 1: s = residual + x w^T + b, torch.ops.pllm.gemm_lt(..., residual=)) instead of by the
next norm (norm_fwd(y, residual) reads y and the residual and writes s and the normalized output).
Interleaved rounds, median microseconds of GEMM + norm."""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

# (model, name, M, N, K, bias, rms)
SHAPES = [("gpt2", "attn_out", 65536, 768, 768, 1, 0), ("gpt2", "fc2", 65536, 768, 3072, 1, 0),
          ("llama", "o", 32768, 2048, 2048, 0, 1), ("llama", "down", 32768, 2048, 5504, 0, 1)]

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=7)
args = ap.parse_args()
from pretraining_llm_amd.ops import _lib  # noqa: E402
_lib.require()
from pretraining_llm_amd.utils.gemm_tuning import enable_tuned_gemms  # noqa: E402
enable_tuned_gemms(0)
P = torch.ops.pllm


def once(fn, reps=5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


for (model, nm, M, N, K, hb, rms) in SHAPES:
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).bfloat16()
    b = (0.1 * torch.randn(N, device="cuda")).bfloat16() if hb else None
    res = torch.randn(M, N, device="cuda").bfloat16()
    g = torch.ones(N, device="cuda").bfloat16()
    nb = None if rms else torch.zeros(N, device="cuda").bfloat16()

    def cur():
        y = F.linear(x, w, b)
        return P.norm_fwd(y, res, g, nb, 1e-5, bool(rms))

    def new():
        s = P.gemm_lt(x, w, b, 0, True, res)[0]
        return P.norm_fwd(s, None, g, nb, 1e-5, bool(rms)), s

    def gemm_only():
        return F.linear(x, w, b)

    def gemm_res_only():
        return P.gemm_lt(x, w, b, 0, True, res)[0]

    fns = {"linear+norm(res)": cur, "gemm_lt(res)+norm": new, "linear": gemm_only, "gemm_lt(res)": gemm_res_only}
    for f in fns.values():
        f(), f()
    ts = {k: [] for k in fns}
    for _ in range(args.rounds):
        for k, f in fns.items():
            ts[k].append(once(f))
    s_ref = (x.float() @ w.float().t() + (b.float() if hb else 0) + res.float())
    s_new = new()[1]
    rel = ((s_new.float() - s_ref).norm() / s_ref.norm()).item()
    print(json.dumps({"model": model, "gemm": nm, "M": M, "N": N, "K": K,
                      **{k: round(statistics.median(v), 1) for k, v in ts.items()}, "rel_err_s": rel}), flush=True)

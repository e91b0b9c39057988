"""Library GEMMs of the training step, y[M, N] = x[M, K] w[N, K]^T (+ b): torch (F.linear with the shipped
TunableOp tables, what the step runs today) vs torch.ops.pllm.gemm_lt (hipBLASLt called directly with its
bias epilogue, autotuned over the heuristic's candidates).  Median microseconds, interleaved rounds.
A data gradient dx = dy w is the same product with w's transposed shadow (x = dy, w = W^T)."""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

SHAPES = {
    "gpt2": [(65536, n, k, b, nm) for (n, k, b, nm) in [
        (2304, 768, 1, "qkv"), (768, 768, 1, "attn_out"), (3072, 768, 1, "fc1"), (768, 3072, 1, "fc2"),
        (50304, 768, 0, "lm_head"), (768, 2304, 0, "qkv_dgrad"), (768, 3072, 0, "fc1_dgrad"),
        (768, 50304, 0, "lm_head_dgrad")]],
    "llama": [(32768, n, k, 0, nm) for (n, k, nm) in [
        (6144, 2048, "qkv"), (2048, 2048, "o"), (2048, 5504, "down"), (50304, 2048, "lm_head"),
        (2048, 6144, "qkv_dgrad"), (2048, 2048, "o_dgrad"), (2048, 11008, "up_dgrad"),
        (2048, 50304, "lm_head_dgrad")]],
    "ref3b": [(16384, n, k, b, nm) for (n, k, b, nm) in [
        (6144, 2048, 1, "qkv"), (8192, 2048, 1, "fc1"), (2048, 8192, 1, "fc2"), (50304, 2048, 1, "lm_head"),
        (2048, 6144, 0, "qkv_dgrad"), (2048, 8192, 0, "fc1_dgrad"), (2048, 50304, 0, "lm_head_dgrad")]],
}

ap = argparse.ArgumentParser()
ap.add_argument("--models", default="gpt2,llama,ref3b")
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--no-tables", action="store_true")
args = ap.parse_args()
from pretraining_llm_amd.ops import _lib  # noqa: E402
_lib.require()
if not args.no_tables:
    from pretraining_llm_amd.utils.gemm_tuning import enable_tuned_gemms
    enable_tuned_gemms(0)


def once(fn, reps=5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


for model in args.models.split(","):
    for (M, N, K, has_b, nm) in SHAPES[model]:
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") * K ** -0.5).bfloat16()
        b = torch.randn(N, device="cuda").bfloat16() if has_b else None
        fns = {"torch": lambda: F.linear(x, w, b), "lt": lambda: torch.ops.pllm.gemm_lt(x, w, b, 0)}
        for f in fns.values():
            f(), f()
        ts = {k: [] for k in fns}
        for _ in range(args.rounds):
            for k, f in fns.items():
                ts[k].append(once(f))
        err = (torch.ops.pllm.gemm_lt(x, w, b, 0)[0].float() - F.linear(x, w, b).float()).abs().max().item()
        med = {k: statistics.median(v) for k, v in ts.items()}
        print(json.dumps({"model": model, "gemm": nm, "M": M, "N": N, "K": K, "bias": has_b,
                          "torch_us": round(med["torch"], 1), "lt_us": round(med["lt"], 1),
                          "lt_vs_torch": round(med["torch"] / med["lt"], 3), "maxdiff": err,
                          "tflops_lt": round(2 * M * N * K / med["lt"] / 1e6, 1)}), flush=True)
        del x, w, b
print("plans (M, N, K, epi, bias, candidates, chosen):", torch.ops.pllm.gemm_lt_plans(), flush=True)

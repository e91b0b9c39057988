"""GPT-2 MLP up-projection forward, three ways (median us): hipBLASLt bias GEMM + the separate GELU pass
(the shipped path), hipBLASLt's own bias+GELU epilogue through torch._addmm_activation (no pre-activation
output), and the plain bias GEMM alone (the floor).  With --tuned the shipped TunableOp tables are loaded."""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tuned", action="store_true")
ap.add_argument("--probe", action="store_true", help="count hipBLASLt candidates per epilogue / bias / aux type")
ap.add_argument("--shapes", default="65536x768x3072,16384x768x3072,65536x1024x4096,16384x2048x8192")
args = ap.parse_args()
from pretraining_llm_amd.ops import _lib  # noqa: E402
_lib.require()
if args.probe:
    BF16, F32, F16 = 14, 0, 2  # hipDataType
    EPI = {"DEFAULT": 1, "BIAS": 4, "RELU": 2, "RELU_BIAS": 6, "GELU": 32, "GELU_BIAS": 36, "GELU_AUX": 160,
           "GELU_AUX_BIAS": 164}
    for s in args.shapes.split(","):
        M, K, N = map(int, s.split("x"))
        for en, ev in EPI.items():
            for bt in (-1, BF16, F32):
                for at in ((-1, BF16, F32, F16) if "AUX" in en else (-1,)):
                    n = torch.ops.pllm.gemm_lt_probe(M, N, K, ev, bt, at)
                    print(f"probe M={M} N={N} K={K} {en} bias_type={bt} aux_type={at}: {n}", flush=True)
    sys.exit(0)
if args.tuned:
    from pretraining_llm_amd.utils.gemm_tuning import enable_tuned_gemms
    enable_tuned_gemms(0)


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e6)
    return statistics.median(ts)


for s in args.shapes.split(","):
    M, K, N = map(int, s.split("x"))
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).bfloat16()
    b = torch.randn(N, device="cuda").bfloat16()
    plain = timeit(lambda: F.linear(x, w, b))
    sep = timeit(lambda: torch.ops.pllm.act_fwd(F.linear(x, w, b), 1))
    epi = timeit(lambda: torch._addmm_activation(b, x, w.t(), use_gelu=True))
    nob = timeit(lambda: F.linear(x, w))
    lt0 = timeit(lambda: torch.ops.pllm.gemm_lt(x, w, None, 0))
    lt0b = timeit(lambda: torch.ops.pllm.gemm_lt(x, w, b, 0))
    lt2 = timeit(lambda: torch.ops.pllm.gemm_lt(x, w, b, 2))
    relu_sep = timeit(lambda: torch.ops.pllm.act_fwd(F.linear(x, w, b), 0))
    relu_addmm = timeit(lambda: torch._addmm_activation(b, x, w.t(), use_gelu=False))
    pre_ref = F.linear(x.float(), w.float(), b.float())
    lt1, e_pre, e_a = float("nan"), float("nan"), float("nan")
    if torch.ops.pllm.gemm_lt_probe(M, N, K, 164, 14, 14) > 0:  # GELU_AUX_BIAS (absent from torch's hipBLASLt)
        lt1 = timeit(lambda: torch.ops.pllm.gemm_lt(x, w, b, 1))
        a, pre = torch.ops.pllm.gemm_lt(x, w, b, 1)
        e_pre = (pre.float() - pre_ref).abs().max().item()
        e_a = (a.float() - F.gelu(pre_ref, approximate="tanh")).abs().max().item()
    r, _ = torch.ops.pllm.gemm_lt(x, w, b, 2)
    e_r = (r.float() - pre_ref.relu()).abs().max().item()
    print(f"M={M} K={K} N={N} tuned={int(args.tuned)} linear_us={plain:.1f} linear_nobias_us={nob:.1f} "
          f"linear+act_us={sep:.1f} addmm_gelu_us={epi:.1f} lt_us={lt0:.1f} lt_bias_us={lt0b:.1f} "
          f"lt_gelu_aux_us={lt1:.1f} lt_relu_us={lt2:.1f} linear+relu_us={relu_sep:.1f} addmm_relu_us={relu_addmm:.1f} err_pre={e_pre:.3g} err_gelu={e_a:.3g} err_relu={e_r:.3g}",
          flush=True)
print("plans (M, N, K, epi, bias, candidates, chosen):", torch.ops.pllm.gemm_lt_plans(), flush=True)

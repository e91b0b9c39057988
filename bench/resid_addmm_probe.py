"""Residual add by the GEMM through torch (addmm, beta = 1, TunableOp tuning in-process) vs the plain GEMM,
at llama-1.3B's MLP down projection (32768 x 2048 x 5504), where hipBLASLt's beta = 1 candidates through
csrc/blaslt.cpp are slow (profiles/r5_residual_in_gemm.md).  Median us of 5 x 5 calls."""
import os
import statistics
import sys
import time

os.environ.setdefault("PYTORCH_TUNABLEOP_ENABLED", "1")
os.environ.setdefault("PYTORCH_TUNABLEOP_TUNING", "1")
os.environ.setdefault("PYTORCH_TUNABLEOP_FILENAME", "/tmp/resid_addmm_probe_tunableop.csv")
import torch  # noqa: E402


def med(fn, reps=5, rounds=5):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(rounds):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) / reps * 1e6)
    return round(statistics.median(ts), 1)


for (M, N, K) in [(32768, 2048, 5504), (32768, 2048, 2048), (65536, 768, 3072)]:
    a = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).bfloat16()
    res = torch.randn(M, N, device="cuda").bfloat16()
    plain = med(lambda: torch.mm(a, w.t()))
    addmm = med(lambda: torch.addmm(res, a, w.t()))
    print({"M": M, "N": N, "K": K, "mm_us": plain, "addmm_beta1_us": addmm}, flush=True)
sys.exit(0)

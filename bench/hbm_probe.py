"""HBM streaming ceiling on this GPU vs the framework's memory-bound kernels: torch copy_,
torch add, and pllm act_fwd (GELU, read+write), at 402 MB bf16 tensors (GPT-2 MLP hidden)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(3):
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / iters)
    return best


def main():
    from pretraining_llm_amd.ops import _lib
    P = _lib.require()
    dev = torch.device("cuda")
    n = 65536 * 3072
    x = torch.randn(n, device=dev).bfloat16()
    y = torch.empty_like(x)
    z = torch.randn(n, device=dev).bfloat16()
    nb = x.numel() * 2
    res = {}
    res["copy_TBps"] = 2 * nb / timeit(lambda: y.copy_(x)) / 1e12
    res["add_TBps"] = 3 * nb / timeit(lambda: torch.add(x, z, out=y)) / 1e12
    res["gelu_fwd_TBps"] = 2 * nb / timeit(lambda: P.act_fwd(x.view(65536, 3072), 1)) / 1e12
    res["gelu_bwd_TBps"] = 3 * nb / timeit(lambda: P.act_bwd(z.view(65536, 3072), x.view(65536, 3072), 1)) / 1e12
    xf = torch.randn(n // 2, device=dev)
    yf = torch.empty_like(xf)
    res["copy_f32_TBps"] = 2 * xf.numel() * 4 / timeit(lambda: yf.copy_(xf)) / 1e12
    print(json.dumps({k: round(v, 3) for k, v in res.items()}))


if __name__ == "__main__":
    main()

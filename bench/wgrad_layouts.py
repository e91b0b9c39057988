"""Weight-gradient dW[P,Q] += dY[M,P]^T X[M,Q] (fp32 accumulate into an fp32 gradient) by operand
layout: the hand-written split-K kernel (token-major operands as they are) vs hipBLASLt through
torch.addmm(out_dtype=float32, out=grad) with (a) both operands token-major ("nt"), (b) dY
transposed first (dYT [P, M]: "nn"), (c) X transposed first (XT [Q, M]) -- transposes timed
separately.  Checks every path against fp32 math on a slice."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(3):
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / iters)
    return best * 1e6


def main():
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    P_ = torch.ops.pllm
    dev = torch.device("cuda")
    cases = [(65536, 2304, 768), (65536, 3072, 768), (65536, 768, 3072), (65536, 50304, 768),
             (32768, 6144, 2048), (32768, 2048, 2048), (32768, 11008, 2048), (32768, 2048, 5504),
             (32768, 50304, 2048)]
    for M, P, Q in cases:
        torch.manual_seed(0)
        dy = (torch.randn(M, P, device=dev) * 0.1).bfloat16()
        x = torch.randn(M, Q, device=dev).bfloat16()
        tgt = torch.zeros(P, Q, device=dev)
        res = {"M": M, "P": P, "Q": Q}
        fl = 2.0 * M * P * Q
        res["hip_us"] = timeit(lambda: P_.wgrad(dy, x, tgt))
        dyT = dy.t().contiguous()
        xT = x.t().contiguous()
        res["transpose_dy_us"] = timeit(lambda: dy.t().contiguous())
        res["transpose_x_us"] = timeit(lambda: x.t().contiguous())
        for tag, a, b in (("nt", dy.t(), x), ("nn", dyT, x), ("tn", dy.t(), xT.t()), ("tt", dyT, xT.t())):
            try:
                torch.addmm(tgt, a, b, out_dtype=torch.float32, out=tgt)
                res[f"{tag}_us"] = timeit(lambda: torch.addmm(tgt, a, b, out_dtype=torch.float32, out=tgt))
                res[f"{tag}_tflops"] = round(fl / res[f"{tag}_us"] / 1e6)
            except Exception as e:  # noqa: BLE001
                res[f"{tag}_err"] = str(e).split("\n")[0][:120]
        # numerics of the in-place fp32 accumulate on a slice
        t2 = torch.ones(P, Q, device=dev)
        torch.addmm(t2, dyT[:, :4096], x[:4096], out_dtype=torch.float32, out=t2)
        ref = 1 + dy[:4096].float().t() @ x[:4096].float()
        res["nn_rel_err"] = ((t2 - ref).norm() / ref.norm()).item()
        res["hip_tflops"] = round(fl / res["hip_us"] / 1e6)
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)
        del dy, x, tgt, dyT, xT, t2


if __name__ == "__main__":
    main()

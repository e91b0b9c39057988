"""wgrad engines with an fp32 gradient target: hand-written split-K kernel (accumulates in place)
vs hipBLASLt through torch.addmm(out_dtype=float32) (bf16 operands, fp32 output)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    dev = torch.device("cuda")
    for M, shapes in ((65536, [(2304, 768), (768, 768), (3072, 768), (768, 3072), (50304, 768)]),
                      (32768, [(6144, 2048), (2048, 2048), (11008, 2048), (2048, 5504), (50304, 2048)])):
        for P, Q in shapes:
            dy = (torch.randn(M, P, device=dev) * 0.1).bfloat16()
            x = torch.randn(M, Q, device=dev).bfloat16()
            tgt = torch.zeros(P, Q, device=dev)
            res = {"M": M, "P": P, "Q": Q}
            try:
                r = torch.addmm(tgt, dy.t(), x, out_dtype=torch.float32)
                ref = dy.float().t()[:, :4096] @ x.float()[:4096]
                res["blas32_ok"] = True
                ts = [timeit(lambda: torch.addmm(tgt, dy.t(), x, out_dtype=torch.float32)) for _ in range(3)]
                res["blas32_us"] = 1e6 * min(ts)
            except Exception as e:  # noqa: BLE001
                res["blas32_err"] = str(e).split("\n")[0][:200]
            ts = [timeit(lambda: torch.ops.pllm.wgrad(dy, x, tgt)) for _ in range(3)]
            res["hip_us"] = 1e6 * min(ts)
            fl = 2.0 * M * P * Q
            for k in ("blas32", "hip"):
                if f"{k}_us" in res:
                    res[f"{k}_tflops"] = fl / res[f"{k}_us"] / 1e6
            print(json.dumps(res), flush=True)
            del dy, x, tgt


if __name__ == "__main__":
    main()

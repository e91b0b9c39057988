"""Weight gradient through hipBLASLt with a bf16 OUTPUT (the precision of the reference's autocast
backward: the mm in bf16, the result cast into the fp32 .grad), vs the hand-written split-K kernel
that accumulates in fp32 straight into the fp32 gradient.

For each GPT-2 / llama wgrad shape dW[P,Q] = dY[M,P]^T X[M,Q]:
  hip      : torch.ops.pllm.wgrad(dy, x, fp32 target)          (hand-written, fp32 accumulate)
  mm_nt    : torch.mm(dy.t(), x) -> bf16 [P,Q]                 (both operands token-major)
  mm_nt_acc: the same + fp32 target.add_(dW)                   (what a bf16-output path costs in all)
With --tune, TunableOp tunes every shape online first (all hipBLASLt solutions + rocBLAS) and the
timed calls use the winners.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tune", action="store_true")
    ap.add_argument("--shapes", default="gpt2")
    args = ap.parse_args()
    if args.tune:
        os.environ["PYTORCH_TUNABLEOP_ENABLED"] = "1"
        os.environ["PYTORCH_TUNABLEOP_TUNING"] = "1"
        os.environ["PYTORCH_TUNABLEOP_FILENAME"] = "/tmp/wgrad_bf16out_tune%d.csv"
        os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS", "300")
    import torch
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    P_ = torch.ops.pllm
    dev = torch.device("cuda")

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

    gpt2 = [(65536, 2304, 768), (65536, 768, 768), (65536, 3072, 768), (65536, 768, 3072), (65536, 50304, 768)]
    llama = [(32768, 6144, 2048), (32768, 2048, 2048), (32768, 11008, 2048), (32768, 2048, 5504),
             (32768, 32000, 2048)]
    cases = {"gpt2": gpt2, "llama": llama, "all": gpt2 + llama}[args.shapes]
    tot = {"hip": 0.0, "mm_nt_acc": 0.0}
    for M, P, Q in cases:
        torch.manual_seed(0)
        dy = (torch.randn(M, P, device=dev) * 0.1).bfloat16()
        x = torch.randn(M, Q, device=dev).bfloat16()
        tgt = torch.zeros(P, Q, device=dev)
        fl = 2.0 * M * P * Q
        res = {"M": M, "P": P, "Q": Q, "tuned": args.tune}
        res["hip_us"] = timeit(lambda: P_.wgrad(dy, x, tgt))
        res["mm_nt_us"] = timeit(lambda: torch.mm(dy.t(), x))
        res["mm_nt_acc_us"] = timeit(lambda: tgt.add_(torch.mm(dy.t(), x)))
        for k in ("hip", "mm_nt"):
            res[k + "_tflops"] = round(fl / res[k + "_us"] / 1e6)
        ref = dy[:8192].float().t() @ x[:8192].float()
        got = torch.mm(dy[:8192].t(), x[:8192]).float()
        res["mm_rel_err"] = ((got - ref).norm() / ref.norm()).item()
        tot["hip"] += res["hip_us"]
        tot["mm_nt_acc"] += res["mm_nt_acc_us"]
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)
        del dy, x, tgt
    print(json.dumps({"total_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()

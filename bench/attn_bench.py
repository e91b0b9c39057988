"""Microbenchmark: causal flash attention fwd / bwd on MI355X, hand-written gfx950 kernels
(torch.ops.pllm.attn_fwd / attn_bwd) vs PyTorch SDPA (ROCm's built-in flash/efficient
attention) on the same random data, interleaved rounds in one process.

Reports TFLOP/s with causal FLOPs counted as half of dense: fwd 2*2*B*H*T*T*D/2,
bwd 2.5x fwd (5 GEMM-shaped products)."""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="64x12x1024x64,8x16x2048x128,8x16x4096x64")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="", help="fwd|bwd: run only our kernel (for profiling)")
    ap.add_argument("--rope-ab", action="store_true", help="our fwd/bwd with vs without fused RoPE tables")
    ap.add_argument("--ours", action="store_true", help="time only the HIP kernels (fwd_us / bwd_us), no SDPA")
    ap.add_argument("--ks-ab", action="store_true",
                    help="backward only: key-stationary kernel (attn_bwd_set_ks(3)) vs the previous kernels "
                         "(set_ks(0)), interleaved rounds")
    args = ap.parse_args()
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    dev = torch.device("cuda")
    for cfg in args.configs.split(","):
        B, H, T, D = (int(v) for v in cfg.split("x"))
        torch.manual_seed(0)
        q = torch.randn(B, T, H, D, device=dev, dtype=torch.bfloat16)
        k = torch.randn(B, T, H, D, device=dev, dtype=torch.bfloat16)
        v = torch.randn(B, T, H, D, device=dev, dtype=torch.bfloat16)
        do = torch.randn(B, T, H, D, device=dev, dtype=torch.bfloat16)
        scale = 1 / math.sqrt(D)
        o, lse = torch.ops.pllm.attn_fwd(q, k, v, True, scale)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        ours_f = lambda: torch.ops.pllm.attn_fwd(q, k, v, True, scale)
        ours_b = lambda: torch.ops.pllm.attn_bwd(do, q, k, v, o, lse, dq, dk, dv, True, scale)
        if args.rope_ab:
            from pretraining_llm_amd import ops
            cos, sin = ops.rope_cache(T, D, 10000.0, dev)
            res = {"cfg": cfg}
            for tag, rc, rs in (("plain", None, None), ("rope", cos, sin)):
                o_, l_ = torch.ops.pllm.attn_fwd(q, k, v, True, scale, rc, rs)
                f_ = lambda: torch.ops.pllm.attn_fwd(q, k, v, True, scale, rc, rs)  # noqa: E731
                b_ = lambda: torch.ops.pllm.attn_bwd(do, q, k, v, o_, l_, dq, dk, dv, True, scale, rc, rs)  # noqa: E731
                res[f"{tag}_fwd_us"] = min(1e6 * timeit(f_) for _ in range(args.rounds))
                res[f"{tag}_bwd_us"] = min(1e6 * timeit(b_) for _ in range(args.rounds))
            # pre-pass arm: rotate q / k of a packed qkv once (rope_qk), plain forward, backward
            # rotating only its outputs (the training path, ops._FlashAttnPacked)
            qkv = torch.cat([q.reshape(B, T, -1), k.reshape(B, T, -1), v.reshape(B, T, -1)], -1)
            qk = torch.ops.pllm.rope_qk(qkv, cos, sin, 3 * H, 2 * H, T)
            qr, kr = qk[..., : H * D].view(B, T, H, D), qk[..., H * D:].view(B, T, H, D)
            o_, l_ = torch.ops.pllm.attn_fwd(qr, kr, v, True, scale)
            pre = lambda: torch.ops.pllm.rope_qk(qkv, cos, sin, 3 * H, 2 * H, T)  # noqa: E731
            f_ = lambda: torch.ops.pllm.attn_fwd(qr, kr, v, True, scale)  # noqa: E731
            b_ = lambda: torch.ops.pllm.attn_bwd(do, qr, kr, v, o_, l_, dq, dk, dv, True, scale, cos, sin, False)  # noqa: E731
            res["prepass_us"] = min(1e6 * timeit(pre) for _ in range(args.rounds))
            res["prepass_fwd_us"] = min(1e6 * timeit(f_) for _ in range(args.rounds))
            res["prepass_bwd_us"] = min(1e6 * timeit(b_) for _ in range(args.rounds))
            print(json.dumps(res), flush=True)
            continue
        if args.ks_ab:
            flops_b = 2.5 * 2 * 2 * B * H * T * T * D / 2
            res = {"cfg": cfg, "ks_bwd_us": [], "old_bwd_us": []}
            for _ in range(args.rounds):
                torch.ops.pllm.attn_bwd_set_ks(3)
                res["ks_bwd_us"].append(1e6 * timeit(ours_b))
                torch.ops.pllm.attn_bwd_set_ks(0)
                res["old_bwd_us"].append(1e6 * timeit(ours_b))
            torch.ops.pllm.attn_bwd_set_ks(2)
            for k_ in ("ks", "old"):
                res[k_ + "_tflops"] = flops_b / (min(res[k_ + "_bwd_us"]) * 1e-6) / 1e12
            print(json.dumps(res), flush=True)
            continue
        if args.ours:
            flops_f = 2 * 2 * B * H * T * T * D / 2
            res = {"cfg": cfg, "fwd_us": [1e6 * timeit(ours_f) for _ in range(args.rounds)],
                   "bwd_us": [1e6 * timeit(ours_b) for _ in range(args.rounds)]}
            res["fwd_tflops"] = flops_f / (min(res["fwd_us"]) * 1e-6) / 1e12
            res["bwd_tflops"] = 2.5 * flops_f / (min(res["bwd_us"]) * 1e-6) / 1e12
            print(json.dumps(res), flush=True)
            continue
        if args.only:
            fn = ours_f if args.only == "fwd" else ours_b
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            continue
        qt, kt, vt = (t.transpose(1, 2).contiguous().requires_grad_() for t in (q, k, v))
        dot = do.transpose(1, 2).contiguous()
        ref_o = F.scaled_dot_product_attention(qt, kt, vt, is_causal=True)
        sdpa_f = lambda: F.scaled_dot_product_attention(qt, kt, vt, is_causal=True)
        sdpa_b = lambda: torch.autograd.grad(ref_o, (qt, kt, vt), dot, retain_graph=True)
        err = ((o.float() - ref_o.transpose(1, 2).float()).norm() / ref_o.float().norm()).item()
        flops_f = 2 * 2 * B * H * T * T * D / 2
        res = {"cfg": cfg, "rel_err_vs_sdpa": err, "ours_fwd_us": [], "sdpa_fwd_us": [], "ours_bwd_us": [],
               "sdpa_bwd_us": []}
        for _ in range(args.rounds):
            res["ours_fwd_us"].append(1e6 * timeit(ours_f))
            res["sdpa_fwd_us"].append(1e6 * timeit(sdpa_f))
            res["ours_bwd_us"].append(1e6 * timeit(ours_b))
            res["sdpa_bwd_us"].append(1e6 * timeit(sdpa_b))
        for k_ in ("ours_fwd", "sdpa_fwd"):
            res[k_ + "_tflops"] = flops_f / (min(res[k_ + "_us"]) * 1e-6) / 1e12
        for k_ in ("ours_bwd", "sdpa_bwd"):
            res[k_ + "_tflops"] = 2.5 * flops_f / (min(res[k_ + "_us"]) * 1e-6) / 1e12
        print(json.dumps(res), flush=True)
        del q, k, v, do, qt, kt, vt


if __name__ == "__main__":
    main()

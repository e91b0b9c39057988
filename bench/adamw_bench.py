"""AdamW + W^T shadow refresh: the fused launch (csrc/adamw.hip adamw_shadow_kernel) vs the flat AdamW
kernel followed by the batched transpose (csrc/transpose.hip), on a model's real parameter layout.

    python bench/adamw_bench.py --model llama-1.3b [--iters 20]

Prints one JSON line: us per optimizer step for both arms (interleaved rounds, same box)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-1.3b")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    from pretraining_llm_amd.models import GPT, get_preset
    from pretraining_llm_amd.ops import _lib
    from pretraining_llm_amd.train.optim import FlatAdamW, no_decay_1d
    _lib.require()
    cfg = get_preset(args.model)
    model = GPT(cfg).to(device="cuda", dtype=torch.bfloat16)
    opt = FlatAdamW(model, lr=1e-4, weight_decay=0.1, max_grad_norm=0.0, decay_filter=no_decay_1d)
    opt.flat_grad.normal_()
    for p in opt._fresh_params:
        p._pllm_grad_fresh = False
    desc = opt._tp_desc
    assert desc is not None, "model has no shadowed matrices"

    ops = torch.ops.pllm

    def run(fused):
        if fused:
            opt.step()
            return
        # the flat AdamW launch, then the separate batched-transpose launch
        opt.step_count += 1
        ops.adamw_(opt.flat_param, opt.master, opt.exp_avg, opt.exp_avg_sq, opt.flat_grad, opt.lr, 0.9, 0.999,
                   opt.eps, opt.weight_decay, opt.step_count, 1.0, None, opt.wd_mask, None)
        ops.transpose_run(desc, opt._tp_tiles)

    res = {"fused_us": [], "separate_us": []}
    for _ in range(args.rounds):
        for fused, key in ((True, "fused_us"), (False, "separate_us")):
            for _ in range(3):
                run(fused)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.iters):
                run(fused)
            b.record()
            torch.cuda.synchronize()
            res[key].append(a.elapsed_time(b) * 1000 / args.iters)
    res.update(model=args.model, params=opt.total, shadowed=sum(p.numel() for p in opt.shadowed))
    print(json.dumps(res))


if __name__ == "__main__":
    main()

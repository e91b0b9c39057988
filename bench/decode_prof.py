"""Decode-step profile helper: GPT-2 small, batch --batch, 128-token prompt, --new greedy tokens
with the hipGraph decode step (run under rocprofv3 --kernel-trace --stats)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--new", type=int, default=64)
    ap.add_argument("--graph", type=int, default=1)
    args = ap.parse_args()
    import torch
    from pretraining_llm_amd import ops
    from pretraining_llm_amd.models import GPT, get_preset
    ops._lib.require()
    torch.manual_seed(0)
    cfg = get_preset("gpt2-small")
    m = GPT(cfg).to("cuda", torch.bfloat16).eval()
    idx = torch.randint(0, cfg.vocab_size, (args.batch, 128), device="cuda")
    m.generate(idx, 4, temperature=0.0, cuda_graph=bool(args.graph))
    torch.cuda.synchronize()
    m.generate(idx, args.new, temperature=0.0, cuda_graph=bool(args.graph))
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()

"""Read the s_memtime stamps of a PLLM_PP_EXP=64 build of csrc/gemm_pp.hip (workgroup 0; per wave:
two K-tiles x 4 phases x {LOAD start, reads issued, DMA issued, vmcnt passed, barrier 1 passed,
MFMAs issued} + the second tile's epilogue start / end) and print per-phase segment cycles.

usage: PLLM_SO=..._C_ppexp64.so python bench/gemm_pp_stamps.py --M 65536 --N 3072 --K 768"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=65536)
    ap.add_argument("--N", type=int, default=3072)
    ap.add_argument("--K", type=int, default=768)
    args = ap.parse_args()
    from pretraining_llm_amd.ops import _lib
    _lib.require()
    P = torch.ops.pllm
    P.gemm_set_config(16, 4, 4)
    a = torch.empty(args.M, args.K, device="cuda").uniform_(-1, 1).bfloat16()
    w = (torch.empty(args.N, args.K, device="cuda").uniform_(-1, 1) / args.K ** 0.5).bfloat16()
    for _ in range(3):
        out = P.gemm_tn(a, w, None, 0)[0]
    torch.cuda.synchronize()
    st = out.reshape(-1)[: 8 * 52 * 4].contiguous().view(torch.int64).view(8, 52).cpu()
    names = ["reads", "dma", "vmcnt", "barrier1", "mfma", "->next"]
    for w_ in range(8):
        row = st[w_]
        for sk in range(2):
            segs = []
            for ph in range(4):
                base = 24 * sk + 6 * ph
                t = [int(row[base + i]) for i in range(6)]
                nxt = int(row[base + 6]) if (ph < 3 or sk == 0) and base + 6 < 48 else None
                d = [t[i + 1] - t[i] for i in range(5)] + ([nxt - t[5]] if nxt is not None else [None])
                segs.append(dict(zip(names, d)))
            print(json.dumps({"wave": w_, "ktile": ["first after epilogue", "mid-tile"][sk], "phases": segs}))
        print(json.dumps({"wave": w_, "epilogue_cycles": int(row[49]) - int(row[48])}))


if __name__ == "__main__":
    main()

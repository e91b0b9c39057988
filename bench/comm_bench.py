"""RCCL collective bandwidth sweep (all-reduce / reduce-scatter / all-gather / all-to-all).

Picks the DP bucket size and TP/EP degree from measurement instead of NVSwitch folklore:
on an MI355X node every GPU has 7 point-to-point xGMI links (~153 GB/s each), so a ring
collective is bound by one link per ring step unless RCCL spreads channels over all links.
The sweep reports, per collective and message size, the time, the algorithm bandwidth
(bytes / time) and the bus bandwidth (the nccl-tests convention: all-reduce x 2(n-1)/n,
reduce-scatter / all-gather / all-to-all x (n-1)/n), which is comparable to the per-GPU
link budget.  The knee of busbw(size) is where a gradient bucket stops paying latency.

  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench/comm_bench.py
  (CPU smoke test: --backend gloo --device cpu --sizes-mb 0.25,1)

rank 0 prints one JSON line per (collective, size).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="nccl")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--sizes-mb", default="1,4,16,32,64,128,256,512")
    ap.add_argument("--ops", default="all_reduce,reduce_scatter,all_gather,all_to_all")
    ap.add_argument("--dtype", default="bfloat16")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rccl-channels", type=int, default=None, help="NCCL_MIN/MAX_NCHANNELS (before init)")
    ap.add_argument("--rccl-env", default="", help="extra 'KEY=VAL,...' RCCL settings")
    args = ap.parse_args(argv)
    from pretraining_llm_amd.utils.dist import apply_rccl_env, parse_env_list
    apply_rccl_env(args.rccl_channels, parse_env_list(args.rccl_env))
    import torch
    import torch.distributed as dist
    from pretraining_llm_amd.utils.dist import init_distributed

    di = init_distributed(args.backend, args.device)
    n, dev = di.world_size, di.device
    dtype = getattr(torch, args.dtype)
    esz = torch.empty((), dtype=dtype).element_size()
    cuda = dev.type == "cuda"

    def sync():
        if cuda:
            torch.cuda.synchronize(dev)

    for op in args.ops.split(","):
        for mb in (float(s) for s in args.sizes_mb.split(",")):
            numel = max(n * 64, int(mb * 2 ** 20) // esz // (n * 64) * (n * 64))
            x = torch.ones(numel, dtype=dtype, device=dev)
            if op == "all_reduce":
                fn = lambda: dist.all_reduce(x)  # noqa: E731
                factor = 2 * (n - 1) / n
            elif op == "reduce_scatter":
                out = torch.empty(numel // n, dtype=dtype, device=dev)
                fn = lambda: dist.reduce_scatter_tensor(out, x)  # noqa: E731
                factor = (n - 1) / n
            elif op == "all_gather":
                src = torch.ones(numel // n, dtype=dtype, device=dev)
                fn = lambda: dist.all_gather_into_tensor(x, src)  # noqa: E731
                factor = (n - 1) / n
            elif op == "all_to_all":
                out = torch.empty_like(x)
                fn = lambda: dist.all_to_all_single(out, x)  # noqa: E731
                factor = (n - 1) / n
            else:
                raise ValueError(op)
            for _ in range(args.warmup):
                fn()
            sync()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(args.iters):
                fn()
            sync()
            dt = (time.perf_counter() - t0) / args.iters
            t = torch.tensor([dt], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
            nbytes = numel * esz
            if di.is_master:
                print(json.dumps({"op": op, "world": n, "backend": args.backend, "dtype": args.dtype,
                                  "size_mb": round(nbytes / 2 ** 20, 3), "time_us": round(dt * 1e6, 1),
                                  "algbw_GBps": round(nbytes / dt / 1e9, 2),
                                  "busbw_GBps": round(nbytes / dt / 1e9 * factor, 2)}), flush=True)
            del x
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

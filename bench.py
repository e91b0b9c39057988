#!/usr/bin/env python
"""Headline benchmark: whole-job tokens/s pretraining GPT-2-small (124M) at seq 1024, bf16.

Contract (driver):  python bench.py --gpus N --steps K --warmup W
  * N = 1: runs in-process on cuda:0;  N > 1: launched by torch.distributed.run,
    one rank per GPU, RCCL data parallel (RANK/LOCAL_RANK/WORLD_SIZE from env).
  * W untimed warmup steps, then EXACTLY K timed optimizer steps bracketed by a
    barrier + device synchronize on both sides; the time is the MAX over ranks.
  * rank 0 prints ONE JSON line.
Every timed step is a full training step: synthetic tokens streamed by the
native loader (pinned, side-stream H2D), forward, backward, bucketed RCCL
all-reduce overlapped with backward, fused AdamW on fp32 masters, zero_grad.
Weights are random-init GPT-2-small (124M, tied embeddings, V=50304);
``--backend torch`` runs the same model on stock PyTorch ops (SDPA,
F.layer_norm, F.cross_entropy, torch AdamW-equivalent math) as the measured
reference-equivalent baseline.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "tokens/sec (whole node) pretraining GPT-2-small seq1024 at 1/2/4/8 MI355X"
# The reference publishes no numbers; its comparison baseline is MEASURED: the same
# GPT-2-small model/optimizer on stock PyTorch-ROCm ops (``--backend torch``: SDPA, F.layer_norm,
# fp32 F.cross_entropy, torch-op AdamW), 1x MI355X, B=64 x 1024 -- BASELINE.md "Measured".
# vs_baseline divides by that number times the GPU count (linear scaling granted to the baseline).
EAGER_BASELINE_TOK_S_PER_GPU = 487050.2
OTHER_METRIC = "tokens/sec (whole node) pretraining {model} seq{seq}"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--batch", type=int, default=int(os.environ.get("PLLM_BENCH_BATCH", "64")),
                    help="micro-batch (sequences) per GPU")
    ap.add_argument("--seq", type=int, default=None, help="sequence length (default: the model's context length)")
    ap.add_argument("--act-ckpt", default=None,
                    help="activation checkpointing on (1) / off (0) / a fraction of the blocks (e.g. 0.5) / "
                         "by HBM budget (auto); default: the preset's")
    ap.add_argument("--backend", default="auto", choices=["auto", "torch"])
    ap.add_argument("--bucket-mb", type=float, default=64.0, help="DP gradient bucket size (MiB)")
    ap.add_argument("--first-bucket-mb", type=float, default=4.0, help="size of the first (earliest) bucket (MiB)")
    ap.add_argument("--rccl-channels", type=int, default=None,
                    help="pin RCCL's channel count (NCCL_MIN/MAX_NCHANNELS) before the communicator is built; "
                         "default: RCCL's own choice")
    ap.add_argument("--rccl-env", default="", help="extra RCCL / torch-NCCL settings, 'KEY=VAL,KEY=VAL'")
    ap.add_argument("--zero", type=int, default=0, choices=[0, 1],
                    help="1 = ZeRO-1: reduce-scatter grads, shard fp32 master/moments, all-gather bf16 weights")
    ap.add_argument("--grad-clip", type=float, default=1.0)
    ap.add_argument("--no-tuned-gemm", action="store_true", help="use the libraries' default GEMM heuristics")
    ap.add_argument("--tune-missing", action="store_true", help="TunableOp-tune GEMM shapes missing from the table")
    ap.add_argument("--cuda-graph", nargs="?", const="1", default="auto", choices=["auto", "0", "1"],
                    help="replay the whole step as one captured hipGraph; auto: the Trainer's own policy "
                         "(train/graph.py graph_step_policy): on for one GPU on the HIP path (+0.5 %%, "
                         "profiles/r3s3_graph_ab.txt), off with N > 1 ranks unless --graph-collectives, off for ZeRO")
    ap.add_argument("--reserve-cus", type=int, default=0,
                    help="CUs the persistent fused-epilogue GEMM grid leaves free (for RCCL kernels overlapping "
                         "the backward at N > 1); 0 = every CU")
    ap.add_argument("--gemm-persistent", default="auto", choices=["auto", "0", "1"],
                    help="persistent ping-pong GEMM / weight-gradient grids; auto: at one GPU only "
                         "(train/graph.py gemm_persistent_policy)")
    ap.add_argument("--graph-collectives", action="store_true",
                    help="capture the RCCL all-reduces inside the step's hipGraph: refused by the step policy (the capture "
                         "aborts in ProcessGroupNCCL's watchdog, train/graph.py); the eager hook-overlapped step runs")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: functional rehearsal on gloo (fp32, tiny shapes); never a measurement")
    ap.add_argument("--verbose", action="store_true")
    return ap.parse_args(argv)


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rccl_version():
    try:
        import torch
        return ".".join(str(v) for v in torch.cuda.nccl.version())
    except Exception:  # informational only: never fail a measured run over it
        return None


def launch_ranks(args, argv) -> int:
    """``--gpus N`` without a torchrun environment: start N ranks (one process per GPU,
    RCCL) through ``torch.distributed.run`` as a CHILD process -- this process never
    touches the GPU -- and return the launcher's exit code."""
    import subprocess
    argv = list(sys.argv[1:] if argv is None else argv)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


def main(argv=None):
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args, argv)
    import torch
    import torch.distributed as dist
    from pretraining_llm_amd import ops
    from pretraining_llm_amd.data import TokenLoader, ensure_synthetic_shard
    from pretraining_llm_amd.models import GPT, get_preset
    from pretraining_llm_amd.parallel.dp import DataParallelEngine
    from pretraining_llm_amd.train.optim import FlatAdamW, no_decay_1d
    from pretraining_llm_amd.utils.dist import apply_rccl_env, comm_env, init_distributed, parse_env_list

    cpu = args.device == "cpu"
    apply_rccl_env(args.rccl_channels, parse_env_list(args.rccl_env))  # before the communicator exists
    di = init_distributed("gloo" if cpu else "nccl", args.device)
    world = di.world_size
    if args.gpus != world:
        print(f"[bench] error: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    dev = di.device
    tuned = False
    if cpu:
        args.no_tuned_gemm = True
        torch.set_num_threads(max(1, min(4, os.cpu_count() or 1)))
    if not args.no_tuned_gemm:
        from pretraining_llm_amd.utils.gemm_tuning import enable_tuned_gemms
        tuned = enable_tuned_gemms(dev.index or 0, tune_missing=args.tune_missing and args.warmup > 0)
    ops.set_backend(args.backend)
    gemm_persistent = None  # (the hand-written GEMMs' grids; HIP path only)
    if args.backend == "auto" and not cpu:
        ops._lib.require()  # the HIP path must be the one that runs: fail loudly if the extension is missing
        from pretraining_llm_amd.train.graph import gemm_persistent_policy
        gemm_persistent = gemm_persistent_policy(world, args.gemm_persistent)
        ops.gemm_config(reserve_cus=args.reserve_cus, persistent=gemm_persistent)

    torch.manual_seed(1234)
    mcfg = get_preset(args.model)
    if args.seq is None:
        args.seq = mcfg.context_length
    if args.seq != mcfg.context_length:
        mcfg = mcfg.replace(context_length=max(args.seq, mcfg.context_length))
    if args.act_ckpt is not None:
        ac = args.act_ckpt
        mcfg = mcfg.replace(activation_checkpointing=ac if ac == "auto" else ac == "1" if ac in ("0", "1") else float(ac))
    model = GPT(mcfg).to(device=dev, dtype=torch.float32 if cpu else torch.bfloat16)
    okw = dict(lr=6e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1, decay_filter=no_decay_1d,
               max_grad_norm=args.grad_clip)
    if args.zero:
        from pretraining_llm_amd.parallel.zero import ShardedFlatAdamW, ZeroDataParallelEngine
        opt = ShardedFlatAdamW(model, bucket_mb=args.bucket_mb, first_bucket_mb=args.first_bucket_mb, **okw)
        engine = ZeroDataParallelEngine(opt, timing=world > 1)
    else:
        opt = FlatAdamW(model, **okw)
        # world > 1: HIP events around every bucket launch and the end-of-backward wait (where did
        # the communication time go), reported in the JSON line's "comm" block
        engine = DataParallelEngine(opt, bucket_mb=args.bucket_mb, first_bucket_mb=args.first_bucket_mb,
                                    timing=world > 1)

    B, T = args.batch, args.seq
    n_tok = max(4_000_000, 4 * B * (T + 1))
    shard = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"pllm_bench_{mcfg.vocab_size}_{n_tok}_r{di.rank}.bin")
    ensure_synthetic_shard(shard, n_tok, mcfg.vocab_size, seed=di.rank, fast=True)
    loader = TokenLoader(shard, B, T, 0, 1, seed=1000 + di.rank, device=dev)

    def step():
        engine.timer.start()
        x, y = loader.next()
        _, loss = model(x, y, return_logits=False)
        loss.backward()
        scale = engine.finish_grad_sync()
        opt.step(grad_scale=scale)
        opt.zero_grad()
        return loss

    from pretraining_llm_amd.train import graph as _graph
    if args.cuda_graph == "auto":
        ok, _why = _graph.graph_step_policy(cuda=not cpu, world=world, dist_backend=di.backend if world > 1 else None,
                                            zero=bool(args.zero),
                                            hip_ops=args.backend == "auto" and bool(getattr(opt, "use_hip", False)),
                                            graph_collectives=args.graph_collectives)
        args.cuda_graph = "1" if ok else "0"
    args.cuda_graph = args.cuda_graph == "1"
    if args.cuda_graph:
        engine.timer.enabled = False  # no event records inside a captured graph
        x0, y0 = loader.next()
        gstep = _graph.GraphedTrainStep(model, opt, engine, B, T, dev, warmup=2).capture(x0, y0, 6e-4)

        def step():  # noqa: F811
            x, y = loader.next()
            return gstep(x, y, 6e-4)

    sync = (lambda: None) if cpu else torch.cuda.synchronize
    model.train()
    for i in range(args.warmup):
        loss = step()
        if args.verbose and di.is_master:
            sync()
            print(f"[bench] warmup {i} loss {float(loss):.4f}", file=sys.stderr)
    if dist.is_initialized():
        dist.barrier()
    sync()
    engine.timer.reset()  # timed steps only
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    sync()
    if dist.is_initialized():
        dist.barrier()
    elapsed = time.perf_counter() - t0
    final_loss = float(loss.detach())
    opt.wait_params()
    ctime = engine.timer.report()
    rank_ms = [1000 * elapsed / args.steps]
    exposed = [ctime.get("exposed_comm_ms") or 0.0]
    if dist.is_initialized():
        # per-rank step time and exposed communication (the slowest rank sets the pace)
        t = torch.tensor([elapsed, exposed[0]], device=dev, dtype=torch.float64)
        parts = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        rank_ms = [float(p[0]) * 1000 / args.steps for p in parts]
        exposed = [float(p[1]) for p in parts]
        elapsed = max(float(p[0]) for p in parts)
    tokens = world * B * T * args.steps
    tps = tokens / elapsed
    flops_tok = mcfg.flops_per_token(T)
    if di.is_master:
        rec = {
            "metric": METRIC if (args.model == "gpt2-small" and T == 1024) else
            OTHER_METRIC.format(model=args.model, seq=T),
            "value": round(tps, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(tps / (EAGER_BASELINE_TOK_S_PER_GPU * world), 3)
                            if (args.model == "gpt2-small" and T == 1024 and args.backend == "auto") else None),
            "baseline": "reference-equivalent eager PyTorch on MI355X, 487.05K tok/s/GPU (BASELINE.md)",
            "dtype": "fp32" if cpu else "bf16",
            "grad_dtype": str(opt.flat_grad.dtype).replace("torch.", ""),
            "data": "synthetic (native token loader over a generated uint16 shard), random-init weights",
            "config": {"model": args.model, "global_batch": B * world, "seq_len": T,
                       "parallelism": f"dp{world}" + ("-zero1" if args.zero else ""), "micro_batch_per_gpu": B, "backend": args.backend,
                       "tokens_per_step": B * T * world, "tuned_gemms": tuned, "cuda_graph": bool(args.cuda_graph),
                       "step_mode": "graph" if args.cuda_graph else "eager",
                       "gemm_reserve_cus": args.reserve_cus,
                       "gemm_persistent": gemm_persistent,
                       "lazy_grad_zeroing": bool(getattr(opt, "lazy_zero", False)),
                       "activation_checkpointing": bool(model.use_checkpointing(torch.empty(B, T, device=dev))),
                       "checkpointed_blocks": int(model.checkpointed_blocks(torch.empty(B, T, device=dev)))},
            "mfu": round(tps / world * flops_tok / 2.5e15, 4),
            "params_M": round(sum(p.numel() for p in opt.params) / 1e6, 2),
            "final_loss": round(final_loss, 4),
            "peak_mem_gb": None if cpu else round(torch.cuda.max_memory_allocated(dev) / 1e9, 2),
            "comm": {"backend": di.backend if world > 1 else None, "world": world,
                     "rccl_version": _rccl_version() if (not cpu and world > 1 and di.backend == "nccl") else None,
                     "n_buckets": len(getattr(engine, "buckets", [])),
                     "bucket_mb": [round(b, 2) for b in engine.bucket_sizes_mb()]
                     if hasattr(engine, "bucket_sizes_mb") else None,
                     # True once the bucket readiness counts were learned: later steps launch each
                     # bucket's collective from the backward hooks (overlapped), not at the end
                     "hook_launched_buckets": getattr(engine, "_expected", None) is not None,
                     "first_bucket_mb": args.first_bucket_mb,
                     # compute-stream stall on RCCL after the backward (ms/step, HIP events), mean
                     # over timed steps; rank 0's and the worst rank's
                     "exposed_comm_ms": ctime.get("exposed_comm_ms"),
                     "exposed_comm_ms_max_rank": round(max(exposed), 3) if world > 1 else None,
                     # last timed step, rank 0: when each bucket's collective was issued and when
                     # the backward ended (ms after the step started)
                     "bucket_launch_ms": ctime.get("bucket_launch_ms"),
                     "backward_end_ms": ctime.get("backward_end_ms"),
                     "rank_step_ms_min": round(min(rank_ms), 3), "rank_step_ms_max": round(max(rank_ms), 3),
                     "rccl_env": comm_env() if world > 1 else {}},
            "device": args.device,
        }
        print(json.dumps(rec), flush=True)
    loader.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())

"""Data-parallel engine on the GPU path (HIP kernels writing gradients straight into the
flat buffer and signalling readiness through ``p._pllm_grad_ready``).

A gpurun box has ONE MI355X and RCCL refuses two ranks on the same device, so the two
ranks here share cuda:0 and talk over gloo (which reduces CUDA tensors through host
staging).  What is under test is the engine's logic on real device kernels -- the
readiness counting learned on the first backward, in-order bucket launch from hooks,
the tied-embedding two-piece gradient, the 1/world scale and the init broadcast --
not the transport; RCCL over xGMI is exercised by the driver's multi-GPU bench.

Checks:
* DP gradient == single-process gradient of the concatenated batch, at fp32 level: both sum
  the same per-rank fp32 gradients (FlatAdamW's default fp32 flat gradient, fp32 all-reduce);
* replicas stay bit-identical after several optimizer steps (SURVEY.md D5 regression).
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _cfg():
    from pretraining_llm_amd.models import get_preset
    # head_dim 64 (the headline attention kernel), V a multiple of 64 for the CE kernel
    return get_preset("gpt2-tiny").replace(vocab_size=1024, context_length=128, n_embed=256, n_head=4)


def _data(world):
    g = torch.Generator().manual_seed(123)
    return torch.randint(0, 1024, (4 * world, 129), generator=g)


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pretraining_llm_amd import ops
    from pretraining_llm_amd.models import GPT
    from pretraining_llm_amd.parallel.dp import DataParallelEngine, params_checksum
    from pretraining_llm_amd.train.optim import FlatAdamW
    ops._lib.require()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = GPT(_cfg()).to(device=dev, dtype=torch.bfloat16)
    if rank == 1:  # desynchronised init: the engine must broadcast rank 0's weights
        with torch.no_grad():
            for p in model.parameters():
                p.add_(0.5)
    opt = FlatAdamW(model, lr=1e-3)
    eng = DataParallelEngine(opt, bucket_mb=0.5, first_bucket_mb=0.1)
    data = _data(world).to(dev)
    x = data[rank * 4:(rank + 1) * 4, :-1].contiguous()
    y = data[rank * 4:(rank + 1) * 4, 1:].contiguous()
    grads = []
    for it in range(2):  # it 0 learns readiness counts; it 1 launches buckets from the hooks
        opt.zero_grad()
        _, loss = model(x, y, return_logits=False)
        loss.backward()
        scale = eng.finish_grad_sync()
        grads.append((opt.flat_grad.float() * scale).cpu())
    launched_in_backward = eng._expected is not None
    sums = []
    for step in range(3):
        opt.zero_grad()
        _, loss = model(x, y, return_logits=False)
        loss.backward()
        scale = eng.finish_grad_sync()
        opt.step(grad_scale=scale)
        cs = params_checksum(opt.params).cpu()
        allc = [torch.zeros_like(cs) for _ in range(world)]
        dist.all_gather(allc, cs)
        sums.append([c.item() for c in allc])
    torch.cuda.synchronize()
    if rank == 0:
        torch.save({"g0": grads[0], "g1": grads[1], "sums": sums, "nb": len(eng.buckets),
                    "learned": launched_in_backward}, os.path.join(outdir, "out.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _single_grad(world):
    from pretraining_llm_amd.models import GPT
    from pretraining_llm_amd.train.optim import FlatAdamW
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = GPT(_cfg()).to(device=dev, dtype=torch.bfloat16)
    opt = FlatAdamW(model, lr=1e-3)
    data = _data(world).to(dev)
    grads = []
    for r in range(world):  # per-rank gradients summed / world == DP average (equal sizes)
        opt.zero_grad()
        _, loss = model(data[r * 4:(r + 1) * 4, :-1].contiguous(), data[r * 4:(r + 1) * 4, 1:].contiguous(),
                        return_logits=False)
        loss.backward()
        grads.append(opt.flat_grad.float().cpu())
    return sum(grads) / world


def test_dp_engine_on_hip_kernels():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        out = torch.load(os.path.join(d, "out.pt"), weights_only=True)
    assert out["nb"] > 3 and out["learned"]
    ref = _single_grad(world)
    for k in ("g0", "g1"):
        got = out[k]
        err = (got - ref).abs().max().item()
        assert err <= 1e-6 * ref.abs().max().item(), (k, err)
        # the overlapped (hook-launched) iteration reduces exactly what the end-of-backward one did
    assert torch.equal(out["g0"], out["g1"])
    for step_sums in out["sums"]:
        assert step_sums[0] == step_sums[1], step_sums


def _zero_worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pretraining_llm_amd import ops
    from pretraining_llm_amd.models import GPT
    from pretraining_llm_amd.parallel.dp import DataParallelEngine
    from pretraining_llm_amd.parallel.zero import ShardedFlatAdamW, ZeroDataParallelEngine
    from pretraining_llm_amd.train.optim import FlatAdamW, no_decay_1d
    ops._lib.require()
    dev = torch.device("cuda", 0)
    data = _data(world).to(dev)
    x = data[rank * 4:(rank + 1) * 4, :-1].contiguous()
    y = data[rank * 4:(rank + 1) * 4, 1:].contiguous()
    kw = dict(lr=1e-3, weight_decay=0.1, decay_filter=no_decay_1d, max_grad_norm=1.0)
    out = {}
    for name in ("dp", "zero"):
        torch.manual_seed(0)
        model = GPT(_cfg()).to(device=dev, dtype=torch.bfloat16)
        if name == "dp":
            opt = FlatAdamW(model, **kw)
            eng = DataParallelEngine(opt, bucket_mb=0.5, first_bucket_mb=0.1)
        else:
            opt = ShardedFlatAdamW(model, bucket_mb=0.5, first_bucket_mb=0.1, **kw)
            eng = ZeroDataParallelEngine(opt)
        for step in range(3):
            opt.zero_grad()
            _, loss = model(x, y, return_logits=False)
            loss.backward()
            opt.step(grad_scale=eng.finish_grad_sync())
        opt.wait_params()  # ZeRO-1 weight all-gathers are consumed lazily by the next forward
        torch.cuda.synchronize()
        out[name] = opt.flat_param[:opt.params[-1].numel() + max(opt.offsets.values())].float().cpu()
        out[name + "_state"] = opt.master.numel()
    if rank == 0:
        torch.save(out, os.path.join(outdir, "zero.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_zero1_on_hip_kernels():
    """ZeRO-1 (reduce-scatter + HIP AdamW on owned bucket parts + all-gather) == replicated DP."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_zero_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        out = torch.load(os.path.join(d, "zero.pt"), weights_only=True)
    n = min(out["dp"].numel(), out["zero"].numel())
    err = (out["dp"][:n] - out["zero"][:n]).abs().max().item()
    assert err <= 1e-2, err  # bf16 weights; grad-norm summation order differs
    assert out["zero_state"] * 2 <= out["dp_state"] + 2 * 64 * world


def _lazy_worker(rank, world, port, outdir):
    """Weight ``b`` is used on rank 0 in every step and on rank 1 only in step 0, so from step 1 on rank 1's
    lazily-zeroed slot of ``b`` still holds its step-0 gradient unless the bucket launch clears it
    (parallel/dp.py DataParallelEngine._launch -> FlatAdamW._clear_unwritten)."""
    import torch.nn as nn
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pretraining_llm_amd import ops
    from pretraining_llm_amd.parallel.dp import DataParallelEngine, params_checksum
    from pretraining_llm_amd.train.optim import FlatAdamW
    ops._lib.require()
    dev = torch.device("cuda", 0)

    class Two(nn.Module):
        def __init__(self):
            super().__init__()
            self.a = nn.Linear(128, 128, bias=False)
            self.b = nn.Linear(128, 128, bias=False)

    out = {}
    for lazy in (False, True):
        torch.manual_seed(0)
        m = Two().to(dev, torch.bfloat16)
        opt = FlatAdamW(m, lr=1e-2, lazy_zero=lazy)
        assert opt.lazy_zero == lazy
        eng = DataParallelEngine(opt, bucket_mb=0.01, first_bucket_mb=0.01)
        g = torch.Generator(device="cpu").manual_seed(7 + rank)
        sums = []
        for step in range(4):
            x = torch.randn(64, 128, generator=g).to(dev).bfloat16()
            opt.zero_grad()
            h = ops.linear(x, m.a.weight)
            if rank == 0 or step == 0:
                h = ops.linear(h, m.b.weight)
            h.float().square().mean().backward()
            opt.step(grad_scale=eng.finish_grad_sync())
            cs = params_checksum(opt.params).cpu()
            allc = [torch.zeros_like(cs) for _ in range(world)]
            dist.all_gather(allc, cs)
            sums.append([c.item() for c in allc])
        eng.remove_hooks()
        torch.cuda.synchronize()
        out["lazy" if lazy else "full"] = (opt.master.detach().float().cpu().clone(), sums)
    if rank == 0:
        torch.save({k: v[0] for k, v in out.items()} | {k + "_sums": v[1] for k, v in out.items()},
                   os.path.join(outdir, "lazy.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_dp_lazy_zero_weight_unused_on_one_rank():
    """World 2, lazy gradient zeroing, a weight unused on ONE rank after step 0: the replicas stay identical and
    follow the fully-zeroed trajectory (a stale slot would add rank 1's step-0 gradient into every later sum)."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_lazy_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        out = torch.load(os.path.join(d, "lazy.pt"), weights_only=True)
    for key in ("full_sums", "lazy_sums"):
        for step_sums in out[key]:
            assert step_sums[0] == step_sums[1], (key, step_sums)
    rel = ((out["lazy"] - out["full"]).norm() / out["full"].norm()).item()
    assert rel < 1e-6, rel


def _rccl_worker(rank, world, port, outdir):
    """One rank on RCCL (backend nccl): the engine with its world > 1 machinery forced on (hooks launching
    bucketed all-reduces during the backward on the communicator's stream, waits, readiness learning) against
    the plain world-1 engine, same seed and data."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from pretraining_llm_amd import ops
    from pretraining_llm_amd.ab import ab_set
    from pretraining_llm_amd.models import GPT
    from pretraining_llm_amd.parallel.dp import DataParallelEngine, params_checksum
    from pretraining_llm_amd.train.optim import FlatAdamW
    ops._lib.require()
    data = _data(1).to(dev)
    x, y = data[:, :-1].contiguous(), data[:, 1:].contiguous()
    out = {"backend": dist.get_backend()}
    for forced in (False, True):
        ab_set("dp_world1", forced)
        torch.manual_seed(0)
        model = GPT(_cfg()).to(device=dev, dtype=torch.bfloat16)
        opt = FlatAdamW(model, lr=1e-3, max_grad_norm=1.0)
        eng = DataParallelEngine(opt, bucket_mb=0.5, first_bucket_mb=0.1)
        in_bwd, sums, grads = [], [], []
        for step in range(4):
            opt.zero_grad()
            _, loss = model(x, y, return_logits=False)
            loss.backward()
            in_bwd.append(eng._next_launch)  # buckets launched by the hooks before the end of the backward
            scale = eng.finish_grad_sync()
            grads.append(opt.flat_grad.float().cpu().clone())
            opt.step(grad_scale=scale)
            sums.append(params_checksum(opt.params).item())
        eng.remove_hooks()
        torch.cuda.synchronize()
        out["forced" if forced else "plain"] = {"sync": eng.sync, "nb": len(eng.buckets), "in_bwd": in_bwd,
                                               "sums": sums, "g": torch.stack(grads)}
    torch.save(out, os.path.join(outdir, "rccl.pt"))
    dist.destroy_process_group()


def test_dp_rccl_world1_rehearsal():
    """The world > 1 data-parallel step over a real RCCL communicator (one rank: a one-GPU box cannot host two
    RCCL ranks): bit-identical gradients and weights to the plain step, and the buckets after the first
    (learning) step launched from the gradient hooks inside the backward."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rccl_worker, args=(1, _free_port(), d), nprocs=1, join=True)
        out = torch.load(os.path.join(d, "rccl.pt"), weights_only=True)
    assert out["backend"] == "nccl"
    f, p = out["forced"], out["plain"]
    assert f["sync"] and not p["sync"]
    assert f["in_bwd"][0] == 0 and all(n == f["nb"] for n in f["in_bwd"][1:]), f["in_bwd"]
    assert torch.equal(f["g"], p["g"])
    assert f["sums"] == p["sums"]

"""Ring (context-parallel) attention on the GPU path: every (query chunk, key chunk) block runs
the HIP flash forward / block-backward kernels and the partial results are LSE-merged; the
sharded output and dQ/dK/dV must match fp32 attention over the whole sequence.

Two ranks share the one MI355X of a gpurun box and ring their K/V over gloo (host-staged);
on a multi-GPU node the same ring runs over RCCL/xGMI.
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
    p = s.getsockname()[1]
    s.close()
    return p


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pretraining_llm_amd import ops
    from pretraining_llm_amd.ops import reference as ref
    from pretraining_llm_amd.parallel import context as cp
    ops._lib.require()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    B, T, H, Hkv, D = 2, 256 * world, 4, 2, 64
    q, k, v, do = (torch.randn(B, T, h, D, generator=g) for h in (H, Hkv, Hkv, H))
    qf, kf, vf = (t.clone().requires_grad_() for t in (q, k, v))
    o_ref, _ = ref.attention(qf, kf, vf, causal=True)
    o_ref.backward(do)
    res = {}
    for layout in ("contiguous", "zigzag"):
        Tl = T // world
        if layout == "zigzag":
            shard = lambda x: cp.zigzag_shard(x, 1)  # noqa: E731
            unshard = lambda x: cp.zigzag_unshard(x.cpu(), 1)  # noqa: E731
        else:
            shard = lambda x: x[:, rank * Tl:(rank + 1) * Tl]  # noqa: E731

            def unshard(x):
                x = x.float().cpu().contiguous()
                parts = [torch.empty_like(x) for _ in range(world)]
                dist.all_gather(parts, x)
                return torch.cat(parts, 1)
        ql, kl, vl = (shard(t).to(dev, torch.bfloat16).contiguous().requires_grad_() for t in (q, k, v))
        o = cp.ring_attention(ql, kl, vl, causal=True, layout=layout)
        o.backward(shard(do).to(dev, torch.bfloat16))
        res[layout] = [_rel(unshard(o.detach().float()), o_ref.detach()),
                       _rel(unshard(ql.grad.float()), qf.grad),
                       _rel(unshard(kl.grad.float()), kf.grad),
                       _rel(unshard(vl.grad.float()), vf.grad)]
    torch.cuda.synchronize()
    torch.save(res, os.path.join(outdir, f"cp{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_ring_attention_on_hip_kernels():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        outs = [torch.load(os.path.join(d, f"cp{r}.pt"), weights_only=True) for r in range(world)]
    for res in outs:
        for layout, errs in res.items():
            assert max(errs) < 3e-2, (layout, errs)

"""Ring (context-parallel) attention vs single-device attention: forward output and
dq/dk/dv, contiguous and zigzag layouts, GQA, gloo world 2 and 4 on CPU."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q_):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pretraining_llm_amd.ops import reference as ref
    from pretraining_llm_amd.parallel import context as cp
    torch.manual_seed(0)
    B, T, H, Hkv, D = 2, 16 * world, 4, 2, 16
    q = torch.randn(B, T, H, D)
    k = torch.randn(B, T, Hkv, D)
    v = torch.randn(B, T, Hkv, D)
    do = torch.randn(B, T, H, D)
    qf, kf, vf = (t.clone().requires_grad_() for t in (q, k, v))
    o_ref, _ = ref.attention(qf, kf, vf, causal=True)
    o_ref.backward(do)
    res = {}
    for layout in ("contiguous", "zigzag"):
        if layout == "zigzag":
            shard = lambda x: cp.zigzag_shard(x, 1)  # noqa: E731
            unshard = lambda x: cp.zigzag_unshard(x, 1)  # noqa: E731
        else:
            Tl = T // world
            shard = lambda x: x[:, rank * Tl:(rank + 1) * Tl]  # noqa: E731

            def unshard(x):
                parts = [torch.empty_like(x) for _ in range(world)]
                dist.all_gather(parts, x.contiguous())
                return torch.cat(parts, 1)
        ql, kl, vl = (shard(t).clone().requires_grad_() for t in (q, k, v))
        o = cp.ring_attention(ql, kl, vl, causal=True, layout=layout)
        o.backward(shard(do))
        res[layout] = [
            (unshard(o.detach()) - o_ref.detach()).abs().max().item(),
            (unshard(ql.grad) - qf.grad).abs().max().item(),
            (unshard(kl.grad) - kf.grad).abs().max().item(),
            (unshard(vl.grad) - vf.grad).abs().max().item(),
        ]
    if rank == 0:
        pos = cp.zigzag_positions(T // world)
        res["positions"] = pos.tolist()
        q_.put(res)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_ring_attention_matches_dense(world):
    ctx = mp.get_context("spawn")
    q_ = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q_)) for r in range(world)]
    for p in procs:
        p.start()
    res = q_.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for layout in ("contiguous", "zigzag"):
        errs = res[layout]
        assert max(errs) < 1e-4, (layout, errs)
    c = 16 // 2
    assert res["positions"] == list(range(0, c)) + list(range((2 * world - 1) * c, 2 * world * c))

"""Tensor / sequence / Ulysses-context parallel layers vs their dense equivalents (gloo, world 2, CPU)."""
import os
import socket
import tempfile

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dense_attn(x, qkv_w, qkv_b, proj_w, proj_b, H):
    from pretraining_llm_amd.ops import reference as ref
    B, T, C = x.shape
    D = C // H
    qkv = F.linear(x, qkv_w, qkv_b).view(B, T, 3, H, D)
    o, _ = ref.attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], causal=True)
    return F.linear(o.reshape(B, T, C), proj_w, proj_b)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pretraining_llm_amd.parallel import tensor as tp
    torch.manual_seed(0)
    B, T, C, H, Fh = 2, 8, 16, 4, 64
    x = torch.randn(B, T, C)
    w1, b1 = torch.randn(Fh, C) * 0.1, torch.randn(Fh) * 0.1
    w2, b2 = torch.randn(C, Fh) * 0.1, torch.randn(C) * 0.1
    qkv_w, qkv_b = torch.randn(3 * C, C) * 0.2, torch.randn(3 * C) * 0.1
    pw, pb = torch.randn(C, C) * 0.2, torch.randn(C) * 0.1
    res = {}

    # --- dense references
    xd = x.clone().requires_grad_()
    yd = F.linear(F.gelu(F.linear(xd, w1, b1), approximate="tanh"), w2, b2)
    yd.sum().backward()
    ad = x.clone().requires_grad_()
    za = _dense_attn(ad, qkv_w, qkv_b, pw, pb, H)
    za.pow(2).sum().backward()

    # --- TP MLP (replicated input)
    mlp = tp.TensorParallelMLP(C, Fh)
    mlp.fc.load_from_dense(w1, b1)
    mlp.proj.load_from_dense(w2, b2)
    xt = x.clone().requires_grad_()
    yt = mlp(xt)
    yt.sum().backward()
    res["mlp_out"] = (yt - yd).abs().max().item()
    res["mlp_dx"] = (xt.grad - xd.grad).abs().max().item()

    # --- TP MLP with sequence parallelism (input/output sharded along T)
    mlp2 = tp.TensorParallelMLP(C, Fh, sequence_parallel=True)
    mlp2.fc.load_from_dense(w1, b1)
    mlp2.proj.load_from_dense(w2, b2)
    xs = x.clone().requires_grad_()
    xl = tp.scatter_to_sequence(xs)
    ys = mlp2(xl)
    ys_full = tp.gather_from_sequence(ys.contiguous())
    (ys.sum()).backward()
    res["sp_out"] = (ys_full - yd).abs().max().item()
    res["sp_dx"] = (xs.grad - xd.grad).abs().max().item()

    # --- TP attention (heads sharded)
    att = tp.TensorParallelAttention(C, H)
    att.load_from_dense(qkv_w, qkv_b, pw, pb)
    at = x.clone().requires_grad_()
    zt = att(at)
    zt.pow(2).sum().backward()
    res["attn_out"] = (zt - za).abs().max().item()
    res["attn_dx"] = (at.grad - ad.grad).abs().max().item()

    # --- Ulysses: sequence-sharded qkv -> head-sharded attention -> back
    uq = x.clone().requires_grad_()
    qkv = F.linear(uq, qkv_w, qkv_b)
    ql = tp.scatter_to_sequence(qkv)
    ol = tp.ulysses_attention(ql, H)
    o_full = tp.gather_from_sequence(ol.contiguous())
    zu = F.linear(o_full, pw, pb)
    res["ulysses_out"] = (zu - za).abs().max().item()
    zu.pow(2).sum().backward()
    # every rank computes the full loss on the gathered output; gradients flowing back through the
    # gather are reduce-scattered, so the replicated input gradient is world x the dense one
    res["ulysses_dx"] = (uq.grad / world - ad.grad).abs().max().item()
    if rank == 0:
        torch.save(res, os.path.join(out, "res.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_tensor_sequence_context_parallel_match_dense():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        res = torch.load(os.path.join(d, "res.pt"), weights_only=True)
    for k, v in res.items():
        assert v < 1e-4, (k, v, res)

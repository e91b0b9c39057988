"""Tensor / sequence / context parallelism wired into GPT + the optimizer (gloo on CPU).

Every case builds the dense model from one seed, shards it with ``parallelize_gpt`` on a
``dp x cp x tp`` mesh, runs one full training step the way ``Trainer.train_step`` does
(forward, backward, DP/ZeRO gradient sync, sequence-parallel replicated-gradient sum,
clipped AdamW) and checks against the dense single-process model on the same global batch:

* the global mean loss,
* every gradient, reassembled into the dense layout (``gather_dense_state``),
* the global gradient norm used for clipping,
* every weight after the optimizer step.

The reference has data parallelism only (scripts/train_transformer.py:122-123); these layouts
are this framework's additions.
"""
import copy
import os
import socket
import tempfile

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


def _cfg(arch):
    from pretraining_llm_amd.models import get_preset
    if arch == "gpt2":
        return get_preset("gpt2-tiny").replace(vocab_size=256, context_length=32, n_embed=64, n_head=4)
    if arch == "llama":
        return get_preset("llama-tiny").replace(vocab_size=256, context_length=32, n_embed=64, n_head=4,
                                                n_kv_head=2, ffn_hidden=96)
    if arch == "ref":
        return get_preset("ref-small").replace(vocab_size=256, context_length=32, n_embed=64, n_head=4,
                                               n_blocks=2)
    raise KeyError(arch)


B_PER_DP, T = 2, 32
MAX_NORM = 0.5  # small enough that clipping is active: the global norm must be right
EPS = 1e-5  # Adam eps well above the fp32 noise of a reordered reduction: |g| ~ eps would flip updates


def _batch(dp):
    g = torch.Generator().manual_seed(7)
    data = torch.randint(0, 256, (B_PER_DP * dp, T + 1), generator=g)
    return data[:, :-1], data[:, 1:]


def _worker(rank, world, port, outdir, arch, tp, cp, sp, zero, cp_mode="ring"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pretraining_llm_amd.models import GPT
    from pretraining_llm_amd.parallel.dp import DataParallelEngine
    from pretraining_llm_amd.parallel.model_parallel import (gather_dense_state, init_parallel_groups,
                                                             parallelize_gpt, sync_replicated_grads)
    from pretraining_llm_amd.train.optim import FlatAdamW
    cfg = _cfg(arch)
    torch.manual_seed(0)
    model = GPT(cfg)
    pg = init_parallel_groups(tp, cp, sp, cp_mode)
    parallelize_gpt(model, pg)
    okw = dict(lr=1e-2, weight_decay=0.1, max_grad_norm=MAX_NORM, eps=EPS)
    if zero:
        from pretraining_llm_amd.parallel.zero import ShardedFlatAdamW, ZeroDataParallelEngine
        opt = ShardedFlatAdamW(model, process_group=pg.grad_group, bucket_mb=0.02, first_bucket_mb=0.01, **okw)
        eng = ZeroDataParallelEngine(opt)
    else:
        opt = FlatAdamW(model, **okw)
        eng = DataParallelEngine(opt, process_group=pg.grad_group, bucket_mb=0.05, first_bucket_mb=0.01)
    if tp > 1:
        opt.set_tensor_parallel(pg.tp_group, tp)
    x, y = _batch(pg.dp)
    x, y = x[pg.dp_rank * B_PER_DP:(pg.dp_rank + 1) * B_PER_DP], y[pg.dp_rank * B_PER_DP:(pg.dp_rank + 1) * B_PER_DP]
    _, loss = model(x, y, return_logits=False)
    loss.backward()
    scale = eng.finish_grad_sync()
    if sp:
        sync_replicated_grads(opt, pg)
        scale /= tp
    out = {}
    if not zero:  # ZeRO keeps only this rank's reduced slice: checked through the step below
        grads = {id(p): opt.grad_view(i).view(p.shape) * scale for i, p in enumerate(opt.params)}
        gd = gather_dense_state(model, GPT(cfg), pg, grads)
        out["grads"] = {n: p.detach().clone() for n, p in gd.named_parameters()}
    out["norm"] = float(opt.grad_norm(scale))
    opt.step(grad_scale=scale)
    opt.wait_params()  # ZeRO-1: the step's weight all-gathers are consumed lazily (next forward)
    wd = gather_dense_state(model, GPT(cfg), pg)
    out["weights"] = {n: p.detach().clone() for n, p in wd.named_parameters()}
    lt = loss.detach().reshape(1).clone()
    dist.all_reduce(lt)
    out["loss"] = float(lt) / world
    if rank == 0:
        torch.save(out, os.path.join(outdir, "out.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _dense(arch, dp):
    from pretraining_llm_amd.models import GPT
    from pretraining_llm_amd.train.optim import FlatAdamW
    cfg = _cfg(arch)
    torch.manual_seed(0)
    model = GPT(cfg)
    opt = FlatAdamW(model, lr=1e-2, weight_decay=0.1, max_grad_norm=MAX_NORM, eps=EPS)
    x, y = _batch(dp)
    _, loss = model(x, y, return_logits=False)
    loss.backward()
    grads = {n: opt.grad_view(i).view(p.shape).clone() for i, (n, p) in enumerate(zip(opt.names, opt.params))}
    norm = float(opt.grad_norm())
    opt.step()
    return {"loss": float(loss.detach()), "grads": grads, "norm": norm,
            "weights": {n: p.detach().clone() for n, p in model.named_parameters()}}


CASES = {
    # name: (world, arch, tp, cp, sequence_parallel, zero)
    "tp2_gpt2": (2, "gpt2", 2, 1, False, False),
    "tp2_sp_gpt2": (2, "gpt2", 2, 1, True, False),
    "tp2_llama_gqa_rope": (2, "llama", 2, 1, False, False),
    "tp2_sp_llama": (2, "llama", 2, 1, True, False),
    "tp2_ref_no_wo": (2, "ref", 2, 1, False, False),
    "cp2_gpt2": (2, "gpt2", 1, 2, False, False),
    "cp2_llama": (2, "llama", 1, 2, False, False),
    "tp2_sp_dp2_zero_llama": (4, "llama", 2, 1, True, True),
    "cp2_dp2_gpt2": (4, "gpt2", 1, 2, False, False),
    "ulysses2_gpt2": (2, "gpt2", 1, 2, False, False, "ulysses"),
    "ulysses2_llama_gqa_rope": (2, "llama", 1, 2, False, False, "ulysses"),
    "ulysses2_dp2_zero_llama": (4, "llama", 1, 2, False, True, "ulysses"),
    # 2-D: tensor x context parallelism (heads over TP, sequence over CP), and sequence
    # parallelism for the reference architecture (no W_o: heads return to sequence shards by an
    # all-to-all)
    "tp2_ulysses2_gpt2": (4, "gpt2", 2, 2, False, False, "ulysses"),
    "tp2_ring2_llama_gqa_rope": (4, "llama", 2, 2, False, False, "ring"),
    "tp2_ring2_ref_no_wo": (4, "ref", 2, 2, False, False, "ring"),
    "tp2_sp_ref_no_wo": (2, "ref", 2, 1, True, False),
}


@pytest.mark.parametrize("case", list(CASES))
def test_model_parallel_step_matches_dense(case):
    world, arch, tp, cp, sp, zero, *mode = CASES[case]
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d, arch, tp, cp, sp, zero, *mode), nprocs=world, join=True)
        got = torch.load(os.path.join(d, "out.pt"), weights_only=True)
    ref = _dense(arch, world // (tp * cp))
    assert abs(got["loss"] - ref["loss"]) < 1e-5, (got["loss"], ref["loss"])
    assert abs(got["norm"] - ref["norm"]) < 1e-4 * ref["norm"], (got["norm"], ref["norm"])
    assert ref["norm"] > MAX_NORM  # clipping active
    if "grads" in got:
        for n, g in ref["grads"].items():
            assert torch.allclose(got["grads"][n], g, atol=1e-6, rtol=1e-4), (n, (got["grads"][n] - g).abs().max())
    for n, w in ref["weights"].items():
        assert torch.allclose(got["weights"][n], w, atol=2e-5, rtol=1e-5), (n, (got["weights"][n] - w).abs().max())


def test_parallel_groups_layout():
    """rank = (dp_rank * cp + cp_rank) * tp + tp_rank with TP innermost; bad sizes raise."""
    from pretraining_llm_amd.parallel.model_parallel import init_parallel_groups
    g = init_parallel_groups(1, 1)
    assert (g.world, g.dp, g.tp, g.cp) == (1, 1, 1, 1) and not g.model_parallel
    with pytest.raises(ValueError):
        init_parallel_groups(1, 1, sequence_parallel=True)
    with pytest.raises(ValueError):
        init_parallel_groups(2, 1)  # world 1 is not divisible by tp 2


def _trainer_cfg(tmp, **kw):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from config.config import PRESET_RUNS, default_config
    cfg = dict(default_config)
    cfg.update(PRESET_RUNS["gpt2-tiny-cpu"])
    cfg.update(dict(t_out_path=os.path.join(tmp, "models", "m.pt"), synthetic_dir=os.path.join(tmp, "syn"),
                    t_train_steps=8, t_eval_steps=4, log_interval=4, t_eval_iters=1, t_batch_size=2, seq_len=64,
                    synthetic_tokens=50_000, device="cpu", max_grad_norm=1.0, eps=1e-5))
    cfg.update(kw)
    return cfg


def _trainer_worker(rank, world, port, tmp, kw):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from pretraining_llm_amd.train import Trainer
    from pretraining_llm_amd.utils.dist import init_distributed
    di = init_distributed("gloo", "cpu")
    a = Trainer(_trainer_cfg(tmp, ckpt_interval=4, **kw), dist_info=di, log=lambda *_: None)
    a.train()
    # resume from the step-4 checkpoint (per-TP-rank shard + optimizer state) and finish again
    b = Trainer(_trainer_cfg(tmp, resume=os.path.join(tmp, "models", "m.latest.pt"),
                             t_out_path=os.path.join(tmp, "models", "b.pt"), **kw), dist_info=di, log=lambda *_: None)
    assert b.step == 4
    b.train()
    err = max((x - y).abs().max().item() for x, y in zip(a.model.parameters(), b.model.parameters()))
    torch.save({"resume_err": err}, os.path.join(tmp, f"r{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("kw", [dict(tp_size=2, sequence_parallel=True), dict(tp_size=2, zero_stage=1), dict(cp_size=2),
                                dict(cp_size=2, cp_mode="ulysses")], ids=["tp2_sp", "tp2_zero1", "cp2", "ulysses2"])
def test_trainer_model_parallel_matches_dense_and_resumes(tmp_path, kw):
    """Trainer with tp_size / cp_size on 2 gloo ranks: the consolidated dense checkpoint after 8
    steps equals a 1-process dense Trainer's weights on the same data, and resuming from the
    step-4 checkpoint reproduces the final weights."""
    from pretraining_llm_amd.models import GPT
    from pretraining_llm_amd.train import Trainer
    from pretraining_llm_amd.utils.checkpoint import load_checkpoint
    mp.spawn(_trainer_worker, args=(2, _free_port(), str(tmp_path), kw), nprocs=2, join=True)
    for r in range(2):
        assert torch.load(tmp_path / f"r{r}.pt", weights_only=True)["resume_err"] < 1e-6
    dense = Trainer(_trainer_cfg(str(tmp_path / "dense")), log=lambda *_: None)
    dense.train()
    ck = load_checkpoint(str(tmp_path / "models" / "m.pt"))
    m = GPT(dense.mcfg)
    m.load_state_dict(ck["model_state_dict"], strict=True)
    for (n, p), q in zip(dense.model.named_parameters(), m.parameters()):
        assert torch.allclose(p, q, atol=5e-5, rtol=1e-4), (n, (p - q).abs().max())


def test_dense_shell_draws_no_rng_and_tp_ranges_aligned():
    """The consolidated-checkpoint model is built without touching the RNG (a saving rank stays in
    step with the others), and the TP-replicated gradient ranges are ALIGN-padded runs (the HIP
    sum of squares needs numel % 8 == 0; an odd-sized replicated parameter must not break it)."""
    import torch.nn as nn
    from pretraining_llm_amd.models import GPT, get_preset
    from pretraining_llm_amd.parallel.model_parallel import build_dense_shell
    from pretraining_llm_amd.train.optim import ALIGN, FlatAdamW
    cfg = get_preset("gpt2-tiny")
    torch.manual_seed(3)
    before = torch.get_rng_state()
    m = build_dense_shell(cfg)
    assert torch.equal(torch.get_rng_state(), before)
    assert sum(p.numel() for p in m.parameters()) == sum(p.numel() for p in GPT(cfg).parameters())

    class Odd(nn.Module):
        def __init__(self):
            super().__init__()
            self.a = nn.Parameter(torch.randn(7))        # replicated, odd size
            self.w = nn.Parameter(torch.randn(16, 8))    # "sharded"
            self.b = nn.Parameter(torch.randn(5))        # replicated, odd size
            self.c = nn.Parameter(torch.randn(3))        # replicated, adjacent to b
    net = Odd()
    net.w._pllm_tp_sharded = True
    opt = FlatAdamW(net)
    opt.set_tensor_parallel(None, 2)
    buf, ranges = opt.replicated_grad_ranges()
    assert all(a % ALIGN == 0 and b % ALIGN == 0 for a, b in ranges) and len(ranges) == 2
    opt.flat_grad.normal_()
    for i, p in enumerate(opt.params):  # padding of the flat gradient is zero, as in training
        o = opt.offsets[i]
        opt.flat_grad[o + p.numel():o + -(-p.numel() // ALIGN) * ALIGN].zero_()
    ss = opt._sumsq(opt.flat_grad)
    rep = sum(opt.grad_view(i).pow(2).sum() for i in (0, 2, 3))
    assert torch.allclose(opt._tp_adjust(ss), ss - rep * 0.5)

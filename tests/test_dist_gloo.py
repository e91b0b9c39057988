"""Multi-process data-parallel tests on CPU with the gloo backend (world size 2).

* bucketed all-reduce gradient == single-process gradient on the concatenated batch
* replicas stay bit-identical over several optimizer steps (regression test for the
  reference's every-other-step sync skip)
* no_sync gradient accumulation parity
"""
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
    port = s.getsockname()[1]
    s.close()
    return port


def _tiny_cfg():
    from pretraining_llm_amd.models import get_preset
    return get_preset("gpt2-tiny").replace(vocab_size=256, context_length=32, n_embed=64, n_head=2)


def _worker(rank, world, port, outdir, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pretraining_llm_amd.models import GPT
    from pretraining_llm_amd.parallel.dp import DataParallelEngine, params_checksum
    from pretraining_llm_amd.train.optim import FlatAdamW
    torch.manual_seed(0)
    cfg = _tiny_cfg()
    model = GPT(cfg)
    # deliberately desynchronise initial weights: the engine must broadcast rank 0's
    if rank == 1:
        with torch.no_grad():
            for p in model.parameters():
                p.add_(1.0)
    opt = FlatAdamW(model, lr=1e-2)
    eng = DataParallelEngine(opt, bucket_mb=0.05, first_bucket_mb=0.01)  # many small buckets
    g = torch.Generator().manual_seed(123)
    data = torch.randint(0, 256, (4 * world, 33), generator=g)
    if mode == "grad":
        x = data[rank * 4:(rank + 1) * 4, :-1]
        y = data[rank * 4:(rank + 1) * 4, 1:]
        for it in range(2):  # second iteration runs with the learned (overlapped) readiness counts
            opt.zero_grad()
            _, loss = model(x, y)
            loss.backward()
            scale = eng.finish_grad_sync()
            grad = opt.flat_grad.clone() * scale
        if rank == 0:
            torch.save({"grad": grad, "buckets": len(eng.buckets)}, os.path.join(outdir, "grad.pt"))
    elif mode == "steps":
        sums = []
        for step in range(4):
            x = data[rank * 4:(rank + 1) * 4, :-1]
            y = data[rank * 4:(rank + 1) * 4, 1:]
            _, loss = model(x, y)
            loss.backward()
            scale = eng.finish_grad_sync()
            opt.step(grad_scale=scale)
            opt.zero_grad()
            cs = params_checksum(opt.params)
            allc = [torch.zeros_like(cs) for _ in range(world)]
            dist.all_gather(allc, cs)
            sums.append([c.item() for c in allc])
        if rank == 0:
            torch.save(sums, os.path.join(outdir, "sums.pt"))
    elif mode == "accum":
        # 2 micro-batches with no_sync on the first == one batch of 8 per rank
        opt.zero_grad()
        for micro in range(2):
            x = data[rank * 4 + micro * 2: rank * 4 + micro * 2 + 2, :-1]
            y = data[rank * 4 + micro * 2: rank * 4 + micro * 2 + 2, 1:]
            ctx = eng.no_sync() if micro == 0 else torch.enable_grad()
            with ctx:
                _, loss = model(x, y)
                loss.backward()
        scale = eng.finish_grad_sync()
        if rank == 0:
            torch.save({"grad": opt.flat_grad.clone() * scale / 2}, os.path.join(outdir, "accum.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _run(mode, world=2):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d, mode), nprocs=world, join=True)
        return {f: torch.load(os.path.join(d, f), weights_only=True) for f in os.listdir(d)}


def _single_process_grad(world=2, rows=None):
    from pretraining_llm_amd.models import GPT
    from pretraining_llm_amd.train.optim import FlatAdamW
    torch.manual_seed(0)
    model = GPT(_tiny_cfg())
    opt = FlatAdamW(model, lr=1e-2)
    g = torch.Generator().manual_seed(123)
    data = torch.randint(0, 256, (4 * world, 33), generator=g)
    # mean over ranks of per-rank mean losses == mean over the concatenated batch (equal sizes)
    _, loss = model(data[:, :-1], data[:, 1:])
    loss.backward()
    return opt.flat_grad.clone()


def test_dp_allreduce_matches_single_process():
    out = _run("grad")
    ref = _single_process_grad()
    got = out["grad.pt"]["grad"]
    assert out["grad.pt"]["buckets"] > 3
    assert torch.allclose(got, ref, atol=2e-6, rtol=1e-4), (got - ref).abs().max()


def test_dp_replicas_stay_identical():
    sums = _run("steps")["sums.pt"]
    for step_sums in sums:
        assert step_sums[0] == step_sums[1], step_sums


def test_dp_no_sync_accumulation():
    acc = _run("accum")["accum.pt"]["grad"]
    ref = _single_process_grad()
    assert torch.allclose(acc, ref, atol=2e-6, rtol=1e-4), (acc - ref).abs().max()


def test_comm_bench_sweep_gloo():
    """bench/comm_bench.py (RCCL bus-bandwidth sweep) runs end-to-end under torchrun (gloo, 2 ranks)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr",
                        "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench", "comm_bench.py"),
                        "--backend", "gloo", "--device", "cpu", "--sizes-mb", "0.1", "--iters", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=240, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-2000:]
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert {x["op"] for x in recs} == {"all_reduce", "reduce_scatter", "all_gather", "all_to_all"}
    assert all(x["busbw_GBps"] > 0 and x["world"] == 2 for x in recs)


def test_bench_self_launches_ranks_cpu():
    """``bench.py --gpus 2`` with no torchrun environment starts 2 ranks itself (gloo on CPU here,
    RCCL on GPUs) and rank 0 reports n_gpus 2 with the time taken as the max over ranks."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--device", "cpu",
                        "--model", "gpt2-tiny", "--steps", "2", "--warmup", "1", "--batch", "2", "--seq", "64",
                        "--rccl-channels", "8", "--rccl-env", "TORCH_NCCL_HIGH_PRIORITY=1", "--bucket-mb", "2",
                        "--first-bucket-mb", "0.5"],
                       capture_output=True, text=True, timeout=300, cwd="/tmp", env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(recs) == 1, r.stdout
    rec = recs[0]
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2" and rec["config"]["global_batch"] == 4
    c = rec["comm"]
    assert c["world"] == 2 and c["hook_launched_buckets"]
    assert rec["config"]["step_mode"] == "eager" and not rec["config"]["cuda_graph"]
    # multi-GPU diagnostics: per-rank step times, the RCCL environment the run had (set before
    # the process group existed), exposed-communication fields (HIP events: None on CPU)
    assert c["rank_step_ms_min"] <= c["rank_step_ms_max"] and abs(c["rank_step_ms_max"] - rec["ms_per_step"]) < 1e-2
    assert c["rccl_env"]["NCCL_MIN_NCHANNELS"] == "8" and c["rccl_env"]["NCCL_MAX_NCHANNELS"] == "8"
    assert c["rccl_env"]["TORCH_NCCL_HIGH_PRIORITY"] == "1"
    assert c["first_bucket_mb"] == 0.5 and c["n_buckets"] >= 2
    assert "exposed_comm_ms" in c and "bucket_launch_ms" in c and "exposed_comm_ms_max_rank" in c
    assert rec["value"] > 0 and abs(rec["value"] - 2 * 2 * 64 * 2 / (rec["ms_per_step"] * 2 / 1000)) / rec["value"] < 0.01


def test_train_cli_under_torchrun_preset(tmp_path):
    """The reference launch contract ``torchrun --nproc_per_node=N scripts/train_transformer.py``
    with a named preset: ``--preset=`` survives torchrun's own argument parser (which takes
    ``--run`` as an abbreviation of its ``--run-path``), 2 gloo ranks train, eval and save."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "tiny.pt"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr",
                        "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(root, "scripts", "train_transformer.py"), "--preset=gpt2-tiny-cpu",
                        "--ddp_backend=gloo", "--t_train_steps=4", "--t_eval_steps=2", "--t_eval_iters=1",
                        "--log_interval=2", "--t_batch_size=2", "--seq_len=64", f"--synthetic_dir={tmp_path}",
                        "--synthetic_tokens=50000", f"--t_out_path={out}"],
                       capture_output=True, text=True, timeout=300, cwd="/tmp",
                       env={**os.environ, "OMP_NUM_THREADS": "2"})
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert "world=2" in r.stdout and "Step 2" in r.stdout, r.stdout[-2000:]
    assert out.exists()


def test_byte_tokenizer_renders_non_byte_ids():
    """The offline byte-level fallback keeps ids outside 0..255 visible in decoded text."""
    from pretraining_llm_amd.data.tokenizer import ByteTokenizer
    t = ByteTokenizer()
    ids = t.encode("héllo") + [1234, 50256] + t.encode("!")
    assert t.decode(ids) == "héllo<|1234|><|50256|>!"
    assert t.decode(t.encode("plain")) == "plain"


@pytest.mark.parametrize("mode", ["default", "graph_collectives"])
def test_trainer_and_bench_take_the_same_step_path(mode, tmp_path):
    """the Trainer's world > 1 step and ``bench.py --gpus N`` take the same path,
    checked by what they DO: 2 gloo ranks (torch.distributed.run) with the step policy stubbed to the
    RCCL branch (GPU, nccl, HIP ops) and a recording eager stand-in for the hipGraph capture
    (tests/_policy_probe.py).  Default: both run the eager hook-overlapped step (no capture object
    built); graph_collectives=True: refused by the policy (it aborts on RCCL, train/graph.py), so both take
    the eager step as well."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "2"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr",
                        "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "tests", "_policy_probe.py"),
                        mode, str(tmp_path)], capture_output=True, text=True, timeout=300, cwd="/tmp", env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    recs = [json.loads(l.split("PROBE ", 1)[1]) for l in r.stdout.splitlines() if "PROBE " in l]
    assert sorted(x["rank"] for x in recs) == [0, 1], r.stdout
    want = "eager"
    for x in recs:
        t, b = x["trainer"], x["bench"]
        assert t["step_mode"] == want, x
        assert b["rc"] in (None, 0), x
        if x["rank"] == 0:
            assert b["step_mode"] == want, x  # rank 0 prints the bench record
        assert t["capture_objects"] == 0 and b["capture_objects"] == 0, x


def test_step_policy_decisions():
    """graph_step_policy's table (the function both launch paths call, see the behavioural test above)."""
    from pretraining_llm_amd.train import graph as g
    for world in (2, 4, 8):
        ok, why = g.graph_step_policy(cuda=True, world=world, dist_backend="nccl")
        assert not ok and "eager" in why
        ok, why = g.graph_step_policy(cuda=True, world=world, dist_backend="nccl", graph_collectives=True)
        assert not ok and "hipErrorCapturedEvent" in why
        assert not g.graph_step_policy(cuda=True, world=world, dist_backend="gloo", graph_collectives=True)[0]
    assert not g.graph_step_policy(cuda=True, world=1, dist_backend="nccl", graph_collectives=True)[0]
    assert g.graph_step_policy(cuda=True, world=1, dist_backend=None) == (True, None)
    assert not g.graph_step_policy(cuda=True, world=1, dist_backend=None, zero=True)[0]
    assert not g.graph_step_policy(cuda=False, world=1, dist_backend=None)[0]
    # persistent GEMM grids: world 1 only by default
    assert g.gemm_persistent_policy(1) and g.gemm_persistent_policy(1, "auto")
    for world in (2, 4, 8):
        assert not g.gemm_persistent_policy(world)
        assert g.gemm_persistent_policy(world, "1") and g.gemm_persistent_policy(world, True)
    assert not g.gemm_persistent_policy(1, "0")


def test_dp_buckets_isolate_oversized_params():
    """A parameter at least a bucket in size gets its own bucket (parallel/dp.py): the tied embedding --
    the last gradient of the backward -- must not drag the first block's parameters into the un-overlappable
    tail bucket.  Buckets still tile the flat gradient buffer in reverse layout order."""
    from pretraining_llm_amd.models import GPT
    from pretraining_llm_amd.parallel.dp import DataParallelEngine
    from pretraining_llm_amd.train.optim import FlatAdamW
    torch.manual_seed(0)
    model = GPT(_tiny_cfg().replace(vocab_size=2048))  # 2048 x 64 fp32 embedding = 0.5 MiB
    opt = FlatAdamW(model, lr=1e-3)
    eng = DataParallelEngine(opt, bucket_mb=0.25, first_bucket_mb=0.01, broadcast_params=False)
    wte = next(i for i, p in enumerate(opt.params) if p.numel() == 2048 * 64)
    own = [b for b in eng.buckets if wte in b["params"]]
    assert len(own) == 1 and own[0]["params"] == [wte]
    # contiguous, non-overlapping, covering every parameter once
    spans = sorted((b["start"], b["end"]) for b in eng.buckets)
    for (s0, e0), (s1, e1) in zip(spans, spans[1:]):
        assert e0 <= s1
    assert sorted(i for b in eng.buckets for i in b["params"]) == list(range(len(opt.params)))
    assert max(eng.bucket_sizes_mb()) <= 0.5 + 1e-6

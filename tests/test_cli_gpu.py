"""Reference entry points on the GPU (subprocesses, so each runs exactly as a user would start it):
the training CLI with a preset (HIP kernels, periodic checkpoint), generate_text.py from that
checkpoint, and the self-launching multi-rank bench (2 ranks sharing the one GPU over gloo: the
functional rehearsal of the driver's N-GPU run)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=240):
    e = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    e.update(env or {})
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        e.pop(k, None)
    return subprocess.run([sys.executable, *args], capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=e)


def test_train_cli_and_generate_gpu(tmp_path):
    ck = tmp_path / "tiny.pt"
    r = _run(["scripts/train_transformer.py", "--preset=gpt2-small", "--override_preset_dims=True", "--n_blocks=2",
              "--n_embed=256", "--n_head=4", "--context_length=256", "--t_batch_size=4", "--t_train_steps=6",
              "--t_eval_steps=3", "--t_eval_iters=1", "--log_interval=3", "--synthetic_data=True",
              f"--synthetic_dir={tmp_path}", "--synthetic_tokens=200000", f"--t_out_path={ck}"])
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert "device=cuda:0" in r.stdout and "Step 3" in r.stdout and ck.exists(), r.stdout[-2000:]
    g = _run(["scripts/generate_text.py", "--model_path", str(ck), "--input_text", "Hello", "--max_new_tokens", "8",
              "--seed", "1"])
    assert g.returncode == 0, g.stderr[-3000:]
    assert "Generated text:" in g.stdout


def test_bench_two_ranks_one_gpu_gloo():
    r = _run(["bench.py", "--gpus", "2", "--model", "gpt2-tiny", "--steps", "2", "--warmup", "1", "--batch", "4",
              "--seq", "128"], env={"PLLM_DIST_BACKEND": "gloo", "PLLM_DIST_ONE_DEVICE": "1"}, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")][-1]
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2" and rec["comm"]["hook_launched_buckets"]
    assert rec["device"] == "cuda" and rec["value"] > 0
    c = rec["comm"]  # HIP-event diagnostics of the multi-rank path
    assert c["exposed_comm_ms"] is not None and c["exposed_comm_ms"] >= 0.0 and c["exposed_comm_ms_max_rank"] >= 0.0
    assert len(c["bucket_launch_ms"]) == c["n_buckets"] and c["backward_end_ms"] > 0
    assert c["rank_step_ms_min"] <= c["rank_step_ms_max"]

"""TORCH_COMPILE on the GPU: the fake impls agree with the real HIP kernels
(torch.library.opcheck), torch.compile traces the model through them, and the Trainer's
TORCH_COMPILE path (hipGraph whole-step replay) trains exactly like eager."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _ext():
    from pretraining_llm_amd.ops import _lib
    _lib.require()


def _op_cases():
    bf, f32 = torch.bfloat16, torch.float32
    r = lambda *s, dt=bf: torch.randn(*s, device=DEV).to(dt)  # noqa: E731
    N, C, V = 256, 512, 1024
    x, w, b = r(N, C), r(C), r(C)
    y, s, mean, rstd = torch.ops.pllm.norm_fwd(x, None, w, b, 1e-5, False)
    B, T, H, D = 2, 128, 4, 64
    q, k, v = r(B, T, H, D), r(B, T, H, D), r(B, T, H, D)
    o, lse = torch.ops.pllm.attn_fwd(q, k, v, True, 0.125)
    idx = torch.randint(0, V, (B, T), device=DEV)
    cos, sin = (t.contiguous() for t in (torch.rand(T, D // 2, device=DEV),) * 2)
    return [
        ("norm_fwd", (x, r(N, C), w, b, 1e-5, False)),
        ("norm_fwd", (x, None, w, None, 1e-5, True)),
        ("norm_bwd", (r(N, C), x, w, mean, rstd, None, True, False)),
        ("norm_bwd_acc", (r(N, C), x, w, mean, rstd, r(N, C), True, False, torch.zeros(C, device=DEV),
                          torch.zeros(C, device=DEV), torch.zeros(C, device=DEV))),
        ("bias_grad", (r(N, C),)),
        ("bias_grad", (r(N, C), torch.zeros(C, device=DEV))),
        ("wgrad", (r(N, 256), r(N, C))),
        ("wgrad", (r(N, 256), r(N, C), torch.zeros(256, C, device=DEV))),
        ("act_fwd", (r(N, C), 1)),
        ("act_bwd", (r(N, C), r(N, C), 0)),
        ("act_bwd_bias", (r(N, C), r(N, C), 1, torch.zeros(C, device=DEV))),
        ("swiglu_fwd", (r(N, 2 * C),)),
        ("swiglu_bwd", (r(N, C), r(N, 2 * C))),
        ("rope", (r(B, T, 3 * H * D), cos, sin, 3 * H, 2 * H, T, 0, False)),
        ("cross_entropy", (r(N, V), torch.randint(0, V, (N,), device=DEV), None, -100)),
        ("cross_entropy", (r(N, V), torch.randint(0, V, (N,), device=DEV), r(N, V), -100,
                           torch.full((1,), 1.0 / N, device=DEV))),
        ("sumsq", (r(4096, dt=f32),)),
        ("grad_norm_clip", (r(4096, dt=f32), 0.5, 1.0)),
        ("embedding_fwd", (idx, r(V, C), r(T, C), 0)),
        ("embedding_bwd", (r(B, T, C), idx, V, T, True)),
        ("embedding_bwd_acc", (r(B, T, C), idx, V, T, True, torch.zeros(V, C, device=DEV),
                               torch.zeros(T, C, device=DEV))),
        ("attn_fwd", (q, k, v, True, 0.125)),
        ("attn_bwd", (r(B, T, H, D), q, k, v, o, lse, torch.empty_like(q), torch.empty_like(k), torch.empty_like(v),
                      True, 0.125)),
        ("attn_decode", (r(B, 1, H, D), k, v, 0.125)),
        ("gemv", (r(4, C), r(768, C), r(768))),
        ("sample", (r(4, V, dt=f32), 0.0, 0)),
        ("gemm_tn", (r(N, C), r(768, C), r(768), 1)),
        ("gemm_tn", (r(N, C), r(768, C), None, 3, r(N, 768), torch.zeros(768, device=DEV))),
    ]


@pytest.mark.parametrize("i", range(28))
def test_opcheck_fake_matches_kernel(i):
    torch.manual_seed(i)
    cases = _op_cases()
    name, args = cases[i]
    torch.library.opcheck(getattr(torch.ops.pllm, name).default, args,
                          test_utils=("test_schema", "test_faketensor"))


@pytest.mark.parametrize("backend", ["eager", "aot_eager"])
def test_torch_compile_model_matches_eager(backend):
    from pretraining_llm_amd.models import GPT, get_preset
    torch._dynamo.reset()
    torch.manual_seed(0)
    cfg = get_preset("gpt2-tiny").replace(context_length=128, vocab_size=1024)
    m = GPT(cfg).to(DEV, torch.bfloat16)
    x = torch.randint(0, 1024, (2, 128), device=DEV)
    _, l0 = m(x, x.roll(-1, 1), return_logits=False)
    l0.backward()
    g0 = {n: p.grad.float().clone() for n, p in m.named_parameters()}
    m.zero_grad(set_to_none=True)
    cm = torch.compile(m, backend=backend)
    _, l1 = cm(x, x.roll(-1, 1), return_logits=False)
    l1.backward()
    assert abs(l0.item() - l1.item()) < 1e-3
    for n, p in m.named_parameters():
        assert (p.grad.float() - g0[n]).norm() <= 1e-2 * g0[n].norm() + 1e-6, n


def test_trainer_torch_compile_selects_graph_step(tmp_path):
    from pretraining_llm_amd.train.trainer import Trainer
    from config.config import default_config
    base = dict(default_config)
    base.update(model_preset="gpt2-tiny", t_batch_size=4, seq_len=128, t_train_steps=10, t_lr=1e-3, warmup_steps=2,
                log_interval=1, t_eval_steps=1000, eval_at_start=False, t_out_path=None, synthetic_data=True,
                synthetic_tokens=200_000, synthetic_dir=str(tmp_path), max_grad_norm=1.0, device="cuda")
    curves = {}
    for comp in (False, True):
        recs = []
        tr = Trainer(dict(base, compile=comp), log=lambda *_: None)
        tr.metrics.log = recs.append
        tr.train()
        assert tr.use_graph == comp and (tr.gstep is not None) == comp
        curves[comp] = [r["train_loss"] for r in recs]
    assert len(curves[True]) == 10
    for a, b in zip(curves[True], curves[False]):
        assert abs(a - b) < 2e-3 * max(1.0, abs(b)), (curves[True], curves[False])


def test_trainer_graph_step_grad_accum_matches_eager(tmp_path, monkeypatch):
    """TORCH_COMPILE parity: the default (no TORCH_COMPILE in the env) on the GPU is the captured
    step, and with grad_accum_steps=2 (both micro-steps captured, the first under no_sync) 10
    graphed steps track eager loss and end at the same weights."""
    from pretraining_llm_amd.train.trainer import Trainer
    from config.config import default_config
    monkeypatch.delenv("TORCH_COMPILE", raising=False)
    base = dict(default_config)
    base.update(model_preset="gpt2-tiny", t_batch_size=4, seq_len=128, t_train_steps=10, t_lr=1e-3, warmup_steps=2,
                log_interval=1, t_eval_steps=1000, eval_at_start=False, t_out_path=None, synthetic_data=True,
                synthetic_tokens=200_000, synthetic_dir=str(tmp_path), max_grad_norm=1.0, device="cuda",
                grad_accum_steps=2)
    curves, weights = {}, {}
    for comp in (None, False):
        recs = []
        tr = Trainer(dict(base, compile=comp), log=lambda *_: None)
        tr.metrics.log = recs.append
        tr.train()
        assert tr.use_graph == (comp is None)
        curves[comp] = [r["train_loss"] for r in recs]
        weights[comp] = tr.opt.master.clone()
    assert len(curves[None]) == 10
    for a, b in zip(curves[None], curves[False]):
        assert abs(a - b) < 2e-3 * max(1.0, abs(b)), (curves[None], curves[False])
    # Adam steps are ~lr in size whatever the gradient's magnitude, so an element whose gradient
    # sits near zero may step either way: compare the weights as a whole
    rel = ((weights[None] - weights[False]).norm() / weights[False].norm()).item()
    assert rel < 1e-3, rel

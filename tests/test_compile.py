"""TORCH_COMPILE compatibility (reference scripts/train_transformer.py:31-33,118-120).

* Every torch.ops.pllm op has a fake (meta) implementation (ops/fake.py): a whole model forward
  on FAKE CUDA tensors traces through the HIP-op path here on a CPU-only machine (the dispatch
  chooses the HIP ops for cuda tensors), for all three architectures, training and eval.
* The Trainer's TORCH_COMPILE path on CPU (torch.compile of the model) trains like eager.
The GPU half (opcheck against the real kernels, AOTAutograd over the model, the hipGraph step
selected by TORCH_COMPILE in the Trainer) is tests/test_compile_gpu.py."""
import pytest
import torch


@pytest.mark.parametrize("preset", ["gpt2-tiny", "llama-tiny", "ref-small"])
def test_model_traces_on_fake_cuda_tensors(preset):
    from torch._subclasses.fake_tensor import FakeTensor, FakeTensorMode
    from pretraining_llm_amd.ops import _lib
    if not _lib.load():
        pytest.skip(f"extension not built: {_lib.error()}")
    from pretraining_llm_amd.models import GPT, get_preset
    cfg = get_preset(preset).replace(vocab_size=512, context_length=128)
    if preset == "ref-small":
        cfg = cfg.replace(n_embed=128, n_head=2, n_blocks=2, ffn_hidden=512)
    old = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    try:
        with FakeTensorMode(allow_non_fake_inputs=True), torch.device("cuda"):
            m = GPT(cfg)
            x = torch.randint(0, 512, (2, 128), device="cuda")
            _, loss = m(x, x, return_logits=False)       # fused LM head + CE (training path)
            with torch.no_grad():
                logits, l2 = m(x, x)
                out = m.generate(x[:, :4], 3, temperature=0.0)   # KV-cache decode kernels
    finally:
        torch.set_default_dtype(old)
    assert isinstance(loss, FakeTensor) and loss.shape == () and loss.dtype == torch.float32 and loss.is_cuda
    assert logits.shape == (2, 128, 512) and logits.dtype == torch.bfloat16
    assert out.shape == (2, 7) and out.dtype == torch.int64


def test_every_op_has_a_fake_impl():
    from pretraining_llm_amd.ops import _lib
    if not _lib.load():
        pytest.skip(f"extension not built: {_lib.error()}")
    import torch._library.simple_registry as reg
    ops = sorted({n.split("::")[1].split(".")[0] for n in torch._C._dispatch_get_all_op_names()
                  if n.startswith("pllm::")})

    def takes_tensors(n):  # configuration / query ops (ints in, ints or nothing out) need no fake kernel
        sch = getattr(torch.ops.pllm, n).default._schema
        return any("Tensor" in str(x.type) for x in list(sch.arguments) + list(sch.returns))

    tensor_ops = [n for n in ops if takes_tensors(n)]
    missing = [n for n in tensor_ops if not reg.singleton.find(f"pllm::{n}").fake_impl.kernel]
    assert len(tensor_ops) >= 20 and not missing, missing


def test_trainer_torch_compile_cpu_matches_eager(tmp_path):
    from pretraining_llm_amd.train.trainer import Trainer
    from config.config import PRESET_RUNS, default_config
    base = dict(default_config)
    base.update(PRESET_RUNS["gpt2-tiny-cpu"])
    base.update(t_train_steps=4, t_eval_steps=100, log_interval=1, eval_at_start=False, t_out_path=None,
                synthetic_dir=str(tmp_path), synthetic_tokens=60_000, t_batch_size=2, seq_len=64)
    losses = {}
    for comp in (False, True):
        recs = []
        tr = Trainer(dict(base, compile=comp, compile_backend="eager"), log=lambda *_: None)
        tr.metrics.log = recs.append
        tr.train()
        assert (tr.fwd is not tr.model) == comp
        losses[comp] = [r["train_loss"] for r in recs]
    assert losses[True] == pytest.approx(losses[False], rel=1e-5)

# scripts/generate_text.py -- text generation from a checkpoint.
#
# Reference: Flink-ddd/pretraining-llm scripts/generate_text.py:7-61
# (generate_text(model_path, input_text, max_new_tokens=100, device='cuda'),
# CLI --model_path --input_text --max_new_tokens, prints "Generated text:\n...").
# Same API and output.  Differences: the model architecture is rebuilt from the
# checkpoint's ``model_config`` when present (else from config.config, like the
# reference), wrapper prefixes are stripped before the strict load (D7), the
# device falls back to CPU when no GPU is present, generation uses the KV cache,
# and --temperature/--top_k/--device/--dtype are optional extras.  --dtype: the
# reference runs the fp32 model on the device (generate_text.py:21-42) -- ``float32``
# does that here too (torch ops, eager decode); the default ``auto`` is bf16 on the
# HIP kernels with the hipGraph decode step on a GPU and fp32 on the CPU.
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from config.config import default_config as config  # noqa: E402


def _dtype(device: str, dtype: str):
    if dtype in (None, "auto"):
        return torch.bfloat16 if device.startswith("cuda") else torch.float32
    return {"bfloat16": torch.bfloat16, "float32": torch.float32}[dtype]


def load_model(model_path: str, device: str, dtype: str = "auto"):
    from pretraining_llm_amd.models import GPT, ModelConfig
    from pretraining_llm_amd.models.config import _ref
    from pretraining_llm_amd.utils.checkpoint import load_checkpoint
    ckpt = load_checkpoint(model_path, map_location="cpu")
    if "model_config" in ckpt:
        cfg = ModelConfig.from_dict(ckpt["model_config"])
    else:
        cfg = _ref(n_head=config['n_head'], n_embed=config['n_embed'], context_length=config['context_length'],
                   vocab_size=config['vocab_size'], n_blocks=config['n_blocks'])
    model = GPT(cfg)
    model.load_state_dict(ckpt['model_state_dict'])
    return model.eval().to(device=device, dtype=_dtype(device, dtype))


def generate_tokens(model_path: str, start_ids, max_new_tokens: int = 100, device: str = 'cuda', dtype: str = "auto",
                    temperature: float = 1.0, top_k=None, seed=None, cuda_graph: bool = True):
    """Token-level generation (prompt ids -> prompt + new ids)."""
    if device.startswith("cuda") and not torch.cuda.is_available():
        device = "cpu"
    model = load_model(model_path, device, dtype)
    context = torch.tensor(list(start_ids), dtype=torch.long, device=device).unsqueeze(0)
    gen = None
    if seed is not None:
        gen = torch.Generator(device=device).manual_seed(int(seed))
    # the hipGraph decode step replays the bf16 HIP kernels; fp32 decodes eagerly like the reference
    graph = cuda_graph and device.startswith("cuda") and _dtype(device, dtype) == torch.bfloat16
    with torch.no_grad():
        return model.generate(context, max_new_tokens=max_new_tokens, temperature=temperature, top_k=top_k,
                              generator=gen, cuda_graph=graph)[0].tolist()


def generate_text(model_path: str, input_text: str, max_new_tokens: int = 100, device: str = 'cuda',
                  temperature: float = 1.0, top_k=None, seed=None, cuda_graph: bool = True, dtype: str = "auto") -> str:
    from pretraining_llm_amd.data.tokenizer import get_tokenizer
    from pretraining_llm_amd.utils.checkpoint import load_checkpoint
    enc = get_tokenizer(config.get('tokenizer_name', 'gpt2'))
    start_ids = enc.encode_ordinary(input_text)
    if not start_ids:
        vocab = load_checkpoint(model_path).get("model_config", {}).get("vocab_size", config['vocab_size'])
        start_ids = [enc.eot_token % vocab]
    tokens = generate_tokens(model_path, start_ids, max_new_tokens, device, dtype, temperature, top_k, seed, cuda_graph)
    return enc.decode(tokens)


def main() -> None:
    parser = argparse.ArgumentParser(description="Generate text using a pre-trained Transformer model.")
    parser.add_argument('--model_path', type=str, help='Path to the saved model checkpoint.')
    parser.add_argument('--input_text', type=str, help='The initial text to start generation from.')
    parser.add_argument('--max_new_tokens', type=int, default=100, help='Maximum number of new tokens to generate.')
    parser.add_argument('--device', type=str, default='cuda')
    parser.add_argument('--temperature', type=float, default=1.0)
    parser.add_argument('--top_k', type=int, default=None)
    parser.add_argument('--seed', type=int, default=None)
    parser.add_argument('--dtype', type=str, default='auto', choices=['auto', 'bfloat16', 'float32'],
                        help="auto: bf16 HIP kernels on a GPU, fp32 on the CPU; float32: the reference's precision")
    parser.add_argument('--no_cuda_graph', action='store_true', help='eager decode steps instead of one hipGraph replay')
    args = parser.parse_args()
    generated = generate_text(args.model_path, args.input_text, args.max_new_tokens, args.device,
                              args.temperature, args.top_k, args.seed, cuda_graph=not args.no_cuda_graph, dtype=args.dtype)
    print(f"Generated text:\n{generated}")


if __name__ == "__main__":
    main()

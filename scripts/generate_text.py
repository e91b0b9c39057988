# scripts/generate_text.py -- text generation from a checkpoint.
#
# Reference: Flink-ddd/pretraining-llm scripts/generate_text.py:7-61
# (generate_text(model_path, input_text, max_new_tokens=100, device='cuda'),
# CLI --model_path --input_text --max_new_tokens, prints "Generated text:\n...").
# Same API and output.  Differences: the model architecture is rebuilt from the
# checkpoint's ``model_config`` when present (else from config.config, like the
# reference), wrapper prefixes are stripped before the strict load (D7), the
# device falls back to CPU when no GPU is present, generation uses the KV cache,
# and --temperature/--top_k/--device are optional extras.
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from config.config import default_config as config  # noqa: E402


def load_model(model_path: str, device: str):
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
    dtype = torch.bfloat16 if device.startswith("cuda") else torch.float32
    return model.eval().to(device=device, dtype=dtype)


def generate_text(model_path: str, input_text: str, max_new_tokens: int = 100, device: str = 'cuda',
                  temperature: float = 1.0, top_k=None, seed=None, cuda_graph: bool = True) -> str:
    if device.startswith("cuda") and not torch.cuda.is_available():
        device = "cpu"
    from pretraining_llm_amd.data.tokenizer import get_tokenizer
    model = load_model(model_path, device)
    enc = get_tokenizer(config.get('tokenizer_name', 'gpt2'))
    start_ids = enc.encode_ordinary(input_text) or [enc.eot_token % model.config.vocab_size]
    context = torch.tensor(start_ids, dtype=torch.long, device=device).unsqueeze(0)
    gen = None
    if seed is not None:
        gen = torch.Generator(device=device).manual_seed(int(seed))
    with torch.no_grad():
        tokens = model.generate(context, max_new_tokens=max_new_tokens, temperature=temperature, top_k=top_k,
                                generator=gen, cuda_graph=cuda_graph and device.startswith("cuda"))[0].tolist()
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
    parser.add_argument('--no_cuda_graph', action='store_true', help='eager decode steps instead of one hipGraph replay')
    args = parser.parse_args()
    generated = generate_text(args.model_path, args.input_text, args.max_new_tokens, args.device,
                              args.temperature, args.top_k, args.seed, cuda_graph=not args.no_cuda_graph)
    print(f"Generated text:\n{generated}")


if __name__ == "__main__":
    main()

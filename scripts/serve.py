# scripts/serve.py -- HTTP generation service over a trained checkpoint (batched KV-cache decode).
#
#   python scripts/serve.py --model_path models/transformer_B.pt --port 8000
#   curl -s localhost:8000/generate -d '{"prompt": "Hello", "max_new_tokens": 32}' -H 'content-type: application/json'
#
# Loads the checkpoint like scripts/generate_text.py (reference-format keys, model_config when
# present) and serves pretraining_llm_amd.inference.server: concurrent requests with the same
# prompt length and sampling settings share one decode batch (hipGraph-replayed steps on the GPU).
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser(description="Serve text generation over HTTP.")
    ap.add_argument("--model_path", required=True)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--max_batch", type=int, default=64)
    ap.add_argument("--max_wait_ms", type=float, default=5.0, help="how long a request waits for batch company")
    ap.add_argument("--no_cuda_graph", action="store_true")
    ap.add_argument("--mode", default="continuous", choices=["continuous", "lockstep"],
                    help="continuous: decode slots at per-sequence positions (requests join/leave every token); "
                         "lockstep: batch only requests with the same prompt length and sampler")
    ap.add_argument("--max_len", type=int, default=None, help="continuous mode: KV-cache length per slot "
                    "(default: the model's context length)")
    args = ap.parse_args()
    import uvicorn

    from config.config import default_config
    from pretraining_llm_amd.data.tokenizer import get_tokenizer
    from pretraining_llm_amd.inference.server import ContinuousGenerationServer, GenerationServer, create_app
    from scripts.generate_text import load_model
    device = args.device if (not args.device.startswith("cuda") or torch.cuda.is_available()) else "cpu"
    model = load_model(args.model_path, device)
    if args.mode == "continuous":
        server = ContinuousGenerationServer(model, max_batch=args.max_batch, max_len=args.max_len,
                                            cuda_graph=not args.no_cuda_graph)
    else:
        server = GenerationServer(model, max_batch=args.max_batch, max_wait_ms=args.max_wait_ms,
                                  cuda_graph=not args.no_cuda_graph)
    app = create_app(server, get_tokenizer(default_config.get("tokenizer_name", "gpt2")))
    try:
        uvicorn.run(app, host=args.host, port=args.port, log_level="info")
    finally:
        server.close()


if __name__ == "__main__":
    main()

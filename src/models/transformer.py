"""Reference module path ``src.models.transformer`` (Transformer)."""
from pretraining_llm_amd.models.compat import Transformer  # noqa: F401


if __name__ == "__main__":
    # demo, as the reference module's (src/models/transformer.py:116-136): loss with targets=input,
    # then generation from a short prompt
    import torch
    model = Transformer(4, 32, 5, 100, 2)
    idx = torch.randint(0, 100, (2, 5))
    logits, loss = model(idx, idx)
    print("Transformer logits", tuple(logits.shape), "loss", float(loss))
    print("generate", model.generate(idx[:, :2], 5).tolist())

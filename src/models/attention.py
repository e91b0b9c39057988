"""Reference module path ``src.models.attention`` (Head, MultiHeadAttention)."""
from pretraining_llm_amd.models.compat import Head, MultiHeadAttention  # noqa: F401


if __name__ == "__main__":
    # shape demo, as the reference module's (src/models/attention.py:98-111)
    import torch
    mha = MultiHeadAttention(n_head=4, n_embed=32, context_length=5)
    x = torch.randn(2, 5, 32)
    print("MultiHeadAttention", tuple(x.shape), "->", tuple(mha(x).shape))

"""Reference module path ``src.models.mlp`` (MLP)."""
from pretraining_llm_amd.models.compat import MLP  # noqa: F401


if __name__ == "__main__":
    # shape demo, as the reference module's (src/models/mlp.py:69-80)
    import torch
    mlp = MLP(16)
    x = torch.randn(2, 3, 16)
    print("MLP", tuple(x.shape), "->", tuple(mlp(x).shape))

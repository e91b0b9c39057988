"""Reference module path ``src.models.transformer_block`` (Block)."""
from pretraining_llm_amd.models.compat import Block  # noqa: F401


if __name__ == "__main__":
    # shape demo, as the reference module's (src/models/transformer_block.py:63-76)
    import torch
    blk = Block(4, 32, 5)
    x = torch.randn(2, 5, 32)
    print("Block", tuple(x.shape), "->", tuple(blk(x).shape))

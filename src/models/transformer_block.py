"""Reference module path ``src.models.transformer_block`` (Block)."""
from pretraining_llm_amd.models.compat import Block  # noqa: F401

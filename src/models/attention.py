"""Reference module path ``src.models.attention`` (Head, MultiHeadAttention)."""
from pretraining_llm_amd.models.compat import Head, MultiHeadAttention  # noqa: F401

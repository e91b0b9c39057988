"""Reference-compatible model package: ``from src.models import MLP, Head, MultiHeadAttention, Block, Transformer``
(reference src/models/__init__.py:2-5), backed by the MI355X-native implementation."""
from pretraining_llm_amd.models.compat import MLP, Head, MultiHeadAttention, Block, Transformer  # noqa: F401

__all__ = ["MLP", "Head", "MultiHeadAttention", "Block", "Transformer"]

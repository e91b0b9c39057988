"""Reference module path ``src.models.transformer`` (Transformer)."""
from pretraining_llm_amd.models.compat import Transformer  # noqa: F401

"""Reference module path ``src.models.mlp`` (MLP)."""
from pretraining_llm_amd.models.compat import MLP  # noqa: F401

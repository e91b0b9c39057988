from .generate import KVCache, generate, sample_next  # noqa: F401

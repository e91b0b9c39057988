from .loader import TokenLoader, get_batch_iterator  # noqa: F401
from .shards import ensure_synthetic_shard, synthetic_tokens, write_tokens, EOT_TOKEN  # noqa: F401

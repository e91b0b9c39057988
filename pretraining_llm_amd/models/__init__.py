from .config import ModelConfig, PRESETS, get_preset  # noqa: F401
from .gpt import GPT, Block as GPTBlock, Attention, MLP as GPTMLP, Norm  # noqa: F401
from .compat import Transformer, Head, MultiHeadAttention, MLP, Block, strip_wrapper_prefixes  # noqa: F401

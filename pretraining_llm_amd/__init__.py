"""MI355X-native (gfx950 / CDNA4) transformer pretraining framework.

Capabilities of Flink-ddd/pretraining-llm, re-designed for AMD Instinct MI355X:
hand-written HIP kernels (``csrc/``) for attention, norms, activations,
cross-entropy, embedding and AdamW; RCCL data parallelism over xGMI
(``parallel/``); a native token loader (``csrc/host``); trainer, checkpointing
and generation in ``train/``, ``utils/``, ``inference/``.
"""
__version__ = "0.1.0"

from .models import GPT, ModelConfig, get_preset  # noqa: F401,E402

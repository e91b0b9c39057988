from .optim import FlatAdamW, no_decay_1d  # noqa: F401
from .trainer import Trainer, lr_at, model_config_from  # noqa: F401

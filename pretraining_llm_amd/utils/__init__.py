from .checkpoint import load_checkpoint, save_checkpoint, unwrap  # noqa: F401
from .dist import DistInfo, init_distributed  # noqa: F401
from .metrics import MetricsLogger, StepTimer, mfu  # noqa: F401

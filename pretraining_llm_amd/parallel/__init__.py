from .dp import DataParallelEngine, all_reduce_mean, params_checksum  # noqa: F401

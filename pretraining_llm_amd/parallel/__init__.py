from .dp import DataParallelEngine, all_reduce_mean, params_checksum  # noqa: F401
from .tensor import (ColumnParallelLinear, RowParallelLinear, TensorParallelAttention,  # noqa: F401
                     TensorParallelMLP, copy_to_tensor_parallel, gather_from_sequence,
                     gather_from_tensor_parallel, head_to_seq_all_to_all, reduce_from_tensor_parallel,
                     reduce_scatter_to_sequence, scatter_to_sequence, seq_to_head_all_to_all,
                     ulysses_attention)
from .context import ring_attention, zigzag_positions, zigzag_shard, zigzag_unshard  # noqa: F401
# ZeRO-1 (parallel/zero.py: ShardedFlatAdamW, ZeroDataParallelEngine) is imported from its module
# directly: it builds on train.optim, which the trainer (train/) imports from here.

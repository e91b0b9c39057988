# config/config.py -- training configuration (reference-compatible).
#
# Every key of the reference's default_config (Flink-ddd/pretraining-llm
# config/config.py:29-47) is kept with its value, and the keys the reference
# scripts read but never defined (ddp_backend, dtype,
# val_path, dataset_name, tokenizer_name) get working defaults.  Framework
# knobs (presets, parallelism, logging, checkpointing) follow.

# --- Configuration ---

# Vocabulary size and transformer configuration (reference "3 Billion" model)
VOCAB_SIZE = 50304
CONTEXT_LENGTH = 512
N_EMBED = 2048
N_HEAD = 16
N_BLOCKS = 64

# Paths to training and development datasets (flat uint16 token files)
TRAIN_PATH = "data/train/pile_train.h5"
DEV_PATH = "data/val/pile_dev.h5"

# Transformer training parameters
T_BATCH_SIZE = 32
T_CONTEXT_LENGTH = 16
T_TRAIN_STEPS = 200000
T_EVAL_STEPS = 1000
T_EVAL_ITERS = 250
T_LR_DECAY_STEP = 50000
T_LR = 5e-4
T_LR_DECAYED = 5e-5
T_OUT_PATH = "models/transformer_B.pt"

DEVICE = 'cuda'

default_config = {
    'vocab_size': VOCAB_SIZE,
    'context_length': CONTEXT_LENGTH,
    'n_embed': N_EMBED,
    'n_head': N_HEAD,
    'n_blocks': N_BLOCKS,
    'train_path': TRAIN_PATH,
    'dev_path': DEV_PATH,
    't_batch_size': T_BATCH_SIZE,
    't_context_length': T_CONTEXT_LENGTH,
    't_train_steps': T_TRAIN_STEPS,
    't_eval_steps': T_EVAL_STEPS,
    't_eval_iters': T_EVAL_ITERS,
    't_lr_decay_step': T_LR_DECAY_STEP,
    't_lr': T_LR,
    't_lr_decayed': T_LR_DECAYED,
    't_out_path': T_OUT_PATH,
    'device': DEVICE,

    # --- keys the reference scripts read but never defined ---------------
    'ddp_backend': 'nccl',            # = RCCL on ROCm (train_transformer.py:17)
    'dtype': 'bfloat16',              # bfloat16 (HIP kernels) | float16 (reference: bf16 compute + loss scaling) | float16_autocast (true fp16, torch ops) | float32 (train/amp.py)
    'loss_scaling': None,             # dynamic loss scaling (GradScaler semantics); None = on iff dtype is float16 / float16_autocast
    'loss_scale_init': 65536.0,
    'loss_scale_growth_interval': 2000,
    'val_path': DEV_PATH,             # alias of dev_path (train_transformer.py:134)
    'dataset_name': 'openwebtext',    # scripts/data_preprocess.py:12, data_download.py:12
    'tokenizer_name': 'gpt2',         # scripts/data_preprocess.py:15

    # --- framework knobs ---------------------------------------------------
    'model_preset': None,             # None -> reference architecture with the dims above;
                                      # else one of pretraining_llm_amd.models.config.PRESETS
    'seq_len': None,                  # training sequence length (None -> model context_length)
    'grad_accum_steps': 1,
    'weight_decay': 0.01,             # torch.optim.AdamW default, applied to all params like the reference
    'weight_decay_all': True,
    'betas': (0.9, 0.999),
    'eps': 1e-8,
    'max_grad_norm': 0.0,             # 0 = no clipping (reference has none)
    'warmup_frac': 0.1,               # reference: 10% linear warmup then constant
    'lr_schedule': 'ref',             # ref | step | cosine
    'seed': 1337,
    'log_interval': None,             # None -> t_eval_steps (reference cadence)
    'eval_at_start': True,
    'ckpt_interval': 0,               # 0 -> save only at the end (reference)
    'resume': None,                   # checkpoint path or 'auto'
    'metrics_path': None,             # JSONL metrics file
    'synthetic_data': False,          # force synthetic token shards
    'allow_synthetic': True,          # fall back to synthetic shards when the data files are missing
    'synthetic_tokens': 2_000_000,
    'synthetic_kind': 'auto',         # markov (order-2 source, learnable) | fast (vectorised) | auto (by size)
    'synthetic_dir': 'data/synthetic',
    'bucket_mb': 64.0,                # DP all-reduce bucket size (xGMI-sized, see parallel/dp.py)
    'first_bucket_mb': 4.0,
    'rccl_channels': None,            # pin RCCL's channel count (NCCL_MIN/MAX_NCHANNELS) before the communicator; None = RCCL's choice
    'rccl_env': None,                 # extra RCCL / torch-NCCL env, dict or 'KEY=VAL,...' (utils/dist.apply_rccl_env)
    'gemm_reserve_cus': 0,            # CUs the persistent fused-epilogue GEMM grid leaves to RCCL kernels (world > 1)
    'gemm_persistent': 'auto',        # persistent ping-pong GEMM grids: auto = world 1 only (train/graph.py)
    'graph_collectives': False,       # refused (eager step): capturing RCCL collectives aborts (train/graph.py)
    'activation_checkpointing': None,
    'override_preset_dims': False,    # with model_preset: the dims above (n_embed, n_head, n_blocks, ...) override the preset's
    'tuned_gemms': True,              # GPU: load the shipped TunableOp GEMM selections (pretraining_llm_amd/tuning/)
    'tp_size': 1,                     # tensor parallelism: heads / FFN columns sharded (parallel/model_parallel.py)
    'sequence_parallel': False,       # with tp_size > 1: norm/residual regions sharded along the sequence
    'cp_size': 1,                     # context parallelism: sequence shards over cp_size ranks
    'cp_mode': 'ring',                # ring (zigzag shards, K/V ring) | ulysses (all-to-all head re-sharding)
    'zero_stage': 0,                  # 1 = shard fp32 master + AdamW moments over DP ranks (parallel/zero.py)
    'profile_dir': None,              # torch.profiler (ROCm activity) chrome traces + kernel table per rank
    'profile_steps': '3:6',           # [start:end) optimizer steps to profile
    'deterministic': False,           # torch.use_deterministic_algorithms + fixed-order kernels only
    'compile': None,                  # None -> env TORCH_COMPILE=="1" (reference toggle): hipGraph step on GPU,
                                      # torch.compile(model) on CPU
    'compile_backend': 'inductor',    # torch.compile backend for the CPU path
    'debug_sync': False,              # AMD_SERIALIZE_KERNEL=3 + HIP_LAUNCH_BLOCKING=1 (set before HIP init)
}

# Named BASELINE.json configurations (override default_config)
PRESET_RUNS = {
    'gpt2-tiny-cpu': dict(model_preset='gpt2-tiny', device='cpu', t_batch_size=8, t_train_steps=50,
                          t_eval_steps=25, t_eval_iters=4, t_lr=1e-3, warmup_frac=0.1, synthetic_data=True,
                          synthetic_tokens=400_000),
    'gpt2-small': dict(model_preset='gpt2-small', t_batch_size=32, t_lr=6e-4, weight_decay=0.1,
                       weight_decay_all=False, betas=(0.9, 0.95), max_grad_norm=1.0, lr_schedule='cosine',
                       t_lr_decayed=6e-5, warmup_frac=0.02),
    'llama-1.3b': dict(model_preset='llama-1.3b', t_batch_size=8, t_lr=3e-4, weight_decay=0.1, weight_decay_all=False,
                       betas=(0.9, 0.95), max_grad_norm=1.0, lr_schedule='cosine', t_lr_decayed=3e-5,
                       warmup_frac=0.02),
    'gpt2-medium-4k': dict(model_preset='gpt2-medium', t_batch_size=8, t_lr=3e-4, weight_decay=0.1,
                           weight_decay_all=False, betas=(0.9, 0.95), max_grad_norm=1.0,
                           activation_checkpointing='auto'),
}

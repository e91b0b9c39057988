# scripts/train_transformer.py -- pretraining entry point.
#
# Reference: Flink-ddd/pretraining-llm scripts/train_transformer.py (env-driven
# DDP bootstrap :14-29, Trainer :35-109, main :112-143).  Same launch contract:
#   python scripts/train_transformer.py                       (single process)
#   torchrun --nproc_per_node=8 scripts/train_transformer.py  (one rank per GPU, RCCL)
# plus ``--preset=<name>`` (config.config.PRESET_RUNS; ``--run=<name>`` is the same flag, but under
# torchrun only ``--preset`` works: torchrun's own parser takes ``--run`` for an abbreviation of
# its ``--run-path``) and ``--key=value`` overrides
# of any default_config key.  ``TORCH_COMPILE=1`` (the reference's toggle) replays the whole
# training step as one captured hipGraph on the GPU (the hot ops are already hand-written gfx950
# kernels; what is left to cut is per-launch host cost) and runs torch.compile on the CPU path.
import argparse
import ast
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from config.config import PRESET_RUNS, default_config  # noqa: E402


def _parse_value(v: str):
    try:
        return ast.literal_eval(v)
    except (ValueError, SyntaxError):
        return v


def build_config(argv=None) -> dict:
    ap = argparse.ArgumentParser(description=__doc__, allow_abbrev=False)
    ap.add_argument("--preset", "--run", dest="run", default=None,
                    help=f"named run preset: {sorted(PRESET_RUNS)} (use --preset under torchrun)")
    args, rest = ap.parse_known_args(argv)
    cfg = dict(default_config)
    if args.run:
        cfg.update(PRESET_RUNS[args.run])
    for item in rest:
        if not item.startswith("--") or "=" not in item:
            raise SystemExit(f"unrecognised argument {item!r} (use --key=value)")
        k, v = item[2:].split("=", 1)
        k = k.replace("-", "_")
        if k not in cfg:
            raise SystemExit(f"unknown config key {k!r}")
        cfg[k] = _parse_value(v)
    if cfg.get("log_interval") is None:
        cfg["log_interval"] = cfg["t_eval_steps"]
    return cfg


def main(argv=None):
    cfg = build_config(argv)
    if cfg.get("debug_sync"):
        # serialize every kernel launch so a fault is attributed to the launch that caused it;
        # must be in the environment before the HIP runtime initialises (torch import below)
        os.environ.setdefault("AMD_SERIALIZE_KERNEL", "3")
        os.environ.setdefault("HIP_LAUNCH_BLOCKING", "1")
    from pretraining_llm_amd.train import Trainer
    from pretraining_llm_amd.utils.dist import destroy
    trainer = Trainer(cfg)
    if trainer.di.is_master:
        n = sum(p.numel() for p in trainer.opt.params)
        print(f"model: {trainer.mcfg.arch} L={trainer.mcfg.n_blocks} C={trainer.mcfg.n_embed} H={trainer.mcfg.n_head} "
              f"T={trainer.seq_len} params={n / 1e6:.1f}M | world={trainer.di.world_size} device={trainer.device} "
              f"dtype={trainer.dtype}")
    trainer.train()
    destroy()


if __name__ == "__main__":
    main()

"""Tuned hipBLASLt/rocBLAS GEMM selection (PyTorch TunableOp) for the library GEMMs.

The plain projection / MLP / LM-head GEMMs run on the vendor libraries.  Their
default heuristics pick poorly for several training shapes on gfx950 (measured
on MI355X, gpt2-small B=32: the K=32768 weight-gradient GEMMs ran at 300-700
TFLOP/s with the default kernel vs up to 2x that with the best candidate), so
the framework ships per-shape selections found by TunableOp on MI355X
(``pretraining_llm_amd/tuning/*.csv``) and loads them at start-up.  Shapes not
in the table are tuned on first use when ``tune_missing`` is set (during the
untimed warmup of bench.py) and otherwise use the library default.
"""
from __future__ import annotations

import glob
import os
import shutil
import tempfile

import torch

from ..ab import ab as _ab

# PLLM_TUNING_DIR: an alternative table directory (A/B of tables)
TUNING_DIR = os.environ.get("PLLM_TUNING_DIR") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning")


_DEFAULT_DIR = None


def _merge_tables(dst: str):
    """Concatenate all shipped tables into one TunableOp CSV (validators once, results deduplicated)."""
    validators, results, seen = [], [], set()
    for p in sorted(glob.glob(os.path.join(TUNING_DIR, "*.csv"))):
        for line in open(p):
            line = line.strip()
            if not line:
                continue
            if line.startswith("Validator"):
                if line not in validators:
                    validators.append(line)
                continue
            key = tuple(line.split(",")[:2])
            if key not in seen:
                seen.add(key)
                results.append(line)
    if not results:
        return False
    with open(dst, "w") as f:
        f.write("\n".join(validators + results) + "\n")
    return True


def enable_tuned_gemms(device_index: int = 0, tune_missing: bool = False, out_dir: str = None,
                       load_tables: bool = True) -> bool:
    """Enable TunableOp with the shipped tables (``load_tables=False``: start empty, i.e. re-tune
    every shape). Returns True if a table was loaded."""
    if not torch.cuda.is_available() or os.environ.get("PLLM_TUNABLEOP", "1") == "0":
        return False
    try:
        import torch.cuda.tunable as tunable
    except Exception:
        return False
    global _DEFAULT_DIR
    if out_dir is None:  # one scratch dir per process (every Trainer / bench of the process reuses it)
        if _DEFAULT_DIR is None:  # (kept at exit: TunableOp may flush tuned results into it then)
            _DEFAULT_DIR = tempfile.mkdtemp(prefix="pllm_tunableop_")
        out_dir = _DEFAULT_DIR
    base = os.path.join(out_dir, "tunableop.csv")
    # TunableOp reads/writes "<stem><device>.csv" per device ordinal
    per_dev = os.path.join(out_dir, f"tunableop{device_index}.csv")
    loaded = _merge_tables(per_dev) if load_tables else False
    tunable.enable(True)
    tunable.tuning_enable(bool(tune_missing))
    if tune_missing:
        # bound the per-shape search (hundreds of hipBLASLt/rocBLAS candidates per shape)
        tunable.set_max_tuning_duration(_ab("tune_ms", 4))
        tunable.set_max_tuning_iterations(_ab("tune_iters", 8))
    tunable.set_filename(base, insert_device_ordinal=True)
    if loaded:
        tunable.read_file(per_dev)
    return loaded


def save_tuned(dst_name: str, device_index: int = 0):
    """Write the current TunableOp results into the shipped tuning dir (used when re-tuning on a box)."""
    import torch.cuda.tunable as tunable
    os.makedirs(TUNING_DIR, exist_ok=True)
    lines = [f"Validator,{k},{v}" for k, v in tunable.get_validators()]
    for res in tunable.get_results():
        lines.append(",".join(str(x) for x in res))
    dst = os.path.join(TUNING_DIR, dst_name)
    with open(dst, "w") as f:
        f.write("\n".join(lines) + "\n")
    return dst

# scripts/data_preprocess.py -- tokenize a corpus into flat uint16 token shards.
#
# Reference: Flink-ddd/pretraining-llm scripts/data_preprocess.py:11-64
# (HF load_dataset(dataset_name) -> train_test_split(test_size=0.0005, seed=42),
# 'test' renamed 'val' -> GPT-2 BPE encode_ordinary + EOT per document, parallel
# map -> each split concatenated into a flat np.uint16 memmap at train_path /
# val_path).  Same output format and split parameters.  Additions: ``--text``
# local text/jsonl inputs (there is no network here), ``--synthetic N`` to write
# seeded synthetic shards instead, and ``--train_path/--val_path`` overrides.
import argparse
import json
import os
import sys
from multiprocessing import Pool, cpu_count

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from config.config import default_config as config  # noqa: E402

_ENC = None


def _init(tok_name):
    global _ENC
    from pretraining_llm_amd.data.tokenizer import get_tokenizer
    _ENC = get_tokenizer(tok_name)


def _encode(text):
    ids = _ENC.encode_ordinary(text)
    ids.append(_ENC.eot_token)
    return ids


def _read_docs(paths):
    docs = []
    for p in paths:
        if p.endswith(".jsonl"):
            with open(p) as f:
                for line in f:
                    line = line.strip()
                    if line:
                        docs.append(json.loads(line).get("text", ""))
        else:
            with open(p, encoding="utf-8", errors="replace") as f:
                docs.extend(d for d in f.read().split("\n\n") if d.strip())
    return docs


def _load_hf_docs(name):
    from datasets import load_dataset
    ds = load_dataset(name)
    split = ds["train"].train_test_split(test_size=0.0005, seed=42, shuffle=True)
    return list(split["train"]["text"]), list(split["test"]["text"])


def _split(docs, seed=42, test_size=0.0005):
    rng = np.random.default_rng(seed)
    perm = rng.permutation(len(docs))
    n_val = max(1, int(round(len(docs) * test_size))) if len(docs) > 1 else 0
    val = [docs[i] for i in perm[:n_val]]
    train = [docs[i] for i in perm[n_val:]]
    return train, val


def write_split(docs, filename, tok_name, num_proc):
    from pretraining_llm_amd.data.shards import write_tokens
    if num_proc > 1 and len(docs) > 64:
        with Pool(num_proc, initializer=_init, initargs=(tok_name,)) as pool:
            ids = pool.map(_encode, docs, chunksize=64)
    else:
        _init(tok_name)
        ids = [_encode(d) for d in docs]
    arr = np.concatenate([np.asarray(x, dtype=np.int64) for x in ids]) if ids else np.zeros(0, np.int64)
    write_tokens(filename, arr)
    print(f"wrote {arr.size:,} tokens to {filename}")
    return arr.size


def main(argv=None):
    ap = argparse.ArgumentParser(description="Tokenize a corpus into uint16 token shards.")
    ap.add_argument("--text", nargs="*", default=None, help="local .txt (documents split on blank lines) or .jsonl")
    ap.add_argument("--dataset_name", default=config.get("dataset_name"))
    ap.add_argument("--tokenizer_name", default=config.get("tokenizer_name", "gpt2"))
    ap.add_argument("--train_path", default=config.get("train_path"))
    ap.add_argument("--val_path", default=config.get("val_path") or config.get("dev_path"))
    ap.add_argument("--synthetic", type=int, default=0, help="write N synthetic tokens per split instead")
    ap.add_argument("--num_proc", type=int, default=min(8, cpu_count()))
    args = ap.parse_args(argv)
    if args.synthetic:
        from pretraining_llm_amd.data.shards import ensure_synthetic_shard
        ensure_synthetic_shard(args.train_path, args.synthetic, config["vocab_size"], seed=1337, stream=0)
        ensure_synthetic_shard(args.val_path, max(1000, args.synthetic // 100), config["vocab_size"], seed=1337,
                               stream=1)
        print(f"wrote synthetic shards {args.train_path}, {args.val_path}")
        return
    if args.text:
        train, val = _split(_read_docs(args.text))
    else:
        train, val = _load_hf_docs(args.dataset_name)
    write_split(train, args.train_path, args.tokenizer_name, args.num_proc)
    write_split(val, args.val_path, args.tokenizer_name, args.num_proc)


if __name__ == "__main__":
    main()

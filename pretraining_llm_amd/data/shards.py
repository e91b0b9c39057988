"""Token shard files: the reference's on-disk format (a flat ``np.uint16`` token
stream, scripts/data_preprocess.py:47-62) plus a synthetic-shard writer so that
no corpus or network is needed.

The synthetic stream is not uniform noise: it is a seeded order-2 Markov
source with sparse transitions (each (prev2, prev1) context has a handful of
likely successors), so a model trained on it shows a real, monotone loss
decrease from ~ln(V) while every statistic stays reproducible from the seed.
"""
from __future__ import annotations

import os

import numpy as np

EOT_TOKEN = 50256  # GPT-2 BPE <|endoftext|> (scripts/data_preprocess.py:31-35)


def write_tokens(path: str, tokens: np.ndarray) -> str:
    """Write a flat uint16 token file (memmap-compatible with the reference loader)."""
    tokens = np.asarray(tokens)
    if tokens.size and (tokens.min() < 0 or tokens.max() > 65535):
        raise ValueError("token ids must fit uint16")
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    arr = np.memmap(path, dtype=np.uint16, mode="w+", shape=(int(tokens.size),))
    arr[:] = tokens.astype(np.uint16)
    arr.flush()
    del arr
    return path


def synthetic_tokens(n_tokens: int, vocab_size: int, seed: int = 0, branching: int = 4,
                     doc_len: int = 2048, stream: int = 0) -> np.ndarray:
    """Seeded order-2 Markov token stream with EOT separators every ~doc_len tokens.
    ``seed`` fixes the source (transition table); ``stream`` selects an independent
    sample path of that same source (train / validation splits)."""
    rng = np.random.default_rng(seed)
    V = int(vocab_size)
    vocab_eff = min(V, 65535)
    # successor table: hash(prev2, prev1) -> `branching` candidate tokens (Zipf-ish weights)
    table_size = 1 << 16
    # successors and noise follow a Zipf law over a random permutation of the vocabulary, so
    # the unigram statistics are skewed like text (fast initial loss drop) and the bigram /
    # trigram structure is there to learn afterwards
    perm = rng.permutation(vocab_eff)
    succ = perm[(rng.zipf(1.3, size=(table_size, branching)) - 1) % vocab_eff]
    w = 1.0 / np.arange(1, branching + 1)
    w = w / w.sum()
    rng = np.random.default_rng([seed, 1000 + stream])
    out = np.empty(n_tokens, dtype=np.int64)
    choice = rng.choice(branching, size=n_tokens, p=w)
    noise = rng.random(n_tokens) < 0.02
    rnd = perm[(rng.zipf(1.3, size=n_tokens) - 1) % vocab_eff]
    p2, p1 = 0, 1
    for i in range(n_tokens):
        if doc_len and i % doc_len == doc_len - 1 and V > EOT_TOKEN:
            t = EOT_TOKEN
        elif noise[i]:
            t = int(rnd[i])
        else:
            h = ((p2 * 1000003) ^ (p1 * 7919)) & (table_size - 1)
            t = int(succ[h, choice[i]])
        out[i] = t
        p2, p1 = p1, t
    return out


def synthetic_tokens_fast(n_tokens: int, vocab_size: int, seed: int = 0) -> np.ndarray:
    """Vectorised variant for large benchmark shards (order-1 structure, O(n) numpy)."""
    rng = np.random.default_rng(seed)
    V = min(int(vocab_size), 65535)
    base = rng.integers(0, V, size=n_tokens, dtype=np.int64)
    # every other token is a deterministic function of its predecessor -> learnable half
    det = (base * 2654435761 + 12345) % V
    out = base.copy()
    out[1::2] = det[0:-1:2][: out[1::2].size]
    return out


def ensure_synthetic_shard(path: str, n_tokens: int, vocab_size: int, seed: int = 0, fast: bool = None,
                           stream: int = 0) -> str:
    """Create ``path`` with synthetic tokens unless it already exists with >= n_tokens tokens."""
    if os.path.exists(path) and os.path.getsize(path) >= 2 * n_tokens:
        return path
    if fast is None:
        fast = n_tokens > 2_000_000
    if fast:
        toks = synthetic_tokens_fast(n_tokens, vocab_size, seed * 7919 + stream)
    else:
        toks = synthetic_tokens(n_tokens, vocab_size, seed, stream=stream)
    tmp = f"{path}.tmp{os.getpid()}"
    write_tokens(tmp, toks)
    os.replace(tmp, path)
    return path

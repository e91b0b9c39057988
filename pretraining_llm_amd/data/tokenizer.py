"""Tokenizer selection.

The reference uses tiktoken's GPT-2 BPE (``r50k_base`` in generate_text.py:35,
``gpt2`` in data_preprocess.py:29; the same merges, EOT = 50256).  tiktoken is
not installed in this environment and there is no network, so the resolution
order is:
  1. tiktoken (``r50k_base`` / ``gpt2``) if importable;
  2. a locally cached Hugging Face GPT-2 tokenizer (``transformers``, offline);
  3. a byte-level fallback (UTF-8 bytes -> ids 0..255, EOT = 50256) so the
     pipeline still runs end to end.  Token ids then differ from GPT-2 BPE:
     parity with the reference tokenization is unpinned in that mode.
"""
from __future__ import annotations

EOT = 50256


class ByteTokenizer:
    name = "bytes"
    eot_token = EOT
    n_vocab = 50257

    def encode_ordinary(self, text: str):
        return list(text.encode("utf-8"))

    def encode(self, text: str):
        return self.encode_ordinary(text)

    def decode(self, ids):
        # runs of byte ids decode as UTF-8; any other id (BPE-range ids a model trained on
        # synthetic or BPE-tokenized shards emits) is rendered as a visible <|id|> marker instead
        # of being dropped, so a generation is never silently empty
        out, run = [], []
        for i in ids:
            i = int(i)
            if 0 <= i < 256:
                run.append(i)
                continue
            if run:
                out.append(bytes(run).decode("utf-8", errors="replace"))
                run = []
            out.append(f"<|{i}|>")
        if run:
            out.append(bytes(run).decode("utf-8", errors="replace"))
        return "".join(out)


class _HFWrap:
    def __init__(self, tok):
        self.tok = tok
        self.name = "hf-gpt2"
        self.eot_token = tok.eos_token_id if tok.eos_token_id is not None else EOT
        self.n_vocab = len(tok)

    def encode_ordinary(self, text):
        return self.tok.encode(text, add_special_tokens=False)

    def encode(self, text):
        return self.encode_ordinary(text)

    def decode(self, ids):
        return self.tok.decode(list(ids))


def get_tokenizer(name: str = "gpt2"):
    try:
        import tiktoken  # type: ignore
        enc = tiktoken.get_encoding("r50k_base" if name in ("gpt2", "r50k_base") else name)
        return enc
    except Exception:
        pass
    try:
        from transformers import GPT2TokenizerFast  # type: ignore
        tok = GPT2TokenizerFast.from_pretrained("gpt2", local_files_only=True)
        wrap = _HFWrap(tok)
        # a cache entry without the BPE vocab/merges loads but encodes everything to []:
        # only accept a tokenizer that round-trips a probe string
        probe = "Hello world"
        ids = wrap.encode_ordinary(probe)
        if ids and wrap.decode(ids) == probe:
            return wrap
    except Exception:
        pass
    return ByteTokenizer()

"""Model configuration and named presets.

The reference defines its model through five flat constants
(`config/config.py:4-8` in Flink-ddd/pretraining-llm: V=50304, T=512, C=2048,
H=16, L=64) and a single architecture (learned positions, pre-LN, per-head
attention without an output projection, ReLU MLP, untied biased LM head;
`src/models/transformer.py:34-39`, `attention.py:29-33`, `mlp.py:24-26`).

Here the architecture is a set of explicit knobs so one model class covers:

* ``arch="ref"``   -- exact reference math and checkpoint layout,
* ``arch="gpt2"``  -- GPT-2 (fused QKV + W_o, GELU(tanh), tied embeddings),
* ``arch="llama"`` -- RoPE + RMSNorm + SwiGLU, no biases, untied head.

Presets mirror the configs named in BASELINE.json.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Optional


@dataclass
class ModelConfig:
    vocab_size: int = 50304
    context_length: int = 1024
    n_embed: int = 768
    n_head: int = 12
    n_blocks: int = 12
    n_kv_head: Optional[int] = None          # GQA; None -> n_head
    ffn_hidden: Optional[int] = None         # None -> 4*C (gelu/relu) or llama rule (swiglu)
    arch: str = "gpt2"                       # ref | gpt2 | llama
    norm: str = "layernorm"                  # layernorm | rmsnorm
    pos: str = "learned"                     # learned | rope
    mlp: str = "gelu"                        # relu | gelu | swiglu
    bias: bool = True                        # biases on linear layers (except lm_head, see head_bias)
    attn_out_proj: bool = True               # W_o (reference has none)
    tie_embeddings: bool = True
    head_bias: bool = False                  # bias on lm_head (reference: True)
    norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    init: str = "gpt2"                       # gpt2 | torch_default
    init_std: float = 0.02
    # True / False, a float fraction of the blocks, or "auto": checkpoint only as many blocks as
    # it takes for a step's activations to fit comfortably in the free HBM (GPT.checkpointed_blocks)
    activation_checkpointing: object = False
    dtype: str = "bfloat16"                  # compute/parameter dtype for training

    def __post_init__(self):
        if self.n_kv_head is None:
            self.n_kv_head = self.n_head
        assert self.n_embed % self.n_head == 0, "n_embed must be divisible by n_head"
        assert self.n_head % self.n_kv_head == 0, "n_head must be divisible by n_kv_head"
        if self.ffn_hidden is None:
            if self.mlp == "swiglu":
                h = int(2 * (4 * self.n_embed) / 3)
                self.ffn_hidden = 256 * ((h + 255) // 256)
            else:
                self.ffn_hidden = 4 * self.n_embed

    @property
    def head_dim(self) -> int:
        return self.n_embed // self.n_head

    def _default_ffn(self, n_embed: int, mlp: str) -> int:
        if mlp == "swiglu":
            h = int(2 * (4 * n_embed) / 3)
            return 256 * ((h + 255) // 256)
        return 4 * n_embed

    def replace(self, **kw) -> "ModelConfig":
        """dataclasses.replace that re-derives dependent defaults (n_kv_head, ffn_hidden)
        when the fields they were derived from change and they were not set explicitly."""
        if "n_head" in kw and "n_kv_head" not in kw and self.n_kv_head == self.n_head:
            kw["n_kv_head"] = None
        if ("n_embed" in kw or "mlp" in kw) and "ffn_hidden" not in kw and \
                self.ffn_hidden == self._default_ffn(self.n_embed, self.mlp):
            kw["ffn_hidden"] = None
        return dataclasses.replace(self, **kw)

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)

    @classmethod
    def from_dict(cls, d: dict) -> "ModelConfig":
        names = {f.name for f in dataclasses.fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in names})

    # ---- accounting ---------------------------------------------------
    def num_params(self, include_embedding: bool = True) -> int:
        C, V, T, L, F = self.n_embed, self.vocab_size, self.context_length, self.n_blocks, self.ffn_hidden
        kv = self.n_kv_head * self.head_dim
        b = 1 if self.bias else 0
        per = 0
        qkv_b = b if self.arch != "ref" else 0                  # reference Head projections are bias-free
        per += C * (C + 2 * kv) + qkv_b * (C + 2 * kv)         # qkv
        if self.attn_out_proj:
            per += C * C + b * C
        if self.mlp == "swiglu":
            per += 3 * C * F + b * (2 * F + C)
        else:
            per += 2 * C * F + b * (F + C)
        nparam_norm = 2 * C if self.norm == "layernorm" else C
        per += 2 * nparam_norm
        n = L * per + nparam_norm
        emb = V * C + (T * C if self.pos == "learned" else 0)
        if include_embedding:
            n += emb
        if not self.tie_embeddings:
            n += V * C + (V if self.head_bias else 0)
        return n

    def matmul_params(self) -> int:
        """Parameters that take part in a GEMM per token (for 6N FLOP accounting)."""
        C, V, L, F = self.n_embed, self.vocab_size, self.n_blocks, self.ffn_hidden
        kv = self.n_kv_head * self.head_dim
        per = C * (C + 2 * kv) + (C * C if self.attn_out_proj else 0)
        per += (3 if self.mlp == "swiglu" else 2) * C * F
        return L * per + V * C

    def flops_per_token(self, seq_len: Optional[int] = None) -> float:
        """Training FLOPs per token: 6*N_matmul + 12*L*T*C (causal attention counted
        dense, the usual PaLM/nanoGPT convention used in BASELINE.md)."""
        T = seq_len or self.context_length
        return 6.0 * self.matmul_params() + 12.0 * self.n_blocks * T * self.n_embed


# ---------------------------------------------------------------------------
# presets (BASELINE.json "configs")
# ---------------------------------------------------------------------------
def _ref(**kw) -> ModelConfig:
    base = dict(arch="ref", norm="layernorm", pos="learned", mlp="relu", bias=True,
                attn_out_proj=False, tie_embeddings=False, head_bias=True,
                init="torch_default")
    base.update(kw)
    return ModelConfig(**base)


def _gpt2(**kw) -> ModelConfig:
    base = dict(arch="gpt2", norm="layernorm", pos="learned", mlp="gelu", bias=True,
                attn_out_proj=True, tie_embeddings=True, head_bias=False, init="gpt2")
    base.update(kw)
    return ModelConfig(**base)


def _llama(**kw) -> ModelConfig:
    base = dict(arch="llama", norm="rmsnorm", pos="rope", mlp="swiglu", bias=False,
                attn_out_proj=True, tie_embeddings=False, head_bias=False, init="gpt2",
                norm_eps=1e-5)
    base.update(kw)
    return ModelConfig(**base)


PRESETS = {
    # reference "3 Billion" config (config/config.py:4-8)
    "ref-3b": lambda: _ref(vocab_size=50304, context_length=512, n_embed=2048, n_head=16, n_blocks=64),
    # reference architecture at GPT-2-small shape
    "ref-small": lambda: _ref(vocab_size=50304, context_length=1024, n_embed=768, n_head=12, n_blocks=12),
    # BASELINE config 1: plumbing on CPU
    "gpt2-tiny": lambda: _gpt2(vocab_size=50304, context_length=256, n_embed=128, n_head=4, n_blocks=2),
    # BASELINE configs 2/3: headline
    "gpt2-small": lambda: _gpt2(vocab_size=50304, context_length=1024, n_embed=768, n_head=12, n_blocks=12),
    # BASELINE config 5: long context
    # (activation checkpointing sized to the HBM: only as many blocks as needed, GPT.checkpointed_blocks)
    "gpt2-medium": lambda: _gpt2(vocab_size=50304, context_length=4096, n_embed=1024, n_head=16, n_blocks=24,
                                 activation_checkpointing="auto"),
    # BASELINE config 4
    "llama-1.3b": lambda: _llama(vocab_size=50304, context_length=2048, n_embed=2048, n_head=16, n_blocks=24,
                                 ffn_hidden=5504),
    "llama-tiny": lambda: _llama(vocab_size=512, context_length=128, n_embed=128, n_head=4, n_blocks=2,
                                 n_kv_head=2, ffn_hidden=256),
}


def get_preset(name: str, **overrides) -> ModelConfig:
    if name not in PRESETS:
        raise KeyError(f"unknown model preset {name!r}; known: {sorted(PRESETS)}")
    return PRESETS[name]().replace(**overrides) if overrides else PRESETS[name]()

"""Decoder-only transformer LM built on the fused gfx950 ops.

Reference parity (Flink-ddd/pretraining-llm):
* ``Transformer.forward(idx, targets) -> (logits, loss)``  -- `src/models/transformer.py:56-78`
* ``forward_embedding`` (fixed for L>1)                      -- `transformer.py:80-94`, `transformer_block.py:49-61`
* ``generate`` (multinomial sampling, context crop)           -- `transformer.py:96-114`, here with a KV cache
* module / state-dict names ``token_embed, position_embed, attn_blocks.{i}.{ln1,attn,ln2,mlp}, layer_norm,
  lm_head, pos_idxs``                                         -- `transformer.py:34-39`

MI355X-first structure (not a translation of the reference's per-head modules):
* one packed QKV GEMM per layer (hipBLASLt) feeding a HIP flash-attention kernel that
  reads Q/K/V strided out of it (llama: RoPE rotates the packed q/k heads first);
* the residual add is fused into the next norm kernel: blocks pass ``(hidden, residual)``
  pairs so no standalone add kernel exists in forward or backward;
* the LM head + cross-entropy writes dlogits during the forward (one pass over logits).
For ``arch="ref"`` a state-dict hook splits/fuses the packed QKV weight into the
reference's per-head ``attn.heads.{h}.{key,query,value}.weight`` (+ ``tril``) layout.
"""
from __future__ import annotations

import math
import numbers
from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.utils.checkpoint import checkpoint

from .. import ops
from .config import ModelConfig


def hbm_free_bytes(device) -> int:
    """Free HBM as the caching allocator sees it: the driver's free bytes plus blocks the
    allocator has reserved but holds no tensor in (an eval pass leaves such blocks behind)."""
    free, _ = torch.cuda.mem_get_info(device)
    return int(free + torch.cuda.memory_reserved(device) - torch.cuda.memory_allocated(device))


class Norm(nn.Module):
    def __init__(self, cfg: ModelConfig):
        super().__init__()
        C = cfg.n_embed
        self.rms = cfg.norm == "rmsnorm"
        self.eps = cfg.norm_eps
        self.weight = nn.Parameter(torch.ones(C))
        self.bias = None if self.rms else nn.Parameter(torch.zeros(C))

    def forward(self, x, residual=None, x_bias=None):
        """Returns (norm(x + residual), x + residual). ``x_bias``: bias of the linear that produced
        x, whose gradient this norm's backward kernel emits (fused bias-grad, HIP path)."""
        if self.rms:
            return ops.rms_norm(x, self.weight, self.eps, residual, x_bias=x_bias)
        return ops.layer_norm(x, self.weight, self.bias, self.eps, residual, x_bias=x_bias)

    def linear(self, x, residual, weight, bias=None, act=None, kv=None):
        """Inference: (act(norm(x + residual) @ weight^T + bias), x + residual) -- one fused
        skinny-GEMM launch for decode-sized inputs (ops.norm_linear, csrc/gemv.hip)."""
        return ops.norm_linear(x, residual, self.weight, self.bias, self.eps, self.rms, weight, bias, act, kv)


class Attention(nn.Module):
    def __init__(self, cfg: ModelConfig, layer_idx: int = 0):
        super().__init__()
        self.cfg = cfg
        self.n_head, self.n_kv_head, self.head_dim = cfg.n_head, cfg.n_kv_head, cfg.head_dim
        C = cfg.n_embed
        qkv_out = (cfg.n_head + 2 * cfg.n_kv_head) * cfg.head_dim
        self.qkv = nn.Linear(C, qkv_out, bias=cfg.bias and cfg.arch != "ref")
        self.proj = nn.Linear(C, C, bias=cfg.bias) if cfg.attn_out_proj else None

    def forward(self, x, rope=None, fuse_out_bias: bool = False):
        return self.forward_res(x, rope, fuse_out_bias)[0]

    def forward_res(self, x, rope=None, fuse_out_bias: bool = False, residual=None):
        """(y + residual, True) when the fused projection adds the block's residual stream in its GEMM
        (ops.resid_gemm_ok), else (y, False) and the caller's norm adds it."""
        qkv = ops.linear(x, self.qkv.weight, self.qkv.bias)
        cos, sin = rope if rope is not None else (None, None)
        if self.proj is not None and ops.attn_proj_ok(qkv, self.n_head, self.n_kv_head, self.proj.weight,
                                                      self.proj.bias):
            # the projection's data gradient also emits the attention backward's row constants
            r = residual if ops.resid_gemm_ok(residual, self.proj.weight) else None
            return ops.attention_proj(qkv, self.n_head, self.n_kv_head, self.proj.weight, self.proj.bias,
                                      rope_cos=cos, rope_sin=sin, bias_grad_external=fuse_out_bias,
                                      residual=r), r is not None
        y = ops.attention_packed(qkv, self.n_head, self.n_kv_head, causal=True, rope_cos=cos, rope_sin=sin)
        if self.proj is not None:
            r = residual if ops.resid_gemm_ok(residual, self.proj.weight) else None
            return ops.linear(y, self.proj.weight, self.proj.bias, bias_grad_external=fuse_out_bias,
                              residual=r), r is not None
        return y, False

    # --- KV-cache decode -------------------------------------------------
    def forward_cached(self, x, cache, layer_idx, pos, rope=None, qkv=None):
        if qkv is None:
            qkv = ops.linear(x, self.qkv.weight, self.qkv.bias)
        B, T, _ = qkv.shape
        H, Hkv, D = self.n_head, self.n_kv_head, self.head_dim
        q = qkv[..., : H * D].view(B, T, H, D)
        k = qkv[..., H * D:(H + Hkv) * D].view(B, T, Hkv, D)
        v = qkv[..., (H + Hkv) * D:].view(B, T, Hkv, D)
        if rope is not None:
            cos, sin = rope
            q = ops.apply_rope(q, cos, sin, pos)
            k = ops.apply_rope(k, cos, sin, pos)
        kc, vc = cache.update(layer_idx, k, v, pos)
        y = ops.attention(q.contiguous(), kc, vc, causal=True)
        y = y.reshape(B, T, H * D)
        if self.proj is not None:
            y = ops.linear(y, self.proj.weight, self.proj.bias)
        return y

    def forward_decode(self, x, cache, layer_idx, pos_t, len_t, rope=None, qkv=None, kv_written=False):
        """One-token step with the position on the DEVICE (``pos_t`` int64 [1], ``len_t`` =
        pos+1 as int32 [1]): no host scalar reaches a kernel argument, so the step can be
        captured once in a hipGraph and replayed at every position (inference/generate.py).
        ``qkv``: the already-projected input (the block fuses ln1 into the projection);
        ``kv_written``: that projection already appended k/v to the cache (no RoPE only)."""
        if qkv is None:
            qkv = ops.linear(x, self.qkv.weight, self.qkv.bias)
        B = qkv.shape[0]
        H, Hkv, D = self.n_head, self.n_kv_head, self.head_dim
        q = qkv[..., : H * D].view(B, 1, H, D)
        k = qkv[..., H * D:(H + Hkv) * D].view(B, 1, Hkv, D)
        v = qkv[..., (H + Hkv) * D:].view(B, 1, Hkv, D)
        per_row = pos_t.numel() > 1  # continuous batching: every sequence at its own position
        if rope is not None:
            cos, sin = rope[0].index_select(0, pos_t), rope[1].index_select(0, pos_t)
            if per_row:  # one table row per sequence: lay the batch out along the time axis
                q = ops.apply_rope(q.reshape(1, B, H, D), cos, sin, 0).view(B, 1, H, D)
                k = ops.apply_rope(k.reshape(1, B, Hkv, D), cos, sin, 0).view(B, 1, Hkv, D)
            else:
                q = ops.apply_rope(q, cos, sin, 0)
                k = ops.apply_rope(k, cos, sin, 0)
        if not kv_written:
            if per_row:
                rows = torch.arange(B, device=pos_t.device)
                cache.k[layer_idx].index_put_((rows, pos_t), k[:, 0])
                cache.v[layer_idx].index_put_((rows, pos_t), v[:, 0])
            else:
                cache.k[layer_idx].index_copy_(1, pos_t, k)
                cache.v[layer_idx].index_copy_(1, pos_t, v)
        y = ops.attention_decode(q.contiguous(), cache.k[layer_idx], cache.v[layer_idx], seqlen=len_t)
        y = y.reshape(B, 1, H * D)
        if self.proj is not None:
            y = ops.linear(y, self.proj.weight, self.proj.bias)
        return y


class MLP(nn.Module):
    def __init__(self, cfg: ModelConfig):
        super().__init__()
        C, Fh = cfg.n_embed, cfg.ffn_hidden
        self.kind = cfg.mlp
        up = 2 * Fh if cfg.mlp == "swiglu" else Fh
        self.hidden = nn.Linear(C, up, bias=cfg.bias)
        self.proj = nn.Linear(Fh, C, bias=cfg.bias)

    def forward_embedding(self, x):
        h = ops.linear(x, self.hidden.weight, self.hidden.bias)
        if self.kind == "gelu":
            return ops.gelu(h)
        if self.kind == "swiglu":
            return ops.swiglu(h)
        return ops.relu(h)

    def project_embedding(self, h):
        return ops.linear(h, self.proj.weight, self.proj.bias)

    def forward(self, x, fuse_out_bias: bool = False):
        """``fuse_out_bias``: the down-projection's bias gradient is emitted by the next norm."""
        return self.forward_res(x, fuse_out_bias)[0]

    def forward_res(self, x, fuse_out_bias: bool = False, residual=None):
        """(y + residual, True) when the fused MLP's down projection adds the residual stream in its GEMM
        (ops.resid_gemm_ok), else (y, False)."""
        if ops.fused_mlp_ok(x, self.hidden.weight, self.hidden.bias, self.proj.weight, self.kind):
            # activation in the GEMM epilogues (csrc/gemm.hip)
            r = residual if ops.resid_gemm_ok(residual, self.proj.weight) else None
            return ops.fused_mlp(x, self.hidden.weight, self.hidden.bias, self.proj.weight, self.proj.bias,
                                 self.kind, out_bias_ext=fuse_out_bias, residual=r), r is not None
        return self._forward_unfused(x, fuse_out_bias), False

    def _forward_unfused(self, x, fuse_out_bias: bool):
        if self.kind == "swiglu" and ops.fused_swiglu_ok(x, self.hidden.weight, self.hidden.bias,
                                                          self.proj.weight, self.proj.bias):
            # SwiGLU backward in the down-projection's data-gradient epilogue (csrc/gemm.hip)
            return ops.fused_swiglu_mlp(x, self.hidden.weight, self.proj.weight)
        fuse_act = ops._hip(x) and self.kind in ("gelu", "relu") and self.hidden.bias is not None \
            and torch.is_grad_enabled()
        h = ops.linear(x, self.hidden.weight, self.hidden.bias, bias_grad_external=fuse_act)
        if self.kind == "gelu":
            a = ops.gelu(h, bias=self.hidden.bias if fuse_act else None)
        elif self.kind == "swiglu":
            a = ops.swiglu(h)
        else:
            a = ops.relu(h) if not fuse_act else ops.relu(h, bias=self.hidden.bias)
        return ops.linear(a, self.proj.weight, self.proj.bias, bias_grad_external=fuse_out_bias)


class Block(nn.Module):
    def __init__(self, cfg: ModelConfig, layer_idx: int = 0):
        super().__init__()
        self.ln1 = Norm(cfg)
        self.attn = Attention(cfg, layer_idx)
        self.ln2 = Norm(cfg)
        self.mlp = MLP(cfg)

    def forward(self, x, residual=None, rope=None, x_bias=None, fuse_mlp_out_bias: bool = False):
        """(x, residual) -> (mlp_out, residual_after_attn); the caller's next norm adds them.

        Fused bias gradients (HIP path): ``x_bias`` is the bias of the layer that produced x (the
        previous block's MLP down projection), emitted by ln1's backward; the attention output
        projection's bias by ln2's backward; with ``fuse_mlp_out_bias`` the caller promises to pass
        this block's ``mlp.proj.bias`` as ``x_bias`` of the next norm."""
        fuse = ops._hip(x) and torch.is_grad_enabled() and self.attn.proj is not None \
            and self.attn.proj.bias is not None and getattr(self.attn, "fused_bias_ok", True)
        h, res = self.ln1(x, residual, x_bias=x_bias)
        # the output projections may add the residual stream in their GEMMs (ops.resid_gemm_ok; the reference's
        # x + attn(ln1(x)) / x + mlp(ln2(x)), /root/reference/src/models/transformer_block.py:44,46): then the
        # next norm gets the stream itself (residual None) and the block returns (stream, None)
        if hasattr(self.attn, "forward_res"):
            a, a_res = self.attn.forward_res(h, rope, fuse, res)
        else:
            a, a_res = self.attn(h, rope, fuse_out_bias=fuse), False
        h2, res2 = self.ln2(a, None if a_res else res, x_bias=self.attn.proj.bias if fuse else None)
        if hasattr(self.mlp, "forward_res"):
            m, m_res = self.mlp.forward_res(h2, fuse and fuse_mlp_out_bias, res2)
        else:
            m, m_res = self.mlp(h2, fuse_out_bias=fuse and fuse_mlp_out_bias), False
        return m, (None if m_res else res2)

    def fused_out_bias(self, x):
        """The bias the next norm must take as ``x_bias`` when fuse_mlp_out_bias=True (or None)."""
        if ops._hip(x) and torch.is_grad_enabled() and self.mlp.proj.bias is not None \
                and self.attn.proj is not None and self.attn.proj.bias is not None \
                and getattr(self.attn, "fused_bias_ok", True) and getattr(self.mlp, "fused_bias_ok", True):
            return self.mlp.proj.bias
        return None

    # Inference steps: each norm runs as the prologue of the projection after it and the MLP
    # activation as the epilogue of the up-projection (Norm.linear -> ops.norm_linear): at
    # decode sizes a block is 4 skinny-GEMM launches + attention; prefill falls back to the
    # unfused kernels.
    def _mlp_infer(self, a, res):
        kind = self.mlp.kind
        act = None if kind == "swiglu" else ("gelu" if kind == "gelu" else "relu")
        h, res2 = self.ln2.linear(a, res, self.mlp.hidden.weight, self.mlp.hidden.bias, act=act)
        if kind == "swiglu":
            h = ops.swiglu(h)
        return ops.linear(h, self.mlp.proj.weight, self.mlp.proj.bias), res2

    def forward_cached(self, x, residual, cache, layer_idx, pos, rope=None):
        qkv, res = self.ln1.linear(x, residual, self.attn.qkv.weight, self.attn.qkv.bias)
        a = self.attn.forward_cached(None, cache, layer_idx, pos, rope, qkv=qkv)
        return self._mlp_infer(a, res)

    def forward_decode(self, x, residual, cache, layer_idx, pos_t, len_t, rope=None):
        # without RoPE the QKV projection's epilogue also appends k/v to the cache
        kv = None
        if rope is None:
            kv = (cache.k[layer_idx], cache.v[layer_idx], pos_t, self.attn.n_head * self.attn.head_dim)
        qkv, res = self.ln1.linear(x, residual, self.attn.qkv.weight, self.attn.qkv.bias, kv=kv)
        a = self.attn.forward_decode(None, cache, layer_idx, pos_t, len_t, rope, qkv=qkv,
                                     kv_written=kv is not None)
        return self._mlp_infer(a, res)

    def forward_embedding(self, x, residual=None, rope=None):
        h, res = self.ln1(x, residual)
        a = self.attn(h, rope)
        h2, res2 = self.ln2(a, res)
        return self.mlp.forward_embedding(h2), res2


class GPT(nn.Module):
    def __init__(self, cfg: ModelConfig):
        super().__init__()
        self.config = cfg
        self.context_length = cfg.context_length
        self.N_BLOCKS = cfg.n_blocks
        C, V = cfg.n_embed, cfg.vocab_size
        self.token_embed = nn.Embedding(V, C)
        self.position_embed = nn.Embedding(cfg.context_length, C) if cfg.pos == "learned" else None
        self.attn_blocks = nn.ModuleList([Block(cfg, i) for i in range(cfg.n_blocks)])
        self.layer_norm = Norm(cfg)
        if cfg.tie_embeddings:
            self.lm_head = None
        else:
            self.lm_head = nn.Linear(C, V, bias=cfg.head_bias)
            # an untied token table is only gathered from, never a GEMM operand: no transposed bf16
            # shadow for the optimizer to refresh every step (train/optim.py)
            self.token_embed.weight._pllm_no_shadow = True
        if self.position_embed is not None:
            self.position_embed.weight._pllm_no_shadow = True
        if cfg.arch == "ref":
            # persistent like the reference (transformer.py:39) so checkpoints match key-for-key
            self.register_buffer("pos_idxs", torch.arange(cfg.context_length), persistent=True)
            from .compat import install_ref_state_dict_hooks
            install_ref_state_dict_hooks(self)
        self._rope = None
        self.parallel = None  # ParallelGroups once parallel.model_parallel.parallelize_gpt ran
        self.reset_parameters()

    # ------------------------------------------------------------------
    def reset_parameters(self):
        cfg = self.config
        if cfg.init == "torch_default":
            for m in self.modules():
                if isinstance(m, (nn.Linear, nn.Embedding)):
                    m.reset_parameters()
            return
        std = cfg.init_std
        proj_std = std / math.sqrt(2 * cfg.n_blocks)
        for name, p in self.named_parameters():
            if p.dim() == 1:
                if name.endswith("bias"):
                    nn.init.zeros_(p)
                else:
                    nn.init.ones_(p)
            elif name.endswith("attn.proj.weight") or name.endswith("mlp.proj.weight"):
                nn.init.normal_(p, 0.0, proj_std)
            else:
                nn.init.normal_(p, 0.0, std)

    @property
    def head_weight(self):
        return self.token_embed.weight if self.lm_head is None else self.lm_head.weight

    @property
    def head_bias(self):
        return None if self.lm_head is None else self.lm_head.bias

    def rope_tables(self, device, length: Optional[int] = None):
        cfg = self.config
        if cfg.pos != "rope":
            return None
        L = length or cfg.context_length
        if self._rope is None or self._rope[0].device != device or self._rope[0].shape[0] < L:
            self._rope = ops.rope_cache(L, cfg.head_dim, cfg.rope_theta, device)
        return self._rope

    def activation_bytes(self, tokens: int) -> int:
        """Estimated bytes of activations a training forward keeps for backward, all layers:
        2 B x (6 C + 2 F) per token and layer (bf16: norm outputs, residual stream, packed QKV,
        attention output, MLP pre/post activation) -- within 2 % of the measured difference
        between checkpointed and full runs of GPT-2 medium at 32K tokens (36.9 vs 14.4 GB)."""
        cfg = self.config
        per = 6 * cfg.n_embed + 2 * cfg.ffn_hidden
        if cfg.pos == "rope":  # rotated q / k of the attention pre-pass (ops._FlashAttnPacked)
            per += (cfg.n_head + cfg.n_kv_head) * cfg.head_dim
        return 2 * per * tokens * cfg.n_blocks

    def checkpointed_blocks(self, idx) -> int:
        """How many of the first blocks recompute their forward in backward.

        ``activation_checkpointing`` is True (all), False (none), a float fraction of the blocks,
        or ``"auto"``: checkpoint only as many blocks as it takes for the kept activations to fit
        in half of the GPU's currently free HBM.  A checkpointed block keeps just its two
        [tokens, C] inputs (x, residual) instead of its ``activation_bytes`` share.  On a 288 GB
        MI355X that keeps GPT-2 medium at 8 x 4096 tokens (23 GB of activations) un-checkpointed
        (308K vs 241K tokens/s, profiles/r1_bench_gpt2medium_s4096.jsonl) and checkpoints a
        growing fraction of the blocks from about 64 x 4096 on, instead of all-or-nothing."""
        mode = self.config.activation_checkpointing
        L = self.config.n_blocks
        if isinstance(mode, bool) or mode is None:
            return L if mode else 0
        if isinstance(mode, numbers.Integral):  # e.g. --activation_checkpointing=1 from the CLI
            return L if mode else 0
        if isinstance(mode, numbers.Real):
            return min(L, max(0, math.ceil(float(mode) * L)))
        if mode != "auto":
            raise ValueError(f"activation_checkpointing={mode!r}: expected bool, float fraction or 'auto'")
        if not idx.is_cuda:
            return 0
        if getattr(self, "_ckpt_auto", None) is None or self._ckpt_auto[0] != idx.numel():
            self._ckpt_auto = (idx.numel(), self.auto_checkpoint_blocks(idx.numel(), 0.5 * hbm_free_bytes(idx.device)))
        return self._ckpt_auto[1]

    def auto_checkpoint_blocks(self, tokens: int, budget_bytes: float) -> int:
        """Fewest checkpointed blocks whose kept activations fit ``budget_bytes`` (all if none do)."""
        L = self.config.n_blocks
        full = self.activation_bytes(tokens)
        if full <= budget_bytes:
            return 0
        per_block = full / L
        saved = per_block - 2 * 2 * self.config.n_embed * tokens  # a checkpointed block keeps x, res
        if saved <= 0:
            return L
        return min(L, math.ceil((full - budget_bytes) / saved))

    def use_checkpointing(self, idx) -> bool:
        """True when at least one block is checkpointed (see ``checkpointed_blocks``)."""
        return self.checkpointed_blocks(idx) > 0

    def num_params(self) -> int:
        return sum(p.numel() for p in self.parameters())

    # ------------------------------------------------------------------
    def _embed(self, idx, positions=None):
        wpe = self.position_embed.weight if self.position_embed is not None else None
        T = idx.shape[1]
        if T > self.config.context_length and wpe is not None and positions is None:
            raise ValueError(f"sequence length {T} > context_length {self.config.context_length}")
        if positions is not None and wpe is not None:
            wpe = wpe.index_select(0, positions)  # a CP / SP shard's global positions
        return ops.embedding(idx, self.token_embed.weight, wpe)

    def _cp_positions(self, idx):
        pg = self.parallel
        if pg is None or pg.cp == 1:
            return None
        if pg.cp_mode == "ulysses":  # contiguous shard
            Tl = idx.shape[1]
            return torch.arange(pg.cp_rank * Tl, (pg.cp_rank + 1) * Tl, device=idx.device)
        from ..parallel.context import zigzag_positions
        return zigzag_positions(idx.shape[1], pg.cp_group, idx.device)

    def _shard_inputs(self, idx, targets):
        """Model parallelism: every rank of a TP / CP group receives the same full batch; CP keeps
        this rank's sequence shard -- zigzag chunks for ring attention, one contiguous chunk for
        Ulysses (sequence parallelism splits after the embedding)."""
        pg = self.parallel
        if pg is not None and pg.cp > 1:
            if pg.cp_mode == "ulysses":
                from ..parallel.tensor import _split_dim
                idx = _split_dim(idx, 1, pg.cp_group)
                targets = _split_dim(targets, 1, pg.cp_group) if targets is not None else None
            else:
                from ..parallel.context import zigzag_shard
                idx = zigzag_shard(idx, 1, pg.cp_group)
                targets = zigzag_shard(targets, 1, pg.cp_group) if targets is not None else None
        return idx, targets

    def _trunk(self, idx):
        pos = self._cp_positions(idx)
        pg = self.parallel
        if pg is not None and pg.sequence_parallel:
            # sequence parallelism: embed only this rank's T/tp tokens (no collective; the
            # replicated embedding tables get this shard's partial gradient like every other
            # replicated parameter, summed over the TP group by sync_replicated_grads)
            from ..parallel.tensor import _split_dim
            T = idx.shape[1]
            if T % pg.tp:
                raise ValueError(f"sequence_parallel: seq_len {T} must be divisible by tp_size {pg.tp}")
            Tl = T // pg.tp
            x = self._embed(_split_dim(idx, 1, pg.tp_group),
                            torch.arange(pg.tp_rank * Tl, (pg.tp_rank + 1) * Tl, device=idx.device))
        else:
            x = self._embed(idx, pos)
        rope = self.rope_tables(idx.device, idx.shape[1] if pos is None else self.config.context_length)
        if rope is not None and pos is not None:
            rope = (rope[0].index_select(0, pos).contiguous(), rope[1].index_select(0, pos).contiguous())
        res = None
        n_ckpt = self.checkpointed_blocks(idx) if self.training and torch.is_grad_enabled() else 0
        x_bias = None  # bias of the layer that produced x (fused into the next norm's backward)
        for i, blk in enumerate(self.attn_blocks):
            if i < n_ckpt:
                x, res = checkpoint(blk, x, res, rope, x_bias, True, use_reentrant=False)
            else:
                x, res = blk(x, res, rope, x_bias, True)
            x_bias = blk.fused_out_bias(x)
        h, _ = self.layer_norm(x, res, x_bias=x_bias)
        return h

    def forward(self, idx: torch.Tensor, targets: Optional[torch.Tensor] = None,
                return_logits: bool = True) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
        """Under tensor/sequence/context parallelism the loss is the mean over THIS rank's tokens
        (SP / CP: its sequence shard); the Trainer scales the gradients accordingly."""
        idx, targets = self._shard_inputs(idx, targets)
        h = self._trunk(idx)
        pg = self.parallel
        if targets is not None and pg is not None and pg.sequence_parallel:
            from ..parallel.tensor import _split_dim
            targets = _split_dim(targets, 1, pg.tp_group)
        B, T, C = h.shape
        if targets is None:
            logits = ops.linear(h, self.head_weight, self.head_bias)
            return logits, None
        if not return_logits:
            # training hot path: LM head GEMM + fused CE that overwrites the logits with dlogits
            return None, ops.lm_head_cross_entropy(h, self.head_weight, self.head_bias, targets)
        logits = ops.linear(h.reshape(B * T, C), self.head_weight, self.head_bias)
        loss = ops.cross_entropy(logits, targets.reshape(B * T))
        return logits.view(B, T, -1), loss

    def forward_embedding(self, idx):
        """(hidden, residual) of the LAST block: hidden = act(mlp.hidden(ln2(res))) [B,T,F],
        res = post-attention residual stream [B,T,C]. Matches the reference for L=1
        (`transformer_block.py:49-61`) and, unlike it, is well-defined for L>1."""
        x = self._embed(idx)
        rope = self.rope_tables(idx.device, idx.shape[1])
        res = None
        for blk in self.attn_blocks[:-1]:
            x, res = blk(x, res, rope)
        return self.attn_blocks[-1].forward_embedding(x, res, rope)

    # ------------------------------------------------------------------
    @torch.no_grad()
    def generate(self, idx: torch.Tensor, max_new_tokens: int, temperature: float = 1.0,
                 top_k: Optional[int] = None, use_cache: bool = True, generator=None,
                 cuda_graph: bool = False, decode_cache: Optional[dict] = None) -> torch.Tensor:
        if self.parallel is not None and self.parallel.model_parallel:
            raise ValueError("generate() runs on a dense model: load the consolidated checkpoint "
                             "(Trainer.save writes one) or parallel.model_parallel.gather_dense_state")
        from ..inference.generate import generate
        return generate(self, idx, max_new_tokens, temperature=temperature, top_k=top_k,
                        use_cache=use_cache, generator=generator, cuda_graph=cuda_graph, decode_cache=decode_cache)

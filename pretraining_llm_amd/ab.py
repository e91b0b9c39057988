"""Debug-only A/B overrides of measured, fixed choices: one environment variable,

    PLLM_AB="key=value,key=value,..."

None of these is part of the supported surface.  Each key flips a choice that was measured and fixed in code
(the record is named next to the key); they stay selectable so a later change can be A/B'd against the fixed
choice on the same box without a rebuild.  The C++ side reads the same variable (csrc/ab.h, pllm::ab_int).

| key | default | what the non-default selects | record |
|---|---|---|---|
| resid_gemm | 1 | 0: the block's residual add in the next norm instead of the projections' GEMMs | r5_residual_in_gemm.md |
| wt_shadow | 1 | 0: data-gradient GEMMs on the weights as stored (no transposed shadows) | r1_prof6_gpt2small_b64_kernel_stats.md (the transposes it replaced) |
| rope_prepass | 1 | 0: RoPE rotated inside the attention kernels' q / k staging | r2_rope_prepass_ab.txt |
| attn_proj_fused | 1 | 0: attention output-projection backward on hipBLASLt + the delta pre-pass | r4_fusion_analysis.md |
| fused_swiglu_fwd | 1 | 0: llama up-projection on hipBLASLt + the SwiGLU kernel | r4_gemm_pp.md |
| lt_relu | 1 | 0: ReLU MLP up-projection on torch + the activation kernel | r4_lt_relu_epilogue.md |
| wgrad_bias | 1 | 0: bias gradients as a separate column-sum pass | r3s3_wgrad_fused_bias_ab.txt |
| wgrad_variant | -- | weight-gradient kernel variant id (torch.ops.pllm.wgrad_set_mfma) | r2_wgrad_4wave_negative.jsonl and the other r2_wgrad_* records |
| wgrad_hy_cost | 1 | 0: the hybrid weight gradient's remainder as one round of slices (ctas / rem) instead of the cost model's count | r6_wgrad_hy_cost.log |
| wgrad_hy | -- | 0 / 1: hybrid whole-tile + sliced-last-round weight-gradient split | r4_wgrad_hybrid.md |
| gemm_persistent | -- | 0 / 1: persistent GEMM grids (default: automatic, train/graph.py) | r4_gemm_persistent_ab.txt |
| dp_world1 | 0 | 1: the DP engine's gradient hooks + bucketed all-reduces at world 1 (a one-rank RCCL rehearsal of the world > 1 step) | tests/test_dp_gpu.py |
| lazy_zero | 1 | 0: zero the whole flat gradient every step | r4_lazy_zero_ab.md |
| ce_chunk_rows | 0 | rows per LM-head + CE chunk (0: automatic) | r2_ce_chunk_sweep.jsonl |
| ce_nt | 1 | 0: plain (not non-temporal) dlogits stores in the CE kernel | csrc/cross_entropy.hip (2,493 vs 2,524 us) |
| tune_ms / tune_iters | 4 / 8 | TunableOp search budget (scripts/tune_gemms.py) | utils/gemm_tuning.py |
| lt_verbose | 0 | 1: print hipBLASLt's candidate timings | -- |
"""
from __future__ import annotations

import os


def _parse() -> dict:
    out = {}
    for item in os.environ.get("PLLM_AB", "").split(","):
        k, eq, v = item.strip().partition("=")
        if k and eq:
            out[k.strip()] = v.strip()
    return out


def ab(key: str, default):
    """The PLLM_AB value of ``key`` converted to ``default``'s type (bool: "1"/"0"), else ``default``.
    Read on every call, so a test can monkeypatch the variable before constructing the object that reads it."""
    v = _parse().get(key)
    if v is None:
        return default
    if isinstance(default, bool):
        return v not in ("0", "false", "False", "")
    if isinstance(default, int):
        return int(v)
    if isinstance(default, float):
        return float(v)
    return v


def ab_set(key: str, value) -> None:
    """Set ``key`` in this process's PLLM_AB (scripts that pin a choice for their children)."""
    d = _parse()
    d[key] = str(int(value) if isinstance(value, bool) else value)
    os.environ["PLLM_AB"] = ",".join(f"{k}={v}" for k, v in d.items())

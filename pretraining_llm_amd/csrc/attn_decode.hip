// Split-KV single-query attention for KV-cache decoding (gfx950).
//
// Reference: generation re-runs the FULL forward for every new token and
// materialises softmax(q k^T) per head (src/models/transformer.py:96-114,
// src/models/attention.py:51-57); SURVEY.md §2.3 K13 asks for a 1 x T_kv decode
// kernel instead.  A decode step is memory-bound (every cached K/V byte is read
// once per token, ~2 FLOP/byte), so this kernel is built around HBM/L2 streaming,
// not MFMA:
//  * grid = (splits, Hkv, B): the key range of one (batch, kv-head) is cut into
//    `splits` contiguous chunks so even B=1 fills the chip (>= ~2 workgroups per
//    CU); all G = H/Hkv query heads of a GQA group share one pass over K/V;
//  * lane layout: a key row of D bf16 is read by D/8 lanes, 16 B each (one
//    128/256 B coalesced segment per row), so a 256-thread workgroup covers
//    256/(D/8) keys per pass; q . k is 8 FMAs per lane + log2(D/8) xor-shuffles;
//  * every key-slice (group of D/8 lanes) keeps its own online-softmax state
//    (running max m, sum l, 8-wide output accumulator per head) over its keys,
//    U keys per iteration with all 2U loads issued first; no LDS or barriers in
//    the main loop.  Slices merge by shuffles inside a wave, then through LDS;
//  * splits > 1 write an fp32 partial (o, log2-sum-exp) per split and a combine
//    kernel merges them (deterministic, fixed order); splits == 1 writes bf16 o.
//  * the key count can come from a device scalar (`seqlen`; or one count per sequence for
//    continuous batching, where every slot of the batch sits at its own position), so a decode step
//    can be captured once in a hipGraph and replayed at every position.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int NT = 256;

template <int D, int G, int U>
__global__ __launch_bounds__(NT) void attn_decode_kernel(DecodeArgs a) {
  constexpr int LPR = D / 8;          // lanes per key row
  constexpr int NKS = NT / LPR;       // key-slices per workgroup
  const int split = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int dp = t % LPR, ks = t / LPR;
  const int S = a.seqlen ? a.seqlen[a.seqlen_per_row ? b : 0] : a.S;
  const int chunk = (S + a.splits - 1) / a.splits;
  const int k0 = split * chunk, k1 = min(S, k0 + chunk);

  // q fragments of the G heads of this group, pre-scaled by scale*log2(e)
  float q[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int h = hk * G + g;
    float f[8];
    unpack8(ld16(a.q + (int64_t)b * a.q_sb + (int64_t)h * a.q_sh + dp * 8), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) q[g][e] = f[e] * a.scale_log2;
  }
  float m[G], l[G], acc[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -INFINITY;
    l[g] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[g][e] = 0.f;
  }
  const uint16_t* kb = a.k + (int64_t)b * a.k_sb + (int64_t)hk * a.k_sh + dp * 8;
  const uint16_t* vb = a.v + (int64_t)b * a.v_sb + (int64_t)hk * a.v_sh + dp * 8;

  for (int j0 = k0 + ks; j0 < k1; j0 += U * NKS) {
    u32x4 kr[U], vr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // all loads first (clamped), then the math
      const int j = min(j0 + u * NKS, k1 - 1);
      kr[u] = ld16(kb + (int64_t)j * a.k_st);
      vr[u] = ld16(vb + (int64_t)j * a.v_st);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float s[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float kf[8];
        unpack8(kr[u], kf);
        float d = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) d = fmaf(q[g][e], kf[e], d);
#pragma unroll
        for (int o = 1; o < LPR; o <<= 1) d += __shfl_xor(d, o, 64);
        s[u] = (j0 + u * NKS < k1) ? d : -INFINITY;
      }
      float mx = m[g];
#pragma unroll
      for (int u = 0; u < U; ++u) mx = fmaxf(mx, s[u]);
      // mx is finite: the first key of this iteration is always valid
      const float corr = fast_exp2(m[g] - mx);
      m[g] = mx;
      l[g] *= corr;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[g][e] *= corr;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float p = fast_exp2(s[u] - mx);
        l[g] += p;
        float vf[8];
        unpack8(vr[u], vf);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[g][e] = fmaf(p, vf[e], acc[g][e]);
      }
    }
  }

  // merge the 64 / LPR key-slices of this wave (lane bits above log2(LPR))
#pragma unroll
  for (int o = LPR; o < 64; o <<= 1) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float m2 = __shfl_xor(m[g], o, 64), l2 = __shfl_xor(l[g], o, 64);
      const float mx = fmaxf(m[g], m2);
      const float c1 = mx == -INFINITY ? 0.f : fast_exp2(m[g] - mx);
      const float c2 = mx == -INFINITY ? 0.f : fast_exp2(m2 - mx);
      l[g] = l[g] * c1 + l2 * c2;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[g][e] = acc[g][e] * c1 + __shfl_xor(acc[g][e], o, 64) * c2;
      m[g] = mx;
    }
  }
  // merge the 4 waves through LDS
  __shared__ float s_ml[4][G][2];
  __shared__ float s_acc[4][G][D];
  if (lane < LPR) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (lane == 0) {
        s_ml[w][g][0] = m[g];
        s_ml[w][g][1] = l[g];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) s_acc[w][g][dp * 8 + e] = acc[g][e];
    }
  }
  __syncthreads();
  for (int i = t; i < G * D; i += NT) {
    const int g = i / D, d = i % D;
    float mx = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) mx = fmaxf(mx, s_ml[ww][g][0]);
    float lsum = 0.f, o = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      const float c = mx == -INFINITY ? 0.f : fast_exp2(s_ml[ww][g][0] - mx);
      lsum += s_ml[ww][g][1] * c;
      o += s_acc[ww][g][d] * c;
    }
    const int h = hk * G + g;
    const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
    if (a.splits == 1) {
      a.o[(int64_t)b * a.o_sb + (int64_t)h * a.o_sh + d] = f2bf_bits(o * inv);
    } else {
      const int64_t row = ((int64_t)b * a.H + h) * a.splits + split;
      a.part_o[row * D + d] = o * inv;
      if (d == 0) a.part_lse[row] = lsum > 0.f ? mx + __log2f(lsum) : -INFINITY;
    }
  }
}

// one wave per (b, h): merge the split partials (fixed order -> deterministic)
template <int D>
__global__ __launch_bounds__(64) void attn_decode_combine_kernel(DecodeArgs a) {
  const int bh = blockIdx.x, lane = threadIdx.x;
  const int b = bh / a.H, h = bh % a.H;
  const float* lse = a.part_lse + (int64_t)bh * a.splits;
  float mx = -INFINITY;
  for (int s = 0; s < a.splits; ++s) mx = fmaxf(mx, lse[s]);
  float o[D / 64 > 0 ? D / 64 : 1] = {};
  float wsum = 0.f;
  for (int s = 0; s < a.splits; ++s) {
    const float c = mx == -INFINITY ? 0.f : fast_exp2(lse[s] - mx);
    wsum += c;
    const float* po = a.part_o + ((int64_t)bh * a.splits + s) * D;
#pragma unroll
    for (int i = 0; i < (D + 63) / 64; ++i)
      if (i * 64 + lane < D) o[i] += c * po[i * 64 + lane];
  }
  const float inv = wsum > 0.f ? 1.f / wsum : 0.f;
#pragma unroll
  for (int i = 0; i < (D + 63) / 64; ++i)
    if (i * 64 + lane < D) a.o[(int64_t)b * a.o_sb + (int64_t)h * a.o_sh + i * 64 + lane] = f2bf_bits(o[i] * inv);
}

template <int D, int G>
void launch(const DecodeArgs& a, hipStream_t st) {
  constexpr int U = G <= 2 ? 4 : 2;
  hipLaunchKernelGGL((attn_decode_kernel<D, G, U>), dim3(a.splits, a.Hkv, a.B), dim3(NT), 0, st, a);
  if (a.splits > 1)
    hipLaunchKernelGGL((attn_decode_combine_kernel<D>), dim3(a.B * a.H), dim3(64), 0, st, a);
}

template <int D>
void dispatch_g(const DecodeArgs& a, hipStream_t st) {
  switch (a.H / a.Hkv) {
    case 1: launch<D, 1>(a, st); break;
    case 2: launch<D, 2>(a, st); break;
    case 4: launch<D, 4>(a, st); break;
    case 8: launch<D, 8>(a, st); break;
    default: break;
  }
}

}  // namespace

namespace pllm {

bool attn_decode_supported(int D, int group) {
  return (D == 32 || D == 64 || D == 128) && (group == 1 || group == 2 || group == 4 || group == 8);
}

int attn_decode_splits(int B, int Hkv, int S_max) {
  // >= ~2 workgroups per CU over the whole grid, >= 64 keys per split
  const int want = (512 + B * Hkv - 1) / (B * Hkv);
  const int cap = (S_max + 63) / 64;
  int s = want < cap ? want : cap;
  return s < 1 ? 1 : (s > 64 ? 64 : s);
}

void attn_decode(const DecodeArgs& a, hipStream_t st) {
  switch (a.D) {
    case 32: dispatch_g<32>(a, st); break;
    case 64: dispatch_g<64>(a, st); break;
    case 128: dispatch_g<128>(a, st); break;
    default: break;
  }
  PL_CHECK_LAUNCH();
}

}  // namespace pllm

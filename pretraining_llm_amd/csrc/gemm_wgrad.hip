// Weight-gradient GEMM for linear layers on gfx950 MFMA (the one-barrier kernel; since round 4 the
// default for fp32 gradient targets is the ping-pong kernel of wgrad_pp.hip, dispatched from wgrad()
// below with the same split-K plan, slab layout and reduce; this kernel serves bf16 targets and
// wgrad_set_mfma(100 / 16 / 32 / 1xx) A/B runs):
//     dW[P, Q] (+)= sum_m dY[m, P] * X[m, Q]          (bf16 in, fp32 accumulate)
// i.e. the reduction runs over the token dimension (M = batch*seq, 65536 for the
// headline config) while the output is small (768x768 .. 50304x768).  Both operands
// are token-major, the "NT" case hipBLASLt serves worst: 0.39-0.99 PFLOP/s in the
// GPT-2-small step against 1.0-1.37 for the forward GEMMs of the same shapes
// (profiles/r1_prof5*).
//
// Design (CDNA4):
//  * split-K over tokens: work item = (token slice, 256x256 output tile), slice-major,
//    and the work items are dealt to the 8 XCDs in contiguous ranges (xcd_remap), so
//    the tiles that share a slice's dY/X panels run on one XCD and share its L2;
//  * 8 waves per workgroup (2 per SIMD) as 2 (P) x 4 (Q), each owning a 128x64 sub-tile
//    as 8x4 v_mfma_f32_16x16x32_bf16 accumulators (or 4x2 32x32x16 ones: wgrad_set_mfma);
//  * operands staged HBM/L2 -> LDS by global_load_lds (16 B per lane, no staging
//    registers): 64-token stages, double-buffered, the next stage's DMA in flight under
//    the current stage's MFMAs, one barrier per stage.  The LDS images are [64][128]
//    halves with the XOR chunk swizzle of attention.hip's Img<128>; the DMA writes
//    lane-linear 1-KiB pieces, so the swizzle is applied to the per-lane SOURCE
//    address instead;
//  * both MFMA fragments come from ds_read_b64_tr_b16 transposed reads (the reduction
//    index is the image row);
//  * one slice: the tile is added straight into the gradient (bf16 or fp32, the optimizer's
//    gradient dtype); several: fp32 partial tiles go to a [S][P][Q] slab summed in a fixed
//    slice order by wgrad_reduce_kernel (deterministic).  Measured and dropped in round 1: a
//    4/5-slot staging ring (4-15 % slower, profiles/r1_wgrad_ring_ab.jsonl) and an in-kernel
//    last-arriver reduction (1.0-3.2x slower, profiles/r1_wgrad_fused_reduce_negative.jsonl).
//    Round 2: a phased variant after the 256² 8-phase GEMM template (4 quadrant phases per K-tile,
//    counted vmcnt(6) with 3 half-tile images in flight, raw barriers, setprio, wave stagger;
//    16x16x32 and 32x32x16) measured 3-10 % SLOWER than this kernel on every GPT-2 / Llama shape
//    (profiles/r2_wgrad_phased_negative_*.jsonl).  PMC (profiles/r2_pmc_wgrad_*head.md): both run
//    the LM-head shape at the same MFMA cycles, 77 % L2 hit rate, 8.4 TB/s L2->LDS, and the
//    wave-cycle count puts the shader clock near 1.7 GHz under this load: ~60 % MFMA-busy at the
//    clock the chip holds.  Also measured slower (6-10 %): fragments of k-step k+1 read into a second
//    register set while step k's 8 MFMAs run, fenced by sched_barriers (256 VGPRs;
//    profiles/r2_wgrad_regpipe_negative.jsonl) -- hipcc's own interleave of 2 reads per 2 MFMAs wins.
//    And 6-14 % slower: 4 waves (one per SIMD) with 128x128 sub-tiles in AGPRs, i.e. 128 instead of
//    192 KiB of LDS reads per stage (profiles/r2_wgrad_4wave_negative.jsonl) -- LDS read volume is not
//    the limiter; the second wave per SIMD covering the per-stage barrier / DMA latency is worth more.
// Requires M % 64 == 0 and P, Q multiples of 8 (checked by the host binding).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "kernels.h"

// Measured and removed (records kept in profiles/): spreading the next stage's DMA over the k-steps
// (0-6 % slower), loader / consumer waves (12-14 % slower), global_load_lds instead of buffer_load ... lds,
// a wave-4-7 DMA stagger, XCD-aligned slice counts (slower in the step, r3s3_wgrad_slices.jsonl) and the
// symmetric (every wave loading) DMA plan (1-8 % slower than the asymmetric one, r3_wgrad_asym_ab.md).

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

PL_DEV f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
PL_DEV f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
PL_DEV s16x4 ds_tr(const uint16_t* p) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p); }
PL_DEV bf16x8 cat_tr(const s16x4& lo, const s16x4& hi) {
  s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}
// buffer-descriptor form (srd_of / blds16): common.h
PL_DEV int acc_row(int i, int half) { return (i & 3) + 8 * (i >> 2) + 4 * half; }

// [rows][128] bf16 image, 16-B chunk ch of row r at ch ^ f(r) (conflict-free tr reads)
PL_DEV int swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
PL_DEV int img_off(int r, int col) { return r * 128 + (((col >> 3) ^ swz(r)) << 3) + (col & 7); }

constexpr int BT = 256;             // output tile (P and Q)
constexpr int BKM = 64;             // tokens per stage
constexpr int NT = 512;             // 8 waves
constexpr int HALF = BKM * 128;     // elements of one [64][128] image
constexpr int STAGE = 4 * HALF;     // A halves 0,1 then B halves 2,3 (64 KiB)

template <int MF, bool OF32>
__global__ __launch_bounds__(NT) void wgrad_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                   const uint16_t* __restrict__ B, int64_t ldb, int M, int P, int Q,
                                                   int S, int slice, float* __restrict__ part, void* __restrict__ out,
                                                   int accumulate, float* __restrict__ bpart) {
  constexpr int QUADS = BKM / 4;  // row-quads per image
  // 1-KiB pieces per wave and stage: waves 0-3 issue all 64 (16 each) and waves 4-7 none, so each
  // SIMD's partner wave computes while the loader wave is stuck issuing its burst
  constexpr int PPW = BKM / 4;
  __shared__ __attribute__((aligned(1024))) uint16_t smem[2 * STAGE];
  const int tiles_q = (Q + BT - 1) / BT, tiles_p = (P + BT - 1) / BT;
  const int ntiles = tiles_p * tiles_q;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int s = lid / ntiles, t = lid % ntiles;
  const int p0 = (t / tiles_q) * BT, q0 = (t % tiles_q) * BT;
  const int m_begin = s * slice;
  const int nstage = (min(M, m_begin + slice) - m_begin) / BKM;
  const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int wp = w >> 2, wq = w & 3;  // wave's 128x64 sub-tile
  const int g1 = (lane >> 4) & 1, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;

  // DMA plan: 64 pieces of 1 KiB per stage (operand x half x 16 row-quads), 8 per wave.
  // Lane l of a piece fills image row 4*quad + l/16, chunk position l%16, which holds
  // logical chunk (l%16) ^ swz(row).  Columns past P/Q are clamped to a valid chunk:
  // they only feed output rows/columns that are never stored.
  int dst[PPW];
#pragma unroll
  for (int k = 0; k < PPW; ++k) {
    const int pc = w * PPW + k, opnd = pc / (2 * QUADS), half = (pc / QUADS) & 1, quad = pc % QUADS;
    dst[k] = (opnd * 2 + half) * HALF + quad * 512;
  }
  const unsigned lds_base = (unsigned)(uintptr_t)smem;
  // buffer form: per-lane byte offsets within a stage (< 64 rows x ld x 2 B), loop-invariant
  uint32_t voff[PPW];
#pragma unroll
  for (int k = 0; k < PPW; ++k) {
    const int pc = w * PPW + k, opnd = pc / (2 * QUADS), half = (pc / QUADS) & 1, quad = pc % QUADS;
    const int row = 4 * quad + (lane >> 4);
    const int col = half * 128 + (((lane & 15) ^ swz(row)) << 3);
    voff[k] = opnd == 0 ? (uint32_t)((row * lda + min(p0 + col, P - 8)) * 2)
                        : (uint32_t)((row * ldb + min(q0 + col, Q - 8)) * 2);
  }
  // pieces [k0, k1) of stage st's DMA plan
  const bool loader = w < 4;
  auto issue = [&](int st) {
    if (!loader) return;
    const int slot = st & 1;
    const int64_t m0 = (int64_t)m_begin + (int64_t)st * BKM;
    const i32x4v sa = srd_of(A + m0 * lda, (uint32_t)(BKM * lda * 2));
    const i32x4v sb = srd_of(B + m0 * ldb, (uint32_t)(BKM * ldb * 2));
#pragma unroll
    for (int k = 0; k < PPW; ++k) {
      const int opnd = (w * PPW + k) / (2 * QUADS);
      blds16(opnd == 0 ? sa : sb, voff[k], lds_base + 2u * (unsigned)(slot * STAGE + dst[k]));
    }
  };

  // MF = 32: 4x2 v_mfma_f32_32x32x16_bf16 accumulators per wave (128x64 sub-tile);
  // MF = 16: 8x4 v_mfma_f32_16x16x32_bf16 accumulators -- same LDS traffic per FLOP.
  constexpr int NI = MF == 32 ? 4 : 8, NJ = MF == 32 ? 2 : 4;
  using Acc = typename std::conditional<MF == 32, f32x16, f32x4>::type;
  constexpr int NE = MF == 32 ? 16 : 4;
  Acc acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int e = 0; e < NE; ++e) acc[i][j][e] = 0.f;

  // Fused bias gradient (bpart != null, MF = 16): the column sums of dY over the slice's tokens,
  // db[p] = sum_m dY[m, p], as MFMAs against an all-ones B fragment -- out[p][q'] = sum_m dY[m, p] for
  // every q' -- run by the workgroups of the first Q tile only, each wave taking 2 of the 8 A
  // fragments of its 128-row half (+2 MFMAs per 32; exact fp32 sums of the bf16 inputs, fixed
  // order).  Replaces a separate column-sum pass over dY (the QKV projection's bias gradient).
  const bool do_b = MF == 16 && bpart != nullptr && (t % tiles_q) == 0;
  f32x4 bacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  const bf16x8 ones = __builtin_bit_cast(bf16x8, u32x4{0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u});
  if (nstage > 0) issue(0);
  for (int st = 0; st < nstage; ++st) {
    const int slot = st & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // stage st landed for every wave; nobody still reads the other slot
    // the next stage's DMA: sixteen 1-KiB pieces per loader wave, issued as one burst after the
    // barrier (profiles/r3_wgrad_stamps.md)
    if (st + 1 < nstage) issue(st + 1);
    const uint16_t* Ai = smem + slot * STAGE + wp * HALF;
    const uint16_t* Bi = smem + slot * STAGE + (2 + (wq >> 1)) * HALF;
    const int bcol = (wq & 1) * 64;
    if constexpr (MF == 32) {
#pragma unroll
      for (int k16 = 0; k16 < BKM / 16; ++k16) {
        const int row = k16 * 16 + 8 * hh + tq;
        bf16x8 af[4], bfr[2];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int col = 32 * i + 16 * g1 + 4 * tp;
          af[i] = cat_tr(ds_tr(Ai + img_off(row, col)), ds_tr(Ai + img_off(row + 4, col)));
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int col = bcol + 32 * j + 16 * g1 + 4 * tp;
          bfr[j] = cat_tr(ds_tr(Bi + img_off(row, col)), ds_tr(Bi + img_off(row + 4, col)));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(af[i], bfr[j], acc[i][j]);
      }
    } else {
      // 16x16x32 operand: lane l holds column l%16, reduction rows 8*(l/16) .. +7
      const int gq = lane >> 4;
#pragma unroll
      for (int k32 = 0; k32 < BKM / 32; ++k32) {
        const int row = k32 * 32 + 8 * gq + tq;
        bf16x8 af[8], bfr[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int col = bcol + 16 * j + 4 * tp;
          bfr[j] = cat_tr(ds_tr(Bi + img_off(row, col)), ds_tr(Bi + img_off(row + 4, col)));
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int col = 16 * i + 4 * tp;
          af[i] = cat_tr(ds_tr(Ai + img_off(row, col)), ds_tr(Ai + img_off(row + 4, col)));
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
        if constexpr (MF == 16) {
          if (do_b) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
              if ((i >> 1) == wq) bacc[i & 1] = mfma16(af[i], ones, bacc[i & 1]);
          }
        }
      }
    }
  }
  // accumulator element e of fragment (i, j) -> output (row p, column q) of the tile
  auto prow = [&](int i, int e) {
    return MF == 32 ? p0 + wp * 128 + 32 * i + acc_row(e, hh) : p0 + wp * 128 + 16 * i + 4 * (lane >> 4) + e;
  };
  auto qcol = [&](int j) { return MF == 32 ? q0 + wq * 64 + 32 * j + r : q0 + wq * 64 + 16 * j + (lane & 15); };
  if (do_b && (lane & 15) == 0) {
    // column 0 of the all-ones product: rows p0 + wp 128 + 16 i + 4 (lane / 16) + e, i = 2 wq + k;
    // slice s's partial row of the fp32 [S][P] slab (summed in slice order by wgrad_reduce_kernel)
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int p = p0 + wp * 128 + 16 * (2 * wq + k) + 4 * (lane >> 4) + e;
        if (p < P) bpart[(int64_t)s * P + p] = bacc[k][e];
      }
  }
  if (S == 1) {
    // single slice: add the tile straight into the gradient
#pragma unroll
    for (int i = 0; i < NI; ++i) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int q = qcol(j), qc = min(q, Q - 1);
        float old[NE];
#pragma unroll
        for (int e = 0; e < NE; ++e) {  // all loads first (clamped, unconditional), then the stores
          const int p = min(prow(i, e), P - 1);
          old[e] = accumulate ? ldg1<OF32>(out, (int64_t)p * Q + qc) : 0.f;
        }
#pragma unroll
        for (int e = 0; e < NE; ++e) {
          const int p = prow(i, e);
          if (p < P && q < Q) stg1<OF32>(out, (int64_t)p * Q + q, acc[i][j][e] + old[e]);
        }
      }
    }
    return;
  }
  // fp32 partial tile -> slab[s][P][Q]
  float* dstp = part + (int64_t)s * P * Q;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int q = qcol(j);
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        const int p = prow(i, e);
        if (p < P && q < Q) dstp[(int64_t)p * Q + q] = acc[i][j][e];
      }
    }
  }
}

// dW[p, q] (+)= sum_s slab[s][p][q]   (8 columns per thread, fixed slice order)
template <bool OF32>
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int S, int64_t PQ,
                                                           void* __restrict__ out, int accumulate) {
  const int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) * 8;
  if (i >= PQ) return;
  char* const o = reinterpret_cast<char*>(out) + i * (OF32 ? 4 : 2);
  float f[8];
  if (accumulate) {
    ld8g<OF32>(o, f);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = 0.f;
  }
  // four slices' loads in flight before their adds (slice order kept: deterministic)
  int s = 0;
  for (; s + 4 <= S; s += 4) {
    f32x4 v[4][2];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f32x4* p = reinterpret_cast<const f32x4*>(part + (s + u) * PQ + i);
      v[u][0] = p[0];
      v[u][1] = p[1];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f[j] += v[u][0][j];
        f[4 + j] += v[u][1][j];
      }
  }
  for (; s < S; ++s) {
    const f32x4* p = reinterpret_cast<const f32x4*>(part + s * PQ + i);
    const f32x4 a = p[0], b = p[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f[j] += a[j];
      f[4 + j] += b[j];
    }
  }
  st8g<OF32>(o, f);
}

}  // namespace

namespace pllm {

// Variant selection (wgrad_set_mfma): 0 = default -- the ping-pong kernel of wgrad_pp.hip where it
// applies (fp32 gradient target), else this file's kernel per shape; 100 = this file's kernel per
// shape; 116 / 132 (or 16 / 32) = this file's kernel with that MFMA shape.
// Same-box A/B of this file's variants (profiles/r3_wgrad_asym_ab.md): the asymmetric DMA is +1-8 %
// over the symmetric kernel; 16x16x32 wins everywhere except the LM-head shapes (P = vocabulary),
// where 32x32x16 does (+0.5-4 %)
static int g_wgrad_mfma = 0;
static bool g_wgrad_pp = true;
void wgrad_set_mfma(int mf) {
  g_wgrad_pp = mf == 0;
  const int v = mf % 100;
  g_wgrad_mfma = v == 0 ? 0 : (v == 16 ? 16 : 32);
}

// A/B switch for slice-count sweeps (bench/wgrad_slices.py): > 0 forces that many slices
static int g_wgrad_force_s = 0;
void wgrad_force_slices(int s) { g_wgrad_force_s = s > 0 ? s : 0; }

void wgrad_plan(int M, int P, int Q, int* S, int* slice) {
  // Split-K slice count from a cost model: rounds of 256 workgroups (one per CU) x stages per
  // slice x ~2.0 us per 256x256x64 stage, plus -- for S > 1 -- the fp32 slab traffic (S slabs
  // written by the main kernel and read back by the reduce) at ~4 TB/s.  The slab term is what
  // keeps S small when P x Q is large (llama MLP: 11008 x 2048 at 16K tokens -> S = 2, not 11).
  // >= 8 stages per slice; near-ties (< 2 %) go to fewer slices.
  const int ntiles = ((P + BT - 1) / BT) * ((Q + BT - 1) / BT);
  const int kst = M / BKM;
  int best = 1;
  double best_t = 1e30, best_eff = 0.0;
  for (int s = 1; s <= 64; ++s) {
    if (s > 1 && kst / s < 8) break;
    const int n = ntiles * s;
    const int rounds = (n + 255) / 256;
    const int st_per = (kst + s - 1) / s;
    double t = rounds * (double)st_per * 2.0e-6;
    if (s > 1) t += (double)P * Q * 4.0 * (2 * s + 1) / 4.0e12;
    if (t < best_t * 0.98) {
      best_t = t;
      best = s;
    }
  }
  if (g_wgrad_force_s > 0) best = std::min(g_wgrad_force_s, std::max(1, kst));
  int st_per = (kst + best - 1) / best;
  *slice = st_per * BKM;
  *S = (kst + st_per - 1) / st_per;
}

int wgrad_bias_slices(int M, int P, int Q) {
  int S, slice;
  wgrad_plan(M, P, Q, &S, &slice);
  return S;
}

// hybrid weight gradients (wgrad_pp_hy), default on: with more tiles than CUs, whole tiles for the whole
// rounds and slices only for the last one -- LM head 65536 x 50304 x 768 3,984 vs 4,081 us, 32768 x 50304 x
// 2048 5,190 vs 5,721 us, GPT-2 step +0.3 %, llama +0.2-0.3 % (profiles/r4_wgrad_hybrid.md).  On the
// persistent grid only (whole rounds of one tile per CU); with a grid per tile the hardware deals the tiles
// anyway.  (Full stream-K -- equal K-tile runs per workgroup -- lost 13-47 %: r4_wgrad_stream_k_negative.md)
static int g_wgrad_hy = 1;
void wgrad_set_hy(int on) { g_wgrad_hy = on; }

static bool wgrad_use_hy(int M, int P, int Q, bool out_f32, bool bias) {
  int full, rem, S, skt;
  return g_wgrad_hy && g_wgrad_pp && out_f32 && !bias && gemm_grid_cap() < (1 << 29) &&
         wgrad_hy_plan(M, P, Q, gemm_grid_cap(), &full, &rem, &S, &skt);
}

int64_t wgrad_ws_floats(int M, int P, int Q, bool out_f32, bool bias) {
  if (wgrad_use_hy(M, P, Q, out_f32, bias)) return wgrad_pp_hy_ws_floats(M, P, Q, gemm_grid_cap());
  int S, slice;
  wgrad_plan(M, P, Q, &S, &slice);
  return S > 1 ? (int64_t)S * P * Q : 0;
}

bool wgrad(const void* dy, int64_t lda, const void* x, int64_t ldb, int M, int P, int Q, float* part, void* out,
           bool out_f32, bool accumulate, hipStream_t st, float* bpart, void* bout, bool bout_f32) {
  if (wgrad_use_hy(M, P, Q, out_f32, bpart != nullptr && bout != nullptr)) {
    wgrad_pp_hy(dy, lda, x, ldb, M, P, Q, part, (float*)out, accumulate, gemm_grid_cap(), st);
    return false;
  }
  int S, slice;
  wgrad_plan(M, P, Q, &S, &slice);
  const int ntiles = ((P + BT - 1) / BT) * ((Q + BT - 1) / BT);
  if (g_wgrad_pp && out_f32 && wgrad_pp_supported(M, P, Q, S, slice)) {
    const bool fb = bpart != nullptr && bout != nullptr;
    wgrad_pp(dy, lda, x, ldb, M, P, Q, S, slice, part, (float*)out, accumulate, fb ? bpart : nullptr,
             gemm_grid_cap(), st);
    if (fb) {
      const dim3 bg((unsigned)((P / 8 + 255) / 256));
      if (bout_f32) hipLaunchKernelGGL(wgrad_reduce_kernel<true>, bg, dim3(256), 0, st, bpart, S, (int64_t)P, bout, 1);
      else hipLaunchKernelGGL(wgrad_reduce_kernel<false>, bg, dim3(256), 0, st, bpart, S, (int64_t)P, bout, 1);
    }
    if (S > 1) {
      const int64_t PQ = (int64_t)P * Q;
      const dim3 rg((unsigned)((PQ / 8 + 255) / 256));
      hipLaunchKernelGGL(wgrad_reduce_kernel<true>, rg, dim3(256), 0, st, part, S, PQ, out, (int)accumulate);
    }
    return fb;
  }
  const int mfma = g_wgrad_mfma != 0 ? g_wgrad_mfma : (P >= 16384 ? 32 : 16);
  // the bias gradient rides along only on the 16x16x32 kernel (see wgrad_kernel)
  const bool fuse_b = bpart != nullptr && bout != nullptr && mfma == 16;
  float* const bp = fuse_b ? bpart : nullptr;
#define PL_WGRAD_LAUNCH(MFV, OF)                                                                           \
  hipLaunchKernelGGL((wgrad_kernel<MFV, OF>), dim3(ntiles * S), dim3(NT), 0, st, (const uint16_t*)dy, lda, \
                     (const uint16_t*)x, ldb, M, P, Q, S, slice, part, out, (int)accumulate, bp)
  if (mfma == 16) {
    if (out_f32) PL_WGRAD_LAUNCH(16, true);
    else PL_WGRAD_LAUNCH(16, false);
  } else {
    if (out_f32) PL_WGRAD_LAUNCH(32, true);
    else PL_WGRAD_LAUNCH(32, false);
  }
#undef PL_WGRAD_LAUNCH
  if (fuse_b) {  // bias gradient: the [S][P] partial rows summed in slice order into bout
    const dim3 bg((unsigned)((P / 8 + 255) / 256));
    if (bout_f32) hipLaunchKernelGGL(wgrad_reduce_kernel<true>, bg, dim3(256), 0, st, bpart, S, (int64_t)P, bout, 1);
    else hipLaunchKernelGGL(wgrad_reduce_kernel<false>, bg, dim3(256), 0, st, bpart, S, (int64_t)P, bout, 1);
  }
  if (S == 1) return fuse_b;
  const int64_t PQ = (int64_t)P * Q;
  const dim3 rg((unsigned)((PQ / 8 + 255) / 256));
  if (out_f32) hipLaunchKernelGGL(wgrad_reduce_kernel<true>, rg, dim3(256), 0, st, part, S, PQ, out, (int)accumulate);
  else hipLaunchKernelGGL(wgrad_reduce_kernel<false>, rg, dim3(256), 0, st, part, S, PQ, out, (int)accumulate);
  return fuse_b;
}

}  // namespace pllm

// Ping-pong TN GEMM with fused epilogues on gfx950 MFMA (round 4):
//     C[M, N] = epi( A[M, K] . B[N, K]^T )          (bf16 in, fp32 accumulate, bf16 out)
// Same contract and epilogues as gemm_tn_kernel (csrc/gemm.hip, which stays as the A/B
// reference); a structurally different main loop, built for the measured bottleneck of that
// kernel: its waves parked 36 % of the time on the one barrier + vmcnt(0) per 64-deep K-tile
// (profiles/r3_gemm_tn.md: MFMA busy 41 % vs hipBLASLt's 52 %).  Reference math: the MLP and
// attention projections of /root/reference/src/models/mlp.py:24-26 and attention.py:29-31.
//
// Design (cdna_hip_programming.md §5 "8-phase", T3/T4/T5; MI355X_MICROARCH.md "Two waves per
// SIMD"):
//  * 256x256 output tile per 512-thread workgroup, persistent over tiles (grouped order, XCD-aware
//    block remap); wave (wr, wc) owns rows wr*128 + [0,128) and columns wc*64 + [0,64): 8 x 4
//    MFMA 16x16x32 accumulators (128 fp32 per lane);
//  * a 64-deep K-tile is 4 PHASES, each one 64x32 quadrant of the wave's tile (16 MFMAs); the
//    two wave groups (waves 0-3 = rows 0-127, waves 4-7 = rows 128-255; one wave of each on every
//    SIMD) run one barrier apart (group 1 takes an extra s_barrier up front), so on every SIMD one
//    wave issues its 16 MFMAs while its partner reads the next quadrant's fragments and issues its
//    share of the next K-tile's DMA: the matrix pipe alternates between the two waves instead of
//    idling at a shared barrier;
//  * K-tile s+1 is DMA'd (buffer_load ... lds, 1 KiB pieces, XOR-swizzled images through the
//    per-lane SOURCE address) during K-tile s's four phases, in the order of first use (A rows of
//    both groups' first quadrant, B columns of the first quadrant, B columns of the second, A rows
//    of the second): every piece has >= 3 phases to land, and each phase waits with a COUNTED
//    vmcnt(4) (never 0 in the main loop) before its barrier;
//  * one VGPR offset per operand and piece parity; a piece's row offset goes into the buffer
//    descriptor's base (scalar), so the DMA plan costs 4 VGPRs instead of one per piece (the
//    spill that sank the round-3 one-wave-per-SIMD variant);
//  * the B image rows are permuted inside each 32-row block (image row 16h + 4g + r <- column
//    8g + 4h + r) so that the accumulators of column tiles 2p and 2p+1 hold 8 CONSECUTIVE output
//    columns per lane: the epilogue stores 16 B per lane straight from registers (no LDS round
//    trip), with bias / GELU / ReLU / GELU' / ReLU' / SwiGLU' / attention-delta math on the way;
//  * the epilogue is NOT a burst at the end of a tile (measured: 128 KiB of stores per CU, issued
//    by every CU at once, parked both wave groups ~4.5k cycles per tile -- 20 % of the kernel at
//    K = 768): the previous tile's epilogue runs one accumulator QUADRANT per phase inside the
//    next tile's first K-tile, each quadrant just before that phase's MFMAs overwrite it; its
//    bias / aux rows come through a per-wave 4 KiB LDS area by DMA issued one phase ahead, and
//    every wait is a count that leaves the stores outstanding (no load of the main loop is issued
//    by the compiler, so no compiler wait drains them).  EPI 5 (SwiGLU backward, 8 KiB of aux per
//    wave and quadrant) keeps the end-of-tile epilogue.
// Requires K % 64 == 0, N % 8 == 0, lda / ldc / ldaux % 8 == 0 (checked by the binding).
#include "common.h"
#include "kernels.h"

// Measured and removed in round 5 (records kept in profiles/): a desynchronising tile split (odd
// workgroups run half of their last tile first and park it; slower, r4_gemm_pp_split_ab.jsonl), a
// start-time stagger of odd workgroups, the K-tile DMA pieces issued among the MFMAs instead of in the
// LOAD segment, a static priority for waves 4-7 instead of per-segment flips, and the
// ablation / s_memtime-stamp diagnostic builds.

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int PT = 256;            // output tile (M and N)
constexpr int PBK = 64;            // K per K-tile
constexpr int PNT = 512;           // 8 waves
constexpr int PIMG = PT * PBK;     // elements of one operand image [256][64]
constexpr int PSLOT = 2 * PIMG;    // A image then B image: 64 KiB
constexpr uint32_t kPOff = 0x80000000u;  // a byte offset past every descriptor built here

PL_DEV bf16x8 ldsf(const uint16_t* p) { return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(p)); }
PL_DEV f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
PL_DEV void pp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
template <int N>
PL_DEV void pp_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// grouped tile order: GROUP_M m-tiles x all n-tiles, m fastest inside a group
PL_DEV void pp_tile(int t, int tiles_m, int tiles_n, int gm, int& tm, int& tn) {
  const int per_group = gm * tiles_n;
  const int grp = t / per_group, first_m = grp * gm, gsize = min(gm, tiles_m - first_m);
  tm = first_m + (t % per_group) % gsize;
  tn = (t % per_group) / gsize;
}

// Two epilogue placements (template flag QE, chosen per call by gemm_pp_quad_epilogue):
//  * end of tile (QE = false): the vector-memory instructions it issues after its last wait
//    (its stores; a lower bound) are what the counted waits of the next tile's first phases
//    leave outstanding;
//  * quadrant epilogues (QE = true; K >= 2048, every EPI but 5, whose 8 KiB of aux rows per wave
//    and quadrant do not fit the LDS): kAuxN DMA ops of the bias / aux rows of one quadrant, and
//    kStQ stores of one quadrant epilogue (C, the EPI 1 pre-activation, the EPI 3 / 4 column-sum
//    partials, the EPI 6 delta on the second column pair).  Measured: faster at K = 3072 / 5504
//    (fewer, longer tiles), slower at K = 768 (the epilogue work lands in the critical LOAD
//    segments of four phases per tile).
#ifndef PL_PP_EPI5_PFD
#define PL_PP_EPI5_PFD 2  // row tiles of SwiGLU-backward aux loads in flight ahead of the one processed
#endif

template <int EPI>
constexpr int kEndStores = (EPI == 1 || EPI == 5) ? 32 : EPI == 7 ? 24 : 16;
// EPI 7 (SwiGLU forward of the llama up-projection, W1 = [gate | up] rows): a tile is 128 output
// columns whose gate AND up weight rows form the 256-row B panel -- wave wc's column pair 0 holds
// gate rows wc*32 + [0,32), its pair 1 the up rows of the same columns -- so every lane holds
// gate and up of the same 8 columns: a = silu(g) * u in registers, [g | u] kept for the backward
template <int EPI>
constexpr int kNT = EPI == 7 ? 128 : PT;
template <int EPI>
constexpr int kAuxN = EPI <= 2 ? 1 : 4;
template <int EPI>
constexpr int kStQ(int q) {
  return EPI == 1 ? 8 : (EPI == 3 || EPI == 4) ? 6 : EPI == 6 ? ((q & 1) ? 8 : 4) : 4;
}

PL_DEV void pp_st16(__amdgpu_buffer_rsrc_t r, uint32_t off, const u32x4& v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
}
PL_DEV float bfr(float x) { return bf2f(f2bf_bits(x)); }  // round to bf16 and back
PL_DEV float pp_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

// ---------------------------------------------------------------------------------------------
// Epilogue of one 256x256 tile, straight from the accumulators.  Lane (r16 = lane & 15,
// g = lane >> 4) holds, for row tile j and column pair p, output row wr*128 + 16j + r16 and the 8
// columns wc*64 + 32p + 8g + [0, 8): acc[2p][j][0..3] then acc[2p+1][j][0..3].
template <int EPI>
PL_DEV void pp_epilogue(f32x4 (&acc)[4][8], const pllm::GemmArgs& g, int tm, int tn, int wr, int wc, int lane) {
  const int M = g.M, N = g.N;
  const int m0 = tm * PT, n0 = tn * PT;
  const int rows_ok = min(PT, M - m0);
  constexpr int W2 = EPI == 5 ? 2 : 1;  // EPI 5: C and aux rows hold two N-wide halves
  const __amdgpu_buffer_rsrc_t crs = rows_rsrc(g.C + (int64_t)m0 * g.ldc, rows_ok, g.ldc, W2 * N);
  const __amdgpu_buffer_rsrc_t ars =
      rows_rsrc(g.aux != nullptr ? g.aux + (int64_t)m0 * g.ldaux : g.C, rows_ok, g.ldaux, W2 * N);
  const int r16 = lane & 15, g4 = lane >> 4;
  const int colw = n0 + wc * 64 + 8 * g4;  // + 32 p
  const bool cok0 = colw < N, cok1 = colw + 32 < N;
  float bias[2][8];
  if constexpr (EPI <= 2) {
    const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(g.bias != nullptr ? g.bias : g.A), (short)0, g.bias != nullptr ? N * 2 : 0, 0x00020000);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const bool ok = p == 0 ? cok0 : cok1;
      unpack8(buf_ld16(brs, ok ? (uint32_t)(colw + 32 * p) * 2u : kPOff), bias[p]);
    }
  }
  float csum[2][8];
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int e = 0; e < 8; ++e) csum[p][e] = 0.f;
  const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(g.delta != nullptr ? g.delta : (float*)g.C), (short)0, EPI == 6 ? (int)(4ll * M * N / 64) : 0,
      0x00020000);
  // aux rows (EPI >= 3) one row tile ahead: the loads of tile j + 1 fly while tile j is processed,
  // and the scheduling barrier at the end of each tile keeps the compiler from hoisting all 16-32
  // loads to the top, where the 128 accumulators are still live (that spilled)
  constexpr int NAX = EPI >= 3 ? (EPI == 5 ? 4 : 2) : 0;
  // EPI 5 (four loads per row tile; all 32 up front do not fit beside the accumulators): a ring of
  // PFD + 1 row tiles, the loads of row tile j + PFD issued before tile j is processed
  constexpr int PFD = PL_PP_EPI5_PFD;
  u32x4 axc[NAX > 0 ? NAX : 1], axn[NAX > 0 ? NAX : 1];
  u32x4 axr[EPI == 5 ? PFD + 1 : 1][NAX > 0 ? NAX : 1];
  auto aux_load = [&](int j, u32x4* dst) {
    if constexpr (NAX > 0) {
      const int rt = wr * 128 + 16 * j + r16;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const bool ok = p == 0 ? cok0 : cok1;
        const uint32_t aoff = ok ? (uint32_t)(((int64_t)rt * g.ldaux + colw + 32 * p) * 2) : kPOff;
        dst[p] = buf_ld16(ars, aoff);
        if constexpr (EPI == 5) dst[2 + p] = buf_ld16(ars, ok ? aoff + (uint32_t)N * 2u : kPOff);
      }
    }
  };
  // EPI 3 / 4 / 6 (two loads per row tile): all 16 issued up front instead -- one round trip
  // per tile, not eight (the pipelined form cost ~1k cycles per row tile under load)
  constexpr bool PRE = EPI == 3 || EPI == 4 || EPI == 6;
  u32x4 axall[PRE ? 8 : 1][2];
  if constexpr (PRE) {
#pragma unroll
    for (int j = 0; j < 8; ++j) aux_load(j, axall[j]);
  } else if constexpr (EPI == 5 && PFD > 1) {
#pragma unroll
    for (int d = 0; d < PFD; ++d) aux_load(d, axr[d]);
  } else {
    aux_load(0, axc);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int rt = wr * 128 + 16 * j + r16;  // row within the tile
    if constexpr (EPI == 5 && PFD > 1) {
      if (j + PFD < 8) aux_load(j + PFD, axr[(j + PFD) % (PFD + 1)]);
#pragma unroll
      for (int x = 0; x < NAX; ++x) axc[x] = axr[j % (PFD + 1)][x];
    } else if constexpr (!PRE) {
      if (j + 1 < 8) aux_load(j + 1, axn);
    } else {
      axc[0] = axall[j][0];
      axc[1] = axall[j][1];
    }
    float dsum = 0.f;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const bool ok = p == 0 ? cok0 : cok1;
      const int col = colw + 32 * p;
      const uint32_t off = ok ? (uint32_t)(((int64_t)rt * g.ldc + col) * 2) : kPOff;
      const uint32_t aoff = ok ? (uint32_t)(((int64_t)rt * g.ldaux + col) * 2) : kPOff;
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc[2 * p][j][e];
        v[4 + e] = acc[2 * p + 1][j][e];
      }
      if constexpr (EPI == 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += bias[p][e];
        pp_st16(crs, off, pack8(v));
      } else if constexpr (EPI == 1) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += bias[p][e];
        const u32x4 pre = pack8(v);
        float f[8];
        unpack8(pre, f);  // the activation reads the bf16-rounded pre-activation
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = gelu_f(f[e]);
        pp_st16(ars, aoff, pre);
        pp_st16(crs, off, pack8(f));
      } else if constexpr (EPI == 2) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e] + bias[p][e], 0.f);
        pp_st16(crs, off, pack8(v));
      } else if constexpr (EPI == 3 || EPI == 4) {
        float a[8];
        unpack8(axc[p], a);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = bfr(v[e]);  // the unfused path's bf16 data gradient
          v[e] = EPI == 3 ? d * gelu_df(a[e]) : (a[e] > 0.f ? d : 0.f);
        }
        const u32x4 o = pack8(v);
        pp_st16(crs, off, o);
        unpack8(o, v);  // the bias gradient sums the bf16-rounded values, like act_bwd_colsum
#pragma unroll
        for (int e = 0; e < 8; ++e) csum[p][e] += v[e];
        __builtin_amdgcn_sched_barrier(0);  // one 8-column group of GELU' math at a time
      } else if constexpr (EPI == 5) {
        float gt[8], up[8], dg[8], du[8];
        unpack8(axc[p], gt);
        unpack8(axc[2 + p], up);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = bfr(v[e]);
          const float sg = pp_sigmoid(gt[e]);
          du[e] = d * (gt[e] * sg);
          dg[e] = d * up[e] * sg * (1.f + gt[e] * (1.f - sg));
        }
        pp_st16(crs, off, pack8(dg));
        pp_st16(crs, ok ? off + (uint32_t)N * 2u : kPOff, pack8(du));
      } else {  // EPI 6: dO stored; delta = sum over the wave's 64 columns (one head) of dO * O
        const u32x4 o = pack8(v);
        pp_st16(crs, off, o);
        float d[8], oo[8];
        unpack8(o, d);
        unpack8(axc[p], oo);
#pragma unroll
        for (int e = 0; e < 8; ++e) dsum = __builtin_fmaf(d[e], oo[e], dsum);
      }
    }
    if constexpr (EPI == 6) {
      // the row's 4 lane groups (g = 0..3: lanes r16, r16 + 16, + 32, + 48) in a fixed order
      dsum += __shfl_xor(dsum, 16, 64);
      dsum += __shfl_xor(dsum, 32, 64);
      const int m = m0 + rt;
      const int bq = m / g.T, tq = m - bq * g.T, hd = (n0 + wc * 64) >> 6;
      const uint32_t doff = (g4 == 0 && m < M && cok0)
                                ? (uint32_t)((((int64_t)bq * (N >> 6) + hd) * g.T + tq) * 4) : kPOff;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, dsum), drs, doff, 0, 0);
    }
    if constexpr (NAX > 0 && !PRE) {
      if constexpr (!(EPI == 5 && PFD > 1)) {
#pragma unroll
        for (int x = 0; x < NAX; ++x) axc[x] = axn[x];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if constexpr (EPI == 3 || EPI == 4) {
    // lanes r16 = 0..15 of a lane group hold the same 8 columns; rows past M contributed zeros
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float s = csum[p][e];
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        s += __shfl_xor(s, 4, 64);
        s += __shfl_xor(s, 8, 64);
        csum[p][e] = s;
      }
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(g.colpart + (int64_t)(2 * tm + wr) * N), (short)0, N * 4, 0x00020000);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const bool ok = (p == 0 ? cok0 : cok1) && r16 == 0;
      const uint32_t po = ok ? (uint32_t)(colw + 32 * p) * 4u : kPOff;
      pp_st16(prs, po, __builtin_bit_cast(u32x4, f32x4{csum[p][0], csum[p][1], csum[p][2], csum[p][3]}));
      pp_st16(prs, ok ? po + 16u : kPOff,
              __builtin_bit_cast(u32x4, f32x4{csum[p][4], csum[p][5], csum[p][6], csum[p][7]}));
    }
  }
}


// EPI 7 epilogue (end of tile): per row tile the lane's gate (pair 0) and up (pair 1) values of
// columns n0 + wc*32 + 8g + [0, 8) -> [g | u] rounded to bf16 into aux [M, 2F] and
// a = silu(g) * u from those bf16 values (swiglu_fwd_kernel's numerics) into C [M, F]: 24 stores
PL_DEV void pp_epilogue_swiglu(f32x4 (&acc)[4][8], const pllm::GemmArgs& g, int tm, int tn, int wr, int wc,
                                 int lane) {
  const int M = g.M, F = g.N;
  const int m0 = tm * PT, n0 = tn * 128;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int col = n0 + wc * 32 + 8 * g4;
  const bool ok = col < F;
  const uint32_t off = ok ? (uint32_t)(((int64_t)r16 * g.ldc + col) * 2) : kPOff;
  const uint32_t aoff = ok ? (uint32_t)(((int64_t)r16 * g.ldaux + col) * 2) : kPOff;
  const int rows_ok = min(PT, M - m0);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int r0 = wr * 128 + 16 * j;
    const int rows_j = max(0, rows_ok - r0);
    const __amdgpu_buffer_rsrc_t crs = rows_rsrc(g.C + (int64_t)(m0 + r0) * g.ldc, rows_j, g.ldc, F);
    const __amdgpu_buffer_rsrc_t ars = rows_rsrc(g.aux + (int64_t)(m0 + r0) * g.ldaux, rows_j, g.ldaux, 2 * F);
    float gt[8], up[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      gt[q] = acc[0][j][q];
      gt[4 + q] = acc[1][j][q];
      up[q] = acc[2][j][q];
      up[4 + q] = acc[3][j][q];
    }
    const u32x4 gp = pack8(gt), upk = pack8(up);
    unpack8(gp, gt);
    unpack8(upk, up);
#pragma unroll
    for (int q = 0; q < 8; ++q) gt[q] = gt[q] * pp_sigmoid(gt[q]) * up[q];
    pp_st16(ars, aoff, gp);
    pp_st16(ars, ok ? aoff + (uint32_t)F * 2u : kPOff, upk);
    pp_st16(crs, off, pack8(gt));
    __builtin_amdgcn_sched_barrier(0);
  }
}

// ---------------------------------------------------------------------------------------------
struct PPCtx {
  const pllm::GemmArgs* g;
  int w, wr, wc, lane;
  unsigned lds;           // byte address of the LDS array
  uint16_t* aux;          // this wave's 4 KiB bias / aux staging area (after the two K-tile slots)
  uint32_t vo[2][2];      // per-lane DMA source offsets of this wave's pieces of groups 0 (A) / 1 (B)
                          // (groups 3 / 2 are the same rows + 64 (A) / + 32 (B): descriptor base)
  uint32_t vaux;          // per-lane source offset of the aux DMA (row lane / 4, 16-B chunk lane % 4)
  unsigned rdA[2], rdB[2];  // per-lane LDS byte offsets of the fragment reads (k32 = 0, 1), slot 0
};

struct PPEpi {  // the tile whose (quadrant) epilogue is in flight
  int tm, tn;
  bool valid;   // false: the kernel's first tile has no predecessor (stores go nowhere)
};

// Descriptors of the DMA target K-tile's A and B panels (256 rows from the K-tile's first column,
// range-checked: rows past M / N read zeros); valid = false: empty ranges (the same instructions
// issue, so the counted waits stay exact; nothing reads that slot again).  Built once per K-tile:
// the pieces differ only in their per-lane offsets (PPCtx::vo), which hold the row.
struct PPSrd {
  i32x4v a, b, b2;  // b2: EPI 7's up-row panel (piece group 2)
};
template <int EPI>
PL_DEV PPSrd pp_srds(const PPCtx& c, int tm, int tn, int kt, bool valid) {
  const pllm::GemmArgs& g = *c.g;
  constexpr int NT = kNT<EPI>;
  const int ra = min(PT, g.M - tm * PT), rb = min(NT, g.N - tn * NT);
  const int64_t kleft2 = (int64_t)(g.K - kt * PBK) * 2;
  const uint32_t ba = valid ? (uint32_t)((int64_t)(ra - 1) * g.lda * 2 + kleft2) : 0u;
  const uint32_t bb = valid ? (uint32_t)((int64_t)(rb - 1) * g.ldb * 2 + kleft2) : 0u;
  const uint16_t* bp = g.B + (int64_t)tn * NT * g.ldb + kt * PBK;
  PPSrd r;
  r.a = srd_of(g.A + (int64_t)tm * PT * g.lda + kt * PBK, ba);
  r.b = srd_of(bp, bb);
  if constexpr (EPI == 7) r.b2 = srd_of(bp + (int64_t)g.N * g.ldb, bb);  // up rows N (= F) further
  return r;
}

// DMA piece group PH (2 pieces per wave) of the target K-tile into LDS slot sl, in the order of
// first use: 0 = A rows 0-63 of both row halves, 1 = B image rows of column pair 0 of every wave,
// 2 = B column pair 1, 3 = A rows 64-127 (distances to first use: 4, 3, 3, 3 phases).
template <int PH>
PL_DEV int pp_blk0(int w) {
  return PH == 0 ? 2 * w + 8 * (w >> 2)
         : PH == 1 ? 8 * (w >> 1) + 2 * (w & 1)
         : PH == 2 ? 4 + 8 * (w >> 1) + 2 * (w & 1)
                   : 8 + 2 * w + 8 * (w >> 2);
}
// shift a descriptor's base by `bytes` (its range shrinks by as much, clamped at 0)
PL_DEV i32x4v srd_shift(const i32x4v& r, uint32_t bytes) {
  const uint64_t a = ((uint64_t)(uint32_t)r[1] << 32 | (uint32_t)r[0]) + bytes;
  i32x4v o;  // (readfirstlane: the asm operand must provably live in SGPRs)
  o[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  o[1] = __builtin_amdgcn_readfirstlane((int)((uint32_t)(a >> 32) & 0xffffu));
  o[2] = __builtin_amdgcn_readfirstlane((uint32_t)r[2] > bytes ? (int)((uint32_t)r[2] - bytes) : 0);
  o[3] = r[3];
  return o;
}
// the descriptor and LDS address of piece group PH (pieces q = 0, 1 at + 1 KiB)
template <int PH, int EPI = 0>
PL_DEV void pp_group(const PPCtx& c, const PPSrd& srd, int sl, i32x4v& r, unsigned& lds0) {
  // (c.lds: the LDS array's own address, so the DMA asm visibly writes it)
  constexpr bool isA = PH == 0 || PH == 3;
  const int blk0 = pp_blk0<PH>(c.w);
  lds0 = c.lds + (unsigned)(sl * PSLOT + (isA ? 0 : PIMG) + blk0 * 512) * 2u;
  // groups 2 / 3: the pieces of groups 1 / 0 shifted by 4 (B: 32 rows) / 8 (A: 64 rows) pieces
  // (EPI 7: group 2 = the up rows of group 1's columns, from their own panel)
  r = PH < 2 ? (isA ? srd.a : srd.b)
             : (EPI == 7 && !isA) ? srd.b2
                                  : srd_shift(isA ? srd.a : srd.b,
                                              (uint32_t)(isA ? 64 * c.g->lda * 2 : 32 * c.g->ldb * 2));
}
template <int PH>
PL_DEV void pp_piece(const PPCtx& c, const i32x4v& r, unsigned lds0, int q) {
  constexpr bool isA = PH == 0 || PH == 3;
  blds16(r, c.vo[isA ? 0 : 1][q], lds0 + 1024u * (unsigned)q);
}
template <int PH, int EPI = 0>
PL_DEV void pp_issue(const PPCtx& c, const PPSrd& srd, int sl) {
  i32x4v r;
  unsigned lds0;
  pp_group<PH, EPI>(c, srd, sl, r, lds0);
#pragma unroll
  for (int q = 0; q < 2; ++q) pp_piece<PH>(c, r, lds0, q);
}

// ---------------------------------------------------------------------------------------------
// Quadrant epilogues.  Quadrant q = (rows half jh, column pair p) = (0,0) (0,1) (1,1) (1,0) of a wave's
// 128x64 tile: rows wr*128 + 16j + r16 (j = 4 jh .. 4 jh + 3), columns wc*64 + 32p + 8g + [0, 8)
// (lane: r16 = lane & 15, g = lane >> 4; acc[2p][j] then acc[2p+1][j]).
//
// The quadrant's bias (EPI <= 2: its 32 columns, 64 B) or aux rows (EPI 3 / 4 / 6: 64 rows x 32
// columns, 4 KiB) are DMA'd into the wave's own LDS area one phase ahead (kAuxN instructions);
// only this wave reads it, so its own counted vmcnt orders the reads.
// quadrant of phase q (snake order: one column-pair fragment set is re-read, not held)
constexpr int pp_qjh(int q) { return q >> 1; }
constexpr int pp_qp(int q) { return (q == 1 || q == 2) ? 1 : 0; }

template <int EPI, int Q>
PL_DEV void pp_aux_issue(const PPCtx& c, const PPEpi& e) {
  const pllm::GemmArgs& g = *c.g;
  constexpr int jh = pp_qjh(Q), p = pp_qp(Q);
  const int col0 = e.tn * PT + c.wc * 64 + 32 * p;
  const unsigned dst = (unsigned)(uintptr_t)c.aux;
  if constexpr (EPI <= 2) {
    const bool has = e.valid && g.bias != nullptr && col0 < g.N;
    const i32x4v srd = srd_of(g.bias != nullptr ? g.bias + (has ? col0 : 0) : g.A, has ? (uint32_t)(g.N - col0) * 2u : 0u);
    blds16(srd, c.lane < 4 ? (uint32_t)c.lane * 16u : kPOff, dst);  // lanes 0-3: 8 columns each
  } else {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int row0 = e.tm * PT + c.wr * 128 + 16 * (4 * jh + jj);
      const bool has = e.valid && row0 < g.M && col0 < g.N;
      const uint32_t bytes = has ? (uint32_t)((int64_t)(g.M - row0 - 1) * g.ldaux * 2 + (int64_t)(g.N - col0) * 2) : 0u;
      const uint16_t* base = has ? g.aux + (int64_t)row0 * g.ldaux + col0 : g.C;
      blds16(srd_of(base, bytes), c.vaux, dst + 1024u * (unsigned)jj);  // [jj][row 0..15][64 B]
    }
  }
}

// The epilogue of quadrant Q of tile e (its aux / bias already in the wave's LDS area and read
// into ax).  EPI 6's delta needs both column pairs of a row: dsum carries pair 0's partial to
// the pair-1 quadrant that follows it.  EPI 3 / 4 write the quadrant's column sums to colpart
// row 4 tm + 2 wr + jh (gemm_colsum_groups = 4 per tile row with this kernel).
template <int EPI, int Q>
PL_DEV void pp_epi_quad(f32x4 (&acc)[4][8], const PPCtx& c, const PPEpi& e, const u32x4 (&ax)[4],
                          float (&dsum)[4]) {
  const pllm::GemmArgs& g = *c.g;
  constexpr int jh = pp_qjh(Q), p = pp_qp(Q);
  constexpr bool first_of_half = (Q & 1) == 0;  // EPI 6: the row half's first column pair
  const int M = g.M, N = g.N;
  const int m0 = e.tm * PT, n0 = e.tn * PT;
  const int rows_ok = e.valid ? min(PT, M - m0) : 0;  // no predecessor: every store is dropped
  const int lane = c.lane, r16 = lane & 15, g4 = lane >> 4;
  const int col = n0 + c.wc * 64 + 32 * p + 8 * g4;
  const bool ok = col < N;
  // per row tile j a descriptor based at its first row (scalar), so the per-lane offsets are
  // the same for every j: one VGPR each instead of eight hoisted row offsets (those spilled)
  const uint32_t off = ok ? (uint32_t)(((int64_t)r16 * g.ldc + col) * 2) : kPOff;
  const uint32_t aoff = ok ? (uint32_t)(((int64_t)r16 * g.ldaux + col) * 2) : kPOff;
  float csum[8];
#pragma unroll
  for (int e2 = 0; e2 < 8; ++e2) csum[e2] = 0.f;
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const int j = 4 * jh + jj;
    const int r0 = c.wr * 128 + 16 * j;  // first row of the row tile within the tile
    const int rows_j = max(0, rows_ok - r0);
    const __amdgpu_buffer_rsrc_t crs = rows_rsrc(g.C + (int64_t)(e.valid ? m0 + r0 : 0) * g.ldc, rows_j, g.ldc, N);
    const __amdgpu_buffer_rsrc_t ars =
        rows_rsrc(g.aux != nullptr ? g.aux + (int64_t)(e.valid ? m0 + r0 : 0) * g.ldaux : g.C, EPI == 1 ? rows_j : 0,
                  g.ldaux, N);
    float v[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[q] = acc[2 * p][j][q];
      v[4 + q] = acc[2 * p + 1][j][q];
    }
    float bias[8];
    if constexpr (EPI <= 2) unpack8(ax[0], bias);  // (kept packed between row tiles)
    if constexpr (EPI == 0) {
      // (written as a max against an opaque -inf: the plain add made hipcc hoist and spill)
      float lo = -INFINITY;
      asm volatile("" : "+v"(lo));
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q] + bias[q], lo);
      pp_st16(crs, off, pack8(v));
    } else if constexpr (EPI == 1) {
      float lo = -INFINITY;  // (as EPI 0)
      asm volatile("" : "+v"(lo));
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q] + bias[q], lo);
      const u32x4 pre = pack8(v);
      float f[8];
      unpack8(pre, f);  // the activation reads the bf16-rounded pre-activation
#pragma unroll
      for (int q = 0; q < 8; ++q) f[q] = gelu_f(f[q]);
      pp_st16(ars, aoff, pre);
      pp_st16(crs, off, pack8(f));
    } else if constexpr (EPI == 2) {
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q] + bias[q], 0.f);
      pp_st16(crs, off, pack8(v));
    } else if constexpr (EPI == 3 || EPI == 4) {
      float a[8];
      unpack8(ax[jj], a);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float d = bfr(v[q]);  // the unfused path's bf16 data gradient
        v[q] = EPI == 3 ? d * gelu_df(a[q]) : (a[q] > 0.f ? d : 0.f);
      }
      const u32x4 o = pack8(v);
      pp_st16(crs, off, o);
      unpack8(o, v);  // the bias gradient sums the bf16-rounded values, like act_bwd_colsum
#pragma unroll
      for (int q = 0; q < 8; ++q) csum[q] += v[q];
    } else {  // EPI 6: dO stored; delta = sum over the wave's 64 columns (one head) of dO * O
      const u32x4 o = pack8(v);
      pp_st16(crs, off, o);
      float d[8], oo[8];
      unpack8(o, d);
      unpack8(ax[jj], oo);
      float sum = first_of_half ? 0.f : dsum[jj];
#pragma unroll
      for (int q = 0; q < 8; ++q) sum = __builtin_fmaf(d[q], oo[q], sum);
      dsum[jj] = sum;
    }
    __builtin_amdgcn_sched_barrier(0);  // one row tile at a time: bounded temporaries
  }
  if constexpr (EPI == 3 || EPI == 4) {
    // lanes r16 = 0..15 of a lane group hold the same 8 columns (fixed butterfly order)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float t = csum[q];
      t += __shfl_xor(t, 1, 64);
      t += __shfl_xor(t, 2, 64);
      t += __shfl_xor(t, 4, 64);
      t += __shfl_xor(t, 8, 64);
      csum[q] = t;
    }
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(g.colpart + (int64_t)(4 * e.tm + 2 * c.wr + jh) * N), (short)0, e.valid ? N * 4 : 0, 0x00020000);
    const uint32_t po = (ok && r16 == 0) ? (uint32_t)col * 4u : kPOff;
    pp_st16(prs, po, __builtin_bit_cast(u32x4, f32x4{csum[0], csum[1], csum[2], csum[3]}));
    pp_st16(prs, po == kPOff ? kPOff : po + 16u, __builtin_bit_cast(u32x4, f32x4{csum[4], csum[5], csum[6], csum[7]}));
  }
  if constexpr (EPI == 6 && !first_of_half) {
    const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(g.delta != nullptr ? g.delta : (float*)g.C), (short)0, e.valid ? (int)(4ll * M * N / 64) : 0,
        0x00020000);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      // the row's 4 lane groups (g = 0..3: lanes r16, r16 + 16, + 32, + 48) in a fixed order
      float sum = dsum[jj];
      sum += __shfl_xor(sum, 16, 64);
      sum += __shfl_xor(sum, 32, 64);
      // a 16-row tile never crosses a sequence (T % 16 == 0, checked by the dispatcher): the
      // (batch, position) split of its first row is scalar, the lanes add their r16
      const int mb = m0 + c.wr * 128 + 16 * (4 * jh + jj);
      const int bq = mb / g.T, tq0 = mb - bq * g.T, hd = (n0 + c.wc * 64) >> 6;
      const uint32_t doff = (g4 == 0 && mb + r16 < M && (n0 + c.wc * 64) < N)
                                ? (uint32_t)((((int64_t)bq * (N >> 6) + hd) * g.T + tq0 + r16) * 4) : kPOff;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, sum), drs, doff, 0, 0);
    }
  }
}

// read quadrant aux / bias out of the wave's LDS area (and make sure the reads have returned
// before the next quadrant's DMA overwrites the area)
template <int EPI>
PL_DEV void pp_aux_read(const PPCtx& c, u32x4 (&ax)[4]) {
  const int r16 = c.lane & 15, g4 = c.lane >> 4;
  if constexpr (EPI <= 2) {
    ax[0] = *reinterpret_cast<const u32x4*>(c.aux + 8 * g4);
  } else {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) ax[jj] = *reinterpret_cast<const u32x4*>(c.aux + 512 * jj + 32 * r16 + 8 * g4);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------------------------
// Counted waits.  Per phase a wave's vector-memory instructions issue in this order: the aux DMA
// of the next quadrant (kAuxN; in the FIRST K-tile's phases 0-2 and the LAST K-tile's phase 3),
// the quadrant's stores (FIRST only), the K-tile DMA (2).  Waits count the instructions issued
// AFTER the ones they need (vmcnt(N) = all but the N youngest are done), so the stores never
// have to complete.  Where a phase belongs to the previous K-tile its kind is only partly known
// (a FIRST K-tile follows a LAST one; nothing else is guaranteed): the count is a lower bound.
template <int EPI, bool QE>
constexpr int pp_phase_ops(bool F, bool L, int q) {
  return 2 + (!QE ? 0 : (((F && q < 3) || (L && q == 3)) ? kAuxN<EPI> : 0) + (F ? kStQ<EPI>(q) : 0));
}
// the DMA wait of phase PH (piece group PH - 2 landed): everything issued in phases PH - 1, PH
template <int EPI, bool QE, bool F, bool L, int PH>
constexpr int pp_dma_wait() {
  int n = pp_phase_ops<EPI, QE>(F, L, PH);
  n += PH >= 1 ? pp_phase_ops<EPI, QE>(F, L, PH - 1) : pp_phase_ops<EPI, QE>(false, F, 3);
  if constexpr (!QE) {
    if (F && PH < 2) n += kEndStores<EPI>;  // the end-of-tile epilogue's stores
  }
  return n > 63 ? 63 : n;
}
// the aux wait of phase PH of a FIRST K-tile (aux issued first in phase PH - 1)
template <int EPI, int PH>
constexpr int pp_aux_wait() {
  return 2 + (PH == 0 ? 0 : kStQ<EPI>(PH - 1));
}

// One phase of a K-tile: the LOAD segment (in a FIRST K-tile the previous tile's quadrant-PH
// epilogue, then the fragment reads for this phase's quadrant, the next K-tile's piece group
// PH, the counted wait), a barrier, the MFMA segment (16 MFMAs into quadrant PH), a barrier.
// The epilogue goes first: the fragments it would otherwise overlap are not live yet.
template <int PH, bool FIRST, bool LAST, int EPI, bool QE>
PL_DEV void pp_phase(const PPCtx& c, f32x4 (&acc)[4][8], bf16x8 (&fa)[2][4], bf16x8 (&fb)[2][2],
                       const uint16_t* slotp, const uint16_t* nslotp, const PPSrd& srd, int nsl,
                       const PPEpi& pe, const PPEpi& ce, float (&dsum)[4]) {
  const int wr = c.wr, wc = c.wc;
  if constexpr (QE) {
    u32x4 ax[4];
    if constexpr (FIRST) {
      pp_vmwait<pp_aux_wait<EPI, PH>()>();
      pp_aux_read<EPI>(c, ax);
    }
    if constexpr (FIRST && PH < 3) pp_aux_issue<EPI, PH + 1>(c, pe);
    if constexpr (LAST && PH == 3) pp_aux_issue<EPI, 0>(c, ce);
    if constexpr (FIRST) pp_epi_quad<EPI, PH>(acc, c, pe, ax, dsum);
    __builtin_amdgcn_sched_barrier(0);
  }
  // ---- fragment reads: 12 / 4 / 8 / 4 (snake order: A rows half + column pair, then pair 1,
  // rows half 1, pair 0 again; one column-pair set of registers)
  {
    const char* sb = reinterpret_cast<const char*>(slotp);
    if constexpr (PH == 0 || PH == 2) {
      const int jh = PH == 0 ? 0 : 1;
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          fa[k][jj] = ldsf(reinterpret_cast<const uint16_t*>(
              sb + c.rdA[k] + (unsigned)((wr * 128 + 16 * (4 * jh + jj)) * PBK * 2)));
    }
    if constexpr (PH != 2) {
      const int p = PH == 1 ? 1 : 0;
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
          fb[k][ii] = ldsf(reinterpret_cast<const uint16_t*>(
              sb + c.rdB[k] + (unsigned)((PIMG + (wc * 64 + 16 * (2 * p + ii)) * PBK) * 2)));
    }
  }
  i32x4v gr;
  unsigned glds;
  pp_group<PH, EPI>(c, srd, nsl, gr, glds);
  pp_piece<PH>(c, gr, glds, 0);
  pp_piece<PH>(c, gr, glds, 1);
  pp_vmwait<pp_dma_wait<EPI, QE, FIRST, LAST, PH>()>();
  pp_barrier();
  // ---- MFMA segment: quadrant (rows half jh, column pair p): (0,0) (0,1) (1,1) (1,0)
  {
    constexpr int jh = pp_qjh(PH);
    constexpr int p = pp_qp(PH);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int ii = 0; ii < 2; ++ii) {
          f32x4& a = acc[2 * p + ii][4 * jh + jj];
          if (FIRST && k == 0) a = mfma16(fb[k][ii], fa[k][jj], f32x4{0.f, 0.f, 0.f, 0.f});
          else a = mfma16(fb[k][ii], fa[k][jj], a);
        }
    __builtin_amdgcn_s_setprio(0);
  }
  pp_barrier();
}

template <bool FIRST, bool LAST, int EPI, bool QE>
PL_DEV void pp_ktile(const PPCtx& c, f32x4 (&acc)[4][8], bf16x8 (&fa)[2][4], bf16x8 (&fb)[2][2],
                       const uint16_t* smem, int s, int ntm, int ntn, int nkt, bool nvalid, const PPEpi& pe,
                       const PPEpi& ce, float (&dsum)[4]) {
  const uint16_t* slotp = smem + (s & 1) * PSLOT;
  const int nsl = (s + 1) & 1;
  const uint16_t* nslotp = smem + nsl * PSLOT;
  const PPSrd srd = pp_srds<EPI>(c, ntm, ntn, nkt, nvalid);  // the DMA carries the next K-tile
  pp_phase<0, FIRST, LAST, EPI, QE>(c, acc, fa, fb, slotp, nslotp, srd, nsl, pe, ce, dsum);
  pp_phase<1, FIRST, LAST, EPI, QE>(c, acc, fa, fb, slotp, nslotp, srd, nsl, pe, ce, dsum);
  pp_phase<2, FIRST, LAST, EPI, QE>(c, acc, fa, fb, slotp, nslotp, srd, nsl, pe, ce, dsum);
  pp_phase<3, FIRST, LAST, EPI, QE>(c, acc, fa, fb, slotp, nslotp, srd, nsl, pe, ce, dsum);
}

template <int EPI, bool QE>
__global__ __launch_bounds__(PNT) void gemm_pp_kernel(pllm::GemmArgs g) {
  // all LDS in ONE array (a second __shared__ object can make hipcc drain the DMA before reads):
  // two 64 KiB K-tile slots, then 8 x 4 KiB per-wave bias / aux areas (quadrant epilogues)
  constexpr int kAuxElems = QE ? 8 * 2048 : 0;
  __shared__ __attribute__((aligned(1024))) uint16_t smem[2 * PSLOT + kAuxElems];
  const int tiles_m = (g.M + PT - 1) / PT, tiles_n = (g.N + kNT<EPI> - 1) / kNT<EPI>, ntiles = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int lid = xcd_remap(blockIdx.x, G);
  if (lid >= ntiles) return;
  PPCtx c;
  c.g = &g;
  const int tid = threadIdx.x, lane = tid & 63;
  c.w = __builtin_amdgcn_readfirstlane(tid >> 6);
  c.wr = c.w >> 2;
  c.wc = c.w & 3;
  c.lane = lane;
  c.lds = (unsigned)(uintptr_t)smem;
  c.aux = smem + 2 * PSLOT + 2048 * c.w;
  c.vaux = (uint32_t)(((int64_t)(lane >> 2) * g.ldaux + 8 * (lane & 3)) * 2);
  {
    // per-lane source offsets of this wave's pieces: lane l of piece blk fills image row
    // 8 * blk + l / 8 at 16-B position l % 8, which holds logical chunk (l % 8) ^ swz(row),
    // swz(row) = (row >> 1) & 7 = (4 * (blk & 1) + l / 16) & 7; B image rows are permuted inside
    // each 32-row block (image row 16h + 4g + r <- column 8g + 4h + r)
    const int prow = 8 * ((lane >> 5) & 1) + ((lane >> 3) & 3);  // B permutation, per-lane part
    auto voA = [&](int blk) {
      const int ch = (lane & 7) ^ ((4 * (blk & 1) + (lane >> 4)) & 7);
      return (uint32_t)(((int64_t)(8 * blk + (lane >> 3)) * g.lda + ch * 8) * 2);
    };
    auto voB = [&](int blk) {
      const int ch = (lane & 7) ^ ((4 * (blk & 1) + (lane >> 4)) & 7);
      // EPI 7: image 32-row block 2 wc + h holds gate (h = 0) / up (h = 1) rows wc*32 + [0, 32)
      const int b32 = EPI == 7 ? (blk >> 2) >> 1 : blk >> 2;
      const int row = 32 * b32 + 16 * (blk & 1) + 4 * ((blk >> 1) & 1) + prow;
      return (uint32_t)(((int64_t)row * g.ldb + ch * 8) * 2);
    };
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      c.vo[0][q] = voA(pp_blk0<0>(c.w) + q);
      c.vo[1][q] = voB(pp_blk0<1>(c.w) + q);
    }
  }
  {
    // fragment reads: image row (16-aligned base) + r16, chunk 4 k32 + g, swizzled by (r16 >> 1) & 7
    const int r16 = lane & 15, g4 = lane >> 4;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const unsigned off = (unsigned)(r16 * PBK + ((((4 * k + g4) ^ ((r16 >> 1) & 7))) << 3)) * 2u;
      c.rdA[k] = off;
      c.rdB[k] = off;
    }
  }
  const int S = g.K / PBK;
  // one full-K segment per tile: tiles lid, lid + G, ...
  const int R = (ntiles - lid + G - 1) / G;
  int tm, tn;
  // prologue: the first segment's first K-tile, all four piece groups, fully landed
  {
    pp_tile(lid, tiles_m, tiles_n, g.group_m, tm, tn);
    const PPSrd srd = pp_srds<EPI>(c, tm, tn, 0, true);
    pp_issue<0, EPI>(c, srd, 0);
    pp_issue<1, EPI>(c, srd, 0);
    pp_issue<2, EPI>(c, srd, 0);
    pp_issue<3, EPI>(c, srd, 0);
  }
  pp_vmwait<0>();
  pp_barrier();
  if (c.wr == 1) pp_barrier();  // the stagger: rows 128-255 run one barrier behind rows 0-127

  f32x4 acc[4][8];
  bf16x8 fa[2][4];
  bf16x8 fb[2][2];
  float dsum[4] = {0.f, 0.f, 0.f, 0.f};
  int s = 0;
  PPEpi pe{tm, tn, false};  // the previous tile (none yet)
  for (int i = 0; i < R; ++i) {
    pp_tile(lid + i * G, tiles_m, tiles_n, g.group_m, tm, tn);
    const PPEpi ce{tm, tn, true};
    const bool more = i + 1 < R;
    int tm2 = tm, tn2 = tn;
    if (more) pp_tile(lid + (i + 1) * G, tiles_m, tiles_n, g.group_m, tm2, tn2);
    // K-tile kt's DMA carries K-tile kt + 1, or the next segment's first K-tile after the last one.
    // The first K-tile is peeled: its MFMAs start the accumulators from zero (with quadrant
    // epilogues: each quadrant right after that quadrant's epilogue of the previous tile).
    // (>= 2 K-tiles per tile: gemm_tn sends K < 128 to the round-3 kernel)
    pp_ktile<true, false, EPI, QE>(c, acc, fa, fb, smem, s, tm, tn, 1, true, pe, ce, dsum);
    ++s;
    for (int kt = 1; kt + 1 < S; ++kt, ++s)
      pp_ktile<false, false, EPI, QE>(c, acc, fa, fb, smem, s, tm, tn, kt + 1, true, pe, ce, dsum);
    pp_ktile<false, true, EPI, QE>(c, acc, fa, fb, smem, s, tm2, tn2, 0, more, pe, ce, dsum);
    ++s;
    if constexpr (!QE) {
      // the end-of-tile epilogue, in this wave's next LOAD slot
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (EPI == 7) pp_epilogue_swiglu(acc, g, tm, tn, c.wr, c.wc, lane);
      else pp_epilogue<EPI>(acc, g, tm, tn, c.wr, c.wc, lane);
      __builtin_amdgcn_sched_barrier(0);
    }
    pe = ce;
  }
  if constexpr (QE) {
    // the last tile's epilogue (its quadrant-0 aux was DMA'd in its last K-tile's phase 3)
    u32x4 ax[4];
    pp_vmwait<0>();
    pp_aux_read<EPI>(c, ax);
    pp_aux_issue<EPI, 1>(c, pe);
    pp_epi_quad<EPI, 0>(acc, c, pe, ax, dsum);
    pp_vmwait<0>();
    pp_aux_read<EPI>(c, ax);
    pp_aux_issue<EPI, 2>(c, pe);
    pp_epi_quad<EPI, 1>(acc, c, pe, ax, dsum);
    pp_vmwait<0>();
    pp_aux_read<EPI>(c, ax);
    pp_aux_issue<EPI, 3>(c, pe);
    pp_epi_quad<EPI, 2>(acc, c, pe, ax, dsum);
    pp_vmwait<0>();
    pp_aux_read<EPI>(c, ax);
    pp_epi_quad<EPI, 3>(acc, c, pe, ax, dsum);
  }
  if (c.wr == 0) pp_barrier();  // balance the stagger
}

}  // namespace

namespace pllm {

// EPI 3 / 4 column-sum partial rows: 4 per tile row with quadrant epilogues, 2 otherwise
int gemm_pp_colsum_groups(int M, int K) { return (gemm_pp_quad_epilogue(K, 3) ? 4 : 2) * ((M + PT - 1) / PT); }

// quadrant epilogues at K >= 2048, except EPI 5 (aux too large for the LDS) and EPI 1 (the GELU's
// VALU work in the LOAD segments: 1410 vs 1344 us for the end-of-tile form + hipBLASLt at the llama
// shape 32768 x 11008 x 2048, gpurun_out/r4pp7_bench.jsonl)
bool gemm_pp_quad_epilogue(int K, int epi) { return K >= 2048 && epi != 5 && epi != 1; }

void gemm_tn_pp(const GemmArgs& a, int epi, int ctas, hipStream_t st) {
  const int nt = epi == 7 ? 128 : PT;
  const int ntiles = ((a.M + PT - 1) / PT) * ((a.N + nt - 1) / nt);
  if (ntiles == 0) return;
  const int grid = ntiles < ctas ? ntiles : ctas;
  const bool qe = gemm_pp_quad_epilogue(a.K, epi);
#define PL_PP_CASE(E)                                                                          \
  do {                                                                                           \
    if (qe) hipLaunchKernelGGL((gemm_pp_kernel<E, E != 5 && E != 1>), dim3(grid), dim3(PNT), 0, st, a); \
    else hipLaunchKernelGGL((gemm_pp_kernel<E, false>), dim3(grid), dim3(PNT), 0, st, a);         \
  } while (0)
  switch (epi) {
    case 0: PL_PP_CASE(0); break;
    case 1: PL_PP_CASE(1); break;
    case 2: PL_PP_CASE(2); break;
    case 3: PL_PP_CASE(3); break;
    case 4: PL_PP_CASE(4); break;
    case 5: PL_PP_CASE(5); break;
    case 6: PL_PP_CASE(6); break;
    default: hipLaunchKernelGGL((gemm_pp_kernel<7, false>), dim3(grid), dim3(PNT), 0, st, a); break;
  }
#undef PL_PP_CASE
}

}  // namespace pllm

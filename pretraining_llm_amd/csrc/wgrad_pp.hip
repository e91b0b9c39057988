// Ping-pong weight-gradient GEMM on gfx950 MFMA (round 4):
//     dW[P, Q] (+)= sum_m dY[m, P] * X[m, Q]          (bf16 in, fp32 accumulate, fp32 out)
// The token-major ("NT") product of every linear layer's backward -- reference math
// /root/reference/src/models/mlp.py:24-26, attention.py:29-31 (autograd's weight gradients) -- on
// the main loop of csrc/gemm_pp.hip instead of gemm_wgrad.hip's one-barrier-per-stage loop.
//
// Why: per-wave stamps of wgrad_kernel (profiles/r3_wgrad_stamps.md) put a third of every 64-token
// stage into issuing its eight 1-KiB LDS-DMA pieces (~140 cycles each) and most of the rest into
// the stage barrier, at ~1.1 PFLOP/s; the same long-K FLOPs in the TN layout run at ~1.8 on
// hipBLASLt.  Here the two wave groups run one barrier apart (as in gemm_pp.hip): on every SIMD one
// wave issues a quadrant's 16 MFMAs while its partner reads the next quadrant's fragments and
// issues its share of the next K-tile's DMA, with counted vmcnt waits (never 0 in the loop).
//
// Layout (what differs from the TN kernel):
//  * 256 x 256 output tile per 512-thread workgroup (P rows x Q columns), wave (wr, wc) owns rows
//    wr*128 + [0, 128) and columns wc*64 + [0, 64) as 8 x 4 accumulators of v_mfma_f32_16x16x32;
//    persistent over work items (token slice, tile) -- split-K slices as wgrad_plan picks them;
//  * a 64-token K-tile is 16 LDS images [64 tokens][32 columns] (64-B rows, 4 KiB): 8 of dY (P
//    columns 32e + [0, 32) of the tile) then 8 of X.  Images this narrow let every DMA piece group
//    hold exactly what one phase first reads: group 0 = the dY images of row half 0 of both wave
//    groups, 1 = the X images of column pair 0 of every wave, 2 = pair 1, 3 = dY row half 1;
//  * the reduction index (token) is the image ROW, so both fragments come from
//    ds_read_b64_tr_b16 transposed reads (two per fragment: 8 consecutive tokens per lane).  The
//    16-B chunk c of image row r sits at c ^ (2 * ((r >> 3) & 1)): the 8 rows x 32 B of one
//    32-lane read group land on 16 distinct 16-B bank slots (conflict-free);
//  * the fragment of column tile t is the MFMA's A operand and the dY fragment its B operand, so
//    a lane's accumulator holds one P row and 4 CONSECUTIVE Q columns: the epilogue stores 16 B of
//    fp32 per lane and accumulator straight from registers (slab partial, or added to the gradient);
//  * bias gradient (dY column sums) by all-ones MFMAs against the dY fragments on the first Q tile's
//    items, each wave taking the row tiles jj == wc of its row halves (+4 MFMAs per 64).
// Requires M % 64 == 0, P % 8 == 0, Q % 8 == 0, row strides % 8 == 0 (checked by the binding).
#include <algorithm>

#include "ab.h"
#include "common.h"
#include "kernels.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int WT = 256;          // output tile (P and Q)
constexpr int WBK = 64;          // tokens per K-tile
constexpr int WNT = 512;         // 8 waves
constexpr int WIMG = WBK * 32;   // elements of one [64][32] image (4 KiB)
constexpr int WSLOT = 16 * WIMG; // 8 dY images then 8 X images: 64 KiB
constexpr uint32_t kWOff = 0x80000000u;  // a byte offset past every descriptor built here

PL_DEV f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
PL_DEV s16x4 ds_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(const uint16_t*)p);
}
PL_DEV bf16x8 frag_tr(const char* p) {
  // rows r and r + 4 of the image (+256 B): 8 consecutive tokens of the lane's column
  const s16x4 lo = ds_tr(p), hi = ds_tr(p + 256);
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}
PL_DEV void wp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
template <int N>
PL_DEV void wp_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// buffer resource from wave-uniform values, provably so (no waterfall loop around its users)
PL_DEV __amdgpu_buffer_rsrc_t wp_rsrc(const void* base, int bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  const uint64_t u = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(a >> 32)) << 32) |
                     (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)u, (short)0, __builtin_amdgcn_readfirstlane(bytes),
                                           0x00020000);
}
// chunk position of logical 16-B chunk c (0..3) in image row r
PL_DEV int wp_swz(int r) { return ((r >> 3) & 1) << 1; }

struct WPArgs {
  const uint16_t* A;  // dY [M, P], row stride lda
  const uint16_t* B;  // X [M, Q], row stride ldb
  int64_t lda, ldb;
  int M, P, Q;
  int S, slice_kt;    // token slices, K-tiles per slice
  float* part;        // S > 1: fp32 [S][P][Q] slab
  float* out;         // S == 1: the fp32 gradient [P, Q]
  int accumulate;     // S == 1: out += tile (else out = tile)
  float* bpart;       // bias gradient partial rows [S][P] (BIAS)
  // hybrid split (HY): items [0, hy_full) are whole tiles (hy_full = whole rounds of the grid), written
  // straight into the gradient; the last hy_rem tiles run as hy_s slices of slice_kt K-tiles each (items
  // hy_full + s hy_rem + j, slice-major), leaving tile-local fp32 pieces [s hy_rem + j][256][256] in `part`
  int hy_full, hy_rem, hy_s;
  int kst;            // K-tiles per tile (M / 64)
};

// one work segment: a tile's K-tiles [kb, ke) and where its accumulators go (dest -1: the gradient,
// added to it when accumulating; slice mode: slab sidx; stream-K: tile-local piece slot dest)
struct WPSeg {
  int tp, tq, kb, ke, dest, sidx;
};

struct WPCtx {
  const WPArgs* g;
  int w, wr, wc, lane;
  unsigned lds;
  uint32_t vo[2][2];  // per-lane DMA source offsets of this wave's pieces of groups 0 (dY) / 1 (X)
  unsigned rd[2];     // per-lane LDS byte offsets of the fragment reads (column half 0 / 16), slot 0
};

// image of piece group PH for wave w (2 pieces each: image rows 32 (w & 1) + [0, 32))
template <int PH>
constexpr int wp_img(int w) {
  return PH == 0 ? (w >> 1) + 2 * (w >> 2)            // dY 0, 1, 4, 5: row half 0 of both groups
         : PH == 3 ? (w >> 1) + 2 * (w >> 2) + 2      // dY 2, 3, 6, 7: row half 1
         : PH == 1 ? 8 + 2 * (w >> 1)                 // X column pair 0 of wave column w >> 1
                   : 9 + 2 * (w >> 1);                // X column pair 1
}

struct WPSrd {
  i32x4v a, b;
};
// descriptors of K-tile kt's dY / X panels (64 token rows from the tile's first column)
PL_DEV WPSrd wp_srds(const WPArgs& g, int tp, int tq, int kt) {
  const int64_t r0 = (int64_t)kt * WBK;
  const int pc = g.P - tp * WT, qc = g.Q - tq * WT;
  WPSrd r;
  r.a = srd_of(g.A + r0 * g.lda + tp * WT, (uint32_t)(((int64_t)(WBK - 1) * g.lda + pc) * 2));
  r.b = srd_of(g.B + r0 * g.ldb + tq * WT, (uint32_t)(((int64_t)(WBK - 1) * g.ldb + qc) * 2));
  return r;
}
// shift a descriptor's base by `bytes` (its range shrinks by as much)
PL_DEV i32x4v wp_shift(const i32x4v& r, uint32_t bytes) {
  const uint64_t a = ((uint64_t)(uint32_t)r[1] << 32 | (uint32_t)r[0]) + bytes;
  i32x4v o;
  o[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  o[1] = __builtin_amdgcn_readfirstlane((int)((uint32_t)(a >> 32) & 0xffffu));
  o[2] = __builtin_amdgcn_readfirstlane((uint32_t)r[2] > bytes ? (int)((uint32_t)r[2] - bytes) : 0);
  o[3] = r[3];
  return o;
}
template <int PH>
PL_DEV void wp_group(const WPCtx& c, const WPSrd& srd, int sl, i32x4v& r, unsigned& lds0) {
  lds0 = c.lds + (unsigned)(sl * WSLOT + wp_img<PH>(c.w) * WIMG + (c.w & 1) * 1024) * 2u;
  // groups 3 / 2: the images of groups 0 / 1 shifted by 64 (dY) / 32 (X) columns
  r = PH == 0 ? srd.a : PH == 1 ? srd.b : PH == 3 ? wp_shift(srd.a, 128u) : wp_shift(srd.b, 64u);
}
template <int PH>
PL_DEV void wp_piece(const WPCtx& c, const i32x4v& r, unsigned lds0, int q) {
  constexpr bool isA = PH == 0 || PH == 3;
  blds16(r, c.vo[isA ? 0 : 1][q], lds0 + 1024u * (unsigned)q);
}
template <int PH>
PL_DEV void wp_issue(const WPCtx& c, const WPSrd& srd, int sl) {
  i32x4v r;
  unsigned lds0;
  wp_group<PH>(c, srd, sl, r, lds0);
#pragma unroll
  for (int q = 0; q < 2; ++q) wp_piece<PH>(c, r, lds0, q);
}

// counted wait of phase PH: piece group PH - 2 landed = all but what this wave issued in phases
// PH - 1 and PH (2 each) -- and, in a tile's first K-tile, the previous tile's 32 epilogue stores
// (a lower bound of what it issued after its last DMA)
template <bool F, int PH>
constexpr int wp_dma_wait() {
  return 4 + ((F && PH < 2) ? 32 : 0);
}

// One phase: fragment reads of quadrant PH (rows half jh, column pair p; snake order (0,0) (0,1)
// (1,1) (1,0)), the next K-tile's piece group PH, the counted wait, a barrier, 16 MFMAs (+ the
// bias MFMAs), a barrier.
template <int PH, bool FIRST, bool BIAS>
PL_DEV void wp_phase(const WPCtx& c, f32x4 (&acc)[4][8], bf16x8 (&fa)[2][4], bf16x8 (&fbp)[2][2][2],
                       f32x4 (&bacc)[2], bool dob, const char* slotp, const WPSrd& srd, int nsl) {
  constexpr int jh = PH >> 1;
  constexpr int p = (PH == 1 || PH == 2) ? 1 : 0;
  if constexpr (PH == 0 || PH == 2) {
    // dY row tiles 4 jh + jj of the wave: image 4 wr + 2 jh + jj / 2, columns 16 (jj & 1)
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        fa[k][jj] = frag_tr(slotp + c.rd[jj & 1] + (unsigned)((4 * c.wr + 2 * jh + (jj >> 1)) * WIMG * 2 + 2048 * k));
  }
  // X column tiles 2 p + ii: image 8 + 2 wc + p, columns 16 ii -- both pairs kept (phase 3 reuses pair 0
  // from phase 0 instead of reading it again: 48 instead of 56 transposed reads per K-tile and wave)
  bf16x8 (&fb)[2][2] = fbp[p];
  if constexpr (PH == 0 || PH == 1) {
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
        fb[k][ii] = frag_tr(slotp + c.rd[ii] + (unsigned)((8 + 2 * c.wc + p) * WIMG * 2 + 2048 * k));
  }
  i32x4v gr;
  unsigned glds;
  wp_group<PH>(c, srd, nsl, gr, glds);
  wp_piece<PH>(c, gr, glds, 0);
  wp_piece<PH>(c, gr, glds, 1);
  wp_vmwait<wp_dma_wait<FIRST, PH>()>();
  wp_barrier();
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
  if constexpr (BIAS && (PH == 0 || PH == 2)) {
    if (dob) {
      // row tile jj == wc of this half: lane l's column sum of P row 16 j + (l & 15) in every element
      const bf16x8 ones = __builtin_bit_cast(bf16x8, u32x4{0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u});
      bf16x8 f0 = fa[0][0], f1 = fa[1][0];
#pragma unroll
      for (int jj = 1; jj < 4; ++jj)
        if (c.wc == jj) {
          f0 = fa[0][jj];
          f1 = fa[1][jj];
        }
      bacc[jh] = mfma16(ones, f0, bacc[jh]);
      bacc[jh] = mfma16(ones, f1, bacc[jh]);
    }
  }
  __builtin_amdgcn_s_setprio(0);
  wp_barrier();
}

template <bool FIRST, bool BIAS>
PL_DEV void wp_ktile(const WPCtx& c, f32x4 (&acc)[4][8], bf16x8 (&fa)[2][4], bf16x8 (&fb)[2][2][2],
                       f32x4 (&bacc)[2], bool dob, const uint16_t* smem, int s, const WPSrd& srd) {
  const char* slotp = reinterpret_cast<const char*>(smem + (s & 1) * WSLOT);
  const int nsl = (s + 1) & 1;
  wp_phase<0, FIRST, BIAS>(c, acc, fa, fb, bacc, dob, slotp, srd, nsl);
  wp_phase<1, FIRST, BIAS>(c, acc, fa, fb, bacc, dob, slotp, srd, nsl);
  wp_phase<2, FIRST, BIAS>(c, acc, fa, fb, bacc, dob, slotp, srd, nsl);
  wp_phase<3, FIRST, BIAS>(c, acc, fa, fb, bacc, dob, slotp, srd, nsl);
}

// work item i -> (slice, P tile, Q tile); slice-major, so the items that share a slice's panels
// are neighbours (one XCD's L2 after xcd_remap)
PL_DEV void wp_item(const WPArgs& g, int i, int tiles_q, int ntiles, int& sidx, int& tp, int& tq) {
  sidx = i / ntiles;
  const int t = i - sidx * ntiles;
  tp = t / tiles_q;
  tq = t - tp * tiles_q;
}

// segment i of workgroup lid (G workgroups; tiles_q tiles per row band, ntiles tiles)
template <bool HY>
PL_DEV WPSeg wp_seg(const WPArgs& g, int lid, int G, int i, int tiles_q, int ntiles) {
  WPSeg s;
  if constexpr (HY) {
    const int it = lid + i * G;
    int t;
    if (it < g.hy_full) {
      t = it;
      s.kb = 0;
      s.ke = g.kst;
      s.dest = -1;
    } else {
      const int j = it - g.hy_full, sl = j / g.hy_rem;
      t = g.hy_full + (j - sl * g.hy_rem);
      s.kb = sl * g.slice_kt;
      s.ke = min(g.kst, s.kb + g.slice_kt);
      s.dest = j;
    }
    s.tp = t / tiles_q;
    s.tq = t - s.tp * tiles_q;
    s.sidx = 0;
  } else {
    wp_item(g, lid + i * G, tiles_q, ntiles, s.sidx, s.tp, s.tq);
    s.kb = s.sidx * g.slice_kt;
    s.ke = min(g.M / WBK, s.kb + g.slice_kt);
    s.dest = g.S > 1 ? s.sidx : -1;
  }
  return s;
}

// segments of workgroup lid
template <bool HY>
PL_DEV int wp_nseg(const WPArgs& g, int lid, int G, int ntiles) {
  const int items = HY ? g.hy_full + g.hy_rem * g.hy_s : ntiles * g.S;
  return lid < items ? (items - lid + G - 1) / G : 0;
}

// the segment's tile: fp32 stores straight from the accumulators (32 per lane, all issued; rows /
// columns out of range go to an offset past the descriptor).  Into the gradient (+= when
// accumulating), the slice's slab, or a stream-K piece slot (tile-local [256][256], no bounds)
template <bool HY>
PL_DEV void wp_epilogue(const WPCtx& c, f32x4 (&acc)[4][8], const WPSeg& sg) {
  const WPArgs& g = *c.g;
  const int r16 = c.lane & 15, g4 = c.lane >> 4;
  const bool piece = HY && sg.dest >= 0;
  float* base = piece ? g.part + (int64_t)sg.dest * (WT * WT)
                      : sg.dest >= 0 ? g.part + (int64_t)sg.dest * g.P * g.Q : g.out;
  const int ld = piece ? WT : g.Q;
  const int row0 = piece ? 0 : sg.tp * WT, col0 = piece ? 0 : sg.tq * WT;
  const int cols_lim = piece ? WT : g.Q;
  const int rows_ok = piece ? WT : min(WT, g.P - sg.tp * WT);
  const bool rmw = sg.dest < 0 && g.accumulate;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int r0 = c.wr * 128 + 16 * j;
    const int rows_j = max(0, min(16, rows_ok - r0));
    const __amdgpu_buffer_rsrc_t rs = wp_rsrc(base + (int64_t)(row0 + (rows_j > 0 ? r0 : 0)) * ld, rows_j * ld * 4);
    f32x4 v[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) v[t] = acc[t][j];
    uint32_t off[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int q = col0 + c.wc * 64 + 16 * t + 4 * g4;
      off[t] = q < cols_lim ? (uint32_t)(r16 * ld + q) * 4u : kWOff;
    }
    if (rmw) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
        v[t] += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off[t], 0, 0));
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[t]), rs, off[t], 0, 0);
    __builtin_amdgcn_sched_barrier(0);  // one row tile at a time (bounded temporaries)
  }
}

template <bool BIAS, bool HY = false>
__global__ __launch_bounds__(WNT) void wgrad_pp_kernel(WPArgs g) {
  __shared__ __attribute__((aligned(1024))) uint16_t smem[2 * WSLOT];
  const int tiles_p = (g.P + WT - 1) / WT, tiles_q = (g.Q + WT - 1) / WT, ntiles = tiles_p * tiles_q;
  const int G = gridDim.x;
  const int lid = xcd_remap(blockIdx.x, G);
  const int R = wp_nseg<HY>(g, lid, G, ntiles);  // segments of this workgroup
  if (R == 0) return;
  WPCtx c;
  c.g = &g;
  const int tid = threadIdx.x, lane = tid & 63;
  c.w = __builtin_amdgcn_readfirstlane(tid >> 6);
  c.wr = c.w >> 2;
  c.wc = c.w & 3;
  c.lane = lane;
  c.lds = (unsigned)(uintptr_t)smem;
  {
    // lane l of a piece fills image row 16 q' + l / 4 (q' = 2 (w & 1) + q) at 16-B position l % 4,
    // which holds logical chunk (l % 4) ^ swz(row): token row, column 32 e + 8 chunk of the panel
    auto vo = [&](int img, int q, int64_t ld) {
      const int row = 16 * (2 * (c.w & 1) + q) + (lane >> 2);
      const int col = 32 * (img & 7) + 8 * ((lane & 3) ^ wp_swz(row));
      return (uint32_t)(((int64_t)row * ld + col) * 2);
    };
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      c.vo[0][q] = vo(wp_img<0>(c.w), q, g.lda);
      c.vo[1][q] = vo(wp_img<1>(c.w), q, g.ldb);
    }
    // fragment reads (16x16x32 operand): lane (gq = l / 16, tq = (l & 15) / 4, tp = l & 3) reads
    // image row 8 gq + tq, columns c0 + 4 tp; the transposed read hands lane l column c0 + l % 16,
    // tokens 8 gq + [0, 4) (and [4, 8) from the second read, 4 rows = 256 B further)
    const int gq = lane >> 4, tq = (lane & 15) >> 2, tpl = lane & 3;
    const int row = 8 * gq + tq;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int col = 16 * h + 4 * tpl;
      c.rd[h] = (unsigned)(row * 32 + ((((col >> 3) ^ wp_swz(row))) << 3) + (col & 7)) * 2u;
    }
  }
  WPSeg sg = wp_seg<HY>(g, lid, G, 0, tiles_q, ntiles);
  {
    const WPSrd srd = wp_srds(g, sg.tp, sg.tq, sg.kb);
    wp_issue<0>(c, srd, 0);
    wp_issue<1>(c, srd, 0);
    wp_issue<2>(c, srd, 0);
    wp_issue<3>(c, srd, 0);
  }
  wp_vmwait<0>();
  wp_barrier();
  if (c.wr == 1) wp_barrier();  // the stagger: rows 128-255 run one barrier behind rows 0-127

  f32x4 acc[4][8];
  bf16x8 fa[2][4];
  bf16x8 fb[2][2][2];
  int s = 0;
  for (int i = 0; i < R; ++i) {
    const bool dob = BIAS && sg.tq == 0;
    f32x4 bacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    const bool more = i + 1 < R;
    // K-tile kt's DMA carries kt + 1, or the next segment's first K-tile after the last one (an
    // empty descriptor after the workgroup's last segment: the same instructions, nothing read)
    for (int kt = sg.kb; kt < sg.ke; ++kt, ++s) {
      WPSrd srd;
      if (kt + 1 < sg.ke) {
        srd = wp_srds(g, sg.tp, sg.tq, kt + 1);
      } else if (more) {
        const WPSeg nx = wp_seg<HY>(g, lid, G, i + 1, tiles_q, ntiles);
        srd = wp_srds(g, nx.tp, nx.tq, nx.kb);
      } else {
        srd = WPSrd{srd_of(g.A, 0u), srd_of(g.B, 0u)};
      }
      if (kt == sg.kb) wp_ktile<true, BIAS>(c, acc, fa, fb, bacc, dob, smem, s, srd);
      else wp_ktile<false, BIAS>(c, acc, fa, fb, bacc, dob, smem, s, srd);
    }
    wp_epilogue<HY>(c, acc, sg);
    if constexpr (BIAS) {
      if (dob) {
        // P rows wr 128 + 16 (4 jh + wc) + lane, from lanes 0-15 (buffer stores: in-order vmcnt)
        const __amdgpu_buffer_rsrc_t brs = wp_rsrc(g.bpart + (int64_t)sg.sidx * g.P, g.P * 4);
#pragma unroll
        for (int jh = 0; jh < 2; ++jh) {
          const int prow = sg.tp * WT + c.wr * 128 + 16 * (4 * jh + c.wc) + lane;
          const uint32_t bo = ((lane >> 4) == 0 && prow < g.P) ? (uint32_t)prow * 4u : kWOff;
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, bacc[jh][0]), brs, bo, 0, 0);
        }
      }
    }
    if (more) sg = wp_seg<HY>(g, lid, G, i + 1, tiles_q, ntiles);
  }
  if (c.wr == 0) wp_barrier();  // balance the stagger
}

// hybrid fix-up: the last hy_rem tiles get out (+)= their hy_s pieces in slice order; one block per
// (tile, 4 rows), one 16-B column group per thread (all of a thread's loads independent)
__global__ __launch_bounds__(256) void wgrad_hy_reduce_kernel(const float* __restrict__ part, float* __restrict__ out,
                                                              int P, int Q, int tiles_q, int hy_full, int hy_rem,
                                                              int hy_s, int accumulate) {
  const int j = blockIdx.x, t = hy_full + j;
  const int tp = t / tiles_q, tq = t - tp * tiles_q;
  const int row = blockIdx.y * 4 + (threadIdx.x >> 6), col = (threadIdx.x & 63) * 4;
  const int grow = tp * WT + row, gcol = tq * WT + col;
  if (grow >= P || gcol >= Q) return;
  f32x4* o = reinterpret_cast<f32x4*>(out + (int64_t)grow * Q + gcol);
  f32x4 f = accumulate ? *o : f32x4{0.f, 0.f, 0.f, 0.f};
  const float* pp = part + (int64_t)j * (WT * WT) + row * WT + col;
  for (int sl = 0; sl < hy_s; ++sl) f += *reinterpret_cast<const f32x4*>(pp + (int64_t)sl * hy_rem * (WT * WT));
  *o = f;
}

}  // namespace

namespace pllm {

// hybrid plan: with more tiles than workgroups, whole tiles for the whole rounds of the grid and the
// remaining tiles as slices (>= 2 K-tiles each); false when it does not apply (no more tiles than
// workgroups: wgrad_plan's uniform slices).  The remainder's slice count comes from wgrad_plan's cost model
// (rounds x K-tiles per slice x ~2 us, plus the tile pieces written and read back at ~4 TB/s) instead of
// "one round of slices" (ctas / rem): llama's gate/up projection (344 tiles on 256 CUs, 88 left) takes 5
// slices in 2 rounds (1.4 tile times) instead of 2 slices in 1 round (1.5) (profiles/r6_wgrad_hy_cost.log)
bool wgrad_hy_plan(int M, int P, int Q, int ctas, int* full, int* rem, int* S, int* slice_kt) {
  const int kst = M / WBK;
  const int ntiles = ((P + WT - 1) / WT) * ((Q + WT - 1) / WT);
  if (M % WBK != 0 || kst < 2 || ctas <= 0 || ntiles <= ctas) return false;
  *full = ntiles / ctas * ctas;
  *rem = ntiles - *full;
  int s = *rem > 0 ? std::max(1, std::min(ctas / *rem, kst / 2)) : 1;
  if (*rem > 0 && ab_int("wgrad_hy_cost", 1)) {
    double best_t = 1e30;
    for (int c = 1; c <= 16 && (c == 1 || kst / c >= 8); ++c) {
      const int per = (kst + c - 1) / c;
      const int rounds = (*rem * c + ctas - 1) / ctas;
      const double t = rounds * (double)per * 2.0e-6 + (c > 1 ? (double)*rem * c * WT * WT * 4.0 * 2 / 4.0e12 : 0.0);
      if (t < best_t * 0.98) {
        best_t = t;
        s = c;
      }
    }
  }
  *slice_kt = (kst + s - 1) / s;
  *S = *rem > 0 ? (kst + *slice_kt - 1) / *slice_kt : 0;
  return true;
}

int64_t wgrad_pp_hy_ws_floats(int M, int P, int Q, int ctas) {
  int full, rem, S, skt;
  return wgrad_hy_plan(M, P, Q, ctas, &full, &rem, &S, &skt) ? (int64_t)rem * S * WT * WT : 0;
}

void wgrad_pp_hy(const void* dy, int64_t lda, const void* x, int64_t ldb, int M, int P, int Q, float* part,
                 float* out, bool accumulate, int ctas, hipStream_t st) {
  int full, rem, S, skt;
  if (!wgrad_hy_plan(M, P, Q, ctas, &full, &rem, &S, &skt)) return;
  WPArgs g;
  g.A = (const uint16_t*)dy;
  g.B = (const uint16_t*)x;
  g.lda = lda;
  g.ldb = ldb;
  g.M = M;
  g.P = P;
  g.Q = Q;
  g.S = 1;
  g.slice_kt = skt;
  g.part = part;
  g.out = out;
  g.accumulate = accumulate ? 1 : 0;
  g.bpart = nullptr;
  g.hy_full = full;
  g.hy_rem = rem;
  g.hy_s = S;
  g.kst = M / WBK;
  const int items = full + rem * S;
  hipLaunchKernelGGL((wgrad_pp_kernel<false, true>), dim3(items < ctas ? items : ctas), dim3(WNT), 0, st, g);
  if (rem > 0)
    hipLaunchKernelGGL(wgrad_hy_reduce_kernel, dim3(rem, WT / 4), dim3(256), 0, st, part, out, P, Q,
                       (Q + WT - 1) / WT, full, rem, S, g.accumulate);
}

bool wgrad_pp_supported(int M, int P, int Q, int S, int slice) {
  (void)P;
  (void)Q;
  // >= 2 K-tiles per slice (the first K-tile is peeled), whole K-tiles
  return M % WBK == 0 && slice % WBK == 0 && slice / WBK >= 2 && S >= 1;
}

void wgrad_pp(const void* dy, int64_t lda, const void* x, int64_t ldb, int M, int P, int Q, int S, int slice,
              float* part, float* out, bool accumulate, float* bpart, int ctas, hipStream_t st) {
  WPArgs g;
  g.A = (const uint16_t*)dy;
  g.B = (const uint16_t*)x;
  g.lda = lda;
  g.ldb = ldb;
  g.M = M;
  g.P = P;
  g.Q = Q;
  g.S = S;
  g.slice_kt = slice / WBK;
  g.part = part;
  g.out = out;
  g.accumulate = accumulate ? 1 : 0;
  g.bpart = bpart;
  g.hy_full = g.hy_rem = g.hy_s = 0;
  g.kst = M / WBK;
  const int ntiles = ((P + WT - 1) / WT) * ((Q + WT - 1) / WT);
  const int items = ntiles * S;
  const int grid = items < ctas ? items : ctas;
  if (bpart != nullptr) hipLaunchKernelGGL(wgrad_pp_kernel<true>, dim3(grid), dim3(WNT), 0, st, g);
  else hipLaunchKernelGGL(wgrad_pp_kernel<false>, dim3(grid), dim3(WNT), 0, st, g);
}

}  // namespace pllm

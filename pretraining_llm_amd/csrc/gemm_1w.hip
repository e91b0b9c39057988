// One-wave-per-SIMD TN GEMM on gfx950 MFMA (round 6):
//     C[M, N] = A[M, K] . B[N, K]^T (+ bias)          (bf16 in, fp32 accumulate, bf16 out)
// Reference math: the projections of /root/reference/src/models/mlp.py:24-26 and attention.py:29-31.
//
// Why this shape (profiles/r6_pmc_gemm_vs_hipblaslt.md): on the GPT-2 shapes hipBLASLt's winning kernel
// (MT256x256x64, MI16x16) runs 4 waves per 256x256 tile -- one per SIMD, 128x128 outputs each -- loads its
// operands straight into LDS (0.13 VMEM and 0.25 LDS instructions per MFMA: the fragment reads only) and
// issues 0.37-0.58 SALU per MFMA; the two-waves-per-SIMD ping-pong kernel of gemm_pp.hip issues 1.2 SALU and
// 0.44 LDS per MFMA, parks 34-39 % of its wave cycles on barriers / counted waits and keeps the matrix pipe
// 53-63 % busy at the measured clock against hipBLASLt's 56-69 %.  This kernel is the one-wave form:
//  * 256x256 tile per 256-thread workgroup, persistent over tiles (grouped order, XCD-aware remap); wave
//    (wr, wc) owns rows wr*128 + [0,128) and columns wc*128 + [0,128): 8 x 8 accumulators of
//    v_mfma_f32_16x16x32_bf16 (256 fp32 per lane; one wave per SIMD, 512 registers);
//  * the operand stream is a ring of 4 LDS stages of one 32-deep K-tile each (A and B images [256][32],
//    16 KiB each), filled by LDS-DMA (buffer_load ... lds, 1 KiB = one 16-row block per instruction, each
//    wave 4 A + 4 B blocks per K-tile) three K-tiles ahead, across tile boundaries;
//  * K-tile q's fragments (8 A + 8 B ds_read_b128) are read during K-tile q - 1's 64 MFMAs into the other
//    half of a double-buffered register set, and K-tile q + 3's DMA is issued among the same MFMAs: per 8
//    MFMAs one A read, one B read and one DMA piece;
//  * ONE barrier per K-tile: after it, K-tile q + 2 has landed for every wave (each waited for its own
//    pieces with a counted vmcnt that leaves K-tile q + 3 in flight) and every wave has read K-tile q - 1's
//    stage, which the next DMA overwrites;
//  * images: 64-B rows, the 16-B chunk g of row r at position g ^ h((r >> 2) & 3), h = {0, 2, 3, 1}: the
//    fragment reads (lane: row l % 16, chunk l / 16) hit 16 distinct 16-B bank slots in every ds_read_b128
//    lane group; the DMA applies the swizzle through its per-lane SOURCE offsets;
//  * B image rows are permuted inside each 32-row pair (image row 16 t + n <- column 8 (n >> 2) + 4 t +
//    (n & 3)), so the accumulators of column tiles 2p and 2p + 1 hold 8 consecutive output columns per lane
//    (the ping-pong kernel's trick): the epilogue stores 16 B per lane from registers.
// Requires K % 64 == 0, N % 8 == 0, lda % 8 == 0 (checked by the binding).
#include "common.h"
#include "kernels.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int OT = 256;             // output tile (M and N)
constexpr int OBK = 32;             // K per stage
constexpr int ONS = 4;              // LDS stages
constexpr int OIMG = OT * OBK;      // elements of one operand image (16 KiB)
constexpr int OSTAGE = 2 * OIMG;    // A image then B image: 32 KiB
constexpr int ONT = 256;            // 4 waves
constexpr uint32_t kOOff = 0x80000000u;  // a byte offset past every descriptor built here
constexpr int kOStores = 32;        // epilogue stores per lane (8 row tiles x 4 column pairs)

PL_DEV f32x4 mf16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
PL_DEV bf16x8 o_ld(const char* p) { return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(p)); }
PL_DEV void o_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
template <int N>
PL_DEV void o_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// chunk position of logical 16-B chunk g in image row r (row within its 16-row block)
PL_DEV int o_swz(int r, int g) { return g ^ ((0x1320 >> (4 * ((r >> 2) & 3))) & 3); }
// 16 B per lane into LDS [m0 + 16 lane] from base + voff + soff (soff: the K-tile's byte offset, scalar)
PL_DEV void o_dma(const i32x4v& srd, uint32_t voff, uint32_t soff, unsigned lds_byte) {
  asm volatile("s_mov_b32 m0, %3\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(srd),
               "s"(__builtin_amdgcn_readfirstlane(soff)), "s"(__builtin_amdgcn_readfirstlane(lds_byte))
               : "memory", "m0");
}

#ifndef PL_W1_GLDS
#define PL_W1_GLDS 0
#endif
// (PL_W1_GLDS A/B: global_load_lds_dwordx4 with a scalar 64-bit base + 32-bit per-lane offsets instead of the
// buffer form; no range check, so the per-lane offsets of rows past M / N are clamped to row 0 per tile)
PL_DEV void o_glds(uint64_t base, uint32_t voff, unsigned lds_byte) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(base),
               "s"(__builtin_amdgcn_readfirstlane(lds_byte))
               : "memory", "m0");
}

// grouped tile order: gm m-tiles x all n-tiles, m fastest inside a group
PL_DEV void o_tile(int t, int tiles_m, int tiles_n, int gm, int& tm, int& tn) {
  const int per_group = gm * tiles_n;
  const int grp = t / per_group, first_m = grp * gm, gsize = min(gm, tiles_m - first_m);
  tm = first_m + (t % per_group) % gsize;
  tn = (t % per_group) / gsize;
}

struct OFrag {
  bf16x8 a[8], b[8];
};

struct OCtx {
  const pllm::GemmArgs* g;
  int lid, G, tiles_m, tiles_n, S, R;
  int w, wr, wc, lane;
  unsigned lds;             // LDS byte address of the ring (DMA targets)
  uint32_t voA[4], voB[4];  // per-lane DMA source offsets of this wave's 4 A / 4 B blocks
  unsigned rd;              // per-lane fragment read offset inside a 16-row block
};

// The DMA cursor: the next K-tile of the stream to load (tile tl of this workgroup, K-tile kt), its
// descriptors (rebuilt only when the stream enters a new tile) and stage
struct ODma {
  i32x4v a, b;
  int tl, kt, q;
  uint64_t ga, gb;       // PL_W1_GLDS: panel bases (tile's first row, column 0)
  uint32_t ca[4], cb[4];  // PL_W1_GLDS: per-lane offsets, rows past M / N clamped to row 0
};
PL_DEV void o_dma_tile(const OCtx& c, ODma& d) {
  const pllm::GemmArgs& g = *c.g;
  if (d.tl < c.R) {
    int tm, tn;
    o_tile(c.lid + d.tl * c.G, c.tiles_m, c.tiles_n, g.group_m, tm, tn);
    const int ra = min(OT, g.M - tm * OT), rb = min(OT, g.N - tn * OT);
    d.a = srd_of(g.A + (int64_t)tm * OT * g.lda, (uint32_t)((int64_t)(ra - 1) * g.lda * 2 + (int64_t)g.K * 2));
    d.b = srd_of(g.B + (int64_t)tn * OT * g.ldb, (uint32_t)((int64_t)(rb - 1) * g.ldb * 2 + (int64_t)g.K * 2));
    if (PL_W1_GLDS) {
      d.ga = (uint64_t)(uintptr_t)(g.A + (int64_t)tm * OT * g.lda);
      d.gb = (uint64_t)(uintptr_t)(g.B + (int64_t)tn * OT * g.ldb);
      const int rr = c.lane >> 2;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int blk = 4 * c.w + k;
        d.ca[k] = 16 * blk + rr < ra ? c.voA[k] : 0u;
        const int brow = 32 * (blk >> 1) + 8 * (rr >> 2) + 4 * (blk & 1) + (rr & 3);
        d.cb[k] = brow < rb ? c.voB[k] : 0u;
      }
    }
  } else {  // past the stream's end: the same instructions on empty ranges (the counted waits stay exact)
    d.a = srd_of(g.A, 0u);
    d.b = srd_of(g.B, 0u);
    if (PL_W1_GLDS) {  // (no range check: row 0 of each operand, read and never used)
      d.ga = (uint64_t)(uintptr_t)g.A;
      d.gb = (uint64_t)(uintptr_t)g.B;
#pragma unroll
      for (int k = 0; k < 4; ++k) d.ca[k] = d.cb[k] = 0u;
    }
  }
}
PL_DEV void o_dma_advance(const OCtx& c, ODma& d) {
  ++d.q;
  if (++d.kt == c.S) {
    d.kt = 0;
    ++d.tl;
    o_dma_tile(c, d);
  }
}
// piece k of the cursor's K-tile (k < 4: A block 4w + k, else B block 4w + k - 4)
PL_DEV void o_piece(const OCtx& c, const ODma& d, int k) {
  const unsigned st = c.lds + (unsigned)((d.q & (ONS - 1)) * OSTAGE * 2);
  const uint32_t koff = (uint32_t)d.kt * OBK * 2u;
  const int blk = 4 * c.w + (k & 3);
  if (PL_W1_GLDS) {
    if (k < 4) o_glds(d.ga + koff, d.ca[k], st + (unsigned)blk * 1024u);
    else o_glds(d.gb + koff, d.cb[k - 4], st + (unsigned)(OIMG * 2 + blk * 1024));
    return;
  }
  if (k < 4) o_dma(d.a, c.voA[k], koff, st + (unsigned)blk * 1024u);
  else o_dma(d.b, c.voB[k - 4], koff, st + (unsigned)(OIMG * 2 + blk * 1024));
}
// two fragments of K-tile q in the order the next K-tile's MFMAs first need them: group i < 4 reads B column
// tiles 2i, 2i + 1 (every row tile's first 8 MFMAs use all eight), group i >= 4 A row tiles 2i - 8, 2i - 7
// (sm: the ring as a generic pointer to the __shared__ array)
PL_DEV void o_read(const OCtx& c, const char* sm, int q, OFrag& f, int i) {
  const char* st = sm + (q & (ONS - 1)) * OSTAGE * 2;
  if (i < 4) {
    f.b[2 * i] = o_ld(st + OIMG * 2 + c.rd + (8 * c.wc + 2 * i) * 1024);
    f.b[2 * i + 1] = o_ld(st + OIMG * 2 + c.rd + (8 * c.wc + 2 * i + 1) * 1024);
  } else {
    f.a[2 * i - 8] = o_ld(st + c.rd + (8 * c.wr + 2 * i - 8) * 1024);
    f.a[2 * i - 7] = o_ld(st + c.rd + (8 * c.wr + 2 * i - 7) * 1024);
  }
}

// one K-tile q: 64 MFMAs on cur; K-tile q + 1's fragments into nxt; the cursor's K-tile (q + 3) by DMA;
// counted wait; barrier
template <bool FIRST>
PL_DEV void o_ktile(const OCtx& c, const char* sm, f32x4 (&acc)[8][8], const OFrag& cur, OFrag& nxt, int q,
                    ODma& d, bool after_epi) {
#ifndef PL_W1_EXP
#define PL_W1_EXP 0
#endif
  // (PL_W1_EXP: timing-only A/B builds -- 1: no DMA, 2: no fragment reads (both wrong results); 3: the DMA
  // piece in the middle of a row tile's 8 MFMAs, the reads after them; 4: all 8 pieces before the MFMAs)
  if (PL_W1_EXP == 4) {
#pragma unroll
    for (int k = 0; k < 8; ++k) o_piece(c, d, k);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (FIRST) acc[i][j] = mf16(cur.b[j], cur.a[i], f32x4{0.f, 0.f, 0.f, 0.f});
      else acc[i][j] = mf16(cur.b[j], cur.a[i], acc[i][j]);
      if (PL_W1_EXP == 3 && j == 3) {
        __builtin_amdgcn_sched_barrier(0);
        o_piece(c, d, i);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (PL_W1_EXP != 2) o_read(c, sm, q + 1, nxt, i);
    if (PL_W1_EXP == 0 || PL_W1_EXP == 2) o_piece(c, d, i);
    __builtin_amdgcn_sched_barrier(0);
  }
  o_dma_advance(c, d);
  // K-tile q + 2 landed (this wave's pieces): all but q + 3's 8 pieces -- and, in a tile's first K-tile, the
  // previous tile's epilogue stores issued between them
  if (after_epi) o_vmwait<8 + kOStores>();
  else o_vmwait<8>();
  o_barrier();
}

// epilogue of tile (tm, tn): lane (r16, g) holds row 16 i + r16 and columns 32 p + 8 g + [0, 8) of its wave's
// 128 x 128 block in acc[i][2p] (first 4) and acc[i][2p + 1]; bias added in fp32, one rounding to bf16
PL_DEV void o_epilogue(const OCtx& c, const f32x4 (&acc)[8][8], int tm, int tn) {
  const pllm::GemmArgs& g = *c.g;
  const int m0 = tm * OT, n0 = tn * OT;
  const int rows_ok = min(OT, g.M - m0);
  int r16 = c.lane & 15;
  asm volatile("" : "+v"(r16));  // (opaque: keeps hipcc from hoisting the row offsets out of the tile loop)
  const int g4 = c.lane >> 4;
  const int colw = n0 + c.wc * 128 + 8 * g4;  // + 32 p
  const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(g.bias != nullptr ? g.bias : g.A), (short)0, g.bias != nullptr ? g.N * 2 : 0, 0x00020000);
#pragma unroll
  for (int p = 0; p < 4; ++p) {  // column pair by column pair: 8 bias values live at a time
    const int col = colw + 32 * p;
    float bias[8];
    unpack8(buf_ld16(brs, col < g.N ? (uint32_t)col * 2u : kOOff), bias);
    // per row tile a descriptor based at its first row (scalar): one per-lane offset for all eight
    const uint32_t off = col < g.N ? (uint32_t)((r16 * (int)g.ldc + col) * 2) : kOOff;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r0 = c.wr * 128 + 16 * i;
      const int rows_i = max(0, min(16, rows_ok - r0));
      const __amdgpu_buffer_rsrc_t crs = rows_rsrc(g.C + (int64_t)(m0 + (rows_i > 0 ? r0 : 0)) * g.ldc, rows_i, g.ldc, g.N);
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc[i][2 * p][e] + bias[e];
        v[4 + e] = acc[i][2 * p + 1][e] + bias[4 + e];
      }
      __builtin_amdgcn_raw_buffer_store_b128(pack8(v), crs, off, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int EPI>
__global__ __launch_bounds__(ONT, 1) void gemm_1w_kernel(pllm::GemmArgs g) {
  __shared__ __attribute__((aligned(1024))) uint16_t smem[ONS * OSTAGE];
  OCtx c;
  c.g = &g;
  c.tiles_m = (g.M + OT - 1) / OT;
  c.tiles_n = (g.N + OT - 1) / OT;
  const int ntiles = c.tiles_m * c.tiles_n;
  c.G = gridDim.x;
  c.lid = xcd_remap(blockIdx.x, c.G);
  if (c.lid >= ntiles) return;
  c.R = (ntiles - c.lid + c.G - 1) / c.G;
  c.S = g.K / OBK;
  const int tid = threadIdx.x;
  c.lane = tid & 63;
  c.w = __builtin_amdgcn_readfirstlane(tid >> 6);
  c.wr = c.w >> 1;
  c.wc = c.w & 1;
  c.lds = (unsigned)(uintptr_t)smem;
  {
    // DMA: lane l fills image row rr = l / 4 of a 16-row block at position l % 4, which holds logical chunk
    // (l % 4) ^ h(rr); B rows permuted inside each 32-row pair (block 2p + t, image row n <- row
    // 32 p + 8 (n >> 2) + 4 t + (n & 3))
    const int rr = c.lane >> 2, ch = o_swz(rr, c.lane & 3);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int blk = 4 * c.w + k, t = blk & 1;
      c.voA[k] = (uint32_t)(((int64_t)(16 * blk + rr) * g.lda + 8 * ch) * 2);
      const int brow = 32 * (blk >> 1) + 8 * (rr >> 2) + 4 * t + (rr & 3);
      c.voB[k] = (uint32_t)(((int64_t)brow * g.ldb + 8 * ch) * 2);
    }
    const int r16 = c.lane & 15, g4 = c.lane >> 4;
    c.rd = (unsigned)(r16 * 64 + o_swz(r16, g4) * 16);
  }
  // prologue: K-tiles 0, 1, 2 of the stream in flight, 0 and 1 landed
  const char* sm = reinterpret_cast<const char*>(smem);
  ODma d;
  d.tl = 0;
  d.kt = 0;
  d.q = 0;
  o_dma_tile(c, d);
#pragma unroll
  for (int q = 0; q < 3; ++q) {
#pragma unroll
    for (int k = 0; k < 8; ++k) o_piece(c, d, k);
    o_dma_advance(c, d);
  }
  o_vmwait<8>();
  o_barrier();
  f32x4 acc[8][8];
  OFrag f0, f1;
#pragma unroll
  for (int i = 0; i < 8; ++i) o_read(c, sm, 0, f0, i);
  int q = 0;
  for (int tl = 0; tl < c.R; ++tl) {
    int tm, tn;
    o_tile(c.lid + tl * c.G, c.tiles_m, c.tiles_n, g.group_m, tm, tn);
    // K-tiles come in pairs (K % 64 == 0): the even one computes on f0, the odd one on f1
    o_ktile<true>(c, sm, acc, f0, f1, q, d, tl > 0);
    o_ktile<false>(c, sm, acc, f1, f0, q + 1, d, false);
    q += 2;
    for (int kt = 2; kt < c.S; kt += 2, q += 2) {
      o_ktile<false>(c, sm, acc, f0, f1, q, d, false);
      o_ktile<false>(c, sm, acc, f1, f0, q + 1, d, false);
    }
    __builtin_amdgcn_sched_barrier(0);
    o_epilogue(c, acc, tm, tn);
    __builtin_amdgcn_sched_barrier(0);
  }
  o_vmwait<0>();
}

}  // namespace

namespace pllm {

bool gemm_1w_supported(int M, int N, int K) { return K % 64 == 0 && K >= 128 && N % 8 == 0 && M > 0 && N > 0; }

void gemm_tn_1w(const GemmArgs& a, int ctas, hipStream_t st) {
  const int ntiles = ((a.M + OT - 1) / OT) * ((a.N + OT - 1) / OT);
  if (ntiles == 0) return;
  const int grid = ntiles < ctas ? ntiles : ctas;
  hipLaunchKernelGGL((gemm_1w_kernel<0>), dim3(grid), dim3(ONT), 0, st, a);
}

}  // namespace pllm

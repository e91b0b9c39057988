// "NT" GEMM with fused MLP epilogues: C[M, N] = A[M, K] . B[N, K]^T (both operands
// K-contiguous, bf16 in, fp32 accumulate), gfx950.
//
// Why a hand-written kernel next to hipBLASLt: the GPT-2 MLP runs GEMM -> GELU as two
// passes in the forward (hipBLASLt has no bf16 GELU+aux epilogue on gfx950: the
// heuristic returns no algorithm, profiles/r1_hipblaslt_epilogue_probe.jsonl) and
// dgrad -> dGELU -> bias-sum as two passes in the backward (its DGELU epilogue runs at
// 214 TFLOP/s).  At B*T = 65,536 tokens each extra pass moves 1.2 GB of HBM traffic.
// Epilogues:
//   EPI 0  C = A B^T (+ bias)                                 plain (A/B against hipBLASLt)
//   EPI 1  H = A B^T + bias (stored, bf16), C = gelu(H)        MLP up-projection forward
//   EPI 2  C = (A B^T) * gelu'(H), bias partials of C           MLP down-projection dgrad
// Tiling (the machine model of gemm_wgrad.hip):
//  * 256 x 256 output tile per workgroup, 8 waves as 2 (M) x 4 (N), each 128 x 64 as 4 x 2
//    v_mfma_f32_32x32x16_bf16 accumulators; 1 workgroup per CU (128 KiB of LDS).  The MFMA
//    takes the B fragment in its A slot, so a lane ends up owning one output ROW and runs
//    of 4 consecutive columns: 8-byte epilogue stores instead of 2-byte ones;
//  * operands staged HBM/L2 -> LDS by global_load_lds (16 B per lane, no staging
//    registers, lane-linear LDS image with the swizzle applied to the SOURCE address);
//    PIPE 0: K staged 64 deep in two slots, one vmcnt(0) + barrier per stage;
//    PIPE 1: K staged 32 deep in a four-slot ring, three stages in flight, counted
//            vmcnt(8/4/0) + raw s_barrier so the DMA stays in flight across barriers
//            (cdna_hip_programming.md "Pipelining across barriers");
//  * LDS image per operand: [256 rows][BK] bf16; 16-B chunk c of row r sits at
//    c ^ ((r >> s) & (BK/8 - 1)) with s chosen so the 16 rows one ds_read_b128 lane group
//    reads land on 16 distinct bank quads -> conflict-free operand reads;
//  * tiles are visited in groups of 8 M-tiles (all N-tiles of a group back to back) after
//    the XCD remap, so an XCD's L2 holds a group's A panels while the weight panels stream.
// Requires K % 64 == 0, N % 8 == 0 (host-checked); M and N edges are clamped/masked.
//
// STATUS: correct (tests/test_kernels_gpu.py::test_gemm_nt_epilogues) but NOT on the training
// path.  Measured at M = 65,536 (profiles/r1_gemm_nt_bench.jsonl) this single-stage-pipeline
// structure reaches 0.72-0.99 PFLOP/s against hipBLASLt's 1.10-1.40 on the same shapes, and
// the fused epilogues lose to hipBLASLt + the separate activation kernels (up-projection
// 532 vs 468 us, dGELU dgrad 619 vs 518 us).  Beating it needs the 8-phase counted-vmcnt
// main loop (cdna_hip_programming.md §5 "The 256² 8-phase template") under these epilogues.
#include "common.h"
#include "kernels.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

PLLM_DEV f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
PLLM_DEV bf16x8 frag(const uint16_t* p) { return __builtin_bit_cast(bf16x8, ld16(p)); }
PLLM_DEV void glds16(const void* src, unsigned lds_byte) {
  // inline asm (see gemm_wgrad.hip): hipcc's waitcnt pass must not drain the prefetch early
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src),
               "s"(__builtin_amdgcn_readfirstlane(lds_byte))
               : "memory", "m0");
}

constexpr int BT = 256;  // output tile (M and N)
constexpr int NT = 512;  // 8 waves
constexpr int GM = 8;    // M-tiles per visiting group

template <int PIPE>
struct Pipe {
  static constexpr int BK = PIPE == 0 ? 64 : 32;   // k per stage
  static constexpr int SLOTS = PIPE == 0 ? 2 : 4;  // LDS stage slots (128 KiB either way)
  static constexpr int AHEAD = PIPE == 0 ? 1 : 3;  // stages issued ahead of the one computed
  static constexpr int CPR = BK / 8;               // 16-B chunks per image row
  static constexpr int SH = CPR == 8 ? 1 : 2;      // swizzle: rows per 256-B bank row = 1 << SH
  static constexpr int IMG = BT * BK;              // elements of one operand image
  static constexpr int STAGE = 2 * IMG;
  static constexpr int RPP = 64 / CPR;             // image rows per 1-KiB wave-instruction piece
  static constexpr int PIECES = 2 * BT / RPP;      // pieces per stage (both operands)
  static constexpr int PPW = PIECES / 8;           // pieces (glds per lane) per wave and stage
};

template <int PIPE>
PLLM_DEV int img_off(int r, int c) {
  using P = Pipe<PIPE>;
  return r * P::BK + ((c ^ ((r >> P::SH) & (P::CPR - 1))) << 3);
}

PLLM_DEV float lo(uint32_t w) { return lo_bf(w); }
PLLM_DEV float hi(uint32_t w) { return hi_bf(w); }

// tile id -> (m0, n0): groups of GM M-tiles, all N-tiles of a group back to back
PLLM_DEV void tile_origin(int t, int tiles_m, int tiles_n, int& m0, int& n0) {
  const int grp = t / (GM * tiles_n), rem = t % (GM * tiles_n);
  const int gm0 = grp * GM, gsz = min(GM, tiles_m - gm0);
  m0 = (gm0 + rem % gsz) * BT;
  n0 = (rem / gsz) * BT;
}

// epilogue: lane owns output row m = .. + 32 i + r; element 4k+q of block (i, j) is column
// n = n0 + 64 wn + 32 j + 8 k + 4 hh + q  -> four consecutive columns per 8-byte access
template <int EPI>
PLLM_DEV void epilogue(const GemmNTArgs& a, f32x16 (&acc)[4][2], int m0, int n0, int wm, int wn, int r, int hh) {
  const int M = a.M, N = a.N;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int nb = n0 + wn * 64 + 32 * j + 4 * hh;
    float bias[16];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int n = nb + 8 * k;
      u32x2 bv = u32x2{0u, 0u};
      if (EPI != 2 && a.bias != nullptr && n < N) bv = *reinterpret_cast<const u32x2*>(a.bias + n);
      bias[4 * k] = lo(bv[0]);
      bias[4 * k + 1] = hi(bv[0]);
      bias[4 * k + 2] = lo(bv[1]);
      bias[4 * k + 3] = hi(bv[1]);
    }
    float cs[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) cs[e] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm * 128 + 32 * i + r;
      const bool mok = m < M;
      const int64_t row = (int64_t)min(m, M - 1) * a.ldc;
      if (EPI == 2) {
        u32x2 hv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)  // all aux loads first (clamped), then the math and stores
          hv[k] = *reinterpret_cast<const u32x2*>(a.aux + row + min(nb + 8 * k, N - 4));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int n = nb + 8 * k;
          const float h[4] = {lo(hv[k][0]), hi(hv[k][0]), lo(hv[k][1]), hi(hv[k][1])};
          float d[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) d[q] = acc[i][j][4 * k + q] * gelu_df(h[q]);
          const u32x2 o = u32x2{pack_bf16x2(d[0], d[1]), pack_bf16x2(d[2], d[3])};
          if (mok && n < N) {
            *reinterpret_cast<u32x2*>(a.C + row + n) = o;
            cs[4 * k] += lo(o[0]);
            cs[4 * k + 1] += hi(o[0]);
            cs[4 * k + 2] += lo(o[1]);
            cs[4 * k + 3] += hi(o[1]);
          }
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int n = nb + 8 * k;
          if (mok && n < N) {
            float v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = acc[i][j][4 * k + q] + bias[4 * k + q];
            const u32x2 hb = u32x2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
            if (EPI == 1) {
              *reinterpret_cast<u32x2*>(a.aux + row + n) = hb;
              const u32x2 g = u32x2{pack_bf16x2(gelu_f(lo(hb[0])), gelu_f(hi(hb[0]))),
                                    pack_bf16x2(gelu_f(lo(hb[1])), gelu_f(hi(hb[1])))};
              *reinterpret_cast<u32x2*>(a.C + row + n) = g;
            } else {
              *reinterpret_cast<u32x2*>(a.C + row + n) = hb;
            }
          }
        }
      }
    }
    if (EPI == 2) {
      // column sums over this wave's 128 rows: the 4 i-blocks (above), then the 32 lanes of
      // each half-wave -> partial row (2 * m-tile + wm) of the bias-gradient workspace
#pragma unroll
      for (int e = 0; e < 16; ++e) {
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) cs[e] += __shfl_xor(cs[e], o, 64);
      }
      if (r == 0) {
        float* pr = a.part + (int64_t)(2 * (m0 / BT) + wm) * N;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int n = nb + 8 * k;
          if (n < N) *reinterpret_cast<f32x4*>(pr + n) = f32x4{cs[4 * k], cs[4 * k + 1], cs[4 * k + 2], cs[4 * k + 3]};
        }
      }
    }
  }
}

// Persistent: one workgroup per CU walks tiles lid, lid + grid, ...; the (tile, k-stage)
// sequence of a workgroup is ONE stage stream, so the DMA of the next tile's first stages
// is in flight while the current tile's epilogue stores drain.
template <int EPI, int PIPE>
__global__ __launch_bounds__(NT) void gemm_nt_kernel(GemmNTArgs a) {
  using P = Pipe<PIPE>;
  constexpr int BK = P::BK, SLOTS = P::SLOTS, AHEAD = P::AHEAD, CPR = P::CPR, IMG = P::IMG, STAGE = P::STAGE;
  constexpr int RPP = P::RPP, PPW = P::PPW, HALF_PIECES = P::PIECES / 2;
  __shared__ __attribute__((aligned(1024))) uint16_t smem[SLOTS * STAGE];
  const int M = a.M, N = a.N;
  const int tiles_m = (M + BT - 1) / BT, tiles_n = (N + BT - 1) / BT, tiles = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int lid = xcd_remap(blockIdx.x, G);
  const int my_tiles = lid < tiles ? (tiles - 1 - lid) / G + 1 : 0;
  const int nstage = a.K / BK;
  const int total = my_tiles * nstage;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int wm = w >> 2, wn = w & 3;

  // DMA plan: lane l of a piece fills image row RPP*g + l/CPR at chunk position l%CPR, which
  // holds logical chunk (l%CPR) ^ swizzle(row).  Rows past M/N are clamped to a valid row:
  // they only feed output rows/columns that are never stored.
  int prow[PPW], pcol[PPW], dst[PPW];
#pragma unroll
  for (int k = 0; k < PPW; ++k) {
    const int pc = w * PPW + k, g = pc % HALF_PIECES;
    prow[k] = RPP * g + lane / CPR;
    pcol[k] = ((lane % CPR) ^ ((prow[k] >> P::SH) & (CPR - 1))) * 8;
    dst[k] = (pc / HALF_PIECES) * IMG + g * 512;
  }
  const unsigned lds_base = (unsigned)(uintptr_t)smem;
  auto issue = [&](int gs) {
    const int t = lid + (gs / nstage) * G, st = gs % nstage, slot = gs % SLOTS;
    int tm0, tn0;
    tile_origin(t, tiles_m, tiles_n, tm0, tn0);
#pragma unroll
    for (int k = 0; k < PPW; ++k) {
      const bool opa = (w * PPW + k) < HALF_PIECES;  // wave-uniform
      const uint16_t* s = opa ? a.A + (int64_t)min(tm0 + prow[k], M - 1) * a.lda
                              : a.B + (int64_t)min(tn0 + prow[k], N - 1) * a.ldb;
      glds16(s + pcol[k] + st * BK, lds_base + 2u * (unsigned)(slot * STAGE + dst[k]));
    }
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

#pragma unroll
  for (int s = 0; s < AHEAD; ++s)
    if (s < total) issue(s);
  for (int gs = 0; gs < total; ++gs) {
    // retire stage gs; the stages issued after it stay in flight across the barrier
    const int pending = min(AHEAD - 1, total - 1 - gs);
    if (PIPE == 0 || pending <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (pending == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's DMA of stage gs landed; slot of gs-1 is free
    asm volatile("" ::: "memory");
    if (gs + AHEAD < total) issue(gs + AHEAD);
    const uint16_t* Ai = smem + (gs % SLOTS) * STAGE;
    const uint16_t* Bi = Ai + IMG;
#pragma unroll
    for (int k16 = 0; k16 < BK / 16; ++k16) {
      const int c = 2 * k16 + hh;
      bf16x8 af[4], bfr[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = frag(Bi + img_off<PIPE>(wn * 64 + 32 * j + r, c));
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag(Ai + img_off<PIPE>(wm * 128 + 32 * i + r, c));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(bfr[j], af[i], acc[i][j]);
    }
    if (gs % nstage == nstage - 1) {
      int m0, n0;
      tile_origin(lid + (gs / nstage) * G, tiles_m, tiles_n, m0, n0);
      epilogue<EPI>(a, acc, m0, n0, wm, wn, r, hh);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    }
  }
}

template <int PIPE>
void launch(const GemmNTArgs& a, int epi, int grid, hipStream_t st) {
  switch (epi) {
    case 0: hipLaunchKernelGGL((gemm_nt_kernel<0, PIPE>), dim3(grid), dim3(NT), 0, st, a); break;
    case 1: hipLaunchKernelGGL((gemm_nt_kernel<1, PIPE>), dim3(grid), dim3(NT), 0, st, a); break;
    default: hipLaunchKernelGGL((gemm_nt_kernel<2, PIPE>), dim3(grid), dim3(NT), 0, st, a); break;
  }
}

}  // namespace

namespace pllm {

// staging pipeline of gemm_nt (0: BK 64 double buffer, 1: BK 32 four-slot ring); bench/gemm_nt_bench.py
static int g_gemm_nt_pipe = 0;
static bool g_gemm_nt_persistent = false;
void gemm_nt_set_pipe(int p) {
  g_gemm_nt_pipe = (p & 1);
  g_gemm_nt_persistent = (p & 2) != 0;
}

int gemm_nt_part_rows(int M) { return 2 * ((M + BT - 1) / BT); }

void gemm_nt(const GemmNTArgs& a, int epi, hipStream_t st) {
  const int tiles = ((a.M + BT - 1) / BT) * ((a.N + BT - 1) / BT);
  if (tiles == 0) return;
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  // one tile per workgroup by default; the persistent form (one workgroup per CU walking its
  // tiles as one stage stream) measured 1.4-1.7x SLOWER (profiles/r1_gemm_nt_persistent_bench.jsonl)
  const int grid = g_gemm_nt_persistent ? (tiles < cus ? tiles : cus) : tiles;
  if (g_gemm_nt_pipe == 0) launch<0>(a, epi, grid, st);
  else launch<1>(a, epi, grid, st);
  PLLM_CHECK_LAUNCH();
}

}  // namespace pllm

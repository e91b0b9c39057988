// Forward / data-gradient GEMM with fused epilogues on gfx950 MFMA:
//     C[M, N] = epi( A[M, K] . B[N, K]^T )          (bf16 in, fp32 accumulate, bf16 out)
// Both operands are K-contiguous ("TN"): the forward linear (A = activations, B = the weight
// [out, in]) and the data gradient through the optimizer's transposed weight shadow
// (A = dY, B = W^T).  It exists for the epilogues hipBLASLt cannot run in bf16 on gfx950
// (profiles/r2_hipblaslt_epilogue_probe.md): the MLP up-projection's bias + GELU / ReLU (the
// pre-activation is kept for the backward) and the MLP down-projection's data gradient fused
// with the activation backward and the up-projection's bias-gradient column sums, which
// otherwise are two full memory-bound passes over the [tokens, 4C] hidden activations
// (act_fwd_kernel, act_bwd_colsum_kernel).  Reference math: the MLP of
// /root/reference/src/models/mlp.py:24-26,39-41 (ReLU) and the GPT-2 preset's GELU.
//
// Design (CDNA4), after csrc/gemm_wgrad.hip:
//  * 256x256 output tile per 512-thread workgroup (8 waves, 2 per SIMD), wave (wm, wn) owns a
//    128x64 sub-tile; tiles grouped GROUP_M m-tiles at a time and dealt to the XCDs in
//    contiguous ranges (xcd_remap) so concurrently running tiles share A / B panels in L2;
//  * K staged 64 at a time HBM/L2 -> LDS by buffer_load ... lds (no staging registers):
//    64 one-KiB pieces per stage (8 rows x 128 B each), double-buffered, one barrier per stage;
//    the 128-B image rows are XOR-swizzled in 16-B chunks (chunk ^ ((row >> 1) & 7)) through the
//    per-lane SOURCE address, which makes the ds_read_b128 fragment reads conflict-free;
//  * MFMA operands swapped (the weight rows feed the A operand), so every accumulator lane holds
//    4 consecutive output columns: the epilogue packs them into 8-B LDS stores, reads the wave's
//    128x64 tile back as rows and writes / reads global memory in whole 128-B rows;
//  * epilogues (EPI): 0 plain (+bias), 1 GELU (C = gelu(pre), aux = pre = acc + bias),
//    2 ReLU (C = relu(acc + bias)), 3 GELU backward (aux = pre in, C = acc * gelu'(pre)),
//    4 ReLU backward (aux = relu output in, C = acc * (aux > 0)), 5 SwiGLU backward (aux = the
//    up-projection's [gate | up] output [M, 2N] in, C = [dgate | dup] [M, 2N]: the llama MLP's
//    down-projection data gradient fused with swiglu_bwd_kernel), 6 attention-output projection data
//    gradient (aux = the attention output O [M, N] in, C = dO = acc, plus delta[b, h, t] = sum over
//    the 64 columns of head h of dO * O: the attention backward's row constants, so its
//    attn_bwd_pre_kernel pass over dO and O disappears; head dim 64); 3 / 4 also write the column
//    sums of C per (tile row, wave row) to an fp32 slab for the bias gradient (fixed order,
//    deterministic).  Every value that the unfused path rounds to bf16 is rounded here too
//    (pre before the activation, the data gradient before the activation backward).
// Requires K % 64 == 0, N % 8 == 0, lda / ldb / ldc / ldaux % 8 == 0 (checked by the binding).
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int GT = 256;             // output tile (M and N)
constexpr int GBK = 64;             // K per stage
constexpr int GNT = 512;            // 8 waves
constexpr int GIMG = GT * GBK;      // elements of one operand image [256][64]
constexpr int GSTAGE = 2 * GIMG;    // A image then B image: 64 KiB

PL_DEV int gswz(int row) { return (row >> 1) & 7; }
PL_DEV int gimg_off(int row, int chunk) { return row * GBK + ((chunk ^ gswz(row)) << 3); }
PL_DEV bf16x8 lds_frag(const uint16_t* p) { return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(p)); }
PL_DEV int acc_row32(int e, int half) { return (e & 3) + 8 * (e >> 2) + 4 * half; }

// grouped tile order: GROUP_M m-tiles x all n-tiles, m fastest inside a group
PL_DEV void tile_of(int t, int tiles_m, int tiles_n, int gm, int& tm, int& tn) {
  const int per_group = gm * tiles_n;
  const int grp = t / per_group, first_m = grp * gm, gsize = min(gm, tiles_m - first_m);
  tm = first_m + (t % per_group) % gsize;
  tn = (t % per_group) / gsize;
}

// buffer store / load of 16 B at a per-lane byte offset; an offset past the descriptor's range
// drops the store / reads zeros, so every lane issues every instruction (exact vmcnt counts)
constexpr uint32_t kOff = 0x80000000u;  // an offset past every descriptor built here (< 2 GiB)
PL_DEV void bst16(__amdgpu_buffer_rsrc_t r, uint32_t off, const u32x4& v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
}
PL_DEV u32x2 bld8(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}

// Epilogue of one 256x256 tile: acc (+ bias) -> bf16 -> the wave's [64][64] LDS region (8 KiB, two
// passes of 64 rows; 8-B granule g of row r at g ^ (r & 15)) -> rows read back as 16 B per lane,
// whole 128-B rows per 8 lanes -> epilogue op -> global by unconditional buffer ops (out-of-range
// lanes get an offset past the descriptor), exactly kEpiOps<MF, EPI> vector-memory instructions
// (EPI 5 issues 64: vmcnt's field holds at most 63, and waiting for one op more is still exact)
template <int MF, int EPI>
constexpr int kEpiOps = EPI == 5 ? 63
                        : EPI == 6 ? 48
                        : EPI == 1 ? 32 + (MF == 32 ? 8 : 4)
                                   : (EPI >= 3 ? 16 + 16 + 2 : 16 + (MF == 32 ? 8 : 4));

PL_DEV float swiglu_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

// (acc columns fragments [I0, I0 + NIE) are the wave's 64 columns)
template <int MF, int EPI, int I0 = 0, typename Acc, int NIA, int NJ>
PL_DEV void gemm_epilogue(const Acc (&acc)[NIA][NJ], uint16_t* tile, const pllm::GemmArgs& g,
                            const __amdgpu_buffer_rsrc_t& brs, int tm, int tn, int wm, int wn, int lane) {
  constexpr int NI = MF == 32 ? 2 : 4;
  static_assert(I0 + NI <= NIA, "column fragments");
  constexpr int NE = MF == 32 ? 16 : 4;
  constexpr int NQ = NE / 4;
  const int M = g.M, N = g.N;
  const int m0 = tm * GT, n0 = tn * GT, ncol0 = n0 + wn * 64;
    const int rows_ok = min(GT, M - m0);
  // EPI 5: C and aux rows hold two N-wide halves ([dgate | dup], [gate | up])
  constexpr int W2 = EPI == 5 ? 2 : 1;
  const __amdgpu_buffer_rsrc_t crs = rows_rsrc(g.C + (int64_t)m0 * g.ldc, rows_ok, g.ldc, W2 * N);
  const __amdgpu_buffer_rsrc_t ars = rows_rsrc(g.aux != nullptr ? g.aux + (int64_t)m0 * g.ldaux : g.C, rows_ok,
                                               g.ldaux, W2 * N);
  // EPI 6: delta [M / T, N / 64, T] fp32 (whole buffer; offsets past it drop the store)
  const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(g.delta != nullptr ? g.delta : (float*)g.C), (short)0, EPI == 6 ? (int)(4ll * M * N / 64) : 0,
      0x00020000);
  const int rsub = lane >> 3, c8 = lane & 7;
  const int col = ncol0 + 8 * c8;
  const bool col_ok = col < N;
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  u32x2 bias[NI][NQ];  // bias of the wave's columns (zeros without one: empty descriptor)
  if constexpr (EPI <= 2) {
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int c = MF == 32 ? 32 * i + 8 * q + 4 * (lane >> 5) : 16 * i + 4 * (lane >> 4);
        bias[i][q] = bld8(brs, (uint32_t)(ncol0 + c) * 2u);
      }
  }
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    // the half's aux rows (EPI >= 3), all 8 (16 for EPI 5) loads issued before the LDS pack: their
    // latency overlaps the pack and each other instead of one load -> use round trip per row
    // block (kEpiOps unchanged: the same instructions, reordered)
    // (two groups of 4 row blocks: group 1's loads go out as group 0's rows are processed; a fully
    // unrolled 8-block loop spilled)
    u32x4 anx[4], anx2[4];
    auto aload = [&](int grp) {
      if constexpr (EPI >= 3) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int rt = wm * 128 + hf * 64 + 8 * (4 * grp + k) + rsub;
          const uint32_t ao = col_ok ? (uint32_t)(((int64_t)rt * g.ldaux + col) * 2) : kOff;
          anx[k] = buf_ld16(ars, ao);
          if constexpr (EPI == 5) anx2[k] = buf_ld16(ars, col_ok ? ao + (uint32_t)N * 2u : kOff);
        }
      }
    };
    aload(0);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
#pragma unroll
      for (int jj = 0; jj < NJ / 2; ++jj) {
        const int j = hf * (NJ / 2) + jj;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          // 4 consecutive columns [c, c + 4) of local row r
          const int c = MF == 32 ? 32 * i + 8 * q + 4 * (lane >> 5) : 16 * i + 4 * (lane >> 4);
          const int r = MF == 32 ? 32 * jj + (lane & 31) : 16 * jj + (lane & 15);
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[I0 + i][j][4 * q + e];
          if constexpr (EPI <= 2) {
            v[0] += lo_bf(bias[i][q][0]);
            v[1] += hi_bf(bias[i][q][0]);
            v[2] += lo_bf(bias[i][q][1]);
            v[3] += hi_bf(bias[i][q][1]);
          }
          const u32x2 pk = {pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
          *reinterpret_cast<u32x2*>(tile + r * 64 + (((c >> 2) ^ (r & 15)) << 2)) = pk;
        }
      }
    }
    // one wave writes and reads its own region: LDS executes a wave's accesses in order
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll 1
    for (int grp = 0; grp < 2; ++grp) {
    u32x4 apre[4], apre2[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      apre[k] = anx[k];
      apre2[k] = anx2[k];
    }
    if (grp == 0) aload(1);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int it = 4 * grp + kk;
      const int r = 8 * it + rsub;
      const int s = r & 15;
      u32x4 v = *reinterpret_cast<const u32x4*>(tile + r * 64 + ((((2 * c8) ^ s) & ~1) << 2));
      if (s & 1) v = u32x4{v[2], v[3], v[0], v[1]};
      const int rt = wm * 128 + hf * 64 + r;  // row within the tile
      const uint32_t off = col_ok ? (uint32_t)(((int64_t)rt * g.ldc + col) * 2) : kOff;
      if constexpr (EPI == 0) {
        bst16(crs, off, v);
      } else if constexpr (EPI == 1 || EPI == 2) {
        float f[8];
        unpack8(v, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = EPI == 1 ? gelu_f(f[e]) : fmaxf(f[e], 0.f);
        if constexpr (EPI == 1) bst16(ars, col_ok ? (uint32_t)(((int64_t)rt * g.ldaux + col) * 2) : kOff, v);
        bst16(crs, off, pack8(f));
      } else if constexpr (EPI == 6) {
        // dO stored as is; its bf16 values times O summed over the wave's 64 columns = one head
        bst16(crs, off, v);
        float d[8], o[8];
        unpack8(v, d);
        unpack8(apre[kk], o);
        float sum = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) sum = __builtin_fmaf(d[e], o[e], sum);
        // the row's 8 lanes (c8 = 0..7, consecutive lanes) in a fixed butterfly order
        sum += __shfl_xor(sum, 1, 64);
        sum += __shfl_xor(sum, 2, 64);
        sum += __shfl_xor(sum, 4, 64);
        const int m = m0 + rt;
        const int bq = m / g.T, tq = m - bq * g.T, hd = ncol0 >> 6;
        const uint32_t doff = (c8 == 0 && m < M && col_ok)
                                  ? (uint32_t)((((int64_t)bq * (N >> 6) + hd) * g.T + tq) * 4) : kOff;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, sum), drs, doff, 0, 0);
      } else if constexpr (EPI == 5) {
        // d = the bf16-rounded data gradient of the SwiGLU output (as swiglu_bwd_kernel reads it)
        float d[8], gt[8], up[8], dg[8], du[8];
        unpack8(v, d);
        unpack8(apre[kk], gt);
        unpack8(apre2[kk], up);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float sg = swiglu_sigmoid(gt[e]);
          du[e] = d[e] * (gt[e] * sg);
          dg[e] = d[e] * up[e] * sg * (1.f + gt[e] * (1.f - sg));
        }
        bst16(crs, off, pack8(dg));
        bst16(crs, col_ok ? off + (uint32_t)N * 2u : kOff, pack8(du));
      } else {
        float f[8], a[8];
        unpack8(v, f);
        unpack8(apre[kk], a);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = EPI == 3 ? f[e] * gelu_df(a[e]) : (a[e] > 0.f ? f[e] : 0.f);
        const u32x4 o = pack8(f);
        bst16(crs, off, o);
        unpack8(o, f);  // the bias gradient sums the bf16-rounded values, like act_bwd_colsum
#pragma unroll
        for (int e = 0; e < 8; ++e) csum[e] += f[e];
      }
    }
    }  // grp
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  if constexpr (EPI == 3 || EPI == 4) {
    // lanes l, l + 8, ..., l + 56 hold the same 8 columns; rows past M contributed zeros
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      csum[e] += __shfl_xor(csum[e], 8, 64);
      csum[e] += __shfl_xor(csum[e], 16, 64);
      csum[e] += __shfl_xor(csum[e], 32, 64);
    }
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(g.colpart + (int64_t)(2 * tm + wm) * N), (short)0, N * 4, 0x00020000);
    const uint32_t po = (lane < 8 && col_ok) ? (uint32_t)col * 4u : kOff;
    bst16(prs, po, __builtin_bit_cast(u32x4, f32x4{csum[0], csum[1], csum[2], csum[3]}));
    bst16(prs, po == kOff ? kOff : po + 16u, __builtin_bit_cast(u32x4, f32x4{csum[4], csum[5], csum[6], csum[7]}));
  }
}

// Persistent: one workgroup per CU walks tiles lid, lid + grid, ...; the DMA pipeline runs across
// tile boundaries (the last stage of a tile prefetches the next tile's first stage), and the
// epilogue's output goes through half of the LDS -- the other half already holds that prefetch --
// so a tile's stores drain under the next tile's first stage instead of stalling every CU at once.
template <int MF, int EPI, bool ASYM>
__global__ __launch_bounds__(GNT) void gemm_tn_kernel(pllm::GemmArgs g) {
  __shared__ __attribute__((aligned(1024))) uint16_t smem[2 * GSTAGE];
  const int M = g.M, N = g.N, K = g.K;
  const int tiles_m = (M + GT - 1) / GT, tiles_n = (N + GT - 1) / GT, ntiles = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int lid = xcd_remap(blockIdx.x, G);
  const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int wm = w >> 2, wn = w & 3;
  const int nstage = K / GBK;
  if (lid >= ntiles) return;

  // ---- DMA plan: piece k of wave w = 8 rows x 128 B (waves 0-3: A rows, 4-7: B rows).  Lane l
  // fills image row 8 * blk + l / 8 at chunk position l % 8, which holds logical chunk
  // (l % 8) ^ gswz(row).  Rows past M / N fall outside the descriptor's range: they read zeros.
  // ASYM: waves 0-3 issue all 64 pieces of a stage (16 each: waves 0-1 A, 2-3 B) and waves 4-7
  // none, so after each barrier the partner wave of every SIMD goes straight to its MFMAs while
  // the loader wave is stuck issuing pieces (a DMA burst costs ~1.1k cycles per stage, CU-wide)
  constexpr int PPW = ASYM ? 16 : 8;
  const int opnd = ASYM ? (w >> 1) & 1 : w >> 2;
  const bool loader = !ASYM || w < 4;
  const int64_t ld = opnd == 0 ? g.lda : g.ldb;
  uint32_t voff[PPW];
#pragma unroll
  for (int k = 0; k < PPW; ++k) {
    const int blk = (ASYM ? (w & 1) * 16 : (w & 3) * 8) + k, row = 8 * blk + (lane >> 3);
    voff[k] = (uint32_t)((row * ld + (((lane & 7) ^ gswz(row)) << 3)) * 2);
  }
  const unsigned lds_base = (unsigned)(uintptr_t)smem;
  auto issue = [&](int t, int st, int slot) {
    if (!loader) return;
    int tm, tn;
    tile_of(t, tiles_m, tiles_n, g.group_m, tm, tn);
    const uint16_t* base = opnd == 0 ? g.A + (int64_t)tm * GT * g.lda : g.B + (int64_t)tn * GT * g.ldb;
    const int rows_ok = opnd == 0 ? min(GT, M - tm * GT) : min(GT, N - tn * GT);
    const int64_t koff = (int64_t)st * GBK * 2;
    const int64_t span = (int64_t)(rows_ok - 1) * ld * 2 + (int64_t)K * 2 - koff;
    const i32x4v srd = srd_of(reinterpret_cast<const char*>(base) + koff, (uint32_t)span);
    const int blk0 = ASYM ? (w & 1) * 16 : (w & 3) * 8;
    const unsigned dst = lds_base + 2u * (unsigned)(slot * GSTAGE + opnd * GIMG + blk0 * 512);
#pragma unroll
    for (int k = 0; k < PPW; ++k) blds16(srd, voff[k], dst + 1024u * k);
  };

  constexpr int NI = MF == 32 ? 2 : 4;  // column fragments (64 columns)
  constexpr int NJ = MF == 32 ? 4 : 8;  // row fragments (128 rows)
  using Acc = typename std::conditional<MF == 32, f32x16, f32x4>::type;
  constexpr int NE = MF == 32 ? 16 : 4;
  const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(g.bias != nullptr ? g.bias : g.A), (short)0, (EPI <= 2 && g.bias != nullptr) ? N * 2 : 0, 0x00020000);

  issue(lid, 0, 0);
  int slot = 0;
  bool first = true;
  for (int t = lid; t < ntiles; t += G) {
    int tm, tn;
    tile_of(t, tiles_m, tiles_n, g.group_m, tm, tn);
    Acc acc[NI][NJ];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int e = 0; e < NE; ++e) acc[i][j][e] = 0.f;
    for (int st = 0; st < nstage; ++st) {
      // the stage's DMA was issued before the previous tile's epilogue: its stores may stay in flight
      if (st == 0 && !first) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kEpiOps<MF, EPI>) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // stage landed for every wave; nobody still reads the other slot
      if (st + 1 < nstage) issue(t, st + 1, slot ^ 1);
      else if (t + G < ntiles) issue(t + G, 0, slot ^ 1);
      const uint16_t* Ai = smem + slot * GSTAGE;         // A image: output rows
      const uint16_t* Bi = smem + slot * GSTAGE + GIMG;  // B image: output columns
      if constexpr (MF == 32) {
#pragma unroll
        for (int k16 = 0; k16 < GBK / 16; ++k16) {
          const int ch = 2 * k16 + (lane >> 5);
          bf16x8 bf[NI], af[NJ];
#pragma unroll
          for (int i = 0; i < NI; ++i) bf[i] = lds_frag(Bi + gimg_off(wn * 64 + 32 * i + (lane & 31), ch));
#pragma unroll
          for (int j = 0; j < NJ; ++j) af[j] = lds_frag(Ai + gimg_off(wm * 128 + 32 * j + (lane & 31), ch));
#pragma unroll
          for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int i = 0; i < NI; ++i)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf[i], af[j], acc[i][j], 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int k32 = 0; k32 < GBK / 32; ++k32) {
          const int ch = 4 * k32 + (lane >> 4);
          bf16x8 bf[NI], af[NJ];
#pragma unroll
          for (int i = 0; i < NI; ++i) bf[i] = lds_frag(Bi + gimg_off(wn * 64 + 16 * i + (lane & 15), ch));
#pragma unroll
          for (int j = 0; j < NJ; ++j) af[j] = lds_frag(Ai + gimg_off(wm * 128 + 16 * j + (lane & 15), ch));
#pragma unroll
          for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int i = 0; i < NI; ++i)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[i], af[j], acc[i][j], 0, 0, 0);
        }
      }
      slot ^= 1;
    }
    first = false;

    // ---- epilogue through the last stage's slot (the other one holds the next tile's prefetch)
    __syncthreads();  // every wave is done with the last stage's images
    gemm_epilogue<MF, EPI>(acc, smem + (slot ^ 1) * GSTAGE + w * (64 * 64), g, brs, tm, tn, wm, wn, lane);
  }
}


}  // namespace

namespace pllm {

static int g_gemm_mfma = 16;
#ifndef PL_GEMM_GROUP_M
#define PL_GEMM_GROUP_M 4  // m-tiles per tile group (L2 reuse of the B panels; A/B builds)
#endif
static int g_gemm_group_m = PL_GEMM_GROUP_M;
// 0: every wave issues its DMA pieces; 2: the asymmetric DMA (waves 0-3 issue all).  Measured and
// removed (profiles/r3_gemm_tn.md): 1 = two k32 phases per K-tile with counted vmcnt across raw
// barriers (3-12 % slower), 3 = one wave per SIMD with 128x128 per wave and the DMA pinned between
// MFMA groups (hipBLASLt's geometry; 4-18 % slower, its fused epilogues up to 40 % slower)
// 4 (default): the ping-pong kernel of gemm_pp.hip (two wave groups one barrier apart, counted
// waits): 4-6 % faster than this file's kernel on every fused epilogue measured (GELU' / SwiGLU' /
// attention delta; gpurun_out/r4pp7_bench.jsonl, r4ab1_swiglu.jsonl), whole GPT-2 step +0.5 %.
// This file's kernel remains the FALLBACK for what the ping-pong loop does not take (a single K-tile,
// K < 128; the delta epilogue with T % 16 != 0); 0 / 2 select it for every shape (tests only)
static int g_gemm_phased = 4;
// CUs the persistent grids leave free, for RCCL kernels overlapping the backward (world > 1)
static int g_gemm_reserve = 0;
// 0: the persistent kernels (gemm_pp / wgrad_pp / this file's) launch one workgroup per tile instead
// of one per CU, so the hardware deals tiles to whichever CUs are free (e.g. beside RCCL kernels)
static int g_gemm_persistent = 1;
void gemm_set_config(int mfma, int group_m, int phased, int reserve_cus, int persistent) {
  if (mfma == 16 || mfma == 32) g_gemm_mfma = mfma;
  if (group_m > 0) g_gemm_group_m = group_m;
  if (phased >= 0) g_gemm_phased = phased;
  if (reserve_cus >= 0) g_gemm_reserve = reserve_cus;
  if (persistent >= 0) g_gemm_persistent = persistent;
}

// column-sum partial rows of the EPI 3 / 4 bias gradient: 2 per tile row here, 4 (one per
// accumulator quadrant row half and wave row) in the ping-pong kernel's quadrant epilogues
// the ping-pong kernel serves a call when selected, with >= 2 K-tiles and (epilogue 6) 16 | T
bool gemm_uses_pp(int K, int epi, int T) { return g_gemm_phased == 4 && K >= 128 && (epi != 6 || T % 16 == 0); }
int gemm_colsum_groups(int M, int K) {
  return gemm_uses_pp(K, 3, 0) ? gemm_pp_colsum_groups(M, K) : 2 * ((M + GT - 1) / GT);
}

static int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

static int gemm_ctas() {
  // persistent grid: one workgroup per CU, minus the CUs reserved for concurrent collectives;
  // non-persistent: no cap (one workgroup per tile / work item)
  if (!g_gemm_persistent) return 1 << 30;
  return num_cus() - g_gemm_reserve > 8 ? num_cus() - g_gemm_reserve : 8;
}
int gemm_grid_cap() { return gemm_ctas(); }

void gemm_tn(const GemmArgs& a0, int epi, hipStream_t st) {
  GemmArgs a = a0;
  a.group_m = g_gemm_group_m;
  const int ntiles = ((a.M + GT - 1) / GT) * ((a.N + GT - 1) / GT);
  if (ntiles == 0) return;
  const int ctas = gemm_ctas();
  if (gemm_uses_pp(a.K, epi, a.T)) {
    gemm_tn_pp(a, epi, ctas, st);
    return;
  }
  const int tiles = ntiles < ctas ? ntiles : ctas;
#define PL_GEMM_CASE(MFV, E)                                                       \
  do {                                                                               \
    if (g_gemm_phased == 2)                                                          \
      hipLaunchKernelGGL((gemm_tn_kernel<MFV, E, true>), dim3(tiles), dim3(GNT), 0, st, a); \
    else                                                                             \
      hipLaunchKernelGGL((gemm_tn_kernel<MFV, E, false>), dim3(tiles), dim3(GNT), 0, st, a); \
  } while (0)
#define PL_GEMM_EPIS(MFV)          \
  switch (epi) {                     \
    case 0: PL_GEMM_CASE(MFV, 0); break; \
    case 1: PL_GEMM_CASE(MFV, 1); break; \
    case 2: PL_GEMM_CASE(MFV, 2); break; \
    case 3: PL_GEMM_CASE(MFV, 3); break; \
    case 4: PL_GEMM_CASE(MFV, 4); break; \
    case 5: PL_GEMM_CASE(MFV, 5); break; \
    default: PL_GEMM_CASE(MFV, 6); break; \
  }
  if (g_gemm_mfma == 16) {
    PL_GEMM_EPIS(16)
  } else {
    PL_GEMM_EPIS(32)
  }
#undef PL_GEMM_EPIS
#undef PL_GEMM_CASE
}

}  // namespace pllm

// Weight-gradient GEMM for linear layers on gfx950 MFMA:
//     dW[P, Q] (+)= sum_m dY[m, P] * X[m, Q]          (bf16 in, fp32 accumulate)
// i.e. the reduction runs over the token dimension (M = batch*seq, 65536 for the
// headline config) while the output is small (768x768 .. 3072x768).  hipBLASLt's
// best candidates for these shapes ran at 0.40-0.82 PFLOP/s on MI355X
// (profiles/r1_prof4*), far below its forward GEMMs, because a 768x768 output has
// only 9 tiles of 256x256 to spread over 256 CUs.
//
// Design (CDNA4):
//  * split-K over tokens: grid = (output tiles) x (S token slices), slice-major so
//    the workgroups that share a slice's dY/X panels run together (L2 reuse);
//  * workgroup tile 256x256, 4 waves each owning a 128x128 sub-tile as 4x4
//    v_mfma_f32_32x32x16_bf16 accumulators (256 accumulator registers: one wave per
//    SIMD with the full 512-entry register file, __launch_bounds__(256, 1));
//  * both operands are token-major in memory, so both MFMA fragments come from
//    ds_read_b64_tr_b16 transposed reads of swizzled [64 tokens][128] LDS images
//    (conflict-free, see Img<128> in attention.hip);
//  * 64-token stages double-buffered through registers: the next stage's 16 x 16-B
//    global loads are issued before the current stage's 64 MFMAs and written to LDS
//    after them, one barrier per stage;
//  * fp32 partial tiles go to a [S][P][Q] slab; a reduce kernel sums the slices in a
//    fixed order and adds the result into the bf16 gradient (the optimizer's flat
//    buffer), so the accumulate is fused and the result is deterministic.
#include "common.h"
#include "kernels.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

PLLM_DEV f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
PLLM_DEV s16x4 ds_tr(const uint16_t* p) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p); }
PLLM_DEV bf16x8 cat_tr(const s16x4& lo, const s16x4& hi) {
  s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}
PLLM_DEV int acc_row(int i, int half) { return (i & 3) + 8 * (i >> 2) + 4 * half; }

// [rows][128] bf16 image, 16-B chunk ch of row r at ch ^ f(r) (conflict-free tr reads)
PLLM_DEV int img_off(int r, int col) {
  const int f = ((r & 3) << 2) | ((r >> 2) & 3);
  return r * 128 + (((col >> 3) ^ f) << 3) + (col & 7);
}

constexpr int BT = 256;          // output tile (P and Q)
constexpr int BKM = 64;          // tokens per stage
constexpr int HALF = BKM * 128;  // elements of one [64][128] image
constexpr int LDS_ELEMS = 2 * 2 * 2 * HALF;  // 2 buffers x {A, B} x 2 halves

__global__ __launch_bounds__(256, 1) void wgrad_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                       const uint16_t* __restrict__ B, int64_t ldb, int M, int P,
                                                       int Q, int S, int slice, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[LDS_ELEMS];
  const int tiles_q = (Q + BT - 1) / BT, tiles_p = (P + BT - 1) / BT;
  const int ntiles = tiles_p * tiles_q;
  const int s = blockIdx.x / ntiles, t = blockIdx.x % ntiles;
  const int p0 = (t / tiles_q) * BT, q0 = (t % tiles_q) * BT;
  const int m_begin = s * slice, m_end = min(M, m_begin + slice);
  const int nstage = (m_end - m_begin + BKM - 1) / BKM;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int wp = w >> 1, wq = w & 1;  // wave's 128x128 sub-tile
  const int g1 = (lane >> 4) & 1, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;

  // staging: 64 rows x 256 cols per operand = 2048 16-B chunks / 256 threads = 8 each
  u32x4 ra[8], rb[8];
  auto gload = [&](int st) {
    const int m0 = m_begin + st * BKM;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = tid + 256 * i, row = c >> 5, col = (c & 31) * 8;
      const int m = m0 + row;
      const bool mok = m < m_end;
      ra[i] = (mok && p0 + col < P) ? ld16(A + (int64_t)m * lda + p0 + col) : u32x4{0u, 0u, 0u, 0u};
      rb[i] = (mok && q0 + col < Q) ? ld16(B + (int64_t)m * ldb + q0 + col) : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto swrite = [&](int buf) {
    uint16_t* base = smem + buf * 4 * HALF;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = tid + 256 * i, row = c >> 5, col = (c & 31) * 8;
      const int half = col >> 7, cc = col & 127;
      st16(base + half * HALF + img_off(row, cc), ra[i]);            // A halves at 0, 1
      st16(base + (2 + half) * HALF + img_off(row, cc), rb[i]);      // B halves at 2, 3
    }
  };

  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  if (nstage > 0) {
    gload(0);
    swrite(0);
  }
  __syncthreads();
  for (int st = 0; st < nstage; ++st) {
    const int buf = st & 1;
    if (st + 1 < nstage) gload(st + 1);
    const uint16_t* Ai = smem + buf * 4 * HALF + wp * HALF;
    const uint16_t* Bi = smem + buf * 4 * HALF + (2 + wq) * HALF;
#pragma unroll
    for (int k16 = 0; k16 < BKM / 16; ++k16) {
      const int row = k16 * 16 + 8 * hh + tq;
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int col = 32 * i + 16 * g1 + 4 * tp;
        af[i] = cat_tr(ds_tr(Ai + img_off(row, col)), ds_tr(Ai + img_off(row + 4, col)));
        bfr[i] = cat_tr(ds_tr(Bi + img_off(row, col)), ds_tr(Bi + img_off(row + 4, col)));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma32(af[i], bfr[j], acc[i][j]);
    }
    if (st + 1 < nstage) swrite(buf ^ 1);
    __syncthreads();
  }
  // fp32 partial tile -> slab[s][P][Q]
  float* out = part + (int64_t)s * P * Q;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = q0 + wq * 128 + 32 * j + r;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int p = p0 + wp * 128 + 32 * i + acc_row(e, hh);
        if (p < P && q < Q) out[(int64_t)p * Q + q] = acc[i][j][e];
      }
    }
  }
}

// dW[p, q] (+)= sum_s slab[s][p][q]   (8 columns per thread, fixed slice order)
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int S, int64_t PQ,
                                                           uint16_t* __restrict__ out, int accumulate) {
  const int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) * 8;
  if (i >= PQ) return;
  float f[8];
  if (accumulate) {
    unpack8(ld16(out + i), f);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = 0.f;
  }
  for (int s = 0; s < S; ++s) {
    const f32x4* p = reinterpret_cast<const f32x4*>(part + s * PQ + i);
    const f32x4 a = p[0], b = p[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f[j] += a[j];
      f[4 + j] += b[j];
    }
  }
  st16(out + i, pack8(f));
}

}  // namespace

namespace pllm {

void wgrad_plan(int M, int P, int Q, int* S, int* slice) {
  const int ntiles = ((P + BT - 1) / BT) * ((Q + BT - 1) / BT);
  int s = (256 + ntiles - 1) / ntiles;               // about one workgroup per CU
  const int max_s = (M + 8 * BKM - 1) / (8 * BKM);    // keep >= 8 stages per slice
  if (s > max_s) s = max_s;
  if (s < 1) s = 1;
  int sl = (M + s - 1) / s;
  sl = (sl + BKM - 1) / BKM * BKM;
  *S = (M + sl - 1) / sl;
  *slice = sl;
}

void wgrad(const void* dy, int64_t lda, const void* x, int64_t ldb, int M, int P, int Q, float* part, void* out,
           bool accumulate, hipStream_t st) {
  int S, slice;
  wgrad_plan(M, P, Q, &S, &slice);
  const int ntiles = ((P + BT - 1) / BT) * ((Q + BT - 1) / BT);
  hipLaunchKernelGGL(wgrad_kernel, dim3(ntiles * S), dim3(256), 0, st, (const uint16_t*)dy, lda, (const uint16_t*)x,
                     ldb, M, P, Q, S, slice, part);
  const int64_t PQ = (int64_t)P * Q;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((PQ / 8 + 255) / 256)), dim3(256), 0, st, part, S, PQ,
                     (uint16_t*)out, (int)accumulate);
}

}  // namespace pllm

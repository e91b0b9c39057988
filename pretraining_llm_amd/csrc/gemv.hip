// Skinny GEMM for decoding: y[M, N] = x[M, K] . W[N, K]^T (+ bias), M <= 8 rows (gfx950).
//
// A batch-1..8 decode step multiplies a handful of token rows by every weight matrix: the
// work is a weight-streaming GEMV (0.25 B of FLOP per weight byte), so MFMA tiles sized
// for training GEMMs mostly idle (hipBLASLt's MT16x16 solutions: 5.7-9.6 us per projection
// at M = 1 for 1.2-4.7 MB of weights, profiles/r1_decode_kernel_stats.md).  Here:
//  * one wave owns 4 consecutive output columns; lane l streams 16-B chunks l, l+64, ... of
//    each column's weight row (coalesced 1-KiB wave reads), the x chunks at the same K
//    offsets are loaded once per step and reused for the 4 columns and all M rows;
//  * fp32 FMAs, then a 64-lane xor-shuffle reduction per (column, row); lane 0 adds the
//    bias and stores;
//  * 4 waves (16 columns) per workgroup -> N / 16 workgroups (3,144 for the 50,304-row LM
//    head: 5 TB/s, profiles/r1_decode_gemv_kernel_stats.md).
// Narrow outputs (N < 8,192: the per-layer projections) would get only 48-192 workgroups
// that way on 256 CUs (N = 768, K = 3,072 ran at 0.67 TB/s), so they take the split-K form:
// one workgroup per 1-4 columns, its 64-256 lanes striding the K chunks of those columns
// together, partial sums reduced across waves through LDS -> 576-768 workgroups.
// Requires K % 8 == 0 and 16-B aligned rows (host-checked).
#include "common.h"
#include "kernels.h"

namespace {

constexpr int GV_THREADS = 256;
constexpr int GV_COLS = 4;  // output columns per wave

template <int M>
__global__ __launch_bounds__(GV_THREADS) void gemv_kernel(const uint16_t* __restrict__ x, int64_t ldx,
                                                          const uint16_t* __restrict__ w, int64_t ldw,
                                                          const uint16_t* __restrict__ bias, uint16_t* __restrict__ y,
                                                          int64_t ldy, int N, int K, int Mr) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = (blockIdx.x * (GV_THREADS / 64) + wave) * GV_COLS;
  if (n0 >= N) return;  // wave-uniform
  const int nch = K >> 3;
  float acc[GV_COLS][M];
#pragma unroll
  for (int c = 0; c < GV_COLS; ++c)
#pragma unroll
    for (int m = 0; m < M; ++m) acc[c][m] = 0.f;
  for (int ch = lane; ch < nch; ch += 64) {
    u32x4 wr[GV_COLS];
#pragma unroll
    for (int c = 0; c < GV_COLS; ++c) {  // weight chunks first (the streamed bytes)
      const int n = min(n0 + c, N - 1);
      wr[c] = ld16_nt(w + (int64_t)n * ldw + ch * 8);
    }
    float xf[M][8];
#pragma unroll
    for (int m = 0; m < M; ++m) {  // rows past the real M (template rounds it up) read nothing
      if (m < Mr) {
        unpack8(ld16(x + (int64_t)m * ldx + ch * 8), xf[m]);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) xf[m][e] = 0.f;
      }
    }
#pragma unroll
    for (int c = 0; c < GV_COLS; ++c) {
      float wf[8];
      unpack8(wr[c], wf);
#pragma unroll
      for (int m = 0; m < M; ++m)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[c][m] = fmaf(wf[e], xf[m][e], acc[c][m]);
    }
  }
#pragma unroll
  for (int c = 0; c < GV_COLS; ++c)
#pragma unroll
    for (int m = 0; m < M; ++m) acc[c][m] = wave_sum(acc[c][m]);
  if (lane == 0) {
#pragma unroll
    for (int c = 0; c < GV_COLS; ++c) {
      const int n = n0 + c;
      if (n < N) {
        const float b = bias ? bf2f(bias[n]) : 0.f;
#pragma unroll
        for (int m = 0; m < M; ++m)
          if (m < Mr) y[(int64_t)m * ldy + n] = f2bf_bits(acc[c][m] + b);
      }
    }
  }
}

// Split-K form: workgroup = T threads over C columns; thread t owns K chunks t, t + T, ...
template <int M, int C, int T>
__global__ __launch_bounds__(T) void gemv_splitk_kernel(const uint16_t* __restrict__ x, int64_t ldx,
                                                        const uint16_t* __restrict__ w, int64_t ldw,
                                                        const uint16_t* __restrict__ bias, uint16_t* __restrict__ y,
                                                        int64_t ldy, int N, int K, int Mr) {
  constexpr int NW = T / 64;
  __shared__ float part[NW][C * M];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = blockIdx.x * C;
  const int nch = K >> 3;
  float acc[C][M];
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int m = 0; m < M; ++m) acc[c][m] = 0.f;
  for (int ch = threadIdx.x; ch < nch; ch += T) {
    u32x4 wr[C];
#pragma unroll
    for (int c = 0; c < C; ++c) wr[c] = ld16_nt(w + (int64_t)min(n0 + c, N - 1) * ldw + ch * 8);
    float xf[M][8];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      if (m < Mr) {
        unpack8(ld16(x + (int64_t)m * ldx + ch * 8), xf[m]);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) xf[m][e] = 0.f;
      }
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      float wf[8];
      unpack8(wr[c], wf);
#pragma unroll
      for (int m = 0; m < M; ++m)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[c][m] = fmaf(wf[e], xf[m][e], acc[c][m]);
    }
  }
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const float v = wave_sum(acc[c][m]);
      if (lane == 0) part[wave][c * M + m] = v;
    }
  __syncthreads();
  const int t = threadIdx.x;
  if (t < C * M) {
    const int c = t / M, m = t % M, n = n0 + c;
    if (n < N && m < Mr) {
      float v = bias ? bf2f(bias[n]) : 0.f;
#pragma unroll
      for (int i = 0; i < NW; ++i) v += part[i][t];
      y[(int64_t)m * ldy + n] = f2bf_bits(v);
    }
  }
}

template <int M>
void launch_splitk(const void* x, int64_t ldx, const void* w, int64_t ldw, const void* bias, void* y, int64_t ldy,
                   int Mr, int N, int K, hipStream_t st) {
  const int nch = K >> 3;
  const int C = N <= 1024 ? 1 : N <= 2048 ? 2 : 4;  // >= 512 workgroups for N >= 512
  const dim3 grid((N + C - 1) / C);
#define LS(CC, TT)                                                                                             \
  hipLaunchKernelGGL((gemv_splitk_kernel<M, CC, TT>), grid, dim3(TT), 0, st, (const uint16_t*)x, ldx,          \
                     (const uint16_t*)w, ldw, (const uint16_t*)bias, (uint16_t*)y, ldy, N, K, Mr)
#define LC(CC)                     \
  if (nch > 128) LS(CC, 256);      \
  else if (nch > 64) LS(CC, 128);  \
  else LS(CC, 64);
  if (C == 1) {
    LC(1)
  } else if (C == 2) {
    LC(2)
  } else {
    LC(4)
  }
#undef LC
#undef LS
}

}  // namespace

namespace pllm {

int gemv_max_rows() { return 8; }

void gemv(const void* x, int64_t ldx, const void* w, int64_t ldw, const void* bias, void* y, int64_t ldy, int M,
          int N, int K, hipStream_t st) {
  if (N < 8192) {
    if (M <= 1) launch_splitk<1>(x, ldx, w, ldw, bias, y, ldy, M, N, K, st);
    else if (M <= 2) launch_splitk<2>(x, ldx, w, ldw, bias, y, ldy, M, N, K, st);
    else if (M <= 4) launch_splitk<4>(x, ldx, w, ldw, bias, y, ldy, M, N, K, st);
    else launch_splitk<8>(x, ldx, w, ldw, bias, y, ldy, M, N, K, st);
    PLLM_CHECK_LAUNCH();
    return;
  }
  const int cols_per_block = GV_COLS * (GV_THREADS / 64);
  const dim3 grid((N + cols_per_block - 1) / cols_per_block);
#define L(MM)                                                                                                  \
  hipLaunchKernelGGL((gemv_kernel<MM>), grid, dim3(GV_THREADS), 0, st, (const uint16_t*)x, ldx,                 \
                     (const uint16_t*)w, ldw, (const uint16_t*)bias, (uint16_t*)y, ldy, N, K, M)
  if (M <= 1) L(1);
  else if (M <= 2) L(2);
  else if (M <= 4) L(4);
  else L(8);
#undef L
  PLLM_CHECK_LAUNCH();
}

}  // namespace pllm

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

PL_DEV float bf16_round(float v) { return bf2f(f2bf_bits(v)); }

// block-wide sums of M per-thread values (all threads get the totals); `red` holds NW x M floats
template <int M, int NW>
PL_DEV void block_sum(float (&v)[M], float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const float t = wave_sum(v[m]);
    if (lane == 0) red[wave * M + m] = t;
  }
  __syncthreads();
#pragma unroll
  for (int m = 0; m < M; ++m) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) t += red[i * M + m];
    v[m] = t;
  }
  __syncthreads();
}

// Split-K form: workgroup = T threads over C columns; thread t owns K chunks t, t + T, ...
// NORM: the GEMM input is norm(x + res) (LayerNorm, or RMSNorm when a.rms), computed in the
// workgroup itself -- each workgroup re-reads the <= 8 L2-resident input rows for one
// statistics pass, and workgroup 0 writes the new residual stream x + res -- so a decode
// block runs no separate norm kernel.  Epilogue: + bias, then GELU (act 1) or ReLU (act 2).
// With a.kc set (decode QKV projection) the K and V columns are also appended to the KV cache at
// the device-side position *a.pos.  Roundings follow the unfused path: x + res, the normalised input and the pre-activation are
// rounded to bf16 where the separate kernels would have stored them.
template <int M, int C, int T, bool NORM>
__global__ __launch_bounds__(T) void gemv_splitk_kernel(const pllm::GemvArgs a) {
  constexpr int NW = T / 64;
  __shared__ float part[NW][C * M];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = blockIdx.x * C;
  const int nch = a.K >> 3, Mr = a.Mr, N = a.N;
  const uint16_t* __restrict__ x = a.x;
  const uint16_t* __restrict__ res = a.res;
  const uint16_t* __restrict__ w = a.w;
  float mean[M], rstd[M];
  // the first weight chunks are requested before the norm statistics so their HBM latency
  // overlaps the statistics pass and its block reduction
  u32x4 wpre[C];
  if (threadIdx.x < nch) {
#pragma unroll
    for (int c = 0; c < C; ++c) wpre[c] = ld16_nt(w + (int64_t)min(n0 + c, N - 1) * a.ldw + threadIdx.x * 8);
  }
  if constexpr (NORM) {
    // one statistics pass (sums of s and s^2 in fp32; var = E[s^2] - E[s]^2 -- a shift by the
    // row's first element cost a dependent load round trip, +1 us per launch); workgroup 0 also
    // writes the residual stream s = x + res
    __shared__ float red[NW * 2 * M];
    float st[2 * M];
#pragma unroll
    for (int m = 0; m < M; ++m) st[m] = st[M + m] = 0.f;
    for (int ch = threadIdx.x; ch < nch; ch += T) {
#pragma unroll
      for (int m = 0; m < M; ++m) {
        if (m < Mr) {
          float f[8];
          unpack8(ld16(x + (int64_t)m * a.ldx + ch * 8), f);
          if (res) {
            float r[8];
            unpack8(ld16(res + (int64_t)m * a.ldr + ch * 8), r);
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] = bf16_round(f[e] + r[e]);
            if (a.s_out && blockIdx.x == 0) st16(a.s_out + (int64_t)m * a.lds + ch * 8, pack8(f));
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            st[m] += f[e];
            st[M + m] += f[e] * f[e];
          }
        }
      }
    }
    block_sum<2 * M, NW>(st, red);
    const float invK = 1.f / (float)a.K;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      mean[m] = a.rms ? 0.f : st[m] * invK;
      rstd[m] = rsqrtf(fmaxf(st[M + m] * invK - mean[m] * mean[m], 0.f) + a.eps);
    }
  }
  float acc[C][M];
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int m = 0; m < M; ++m) acc[c][m] = 0.f;
  for (int ch = threadIdx.x; ch < nch; ch += T) {
    u32x4 wr[C];
    if (ch == (int)threadIdx.x) {
#pragma unroll
      for (int c = 0; c < C; ++c) wr[c] = wpre[c];
    } else {
#pragma unroll
      for (int c = 0; c < C; ++c) wr[c] = ld16_nt(w + (int64_t)min(n0 + c, N - 1) * a.ldw + ch * 8);
    }
    float g[8], bt[8];
    if constexpr (NORM) {
      unpack8(ld16(a.gamma + ch * 8), g);
      if (a.beta) {
        unpack8(ld16(a.beta + ch * 8), bt);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) bt[e] = 0.f;
      }
    }
    float xf[M][8];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      if (m < Mr) {
        unpack8(ld16(x + (int64_t)m * a.ldx + ch * 8), xf[m]);
        if constexpr (NORM) {
          if (res) {
            float r[8];
            unpack8(ld16(res + (int64_t)m * a.ldr + ch * 8), r);
#pragma unroll
            for (int e = 0; e < 8; ++e) xf[m][e] = bf16_round(xf[m][e] + r[e]);
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) xf[m][e] = bf16_round((xf[m][e] - mean[m]) * rstd[m] * g[e] + bt[e]);
        }
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
      float v = a.bias ? bf2f(a.bias[n]) : 0.f;
#pragma unroll
      for (int i = 0; i < NW; ++i) v += part[i][t];
      if (a.act == 1) v = gelu_f(bf16_round(v));
      else if (a.act == 2) v = fmaxf(v, 0.f);
      const uint16_t o = f2bf_bits(v);
      a.y[(int64_t)m * a.ldy + n] = o;
      const int64_t p = a.kc ? a.pos[a.pos_per_row ? m : 0] : -1;
      if (a.kc && n >= a.q_cols && p >= 0 && p < a.kv_smax) {  // KV-cache append (no copy kernels)
        const int j = n - a.q_cols;
        const int64_t at = (int64_t)m * a.kv_ldb + p * a.kv_cols;
        if (j < a.kv_cols) a.kc[at + j] = o;
        else a.vc[at + j - a.kv_cols] = o;
      }
    }
  }
}

template <int M, bool NORM>
void launch_splitk(const pllm::GemvArgs& a, hipStream_t st) {
  const int nch = a.K >> 3;
  const int C = a.N <= 1024 ? 1 : a.N <= 2048 ? 2 : 4;  // >= 512 workgroups for N >= 512
  const dim3 grid((a.N + C - 1) / C);
#define LS(CC, TT) hipLaunchKernelGGL((gemv_splitk_kernel<M, CC, TT, NORM>), grid, dim3(TT), 0, st, a)
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

template <bool NORM>
void dispatch_splitk(const pllm::GemvArgs& a, hipStream_t st) {
  if (a.Mr <= 1) launch_splitk<1, NORM>(a, st);
  else if (a.Mr <= 2) launch_splitk<2, NORM>(a, st);
  else if (a.Mr <= 4) launch_splitk<4, NORM>(a, st);
  else launch_splitk<8, NORM>(a, st);
}

}  // namespace

namespace pllm {

int gemv_max_rows() { return 8; }

void gemv(const GemvArgs& a, hipStream_t st) {
  if (a.gamma) {
    dispatch_splitk<true>(a, st);
  } else if (a.N < 8192 || a.act != 0 || a.kc) {
    dispatch_splitk<false>(a, st);
  } else {
    const int cols_per_block = GV_COLS * (GV_THREADS / 64);
    const dim3 grid((a.N + cols_per_block - 1) / cols_per_block);
#define L(MM)                                                                                                  \
  hipLaunchKernelGGL((gemv_kernel<MM>), grid, dim3(GV_THREADS), 0, st, a.x, a.ldx, a.w, a.ldw, a.bias, a.y,     \
                     a.ldy, a.N, a.K, a.Mr)
    if (a.Mr <= 1) L(1);
    else if (a.Mr <= 2) L(2);
    else if (a.Mr <= 4) L(4);
    else L(8);
#undef L
  }
  PL_CHECK_LAUNCH();
}

}  // namespace pllm

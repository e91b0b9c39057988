// LayerNorm / RMSNorm with a fused residual add, forward and backward (gfx950).
//
// Reference math: nn.LayerNorm(C) with affine weight+bias applied pre-attention
// and pre-MLP (reference src/models/transformer_block.py:28-31,44-46) and as the
// final norm (transformer.py:37,70).  The residual adds `x + attn(...)` /
// `x + mlp(...)` (transformer_block.py:44,46) are folded into the NEXT norm:
//
//   fwd:  s = x + r  (stored, bf16) ;  y = (s - mean) * rstd * w + b
//   bwd:  dx = d(norm)/ds . dy + ds_next      (ds_next = grad of the residual stream)
//
// Gradients of the affine parameters are written/accumulated in the optimizer's gradient
// dtype (bf16 or fp32, FlatAdamW grad_dtype); activations stay bf16.
//
// Layout / mapping: one wave64 per row, 8 bf16 (16 B) per lane per chunk, the
// row held in registers between the two reduction passes (exact two-pass
// variance, no E[x^2]-E[x]^2 cancellation).  dw/db are reduced per workgroup
// into an fp32 [G, C] slab and summed by a second, column-parallel kernel, so
// the weight gradient is deterministic (no float atomics).
#include "common.h"
#include "kernels.h"

namespace {

constexpr int ROWS_PER_BLOCK = 4;  // 4 waves, one row each

// One row per wave, full grid (C > 1024 or few rows: measured faster there than the persistent form below)
template <int K>  // chunks of 8 elements per lane (C <= 512*K)
__global__ __launch_bounds__(256) void norm_fwd_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ res, const uint16_t* __restrict__ w,
    const uint16_t* __restrict__ b, uint16_t* __restrict__ y, uint16_t* __restrict__ s_out,
    float* __restrict__ mean_out, float* __restrict__ rstd_out, int N, int C, float eps, int rms) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
  if (row >= N) return;
  const int nch = C >> 3;
  const size_t base = (size_t)row * C;
  float v[K][8];
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int c = lane + 64 * k;
    if (c < nch) {
      u32x4 xv = ld16(x + base + c * 8);
      unpack8(xv, v[k]);
      if (res) {
        float r8[8];
        unpack8(ld16(res + base + c * 8), r8);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] += r8[j];
        u32x4 sv = pack8(v[k]);
        st16(s_out + base + c * 8, sv);
        unpack8(sv, v[k]);  // normalise exactly the bf16 value that backward will see
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) sum += v[k][j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[k][j] = 0.f;
    }
  }
  const float invC = 1.f / (float)C;
  float mean = 0.f;
  if (!rms) mean = wave_sum(sum) * invC;
  float sq = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int c = lane + 64 * k;
    if (c < nch) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[k][j] - mean;
        sq += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(sq) * invC + eps);
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int c = lane + 64 * k;
    if (c < nch) {
      float w8[8], o[8];
      unpack8(ld16(w + c * 8), w8);
      if (b) {
        float b8[8];
        unpack8(ld16(b + c * 8), b8);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (v[k][j] - mean) * rstd * w8[j] + b8[j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (v[k][j] - mean) * rstd * w8[j];
      }
      st16(y + base + c * 8, pack8(o));
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}


// One wave per row, rows strided over a persistent grid (8 blocks of 4 waves per CU); the NEXT row's x (and
// residual) loads are issued before the current row is reduced, so every wave keeps two rows of loads in flight
// at full occupancy (one row per wave at a time ran at ~4 TB/s at 65536 x 768; two rows per wave with half the
// waves was slower still, profiles/r6_norm_fwd_two_rows_negative.log).  The weight / bias chunks are loaded once
// before the loop: a load issued after the prefetch would make its wait drain the prefetch too.
template <int K>  // chunks of 8 elements per lane (C <= 512*K)
__global__ __launch_bounds__(256) void norm_fwd_pf_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ res, const uint16_t* __restrict__ w,
    const uint16_t* __restrict__ b, uint16_t* __restrict__ y, uint16_t* __restrict__ s_out,
    float* __restrict__ mean_out, float* __restrict__ rstd_out, int N, int C, float eps, int rms) {
  const int lane = threadIdx.x & 63;
  const int stride = gridDim.x * ROWS_PER_BLOCK;
  int row = blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
  if (row >= N) return;
  const int nch = C >> 3;
  const u32x4 zero4 = u32x4{0u, 0u, 0u, 0u};
  u32x4 wv[K], bv[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int c = lane + 64 * k;
    wv[k] = c < nch ? ld16(w + c * 8) : zero4;
    bv[k] = (b && c < nch) ? ld16(b + c * 8) : zero4;
  }
  // loads of row min(r, N - 1): always issued (no conditional VMEM, so the compiler's counted waits stay exact)
  auto load = [&](int r, u32x4* X, u32x4* R) __attribute__((always_inline)) {
    const size_t base = (size_t)min(r, N - 1) * C;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int c = lane + 64 * k;
      X[k] = c < nch ? ld16(x + base + c * 8) : zero4;
      R[k] = (res && c < nch) ? ld16(res + base + c * 8) : zero4;
    }
  };
  const float invC = 1.f / (float)C;
  auto process = [&](int row, const u32x4* cx, const u32x4* cr) __attribute__((always_inline)) {
    const size_t base = (size_t)row * C;
    float v[K][8];
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int c = lane + 64 * k;
      unpack8(cx[k], v[k]);
      if (c < nch) {
        if (res) {
          float r8[8];
          unpack8(cr[k], r8);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[k][j] += r8[j];
          u32x4 sv = pack8(v[k]);
          st16(s_out + base + c * 8, sv);
          unpack8(sv, v[k]);  // normalise exactly the bf16 value that backward will see
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) sum += v[k][j];
      }
    }
    float mean = 0.f;
    if (!rms) mean = wave_sum(sum) * invC;
    float sq = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int c = lane + 64 * k;
      if (c < nch) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = v[k][j] - mean;
          sq += d * d;
        }
      }
    }
    const float rstd = rsqrtf(wave_sum(sq) * invC + eps);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int c = lane + 64 * k;
      if (c < nch) {
        float w8[8], b8[8], o[8];
        unpack8(wv[k], w8);
        unpack8(bv[k], b8);  // (zeros without a bias)
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (v[k][j] - mean) * rstd * w8[j] + b8[j];
        st16(y + base + c * 8, pack8(o));
      }
    }
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  };
  // two register sets, rows alternating between them: while one row is reduced the next one's loads (and the
  // one after, issued right after the reduce) are in flight -- no register copies, so no vmcnt(0) at the latch
  u32x4 ax[K], ar[K], bx[K], br[K];
  load(row, ax, ar);
  load(row + stride, bx, br);
  for (; row < N; row += 2 * stride) {
    process(row, ax, ar);
    load(row + 2 * stride, ax, ar);
    if (row + stride < N) process(row + stride, bx, br);
    load(row + 3 * stride, bx, br);
  }
}


// Backward.  One wave per row, rows strided over a <=512-block grid; the NEXT
// row's operands are loaded before the current row is processed, so each wave
// keeps two rows of loads in flight (the loop is latency-bound otherwise).
// Per-block column partials of dw, db and (XB) of dx itself are combined across
// the 4 waves through LDS and written to fp32 [G, C] slabs; col_reduce_kernel
// finishes them.  The dx column sums are the bias gradient of the linear layer
// that produced x (attention output projection / MLP down projection), fused
// here instead of a separate pass over dy.
template <int K, bool XB>
__global__ __launch_bounds__(256) void norm_bwd_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ s, const uint16_t* __restrict__ w,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in, const uint16_t* __restrict__ ds,
    uint16_t* __restrict__ dx, float* __restrict__ dw_part, float* __restrict__ db_part,
    float* __restrict__ xb_part, int N, int C, int rms) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nch = C >> 3;
  const float invC = 1.f / (float)C;
  const u32x4 zero4 = {0u, 0u, 0u, 0u};
  u32x4 wr[K];
  float dwa[K][8], dba[K][8], xba[K][8];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int c = lane + 64 * k;
    wr[k] = c < nch ? ld16(w + c * 8) : zero4;
#pragma unroll
    for (int j = 0; j < 8; ++j) dwa[k][j] = dba[k][j] = xba[k][j] = 0.f;
  }
  const int stride = gridDim.x * ROWS_PER_BLOCK;
  int row = blockIdx.x * ROWS_PER_BLOCK + wid;
  u32x4 cs[K], cd[K], cr[K];
  float cmean = 0.f, crstd = 0.f;
  auto load = [&](int r, u32x4* S, u32x4* Dy, u32x4* R, float& mu, float& rs) {
    const size_t base = (size_t)r * C;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int c = lane + 64 * k;
      const bool in = c < nch;
#ifndef PL_NORM_NTS
#define PL_NORM_NTS 1
#endif
      // the forward's residual stream, cold by now, by non-temporal loads: 79-82 vs 86-88 us at 65536 x 768,
      // 103 vs 107.5 us at 32768 x 2048 (profiles/r6_norm_bwd_nt_loads.log)
      S[k] = in ? (PL_NORM_NTS ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(s + base + c * 8))
                               : ld16(s + base + c * 8))
                : zero4;
      Dy[k] = in ? ld16(dy + base + c * 8) : zero4;
      R[k] = (in && ds) ? ld16(ds + base + c * 8) : zero4;
    }
    mu = rms ? 0.f : mean_in[r];
    rs = rstd_in[r];
  };
  if (row < N) load(row, cs, cd, cr, cmean, crstd);
  for (; row < N; row += stride) {
    const int nrow = row + stride;
    u32x4 ns[K], nd[K], nr[K];
    float nmean = 0.f, nrstd = 0.f;
    if (nrow < N) load(nrow, ns, nd, nr, nmean, nrstd);
    const size_t base = (size_t)row * C;
    float xh[K][8], g[K][8];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float d8[8], w8[8];
      unpack8(cs[k], xh[k]);
      unpack8(cd[k], d8);
      unpack8(wr[k], w8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xh[k][j] = (xh[k][j] - cmean) * crstd;
        g[k][j] = d8[j] * w8[j];
        sg += g[k][j];
        sgx += g[k][j] * xh[k][j];
        dwa[k][j] += d8[j] * xh[k][j];
        dba[k][j] += d8[j];
      }
    }
    const float mg = rms ? 0.f : wave_sum(sg) * invC;
    const float mgx = wave_sum(sgx) * invC;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int c = lane + 64 * k;
      float o[8], r8[8];
      unpack8(cr[k], r8);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = crstd * (g[k][j] - mg - xh[k][j] * mgx) + r8[j];
      const u32x4 ov = pack8(o);
      if (c < nch) st16(dx + base + c * 8, ov);
      if (XB) {
        unpack8(ov, o);  // sum exactly the bf16 values the producer's backward sees
#pragma unroll
        for (int j = 0; j < 8; ++j) xba[k][j] += o[j];
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      cs[k] = ns[k];
      cd[k] = nd[k];
      cr[k] = nr[k];
    }
    cmean = nmean;
    crstd = nrstd;
  }
  // combine the 4 waves' partials through LDS (one quantity at a time: [4][C] floats)
  extern __shared__ __attribute__((aligned(16))) float red[];
  auto flush = [&](float (*acc)[8], float* part) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int c = lane + 64 * k;
      if (c < nch) {
#pragma unroll
        for (int j = 0; j < 8; ++j) red[wid * C + c * 8 + j] = acc[k][j];
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < C; i += blockDim.x)
      part[(size_t)blockIdx.x * C + i] = (red[i] + red[C + i]) + (red[2 * C + i] + red[3 * C + i]);
    __syncthreads();
  };
  flush(dwa, dw_part);
  if (db_part) flush(dba, db_part);
  if (XB) flush(xba, xb_part);
}

// column sums of an fp32 [G, C] slab -> [C] gradient (bf16 or fp32: OF32).  One 1024-thread
// block per 64 columns: 16 waves each sum a strided subset of the G rows (coalesced 256 B per
// wave-row), then a fixed-order LDS combine -> deterministic.
template <bool OF32>
__global__ __launch_bounds__(1024) void col_reduce_kernel(const float* __restrict__ part, int G, int C,
                                                          void* __restrict__ out, int accumulate) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, g0 = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float a0 = 0.f, a1 = 0.f;
  if (c < C) {
    int g = g0;
    for (; g + 16 < G; g += 32) {
      a0 += part[(size_t)g * C + c];
      a1 += part[(size_t)(g + 16) * C + c];
    }
    if (g < G) a0 += part[(size_t)g * C + c];
  }
  red[g0][lane] = a0 + a1;
  __syncthreads();
  if (threadIdx.x < 64 && c < C) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += red[i][lane];
    stg1<OF32>(out, c, accumulate ? s + ldg1<OF32>(out, c) : s);
  }
}

// Up to three column reductions of the same [G, C] geometry in ONE launch (blockIdx.y picks the
// slab): a LayerNorm backward's weight, bias and producer-bias gradients.  Three 6.8-us launches
// of 12 blocks each were 0.66 ms of the GPT-2-small step (profiles/r2_prof6_gpt2small_b64_kernel_stats.md).
struct ColReduceSet {
  const float* part[3];
  void* out[3];
  int accumulate[3];
};
template <bool OF32>
__global__ __launch_bounds__(1024) void col_reduce_set_kernel(ColReduceSet set, int G, int C) {
  __shared__ float red[16][64];
  const int y = blockIdx.y;
  const float* __restrict__ part = set.part[y];
  const int lane = threadIdx.x & 63, g0 = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float a0 = 0.f, a1 = 0.f;
  if (c < C) {
    int g = g0;
    for (; g + 16 < G; g += 32) {
      a0 += part[(size_t)g * C + c];
      a1 += part[(size_t)(g + 16) * C + c];
    }
    if (g < G) a0 += part[(size_t)g * C + c];
  }
  red[g0][lane] = a0 + a1;
  __syncthreads();
  if (threadIdx.x < 64 && c < C) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += red[i][lane];
    stg1<OF32>(set.out[y], c, set.accumulate[y] ? s + ldg1<OF32>(set.out[y], c) : s);
  }
}

// per-block column partial sums of a bf16 [N, C] matrix (bias gradient of a linear
// layer whose output gradient is x).  Block = 256 threads = 4 row lanes x 64 column
// chunks of 8 -> one 512-column panel; grid = (panels, row groups).
__global__ __launch_bounds__(256) void colsum_partial_kernel(const uint16_t* __restrict__ x, int N, int C,
                                                             float* __restrict__ part) {
  __shared__ float red[4][512];
  const int lane = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c8 = blockIdx.x * 64 + lane;  // 8-column chunk index
  const int nch = C >> 3;
  const int rows_per = (N + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * rows_per, r1 = min(N, r0 + rows_per);
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c8 < nch) {
    int r = r0 + rl;
    for (; r + 4 < r1; r += 8) {
      float f[8], h[8];
      unpack8(ld16(x + (size_t)r * C + c8 * 8), f);
      unpack8(ld16(x + (size_t)(r + 4) * C + c8 * 8), h);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += f[j] + h[j];
    }
    if (r < r1) {
      float f[8];
      unpack8(ld16(x + (size_t)r * C + c8 * 8), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += f[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rl][lane * 8 + j] = a[j];
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 256) {
    const int c = blockIdx.x * 512 + i;
    if (c < C) part[(size_t)blockIdx.y * C + c] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
  }
}

}  // namespace

namespace pllm {

void norm_fwd(const void* x, const void* res, const void* w, const void* b, void* y, void* s, float* mean,
              float* rstd, int N, int C, float eps, bool rms, hipStream_t st) {
  const int blocks = (N + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK;
  const int K = (C + 511) / 512;
  // rows of <= 1,024 elements and >= 4 rows per wave of the persistent grid (8 blocks of 4 waves per CU):
  // the persistent two-row-prefetch kernel -- 36-37 vs 41-43 us at 65536 x 768 -- else one row per wave, full
  // grid (32768 x 2048: 45 vs 47 us; 16384 x 1024: 14.7 vs 15.4 us) (profiles/r6_norm_fwd_prefetch.log)
  const bool pf = K <= 2 && blocks >= 4 * 2048;
  dim3 grid(pf ? 2048 : blocks), block(256);
#define L(KK)                                                                                                  \
  do {                                                                                                         \
    if (pf)                                                                                                    \
      hipLaunchKernelGGL(norm_fwd_pf_kernel<KK>, grid, block, 0, st, (const uint16_t*)x, (const uint16_t*)res, \
                         (const uint16_t*)w, (const uint16_t*)b, (uint16_t*)y, (uint16_t*)s, mean, rstd, N, C,  \
                         eps, (int)rms);                                                                       \
    else                                                                                                       \
      hipLaunchKernelGGL(norm_fwd_kernel<KK>, grid, block, 0, st, (const uint16_t*)x, (const uint16_t*)res,    \
                         (const uint16_t*)w, (const uint16_t*)b, (uint16_t*)y, (uint16_t*)s, mean, rstd, N, C,  \
                         eps, (int)rms);                                                                       \
  } while (0)
  if (K <= 1) L(1);
  else if (K <= 2) L(2);
  else if (K <= 4) L(4);
  else L(8);
#undef L
}

// rows of > 1,024 elements (K >= 4, 256 VGPRs): 256 workgroups -- 98-99 vs 102-104 us at 32768 x 2048 --
// else 512 (at 65536 x 768: 78-85 us, 110 with 256, 92 with 1,024) (profiles/r6_norm_grid_sweep.log)
int norm_bwd_grid(int N, int C) {
  int g = (N + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK;
  const int cap = C > 1024 ? 256 : 512;
  return g < cap ? g : cap;
}

void col_reduce(const float* part, int G, int C, void* out, bool out_f32, bool accumulate, hipStream_t st) {
  if (out_f32)
    hipLaunchKernelGGL(col_reduce_kernel<true>, dim3((C + 63) / 64), dim3(1024), 0, st, part, G, C, out,
                       (int)accumulate);
  else
    hipLaunchKernelGGL(col_reduce_kernel<false>, dim3((C + 63) / 64), dim3(1024), 0, st, part, G, C, out,
                       (int)accumulate);
}

void norm_bwd(const void* dy, const void* s, const void* w, const float* mean, const float* rstd, const void* ds,
              void* dx, float* dw_part, float* db_part, void* dw, void* db, bool grad_f32, int N, int C, bool rms,
              bool accumulate, float* xb_part, void* xb, bool xb_accumulate, hipStream_t st) {
  const int G = norm_bwd_grid(N, C);
  const int K = (C + 511) / 512;
  const size_t lds = (size_t)4 * C * sizeof(float);
#define L(KK, XBB)                                                                                              \
  hipLaunchKernelGGL((norm_bwd_kernel<KK, XBB>), dim3(G), dim3(256), lds, st, (const uint16_t*)dy,            \
                     (const uint16_t*)s, (const uint16_t*)w, mean, rstd, (const uint16_t*)ds, (uint16_t*)dx, dw_part, \
                     db_part, xb_part, N, C, (int)rms)
  const bool xbf = xb_part != nullptr;
  if (K <= 1) { if (xbf) L(1, true); else L(1, false); }
  else if (K <= 2) { if (xbf) L(2, true); else L(2, false); }
  else if (K <= 4) { if (xbf) L(4, true); else L(4, false); }
  else { if (xbf) L(8, true); else L(8, false); }
#undef L
  // the (bit-identical) per-slab reductions of col_reduce, batched into one launch
  ColReduceSet set{};
  int n = 0;
  set.part[n] = dw_part, set.out[n] = dw, set.accumulate[n++] = (int)accumulate;
  if (db_part && db) set.part[n] = db_part, set.out[n] = db, set.accumulate[n++] = (int)accumulate;
  if (xbf && xb) set.part[n] = xb_part, set.out[n] = xb, set.accumulate[n++] = (int)xb_accumulate;
  const dim3 rg((C + 63) / 64, n);
  if (grad_f32) hipLaunchKernelGGL(col_reduce_set_kernel<true>, rg, dim3(1024), 0, st, set, G, C);
  else hipLaunchKernelGGL(col_reduce_set_kernel<false>, rg, dim3(1024), 0, st, set, G, C);
}

int colsum_groups(int N) {
  int g = N / 256;
  return g < 1 ? 1 : (g > 256 ? 256 : g);
}

void bias_grad(const void* x, int N, int C, float* part, void* out, bool out_f32, bool accumulate, hipStream_t st) {
  const int G = colsum_groups(N);
  hipLaunchKernelGGL(colsum_partial_kernel, dim3((C + 511) / 512, G), dim3(256), 0, st, (const uint16_t*)x, N, C,
                     part);
  col_reduce(part, G, C, out, out_f32, accumulate, st);
}

}  // namespace pllm

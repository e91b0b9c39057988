// Token + learned-position embedding, forward and deterministic backward (gfx950).
//
// Reference: token_embed(idx) + position_embed(pos_idxs[:T])
// (src/models/transformer.py:41-54).  The backward of an embedding is a
// scatter-add; instead of float atomics (order-dependent results) the token
// ids are sorted once (torch.sort, stable) and each run of equal ids is summed
// by one wave in a fixed order, so dW_te is bitwise reproducible.
#include "common.h"
#include "kernels.h"

namespace {

__global__ __launch_bounds__(256) void embed_fwd_kernel(const int64_t* __restrict__ idx, const uint16_t* __restrict__ wte,
                                                        const uint16_t* __restrict__ wpe, uint16_t* __restrict__ out,
                                                        int64_t N, int T, int C, int pos_offset, int64_t V) {
  const int cv = C >> 3;
  const int64_t total = N * cv;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = i / cv;
    const int c = (int)(i - n * cv);
    const int64_t tok = idx[n];
    if (c == 0) PLLM_DCHECK(tok >= 0 && tok < V, "token id in [0, vocab)", tok);
    // out-of-range ids read nothing (row of zeros) instead of faulting the GPU
    u32x4 v = (tok >= 0 && tok < V) ? ld16(wte + tok * C + c * 8) : u32x4{0u, 0u, 0u, 0u};
    if (wpe) {
      float a[8], p[8];
      unpack8(v, a);
      unpack8(ld16(wpe + (int64_t)((n % T) + pos_offset) * C + c * 8), p);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += p[j];
      v = pack8(a);
    }
    st16(out + n * C + c * 8, v);
  }
}

// one wave per sorted position; only the first position of each run of equal
// ids does work: it sums the dx rows of the whole run in sorted (stable) order.
__global__ __launch_bounds__(256) void embed_bwd_tok_kernel(const uint16_t* __restrict__ dx, const int32_t* __restrict__ sorted,
                                                            const int32_t* __restrict__ perm, uint16_t* __restrict__ dwte,
                                                            int64_t N, int C, int64_t V) {
  const int64_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= N) return;
  const int id = sorted[i];
  if (id < 0 || id >= V) return;  // out-of-range ids contribute nothing (forward read zeros)
  if (i > 0 && sorted[i - 1] == id) return;
  int64_t end = i + 1;
  while (end < N && sorted[end] == id) ++end;
  const int cv = C >> 3;
  for (int c = lane; c < cv; c += 64) {
    float acc[8];
    unpack8(ld16(dwte + (int64_t)id * C + c * 8), acc);  // accumulate into the destination
    for (int64_t j = i; j < end; ++j) {
      float f[8];
      unpack8(ld16(dx + (int64_t)perm[j] * C + c * 8), f);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += f[k];
    }
    st16(dwte + (int64_t)id * C + c * 8, pack8(acc));
  }
}

// dwpe[t] = sum_b dx[b, t]   (thread per (t, 8-col chunk), fixed b order)
__global__ __launch_bounds__(256) void embed_bwd_pos_kernel(const uint16_t* __restrict__ dx, uint16_t* __restrict__ dwpe,
                                                            int Bn, int T, int C) {
  const int cv = C >> 3;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= (int64_t)T * cv) return;
  const int t = (int)(i / cv), c = (int)(i % cv);
  float acc[8];
  unpack8(ld16(dwpe + (int64_t)t * C + c * 8), acc);  // accumulate into the destination
  for (int b = 0; b < Bn; ++b) {
    float f[8];
    unpack8(ld16(dx + ((int64_t)b * T + t) * C + c * 8), f);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += f[k];
  }
  st16(dwpe + (int64_t)t * C + c * 8, pack8(acc));
}

}  // namespace

namespace pllm {

void embedding_fwd(const int64_t* idx, const void* wte, const void* wpe, void* out, int64_t N, int T, int C,
                   int pos_offset, int64_t V, hipStream_t st) {
  int64_t work = N * (C / 8);
  int grid = (int)((work + 255) / 256);
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(grid), dim3(256), 0, st, idx, (const uint16_t*)wte, (const uint16_t*)wpe,
                     (uint16_t*)out, N, T, C, pos_offset, V);
}

void embedding_bwd(const void* dx, const int32_t* sorted, const int32_t* perm, void* dwte, void* dwpe, int64_t N,
                   int Bn, int T, int C, int64_t V, hipStream_t st) {
  hipLaunchKernelGGL(embed_bwd_tok_kernel, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, st, (const uint16_t*)dx, sorted,
                     perm, (uint16_t*)dwte, N, C, V);
  if (dwpe) {
    const int64_t work = (int64_t)T * (C / 8);
    hipLaunchKernelGGL(embed_bwd_pos_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, st,
                       (const uint16_t*)dx, (uint16_t*)dwpe, Bn, T, C);
  }
}

}  // namespace pllm

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
// dwte / dwpe are the optimizer's gradient views: bf16 or fp32 (F32)
template <bool F32>
__global__ __launch_bounds__(256) void embed_bwd_tok_kernel(const uint16_t* __restrict__ dx, const int32_t* __restrict__ sorted,
                                                            const int32_t* __restrict__ perm, void* __restrict__ dwte,
                                                            int64_t N, int C, int64_t V) {
  constexpr int ES = F32 ? 4 : 2;
  char* const gw = reinterpret_cast<char*>(dwte);
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
    ld8g<F32>(gw + ((int64_t)id * C + c * 8) * ES, acc);  // accumulate into the destination
    for (int64_t j = i; j < end; ++j) {
      float f[8];
      unpack8(ld16(dx + (int64_t)perm[j] * C + c * 8), f);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += f[k];
    }
    st8g<F32>(gw + ((int64_t)id * C + c * 8) * ES, acc);
  }
}

// dwpe[t] = sum_b dx[b, t]   (thread per (t, 8-col chunk), fixed b order)
template <bool F32>
__global__ __launch_bounds__(256) void embed_bwd_pos_kernel(const uint16_t* __restrict__ dx, void* __restrict__ dwpe,
                                                            int Bn, int T, int C) {
  constexpr int ES = F32 ? 4 : 2;
  char* const gw = reinterpret_cast<char*>(dwpe);
  const int cv = C >> 3;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= (int64_t)T * cv) return;
  const int t = (int)(i / cv), c = (int)(i % cv);
  float acc[8];
  ld8g<F32>(gw + ((int64_t)t * C + c * 8) * ES, acc);  // accumulate into the destination
  for (int b = 0; b < Bn; ++b) {
    float f[8];
    unpack8(ld16(dx + ((int64_t)b * T + t) * C + c * 8), f);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += f[k];
  }
  st8g<F32>(gw + ((int64_t)t * C + c * 8) * ES, acc);
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

void embedding_bwd(const void* dx, const int32_t* sorted, const int32_t* perm, void* dwte, void* dwpe, bool grad_f32,
                   int64_t N, int Bn, int T, int C, int64_t V, hipStream_t st) {
  const dim3 tg((unsigned)((N + 3) / 4)), pg((unsigned)(((int64_t)T * (C / 8) + 255) / 256));
  if (grad_f32) {
    hipLaunchKernelGGL(embed_bwd_tok_kernel<true>, tg, dim3(256), 0, st, (const uint16_t*)dx, sorted, perm, dwte, N, C, V);
    if (dwpe) hipLaunchKernelGGL(embed_bwd_pos_kernel<true>, pg, dim3(256), 0, st, (const uint16_t*)dx, dwpe, Bn, T, C);
  } else {
    hipLaunchKernelGGL(embed_bwd_tok_kernel<false>, tg, dim3(256), 0, st, (const uint16_t*)dx, sorted, perm, dwte, N, C, V);
    if (dwpe) hipLaunchKernelGGL(embed_bwd_pos_kernel<false>, pg, dim3(256), 0, st, (const uint16_t*)dx, dwpe, Bn, T, C);
  }
}

}  // namespace pllm

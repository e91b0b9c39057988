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
    if (c == 0) PL_DCHECK(tok >= 0 && tok < V, "token id in [0, vocab)", tok);
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

// Token-embedding backward over the stably sorted ids, in fixed chunks of EK sorted positions
// (skew-robust: a Zipf-distributed batch -- real text, or the learnable synthetic shards -- has
// runs of tens of thousands of equal ids; the first version summed each run with one wave and
// took 13 ms per GPT-2-small step on such data against 0.07 ms on uniform ids).
//   phase 1 (one workgroup per chunk, one thread per 8-column chunk): walk the chunk's positions
//     in sorted order summing gathered dx rows per run.  A run that starts and ends inside the
//     chunk is complete and is added straight into dW[id] (no other workgroup touches that row).
//     A run crossing the chunk's START leaves its in-chunk sum in head[j] (the prefix, or the
//     whole chunk when the run also crosses the end); a run that starts inside the chunk and
//     crosses its END leaves its sum in tail[j].
//   phase 2 (one workgroup per chunk that owns such a crossing run): tail[j] + head[j+1] + ...
//     in chunk order until the chunk where the run ends, added into dW[id].
// Every row of dW is written by exactly one thread, every sum runs in a fixed order: bitwise
// reproducible, no atomics.  dwte: the optimizer's gradient view, bf16 or fp32 (F32).
constexpr int EK = 64;

template <bool F32>
__global__ __launch_bounds__(256) void embed_bwd_chunk_kernel(const uint16_t* __restrict__ dx,
                                                              const int32_t* __restrict__ sorted,
                                                              const int32_t* __restrict__ perm, void* __restrict__ dwte,
                                                              float* __restrict__ head, float* __restrict__ tail,
                                                              int64_t N, int C, int64_t V) {
  constexpr int ES = F32 ? 4 : 2;
  char* const gw = reinterpret_cast<char*>(dwte);
  const int64_t j = blockIdx.x, p0 = j * EK, p1 = min(N, p0 + EK);
  const int cv = C >> 3;
  // run boundaries of the chunk are wave-uniform: every thread walks the same ids
  const int first_id = sorted[p0];
  const bool from_prev = p0 > 0 && sorted[p0 - 1] == first_id;
  const bool to_next = p1 < N && sorted[p1] == sorted[p1 - 1];
  for (int c = threadIdx.x; c < cv; c += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    bool started_here = !from_prev;
    for (int64_t g = p0; g < p1; g += 8) {
      // 8 gathered rows in flight, then summed in sorted order
      u32x4 rows[8];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        rows[k] = g + k < p1 ? ld16(dx + (int64_t)perm[g + k] * C + c * 8) : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int64_t p = g + k;
        if (p >= p1) break;
        float f[8];
        unpack8(rows[k], f);
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] += f[q];
        const int id = sorted[p];
        if (p + 1 < p1 && sorted[p + 1] == id) continue;  // run goes on inside the chunk
        const bool crosses_end = p + 1 == p1 && to_next;
        float* part = !started_here ? head + j * C : (crosses_end ? tail + j * C : nullptr);
        if (part) {
          st16(part + c * 8, u32x4{__float_as_uint(acc[0]), __float_as_uint(acc[1]), __float_as_uint(acc[2]),
                                   __float_as_uint(acc[3])});
          st16(part + c * 8 + 4, u32x4{__float_as_uint(acc[4]), __float_as_uint(acc[5]), __float_as_uint(acc[6]),
                                       __float_as_uint(acc[7])});
        } else if (id >= 0 && id < V) {  // out-of-range ids contribute nothing (the forward read zeros)
          float o[8];
          ld8g<F32>(gw + ((int64_t)id * C + c * 8) * ES, o);
#pragma unroll
          for (int q = 0; q < 8; ++q) o[q] += acc[q];
          st8g<F32>(gw + ((int64_t)id * C + c * 8) * ES, o);
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] = 0.f;
        started_here = true;
      }
    }
  }
}

template <bool F32>
__global__ __launch_bounds__(256) void embed_bwd_carry_kernel(const int32_t* __restrict__ sorted,
                                                              void* __restrict__ dwte, const float* __restrict__ head,
                                                              const float* __restrict__ tail, int64_t N, int C,
                                                              int64_t V) {
  constexpr int ES = F32 ? 4 : 2;
  char* const gw = reinterpret_cast<char*>(dwte);
  const int64_t nch = (N + EK - 1) / EK;
  const int64_t j = blockIdx.x, p0 = j * EK, p1 = min(N, p0 + EK);
  const int id = sorted[p1 - 1];
  // chunk j owns a crossing run iff its last run continues into chunk j+1 and started in chunk j
  if (!(p1 < N && sorted[p1] == id)) return;
  if (p0 > 0 && sorted[p0] == id && sorted[p0 - 1] == id) return;
  if (id < 0 || id >= V) return;
  const int cv = C >> 3;
  for (int c = threadIdx.x; c < cv; c += blockDim.x) {
    float acc[8];
    const f32x4* t = reinterpret_cast<const f32x4*>(tail + j * C + c * 8);
    const f32x4 t0 = t[0], t1 = t[1];
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = t0[k], acc[4 + k] = t1[k];
    for (int64_t jj = j + 1; jj < nch; ++jj) {
      const f32x4* h = reinterpret_cast<const f32x4*>(head + jj * C + c * 8);
      const f32x4 h0 = h[0], h1 = h[1];
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] += h0[k], acc[4 + k] += h1[k];
      const int64_t e = min(N, (jj + 1) * EK);
      if (!(e < N && sorted[e - 1] == id && sorted[e] == id)) break;  // the run ends in chunk jj
    }
    float o[8];
    ld8g<F32>(gw + ((int64_t)id * C + c * 8) * ES, o);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] += acc[k];
    st8g<F32>(gw + ((int64_t)id * C + c * 8) * ES, o);
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

int64_t embedding_bwd_chunks(int64_t N) { return (N + EK - 1) / EK; }

void embedding_bwd(const void* dx, const int32_t* sorted, const int32_t* perm, void* dwte, void* dwpe, bool grad_f32,
                   float* part, int64_t N, int Bn, int T, int C, int64_t V, hipStream_t st) {
  const int64_t nch = embedding_bwd_chunks(N);
  float* head = part;
  float* tail = part + nch * C;
  const int cv = C / 8;
  const dim3 cg((unsigned)nch), cb((unsigned)(cv >= 256 ? 256 : (cv + 63) / 64 * 64));
  const dim3 pg((unsigned)(((int64_t)T * (C / 8) + 255) / 256));
#define L(F)                                                                                                  \
  hipLaunchKernelGGL(embed_bwd_chunk_kernel<F>, cg, cb, 0, st, (const uint16_t*)dx, sorted, perm, dwte, head, \
                     tail, N, C, V);                                                                          \
  hipLaunchKernelGGL(embed_bwd_carry_kernel<F>, cg, cb, 0, st, sorted, dwte, head, tail, N, C, V);            \
  if (dwpe) hipLaunchKernelGGL(embed_bwd_pos_kernel<F>, pg, dim3(256), 0, st, (const uint16_t*)dx, dwpe, Bn, T, C)
  if (grad_f32) { L(true); } else { L(false); }
#undef L
}

}  // namespace pllm

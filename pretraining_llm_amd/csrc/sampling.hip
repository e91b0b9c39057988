// Fused next-token sampling for generation (gfx950).
//
// Reference: softmax of the last position's logits, then torch.multinomial
// (src/models/transformer.py:111-112) -- a softmax pass, a normalisation pass, a
// cumulative-sum pass and a search, each a separate launch per generated token.
// Here one workgroup per sequence draws the token in ONE pass over the logits with
// the Gumbel-max trick:
//     token = argmax_i ( logit_i / T + G_i ),   G_i = -log(-log(U_i)),  U_i ~ U(0,1)
// which is an exact sample of softmax(logits / T).  U_i comes from a counter-based
// hash of (seed, row, i), so a draw is reproducible from the seed and needs no RNG
// state on the device.  T == 0 is greedy argmax.  Masked (-inf) logits are never
// drawn.  Ties resolve to the lowest index, like torch.argmax.
#include "common.h"
#include "kernels.h"

namespace {

PL_DEV uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// (value, index) argmax with lowest-index tie break
PL_DEV void better(float& v, int& i, float v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) {
    v = v2;
    i = i2;
  }
}

template <typename T>
PL_DEV float load_logit(const T* p, int64_t i);
template <>
PL_DEV float load_logit<float>(const float* p, int64_t i) { return p[i]; }
template <>
PL_DEV float load_logit<uint16_t>(const uint16_t* p, int64_t i) { return bf2f(p[i]); }

template <typename T>
__global__ __launch_bounds__(1024) void sample_kernel(const T* __restrict__ logits, int64_t ld, int V, float inv_temp,
                                                      int greedy, uint64_t seed, int64_t* __restrict__ out) {
  __shared__ float sv[16];
  __shared__ int si[16];
  const int row = blockIdx.x;
  const T* x = logits + row * ld;
  const uint64_t rkey = mix64(seed ^ (0x9e3779b97f4a7c15ull * (uint64_t)(row + 1)));
  float best = -INFINITY;
  int bi = 0x7fffffff;
  // SU independent loads in flight per thread before any compare: a plain strided loop kept
  // one load outstanding at a time (21.5 us for one 50,304-logit row,
  // profiles/r1_decode_gemv_kernel_stats.md)
  constexpr int SU = 16;
  for (int i0 = threadIdx.x; i0 < V; i0 += blockDim.x * SU) {
    float sv_[SU];
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const int i = i0 + u * blockDim.x;
      sv_[u] = i < V ? load_logit<T>(x, i) : NAN;
    }
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const int i = i0 + u * blockDim.x;
      float s = sv_[u];
      if (!greedy) {
        const uint64_t h = mix64(rkey + (uint64_t)i);
        const float uu = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);  // (0, 1)
        s = s * inv_temp - __logf(-__logf(uu));
      }
      if (s == s) better(best, bi, s, i);  // NaN logits (and the tail padding) are never drawn
    }
  }
  // wave then block argmax
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float v2 = __shfl_xor(best, o, 64);
    const int i2 = __shfl_xor(bi, o, 64);
    better(best, bi, v2, i2);
  }
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nw = blockDim.x >> 6;
  if (l == 0) {
    sv[w] = best;
    si[w] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < nw; ++k) better(best, bi, sv[k], si[k]);
    // every logit -inf/NaN: fall back to token 0 instead of an out-of-range id
    out[row] = bi < V ? bi : 0;
  }
}

}  // namespace

namespace pllm {

void sample_tokens(const void* logits, bool bf16_in, int64_t ld, int B, int V, float temperature, uint64_t seed,
                   int64_t* out, hipStream_t st) {
  const int greedy = temperature <= 0.f;
  const float inv_t = greedy ? 1.f : 1.f / temperature;
  if (bf16_in)
    hipLaunchKernelGGL(sample_kernel<uint16_t>, dim3(B), dim3(1024), 0, st, (const uint16_t*)logits, ld, V, inv_t,
                       greedy, seed, out);
  else
    hipLaunchKernelGGL(sample_kernel<float>, dim3(B), dim3(1024), 0, st, (const float*)logits, ld, V, inv_t, greedy,
                       seed, out);
}

}  // namespace pllm

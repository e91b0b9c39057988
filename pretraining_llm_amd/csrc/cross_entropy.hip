// Fused softmax cross-entropy, forward + backward in one pass (gfx950).
//
// Reference: F.cross_entropy(logits.view(B*T, V), targets.view(B*T)) in fp32
// under autocast (src/models/transformer.py:72-77).  Here one workgroup of
// 512 threads owns one row of bf16 logits; the row (V = 50304 -> 98 KiB) stays
// in registers (CH chunks of 8 bf16 per lane), so the logits are read from HBM
// exactly once and, in training, overwritten in place by
//     dlogits = (softmax(x) - onehot(t)) * inv_n          (inv_n = 1 / #valid)
// so no probability tensor and no second logits-sized buffer ever exist.
#include <cstdlib>

#include "ab.h"
#include "common.h"
#include "kernels.h"

namespace {

constexpr int CE_THREADS = 512;
// each lane's (max, exp-sum) pair merged in ONE block reduction (2 barriers per row instead of 5 for
// separate max / sum reductions): 2,524 vs 2,551 us at 65536 x 50304 (bench/ce_bench.py, round 4)

// one row per block: stores of the gradient with the non-temporal hint when NTS (A/B)
template <int CH, bool WRITE_GRAD, int CE_THREADS = 512, bool NTS = false>
__global__ __launch_bounds__(CE_THREADS) void ce_kernel(const uint16_t* __restrict__ logits, int64_t ld,
                                                         const int64_t* __restrict__ targets, int V,
                                                         int ignore_index, float* __restrict__ loss,
                                                         uint16_t* __restrict__ dlogits, const float* __restrict__ inv_n) {
  // The row is held PACKED (bf16, 4 VGPRs per 8 logits) so a 512-thread block needs ~52
  // VGPRs for V = 50304 and several blocks fit per CU; exp2 is recomputed in the output
  // pass instead of being stored (VALU is idle in this HBM-bound kernel).
  constexpr float LOG2E = 1.4426950408889634f;
  constexpr int CE_WAVES = CE_THREADS / 64;
  __shared__ float scratch[2 * CE_WAVES];
  const int row = blockIdx.x;
  const uint16_t* x = logits + (size_t)row * ld;
  const int nch = V >> 3;
  u32x4 v[CH];
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int c = threadIdx.x + CE_THREADS * k;
#ifndef PL_CE_NTL
#define PL_CE_NTL 1
#endif
    // non-temporal loads of the once-read logits: 2,370 vs 2,490 us at 65536 x 50304, 3 interleaved rounds
    // (profiles/r6_ce_nt_loads.log)
    if (PL_CE_NTL)
      v[k] = c < nch ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(x + c * 8))
                     : u32x4{0xff80ff80u, 0xff80ff80u, 0xff80ff80u, 0xff80ff80u};
    else
      v[k] = c < nch ? ld16(x + c * 8) : u32x4{0xff80ff80u, 0xff80ff80u, 0xff80ff80u, 0xff80ff80u};  // -inf
  }
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    float f[8];
    unpack8(v[k], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, f[j]);
  }
  // scalar tail when V % 8 != 0
  const int tail0 = nch * 8;
  float tv = -INFINITY;
  const int tj = tail0 + threadIdx.x;
  if (tj < V) {
    tv = bf2f(x[tj]);
    m = fmaxf(m, tv);
  }
  const int64_t t = targets[row];
  const bool valid = t != (int64_t)ignore_index && t >= 0 && t < V;
  float mc, s;
  {
    // the lane's own max, its exp-sum against it, then ONE block reduction of (max, sum) pairs
    // (2 barriers instead of 4; the target logit is read before any lane can overwrite it)
    const float xt = (threadIdx.x == 0 && valid) ? bf2f(x[t]) : 0.f;
    const float ml = m == -INFINITY ? 0.f : m * LOG2E;
#pragma unroll
    for (int k = 0; k < CH; ++k) asm volatile("" : "+v"(v[k]));
    float sl = 0.f;
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      float f[8];
      unpack8(v[k], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) sl += fast_exp2(__builtin_fmaf(f[j], LOG2E, -ml));
    }
    if (tj < V) sl += fast_exp2(__builtin_fmaf(tv, LOG2E, -ml));
    // wave: pairwise (m, s) merge, then across waves through LDS
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(sl, o, 64);
      const float mn = fmaxf(m, m2);
      const float mnl = mn == -INFINITY ? 0.f : mn * LOG2E;
      sl = (m == -INFINITY ? 0.f : sl * fast_exp2(m * LOG2E - mnl)) +
           (m2 == -INFINITY ? 0.f : s2 * fast_exp2(m2 * LOG2E - mnl));
      m = mn;
    }
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (l == 0) {
      scratch[w] = m;
      scratch[CE_WAVES + w] = sl;
    }
    __syncthreads();
    float mb = -INFINITY;
#pragma unroll
    for (int i = 0; i < CE_WAVES; ++i) mb = fmaxf(mb, scratch[i]);
    mc = mb * LOG2E;
    float sb = 0.f;
#pragma unroll
    for (int i = 0; i < CE_WAVES; ++i) {
      const float mi = scratch[i];
      if (mi != -INFINITY) sb += scratch[CE_WAVES + i] * fast_exp2(mi * LOG2E - mc);
    }
    m = mb;
    s = sb;
#pragma unroll
    for (int k = 0; k < CH; ++k) asm volatile("" : "+v"(v[k]));
    if (threadIdx.x == 0) PL_DCHECK(t == (int64_t)ignore_index || (t >= 0 && t < V), "target in [0, vocab) or ignore_index", t);
    if (threadIdx.x == 0) loss[row] = valid ? (__logf(s) + m - xt) : 0.f;
    if (!WRITE_GRAD) return;
    __syncthreads();  // lane 0's target-logit read (consumed by the loss above) precedes every store
  }
  const float in = *inv_n;
  const float scale = valid ? in / s : 0.f;
  uint16_t* dx = dlogits + (size_t)row * ld;
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int c = threadIdx.x + CE_THREADS * k;
    if (c < nch) {
      float f[8];
      unpack8(v[k], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = fast_exp2(__builtin_fmaf(f[j], LOG2E, -mc)) * scale;
      if (valid && (int)(t >> 3) == c) f[t & 7] -= in;
      if constexpr (NTS) __builtin_nontemporal_store(pack8(f), reinterpret_cast<u32x4*>(dx + c * 8));
      else st16(dx + c * 8, pack8(f));
    }
  }
  if (tj < V) {
    float o = fast_exp2(__builtin_fmaf(tv, LOG2E, -mc)) * scale;
    if (valid && tj == t) o -= in;
    dx[tj] = f2bf_bits(o);
  }
}

}  // namespace

namespace pllm {

template <int NT, bool NTS>
void ce_launch(const void* logits, int64_t ld, const int64_t* targets, int N, int V, int ignore_index, float* loss,
               void* dlogits, const float* inv_n, hipStream_t st) {
  const int nch = V / 8;
  const int CH = (nch + NT - 1) / NT;
  const bool g = dlogits != nullptr;
#define L(C)                                                                                               \
  do {                                                                                                     \
    if (g)                                                                                                 \
      hipLaunchKernelGGL((ce_kernel<C, true, NT, NTS>), dim3(N), dim3(NT), 0, st, (const uint16_t*)logits, ld, \
                         targets, V, ignore_index, loss, (uint16_t*)dlogits, inv_n);                       \
    else                                                                                                   \
      hipLaunchKernelGGL((ce_kernel<C, false, NT, NTS>), dim3(N), dim3(NT), 0, st, (const uint16_t*)logits, ld, \
                         targets, V, ignore_index, loss, (uint16_t*)nullptr, inv_n);                       \
  } while (0)
  if (CH <= 1) L(1);
  else if (CH <= 2) L(2);
  else if (CH <= 4) L(4);
  else if (CH <= 8) L(8);
  else if (CH <= 13) L(13);
  else if (CH <= 16) L(16);
  else L(32);
#undef L
}

void cross_entropy(const void* logits, int64_t ld, const int64_t* targets, int N, int V, int ignore_index,
                   float* loss, void* dlogits, const float* inv_n, hipStream_t st) {
  // non-temporal gradient stores: 2,493 vs 2,524 us at 65536 x 50304 (PLLM_AB=ce_nt=0: plain stores);
  // 256- / 1024-thread blocks measured 2,533 / 2,641 us (scripts/gpu/r4_ce2.sh, 3 interleaved rounds)
  static const bool nts = pllm::ab_int("ce_nt", 1) != 0;
  if (nts) ce_launch<CE_THREADS, true>(logits, ld, targets, N, V, ignore_index, loss, dlogits, inv_n, st);
  else ce_launch<CE_THREADS, false>(logits, ld, targets, N, V, ignore_index, loss, dlogits, inv_n, st);
}

int cross_entropy_max_vocab() { return CE_THREADS * 8 * 32 + CE_THREADS; }

}  // namespace pllm

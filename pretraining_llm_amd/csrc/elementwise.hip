// Memory-bound elementwise kernels (gfx950): activations and RoPE.
//
// * ReLU   -- reference MLP activation (src/models/mlp.py:25,39-41)
// * GELU   -- tanh form, GPT-2 preset
// * SwiGLU -- Llama preset, input laid out [gate | up] along the last dim
// * RoPE   -- rotate-half convention on the q and k heads of a packed qkv row
//
// Every kernel moves 16 B (8 x bf16) per lane per access over a FULL grid (one 16-B vector per
// thread; the loops still grid-stride for safety): a grid capped at 2048 blocks with
// grid-stride loops streamed 5.1 TB/s where the full grid streams 6.0-6.2 TB/s on MI355X
// (GELU fwd / bwd at 402 MB, bench/hbm_probe.py, profiles/r2_elementwise_grid_ab.txt).
#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace {

PL_DEV float sigmoid_f(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

inline int ew_grid(size_t n_vec) {
  size_t g = (n_vec + 255) / 256;
  return (int)(g < (1u << 30) ? (g > 0 ? g : 1) : (1u << 30));
}

// op: 0 relu, 1 gelu
template <int OP>
__global__ __launch_bounds__(256) void act_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                      size_t nvec) {
  // two 16-B vectors per thread per iteration: both loads are in flight before the math
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += 2 * stride) {
    const bool two = i + stride < nvec;
    const u32x4 va = ld16(x + i * 8);
    const u32x4 vb = two ? ld16(x + (i + stride) * 8) : va;
    float f[8], g[8];
    unpack8(va, f);
    unpack8(vb, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      f[j] = OP == 0 ? fmaxf(f[j], 0.f) : gelu_f(f[j]);
      g[j] = OP == 0 ? fmaxf(g[j], 0.f) : gelu_f(g[j]);
    }
    st16(y + i * 8, pack8(f));
    if (two) st16(y + (i + stride) * 8, pack8(g));
  }
}

// relu bwd takes the OUTPUT (y>0 <=> x>0), gelu bwd takes the input
template <int OP>
__global__ __launch_bounds__(256) void act_bwd_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ xin,
                                                      uint16_t* __restrict__ dx, size_t nvec) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    float g[8], a[8];
    unpack8(ld16(dy + i * 8), g);
    unpack8(ld16(xin + i * 8), a);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = OP == 0 ? (a[j] > 0.f ? g[j] : 0.f) : g[j] * gelu_df(a[j]);
    st16(dx + i * 8, pack8(g));
  }
}

// Activation backward that also produces the bias gradient of the linear layer
// feeding the activation (= column sums of dx), in the same pass over dy:
// grid = (512-column panels, row groups); per-block column partials -> fp32 slab.
template <int OP>
__global__ __launch_bounds__(256) void act_bwd_colsum_kernel(const uint16_t* __restrict__ dy,
                                                             const uint16_t* __restrict__ xin, uint16_t* __restrict__ dx,
                                                             int N, int C, float* __restrict__ part) {
  __shared__ float red[4][512];
  const int lane = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c8 = blockIdx.x * 64 + lane;
  const int nch = C >> 3;
  const int rows_per = (N + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * rows_per, r1 = min(N, r0 + rows_per);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c8 < nch) {
    // two rows per iteration: four 16-B loads in flight before the math
    for (int r = r0 + rl; r < r1; r += 8) {
      const bool two = r + 4 < r1;
      const size_t off = (size_t)r * C + c8 * 8, off2 = off + (size_t)4 * C;
      const u32x4 d0 = ld16(dy + off), x0 = ld16(xin + off);
      const u32x4 d1 = two ? ld16(dy + off2) : d0, x1 = two ? ld16(xin + off2) : x0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h == 1 && !two) break;
        float g[8], a[8];
        unpack8(h ? d1 : d0, g);
        unpack8(h ? x1 : x0, a);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = OP == 0 ? (a[j] > 0.f ? g[j] : 0.f) : g[j] * gelu_df(a[j]);
        const u32x4 o = pack8(g);
        st16(dx + (h ? off2 : off), o);
        unpack8(o, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += g[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rl][lane * 8 + j] = acc[j];
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 256) {
    const int c = blockIdx.x * 512 + i;
    if (c < C) part[(size_t)blockIdx.y * C + c] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
  }
}

// SwiGLU: gu [rows, 2F] -> y [rows, F];  F % 8 == 0
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const uint16_t* __restrict__ gu, uint16_t* __restrict__ y,
                                                         size_t rows, int F) {
  const int fv = F >> 3;
  const size_t nvec = rows * fv;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    const size_t r = i / fv;
    const int c = (int)(i - r * fv);
    float g[8], u[8];
    unpack8(ld16(gu + r * 2 * F + c * 8), g);
    unpack8(ld16(gu + r * 2 * F + F + c * 8), u);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = g[j] * sigmoid_f(g[j]) * u[j];
    st16(y + r * F + c * 8, pack8(g));
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ gu,
                                                         uint16_t* __restrict__ dgu, size_t rows, int F) {
  const int fv = F >> 3;
  const size_t nvec = rows * fv;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    const size_t r = i / fv;
    const int c = (int)(i - r * fv);
    float g[8], u[8], d[8], dg[8], du[8];
    unpack8(ld16(gu + r * 2 * F + c * 8), g);
    unpack8(ld16(gu + r * 2 * F + F + c * 8), u);
    unpack8(ld16(dy + r * F + c * 8), d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float sg = sigmoid_f(g[j]);
      const float silu = g[j] * sg;
      du[j] = d[j] * silu;
      dg[j] = d[j] * u[j] * sg * (1.f + g[j] * (1.f - sg));
    }
    st16(dgu + r * 2 * F + c * 8, pack8(dg));
    st16(dgu + r * 2 * F + F + c * 8, pack8(du));
  }
}

// RoPE over the first n_rot heads of each packed row [rows, n_heads_total*D]
// (q heads then k heads); the remaining heads (v) are copied when out != in.
// cos/sin: fp32 [T, D/2]; row r has position (r % T) + pos_offset.
// dir = +1 forward rotation, -1 inverse (backward).
// out_heads: heads written per output row (n_heads_total: full copy; n_rot: the rotated q and k
// heads only, into a [rows, n_rot*D] buffer -- the attention pre-pass)
__global__ __launch_bounds__(256) void rope_kernel(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                                   const float* __restrict__ cosb, const float* __restrict__ sinb,
                                                   size_t rows, int T, int n_heads_total, int n_rot, int D,
                                                   int pos_offset, float dir, int out_heads) {
  const int half = D >> 1;
  const int hv = half >> 3;  // 8-element groups per half
  const size_t W = (size_t)n_heads_total * D, WO = (size_t)out_heads * D;
  const size_t nwork = rows * out_heads * hv;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nwork; i += (size_t)gridDim.x * blockDim.x) {
    const int g = (int)(i % hv);
    const size_t rh = i / hv;
    const int h = (int)(rh % out_heads);
    const size_t r = rh / out_heads;
    const uint16_t* src = in + r * W + (size_t)h * D;
    uint16_t* dst = out + r * WO + (size_t)h * D;
    u32x4 lo = ld16(src + g * 8), hi = ld16(src + half + g * 8);
    if (h < n_rot) {
      const int t = (int)(r % T) + pos_offset;
      float a[8], b[8], o1[8], o2[8];
      unpack8(lo, a);
      unpack8(hi, b);
      const float* cp = cosb + (size_t)t * half + g * 8;
      const float* sp = sinb + (size_t)t * half + g * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float c = cp[j], s = sp[j] * dir;
        o1[j] = a[j] * c - b[j] * s;
        o2[j] = b[j] * c + a[j] * s;
      }
      st16(dst + g * 8, pack8(o1));
      st16(dst + half + g * 8, pack8(o2));
    } else if (dst != src) {
      st16(dst + g * 8, lo);
      st16(dst + half + g * 8, hi);
    }
  }
}

// x *= s[0] in place (bf16 or fp32), a no-op launch when s[0] == 1 (x * 1 == x bit for bit): the LM-head
// backward's scale by the upstream gradient is 1 in every plain training step, so the 100-250 MB pass it
// used to cost (torch mul) is read only when a loss scale / accumulation factor makes it needed
template <bool F32>
__global__ __launch_bounds__(256) void scale_kernel(void* __restrict__ xv, const float* __restrict__ s, size_t nvec) {
  const float sc = *s;
  if (sc == 1.f) return;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    if constexpr (F32) {
      f32x4* x = reinterpret_cast<f32x4*>(xv) + 2 * i;
      f32x4 a = x[0], b = x[1];
      x[0] = a * sc;
      x[1] = b * sc;
    } else {
      uint16_t* x = reinterpret_cast<uint16_t*>(xv);
      float f[8];
      unpack8(ld16(x + i * 8), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= sc;
      st16(x + i * 8, pack8(f));
    }
  }
}


// Ring attention's LSE merge (parallel/context.py _merge; the reference has no context parallelism,
// its attention is /root/reference/src/models/attention.py:47-57): a partial block result (o bf16,
// lse fp32) folded into the fp32 accumulators in place --
//   new = logaddexp(lse_acc, lse); o_acc = o_acc e^(lse_acc - new) + o e^(lse - new); lse_acc = new
// (a weight whose exponent is -inf - -inf is 0, as torch's nan_to_num).  One lane per 8 head
// elements; a row's D / 8 <= 16 lanes sit in one wave, which reads lse_acc before its lane 0
// writes it.  Replaces five fp32 torch passes per block pair.
struct LseMergeArgs {
  float* o_acc;
  float* lse_acc;
  const uint16_t* o;
  const float* lse;
  int64_t oa_b, oa_t, oa_h, la_b, la_h, la_t, o_b, o_t, o_h, l_b, l_h, l_t;
  int B, T, H, D;
};
__global__ __launch_bounds__(256) void lse_merge_kernel(LseMergeArgs a) {
  const int cpr = a.D / 8;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t row = gid / cpr;
  const int c = (int)(gid - row * cpr);
  if (row >= (int64_t)a.B * a.T * a.H) return;
  const int h = (int)(row % a.H);
  const int64_t bt = row / a.H;
  const int t = (int)(bt % a.T), b = (int)(bt / a.T);
  float* lap = a.lse_acc + b * a.la_b + h * a.la_h + t * a.la_t;
  const float la = *lap, lb = a.lse[b * a.l_b + h * a.l_h + t * a.l_t];
  const float mx = fmaxf(la, lb);
  const float nw = mx == -INFINITY ? -INFINITY : mx + log1pf(__expf(-fabsf(la - lb)));
  const float wa = la == -INFINITY ? 0.f : __expf(la - nw);
  const float wb = lb == -INFINITY ? 0.f : __expf(lb - nw);
  float* oa = a.o_acc + b * a.oa_b + t * a.oa_t + h * a.oa_h + 8 * c;
  float x[8];
  unpack8(*reinterpret_cast<const u32x4*>(a.o + b * a.o_b + t * a.o_t + h * a.o_h + 8 * c), x);
  f32x4* o4 = reinterpret_cast<f32x4*>(oa);
  f32x4 v0 = o4[0], v1 = o4[1];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v0[e] = v0[e] * wa + x[e] * wb;
    v1[e] = v1[e] * wa + x[4 + e] * wb;
  }
  o4[0] = v0;
  o4[1] = v1;
  if (c == 0) *lap = nw;
}

// zero n [start, end) byte ranges of a buffer (16-B aligned; desc int64 [n][3] = start, end, bytes of the
// ranges before this one): ONE flat grid over the ranges' total bytes, each thread finding its range by a
// scan of the (few) descriptors -- the optimizer's lazily zeroed gradient buffer clears its accumulate-only
// slots in one launch whose size follows the bytes, not the range count (train/optim.py)
__global__ __launch_bounds__(256) void zero_ranges_kernel(char* __restrict__ buf, const int64_t* __restrict__ desc,
                                                          int n, int64_t total) {
  const u32x4 z = {0u, 0u, 0u, 0u};
  for (int64_t v = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; v < total;
       v += (int64_t)gridDim.x * blockDim.x * 16) {
    int r = 0;
    while (r + 1 < n && desc[3 * (r + 1) + 2] <= v) ++r;
    *reinterpret_cast<u32x4*>(buf + desc[3 * r] + (v - desc[3 * r + 2])) = z;
  }
}

}  // namespace

namespace pllm {

void zero_ranges(void* buf, const int64_t* desc, int n, int64_t total_bytes, hipStream_t st) {
  if (n <= 0 || total_bytes <= 0) return;
  const int64_t vec = (total_bytes + 15) / 16;
  const int gx = (int)std::min<int64_t>(std::max<int64_t>(1, (vec + 255) / 256), 1 << 20);
  hipLaunchKernelGGL(zero_ranges_kernel, dim3(gx), dim3(256), 0, st, (char*)buf, desc, n, total_bytes);
}


void act_fwd(int op, const void* x, void* y, size_t n, hipStream_t st) {
  const size_t nv = n / 8;
  if (op == 0)
    hipLaunchKernelGGL(act_fwd_kernel<0>, dim3(ew_grid(nv)), dim3(256), 0, st, (const uint16_t*)x, (uint16_t*)y, nv);
  else
    hipLaunchKernelGGL(act_fwd_kernel<1>, dim3(ew_grid(nv)), dim3(256), 0, st, (const uint16_t*)x, (uint16_t*)y, nv);
}

void act_bwd(int op, const void* dy, const void* xin, void* dx, size_t n, hipStream_t st) {
  const size_t nv = n / 8;
  if (op == 0)
    hipLaunchKernelGGL(act_bwd_kernel<0>, dim3(ew_grid(nv)), dim3(256), 0, st, (const uint16_t*)dy,
                       (const uint16_t*)xin, (uint16_t*)dx, nv);
  else
    hipLaunchKernelGGL(act_bwd_kernel<1>, dim3(ew_grid(nv)), dim3(256), 0, st, (const uint16_t*)dy,
                       (const uint16_t*)xin, (uint16_t*)dx, nv);
}

void act_bwd_bias(int op, const void* dy, const void* xin, void* dx, int N, int C, float* part, void* bias_grad,
                  bool grad_f32, bool accumulate, hipStream_t st) {
  const int G = colsum_groups(N);
  dim3 grid((C + 511) / 512, G);
  if (op == 0)
    hipLaunchKernelGGL(act_bwd_colsum_kernel<0>, grid, dim3(256), 0, st, (const uint16_t*)dy, (const uint16_t*)xin,
                       (uint16_t*)dx, N, C, part);
  else
    hipLaunchKernelGGL(act_bwd_colsum_kernel<1>, grid, dim3(256), 0, st, (const uint16_t*)dy, (const uint16_t*)xin,
                       (uint16_t*)dx, N, C, part);
  col_reduce(part, G, C, bias_grad, grad_f32, accumulate, st);
}

void swiglu_fwd(const void* gu, void* y, size_t rows, int F, hipStream_t st) {
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(ew_grid(rows * (F / 8))), dim3(256), 0, st, (const uint16_t*)gu,
                     (uint16_t*)y, rows, F);
}

void swiglu_bwd(const void* dy, const void* gu, void* dgu, size_t rows, int F, hipStream_t st) {
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(ew_grid(rows * (F / 8))), dim3(256), 0, st, (const uint16_t*)dy,
                     (const uint16_t*)gu, (uint16_t*)dgu, rows, F);
}

void rope(const void* in, void* out, const float* cosb, const float* sinb, size_t rows, int T, int n_heads_total,
          int n_rot, int D, int pos_offset, bool inverse, hipStream_t st, int out_heads) {
  if (out_heads <= 0) out_heads = n_heads_total;
  const size_t nwork = rows * out_heads * (D / 16);
  hipLaunchKernelGGL(rope_kernel, dim3(ew_grid(nwork)), dim3(256), 0, st, (const uint16_t*)in, (uint16_t*)out, cosb,
                     sinb, rows, T, n_heads_total, n_rot, D, pos_offset, inverse ? -1.f : 1.f, out_heads);
}

void scale_inplace(void* x, bool f32, const float* s, size_t n, hipStream_t st) {
  const size_t nv = n / 8;
  if (f32) hipLaunchKernelGGL(scale_kernel<true>, dim3(ew_grid(nv)), dim3(256), 0, st, x, s, nv);
  else hipLaunchKernelGGL(scale_kernel<false>, dim3(ew_grid(nv)), dim3(256), 0, st, x, s, nv);
}

void lse_merge(float* o_acc, float* lse_acc, const void* o, const float* lse, const int64_t* st, int B, int T, int H,
               int D, hipStream_t stream) {
  LseMergeArgs a{o_acc, lse_acc, (const uint16_t*)o, lse, st[0], st[1], st[2], st[3], st[4], st[5], st[6],
                 st[7], st[8], st[9], st[10], st[11], B, T, H, D};
  const int64_t n = (int64_t)B * T * H * (D / 8);
  hipLaunchKernelGGL(lse_merge_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, a);
}

}  // namespace pllm

// Fused multi-tensor AdamW over ONE flat parameter buffer, plus the global
// gradient-norm reduction used for clipping (gfx950).
//
// Reference: torch.optim.AdamW(model.parameters(), lr=t_lr) with defaults
// betas (0.9, 0.999), eps 1e-8, weight_decay 0.01 (scripts/train_transformer.py:126),
// i.e. per element
//     p *= 1 - lr*wd ;  m = b1*m + (1-b1)*g ;  v = b2*v + (1-b2)*g^2
//     p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)
// The reference runs this as ~5 foreach kernels over 3590 tensors plus
// autocast weight casts every forward; here it is ONE launch over a contiguous
// fp32 master buffer that also writes the bf16 compute weights the next forward
// reads (no separate cast pass).  Weight decay is selected per 64-element block
// by a byte mask (parameters are 64-aligned in the flat buffer), and the step's
// scalars can come from a device buffer so the launch can live in a hipGraph.
#include "common.h"
#include "kernels.h"

namespace {

// full grids for the streaming kernels (one vector per thread): a capped grid with
// grid-stride loops streams ~15 % slower on MI355X (see elementwise.hip)
inline int grid_for(size_t nvec) {
  size_t g = (nvec + 255) / 256;
  return (int)(g < (1u << 30) ? (g > 0 ? g : 1) : (1u << 30));
}

struct AdamHyper {
  float lr, b1, b2, eps, wd, inv_bc1, inv_sqrt_bc2, gs;
};

PLLM_DEV AdamHyper adam_hyper(float lr, float b1, float b2, float eps, float wd, float inv_bc1, float inv_sqrt_bc2,
                              float grad_scale, const float* scale_ptr, const float* hyper) {
  if (hyper) {  // [lr, 1/bc1, 1/sqrt(bc2)] written by the host before a graph replay
    lr = hyper[0];
    inv_bc1 = hyper[1];
    inv_sqrt_bc2 = hyper[2];
  }
  return AdamHyper{lr, b1, b2, eps, wd, inv_bc1, inv_sqrt_bc2, grad_scale * (scale_ptr ? *scale_ptr : 1.f)};
}

// AdamW on the 8 elements of vector i of the flat buffers; returns the new fp32 weights in pp
template <bool GRAD_F32>
PLLM_DEV void adamw8(size_t i, float* __restrict__ master, float* __restrict__ m, float* __restrict__ v,
                     const void* __restrict__ grad, const uint8_t* __restrict__ wd_blocks, const AdamHyper& h,
                     float (&pp)[8]) {
  // weight decay applies per 64-element block (params are 64-aligned in the flat buffer)
  const float decay = (wd_blocks == nullptr || wd_blocks[i >> 3]) ? 1.f - h.lr * h.wd : 1.f;
  const float step = h.lr * h.inv_bc1;
  float g[8];
  if (GRAD_F32) {
    const f32x4* gp = reinterpret_cast<const f32x4*>(grad) + 2 * i;
    f32x4 a = gp[0], b = gp[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      g[j] = a[j];
      g[4 + j] = b[j];
    }
  } else {
    unpack8(ld16(reinterpret_cast<const uint16_t*>(grad) + i * 8), g);
  }
  f32x4* pm = reinterpret_cast<f32x4*>(master) + 2 * i;
  f32x4* mm = reinterpret_cast<f32x4*>(m) + 2 * i;
  f32x4* vm = reinterpret_cast<f32x4*>(v) + 2 * i;
  f32x4 p0 = pm[0], p1 = pm[1], m0 = mm[0], m1 = mm[1], v0 = vm[0], v1 = vm[1];
  float mo[8], vo[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    pp[j] = p0[j];
    pp[4 + j] = p1[j];
    mo[j] = m0[j];
    mo[4 + j] = m1[j];
    vo[j] = v0[j];
    vo[4 + j] = v1[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float gg = g[j] * h.gs;
    mo[j] = h.b1 * mo[j] + (1.f - h.b1) * gg;
    vo[j] = h.b2 * vo[j] + (1.f - h.b2) * gg * gg;
    const float denom = sqrtf(vo[j]) * h.inv_sqrt_bc2 + h.eps;
    pp[j] = pp[j] * decay - step * mo[j] / denom;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    p0[j] = pp[j];
    p1[j] = pp[4 + j];
    m0[j] = mo[j];
    m1[j] = mo[4 + j];
    v0[j] = vo[j];
    v1[j] = vo[4 + j];
  }
  pm[0] = p0;
  pm[1] = p1;
  mm[0] = m0;
  mm[1] = m1;
  vm[0] = v0;
  vm[1] = v1;
}

template <bool GRAD_F32>
__global__ __launch_bounds__(256) void adamw_kernel(uint16_t* __restrict__ param, float* __restrict__ master,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    const void* __restrict__ grad, size_t nvec, float lr,
                                                    float b1, float b2, float eps, float wd, float inv_bc1,
                                                    float inv_sqrt_bc2, float grad_scale,
                                                    const float* __restrict__ scale_ptr,
                                                    const uint8_t* __restrict__ wd_blocks,
                                                    const float* __restrict__ hyper) {
  const AdamHyper h = adam_hyper(lr, b1, b2, eps, wd, inv_bc1, inv_sqrt_bc2, grad_scale, scale_ptr, hyper);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    float pp[8];
    adamw8<GRAD_F32>(i, master, m, v, grad, wd_blocks, h, pp);
    if (param) st16(param + i * 8, pack8(pp));
  }
}

// AdamW fused with the W^T shadow refresh (verdict r4 item 5: the separate transpose pass re-read every
// bf16 weight right after this kernel wrote it).  Blocks [0, tiles): one 64 x 64 tile of a shadowed
// matrix each (transpose_plan's table: src = the matrix inside the flat bf16 buffer, dst = its shadow):
// AdamW on the tile's 4096 elements (8 threads per 64-element row: 256-B runs of every fp32 buffer),
// the bf16 weights stored in place AND staged in LDS, then the tile's transpose stored to the shadow
// (16 B per lane, as transpose.hip).  Blocks [tiles, ...): the elements outside shadowed matrices,
// 256 vectors per block over the runs table (start vector, end vector, first block).
constexpr int ATT = 64, APITCH = ATT + 2;

template <bool GRAD_F32>
__global__ __launch_bounds__(256) void adamw_shadow_kernel(
    uint16_t* __restrict__ param, float* __restrict__ master, float* __restrict__ m, float* __restrict__ v,
    const void* __restrict__ grad, float lr, float b1, float b2, float eps, float wd, float inv_bc1,
    float inv_sqrt_bc2, float grad_scale, const float* __restrict__ scale_ptr, const uint8_t* __restrict__ wd_blocks,
    const float* __restrict__ hyper, const int64_t* __restrict__ desc, int ndesc, int tiles,
    const int64_t* __restrict__ runs, int nruns) {
  __shared__ uint16_t tile[ATT * APITCH];
  const AdamHyper h = adam_hyper(lr, b1, b2, eps, wd, inv_bc1, inv_sqrt_bc2, grad_scale, scale_ptr, hyper);
  const int t = blockIdx.x;
  if (t >= tiles) {
    const int fb = t - tiles;
    int lo = 0, hi = nruns - 1;  // last run whose first block <= fb (block-uniform: scalar loads)
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (runs[mid * 3 + 2] <= fb) lo = mid;
      else hi = mid - 1;
    }
    const int64_t* r = runs + lo * 3;
    const size_t i = (size_t)r[0] + (size_t)(fb - r[2]) * 256 + threadIdx.x;
    if (i < (size_t)r[1]) {
      float pp[8];
      adamw8<GRAD_F32>(i, master, m, v, grad, wd_blocks, h, pp);
      st16(param + i * 8, pack8(pp));
    }
    return;
  }
  int lo = 0, hi = ndesc - 1;  // the matrix owning tile t
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (desc[mid * 6 + 4] <= t) lo = mid;
    else hi = mid - 1;
  }
  const int64_t* d = desc + lo * 6;
  const size_t base = (size_t)((const uint16_t*)(uintptr_t)d[0] - param);  // element offset of the matrix
  uint16_t* dst = reinterpret_cast<uint16_t*>(d[1]);
  const int R = (int)d[2], C = (int)d[3];
  const int local = t - (int)d[4], tiles_c = (int)d[5];
  const int r0 = (local / tiles_c) * ATT, c0 = (local % tiles_c) * ATT;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int ch = threadIdx.x + 256 * k, rr = ch >> 3, cc = (ch & 7) * 8;
    const int r = r0 + rr, c = c0 + cc;
    if (r < R && c < C) {  // C % 8 == 0: a chunk is whole or absent
      const size_t i = (base + (size_t)r * C + c) >> 3;
      float pp[8];
      adamw8<GRAD_F32>(i, master, m, v, grad, wd_blocks, h, pp);
      const u32x4 pk = pack8(pp);
      st16(param + i * 8, pk);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        tile[rr * APITCH + cc + 2 * j] = (uint16_t)(pk[j] & 0xffffu);
        tile[rr * APITCH + cc + 2 * j + 1] = (uint16_t)(pk[j] >> 16);
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int ch = threadIdx.x + 256 * k, oc_r = ch >> 3, oc_c = (ch & 7) * 8;
    const int orow = c0 + oc_r, ocol = r0 + oc_c;  // dst is [C][R]; R % 8 == 0
    if (orow >= C || ocol >= R) continue;
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      o[j] = (uint32_t)tile[(oc_c + 2 * j) * APITCH + oc_r] | ((uint32_t)tile[(oc_c + 2 * j + 1) * APITCH + oc_r] << 16);
    st16(dst + (int64_t)orow * R + ocol, o);
  }
}

// per-block partial sums of squares of a flat bf16 (or fp32) gradient
template <bool F32>
__global__ __launch_bounds__(256) void sumsq_kernel(const void* __restrict__ x, size_t nvec, float* __restrict__ part) {
  __shared__ float scratch[4];
  float acc = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    float f[8];
    if (F32) {
      const f32x4* p = reinterpret_cast<const f32x4*>(x) + 2 * i;
      f32x4 a = p[0], b = p[1];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f[j] = a[j];
        f[4 + j] = b[j];
      }
    } else {
      unpack8(ld16(reinterpret_cast<const uint16_t*>(x) + i * 8), f);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += f[j] * f[j];
  }
  acc = block_sum<4>(acc, scratch);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

}  // namespace

namespace pllm {

void adamw_flat(void* param_bf16, float* master, float* m, float* v, const void* grad, bool grad_f32, size_t n,
                float lr, float b1, float b2, float eps, float wd, int step, float grad_scale,
                const float* scale_ptr, const uint8_t* wd_blocks, const float* hyper, hipStream_t st) {
  const size_t nv = n / 8;
  const float bc1 = 1.f - powf(b1, (float)(step > 0 ? step : 1));
  const float bc2 = 1.f - powf(b2, (float)(step > 0 ? step : 1));
  const float inv_bc1 = 1.f / bc1, inv_sqrt_bc2 = 1.f / sqrtf(bc2);
  if (grad_f32)
    hipLaunchKernelGGL(adamw_kernel<true>, dim3(grid_for(nv)), dim3(256), 0, st, (uint16_t*)param_bf16, master, m, v,
                       grad, nv, lr, b1, b2, eps, wd, inv_bc1, inv_sqrt_bc2, grad_scale, scale_ptr, wd_blocks, hyper);
  else
    hipLaunchKernelGGL(adamw_kernel<false>, dim3(grid_for(nv)), dim3(256), 0, st, (uint16_t*)param_bf16, master, m,
                       v, grad, nv, lr, b1, b2, eps, wd, inv_bc1, inv_sqrt_bc2, grad_scale, scale_ptr, wd_blocks, hyper);
}

void adamw_shadow(void* param_bf16, float* master, float* m, float* v, const void* grad, bool grad_f32, float lr,
                  float b1, float b2, float eps, float wd, int step, float grad_scale, const float* scale_ptr,
                  const uint8_t* wd_blocks, const float* hyper, const int64_t* desc, int ndesc, int tiles,
                  const int64_t* runs, int nruns, int flat_blocks, hipStream_t st) {
  const float bc1 = 1.f - powf(b1, (float)(step > 0 ? step : 1));
  const float bc2 = 1.f - powf(b2, (float)(step > 0 ? step : 1));
  const float inv_bc1 = 1.f / bc1, inv_sqrt_bc2 = 1.f / sqrtf(bc2);
  const int grid = tiles + flat_blocks;
  if (grid <= 0) return;
  if (grad_f32)
    hipLaunchKernelGGL(adamw_shadow_kernel<true>, dim3(grid), dim3(256), 0, st, (uint16_t*)param_bf16, master, m, v,
                       grad, lr, b1, b2, eps, wd, inv_bc1, inv_sqrt_bc2, grad_scale, scale_ptr, wd_blocks, hyper, desc,
                       ndesc, tiles, runs, nruns);
  else
    hipLaunchKernelGGL(adamw_shadow_kernel<false>, dim3(grid), dim3(256), 0, st, (uint16_t*)param_bf16, master, m, v,
                       grad, lr, b1, b2, eps, wd, inv_bc1, inv_sqrt_bc2, grad_scale, scale_ptr, wd_blocks, hyper, desc,
                       ndesc, tiles, runs, nruns);
}

int sumsq_blocks(size_t n) { return grid_for(n / 8) < 1024 ? grid_for(n / 8) : 1024; }

void sumsq(const void* x, bool f32, size_t n, float* part, hipStream_t st) {
  const size_t nv = n / 8;
  const int G = sumsq_blocks(n);
  if (f32)
    hipLaunchKernelGGL(sumsq_kernel<true>, dim3(G), dim3(256), 0, st, x, nv, part);
  else
    hipLaunchKernelGGL(sumsq_kernel<false>, dim3(G), dim3(256), 0, st, x, nv, part);
}

}  // namespace pllm

// Batched bf16 matrix transpose: refreshes the optimizer's W^T shadows of every 2-D
// weight in ONE launch after each step (train/optim.py FlatAdamW.refresh_shadows).
// A descriptor table (built once: the flat parameter buffer never moves) lists
// (src, dst, rows, cols, first tile) per matrix; a persistent grid of workgroups walks
// the 64x64 tiles, each transposed through LDS with 16-B global loads and stores.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int TT = 64;       // tile edge
constexpr int PITCH = TT + 2;  // LDS row pitch (elements): breaks the column-read bank pattern

__global__ __launch_bounds__(256) void transpose_batch_kernel(const int64_t* __restrict__ desc, int n, int total) {
  __shared__ uint16_t tile[TT * PITCH];
  // Persistent grid-stride loop over tiles.  Tile ids only grow, so the owning matrix is found
  // by continuing the table scan from the previous tile's matrix (amortised O(1) per tile; a
  // fresh linear scan per tile made the 195-matrix reference-3B refresh take 57 ms).
  int m = 0;
  for (int t = blockIdx.x; t < total; t += gridDim.x) {
    while (m + 1 < n && desc[(m + 1) * 6 + 4] <= t) ++m;
    const int64_t* d = desc + m * 6;
    const uint16_t* src = reinterpret_cast<const uint16_t*>(d[0]);
    uint16_t* dst = reinterpret_cast<uint16_t*>(d[1]);
    const int R = (int)d[2], C = (int)d[3];
    const int local = t - (int)d[4], tiles_c = (int)d[5];
    const int r0 = (local / tiles_c) * TT, c0 = (local % tiles_c) * TT;
    __syncthreads();  // the previous tile's LDS reads are done
    // load: 64 rows x 8 chunks of 8 elements
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int ch = threadIdx.x + 256 * k, rr = ch >> 3, cc = (ch & 7) * 8;
      const int r = r0 + rr, c = c0 + cc;
      if (r < R && c + 8 <= C) {
        const u32x4 v = ld16(src + (int64_t)r * C + c);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          tile[rr * PITCH + cc + 2 * j] = (uint16_t)(v[j] & 0xffffu);
          tile[rr * PITCH + cc + 2 * j + 1] = (uint16_t)(v[j] >> 16);
        }
      } else if (r < R) {
        for (int j = 0; j < 8; ++j)
          if (c + j < C) tile[rr * PITCH + cc + j] = src[(int64_t)r * C + c + j];
      }
    }
    __syncthreads();
    // store: output rows are input columns; 8 consecutive output elements per thread
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int ch = threadIdx.x + 256 * k, oc_r = ch >> 3, oc_c = (ch & 7) * 8;
      const int orow = c0 + oc_r, ocol = r0 + oc_c;  // dst is [C][R]
      if (orow >= C) continue;
      uint16_t e[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) e[j] = tile[(oc_c + j) * PITCH + oc_r];
      if (ocol + 8 <= R) {
        u32x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = (uint32_t)e[2 * j] | ((uint32_t)e[2 * j + 1] << 16);
        st16(dst + (int64_t)orow * R + ocol, v);
      } else {
        for (int j = 0; j < 8; ++j)
          if (ocol + j < R) dst[(int64_t)orow * R + ocol + j] = e[j];
      }
    }
  }
}

}  // namespace

namespace pllm {

int transpose_tiles(int R, int C) { return ((R + TT - 1) / TT) * ((C + TT - 1) / TT); }

void transpose_batch(const int64_t* desc, int n, int total_tiles, hipStream_t st) {
  const int grid = total_tiles < 256 * 8 ? total_tiles : 256 * 8;  // 8 workgroups per CU
  if (total_tiles > 0)
    hipLaunchKernelGGL(transpose_batch_kernel, dim3(grid), dim3(256), 0, st, desc, n, total_tiles);
}

}  // namespace pllm

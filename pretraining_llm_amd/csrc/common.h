// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels.
//
// Conventions used by every kernel in this directory:
//  * wave64: lane = threadIdx.x & 63, reductions use 64-wide shuffles;
//  * bf16 tensors are moved 16 bytes per lane (8 x bf16) whenever the row
//    length allows it (cdna_hip_programming.md Guideline 13);
//  * f32 -> bf16 conversion is a plain __bf16 cast (hipcc emits
//    v_cvt_pk_bf16_f32, round-to-nearest-even, NaN-preserving);
//  * no torch headers here: the .hip files compile in seconds and the torch
//    glue lives in bindings.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PL_DEV __device__ __forceinline__

typedef __bf16 bf16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x8 __attribute__((ext_vector_type(8)));   // 8 x bf16 MFMA fragment
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

PL_DEV float bf2f(uint16_t u) { return __uint_as_float(((uint32_t)u) << 16); }
PL_DEV float bf2f(bf16 b) { return (float)b; }
PL_DEV uint16_t f2bf_bits(float f) {
  bf16 b = (bf16)f;
  return *reinterpret_cast<uint16_t*>(&b);
}
// two floats -> packed bf16x2 in one dword (lo in bits 0..15)
PL_DEV uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)f2bf_bits(lo) | ((uint32_t)f2bf_bits(hi) << 16);
}
// Bare v_exp_f32 (2^x).  exp2f() lowers to a denormal-safe sequence (range test,
// bias, v_exp, rescale: ~6 VALU) because f32 denormals are on by default; every
// caller here feeds softmax-style sums where a flushed 2^-126 tail is harmless,
// so the hot loops keep one transcendental per element.
PL_DEV float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
PL_DEV float lo_bf(uint32_t w) { return __uint_as_float(w << 16); }
PL_DEV float hi_bf(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// 8 bf16 <-> 8 floats through one 16-byte vector
PL_DEV void unpack8(const u32x4& v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = lo_bf(v[i]);
    f[2 * i + 1] = hi_bf(v[i]);
  }
}
PL_DEV u32x4 pack8(const float* f) {
  u32x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = pack_bf16x2(f[2 * i], f[2 * i + 1]);
  return v;
}
PL_DEV u32x4 ld16(const void* p) { return *reinterpret_cast<const u32x4*>(p); }
PL_DEV void st16(void* p, const u32x4& v) { *reinterpret_cast<u32x4*>(p) = v; }
PL_DEV u32x4 ld16_nt(const void* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}
PL_DEV void st16_nt(void* p, const u32x4& v) {
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
}

// ---- gradient buffers: bf16 or fp32 (FlatAdamW grad_dtype) ----------------
// 8 consecutive gradient values <-> 8 floats: 16 B (bf16) or 32 B (fp32) per lane
template <bool F32>
PL_DEV void ld8g(const void* p, float* f) {
  if constexpr (F32) {
    const f32x4* q = reinterpret_cast<const f32x4*>(p);
    const f32x4 a = q[0], b = q[1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[i] = a[i];
      f[4 + i] = b[i];
    }
  } else {
    unpack8(ld16(p), f);
  }
}
template <bool F32>
PL_DEV void st8g(void* p, const float* f) {
  if constexpr (F32) {
    f32x4* q = reinterpret_cast<f32x4*>(p);
    q[0] = f32x4{f[0], f[1], f[2], f[3]};
    q[1] = f32x4{f[4], f[5], f[6], f[7]};
  } else {
    st16(p, pack8(f));
  }
}
// one gradient element
template <bool F32>
PL_DEV float ldg1(const void* p, int64_t i) {
  if constexpr (F32) return reinterpret_cast<const float*>(p)[i];
  else return bf2f(reinterpret_cast<const uint16_t*>(p)[i]);
}
template <bool F32>
PL_DEV void stg1(void* p, int64_t i, float v) {
  if constexpr (F32) reinterpret_cast<float*>(p)[i] = v;
  else reinterpret_cast<uint16_t*>(p)[i] = f2bf_bits(v);
}

// ---- wave64 / block reductions -------------------------------------------
PL_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// tanh-form GELU shared by the activation, fused-epilogue GEMM and decode kernels
constexpr float kGeluK = 0.7978845608028654f;  // sqrt(2/pi)
constexpr float kGeluC = 0.044715f;
PL_DEV float tanh_fast(float u) {
  // tanh(u) = 1 - 2 / (exp(2u) + 1); saturates correctly for |u| large.  v_rcp_f32 instead
  // of an IEEE division: the division's scale/fixup sequence made GELU VALU-bound
  // (~25 VALU ops per element at 8 elements per 16-B access) instead of HBM-bound.
  return 1.f - 2.f * __builtin_amdgcn_rcpf(__expf(2.f * u) + 1.f);
}
PL_DEV float gelu_f(float x) {
  const float t = tanh_fast(kGeluK * (x + kGeluC * x * x * x));
  return 0.5f * x * (1.f + t);
}
PL_DEV float gelu_df(float x) {
  // d/dx of the tanh GELU in sigmoid form: 0.5 (1 + tanh u) = s = sigmoid(2u), u = k (x + c x^3),
  // so the derivative is s + x s (1 - s) 2k (1 + 3c x^2): one exp2 (argument folded into an FMA),
  // one rcp and ~9 more VALU ops instead of the tanh form's ~15 (GELU backward + column sums
  // 251 -> 248 us at 65536 x 3072, profiles/r2_gelu_df_sigmoid_ab.txt).  x -> -inf: s -> 0,
  // result 0; x -> +inf: s -> 1, result 1.
  constexpr float kLog2e = 1.4426950408889634f;
  const float x2 = x * x;
  const float e = fast_exp2(x * __builtin_fmaf(-2.f * kGeluK * kGeluC * kLog2e, x2, -2.f * kGeluK * kLog2e));
  const float s = __builtin_amdgcn_rcpf(1.f + e);
  const float q = x * __builtin_fmaf(6.f * kGeluK * kGeluC, x2, 2.f * kGeluK);
  return __builtin_fmaf(q * s, 1.f - s, s);
}
PL_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum over NW waves through a small LDS scratch (NW <= 16).
template <int NW>
PL_DEV float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) scratch[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) r += scratch[i];
  __syncthreads();
  return r;
}
template <int NW>
PL_DEV float block_max(float v, float* scratch) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) scratch[w] = v;
  __syncthreads();
  float r = -INFINITY;
#pragma unroll
  for (int i = 0; i < NW; ++i) r = fmaxf(r, scratch[i]);
  __syncthreads();
  return r;
}

// Bijective XCD-aware remap of a 1-D block id (cdna_hip_programming.md §5, T1):
// blocks that the dispatcher deals to the same XCD (id % 8) get a contiguous
// range of logical ids, so neighbouring tiles share that XCD's L2.
PL_DEV int xcd_remap(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// Retire every outstanding vector-memory load (s_waitcnt vmcnt(0); gfx9 encoding: expcnt 7,
// lgkmcnt 15).  A real S_WAITCNT the compiler's waitcnt pass understands -- unlike inline asm --
// so registers loaded before a loop (Q fragments, K/V rows) count as ready inside it.  Without
// it the pass merges the loop's pending prefetch with those loads and emits vmcnt(0) in front
// of the first MFMA of EVERY iteration, which serialises the prefetch it was meant to overlap.
PL_DEV void vm_wait_all() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// Buffer loads over the rows [0, rows) of one (batch, head) slice of a row-strided bf16 matrix
// (cdna_hip_programming.md T8/T20): a wave-uniform descriptor plus a 32-bit per-lane byte offset
// replaces per-load 64-bit address arithmetic, and the hardware range check returns zeros for
// rows >= rows (no per-load branch).  Requires (rows - 1) * stride + width < 2^31 elements.
PL_DEV __amdgpu_buffer_rsrc_t rows_rsrc(const uint16_t* base, int rows, int64_t stride, int width) {
  const int bytes = rows > 0 ? (int)(((int64_t)(rows - 1) * stride + width) * 2) : 0;
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, bytes, 0x00020000);
}
PL_DEV u32x4 buf_ld16(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0u, 0));
}

// global -> LDS DMA of 16 B per lane into [m0 + 16 * lane] (m0 = wave-uniform LDS byte address)
// through a buffer descriptor: a wave-uniform base (4 SGPRs, range-checked: out-of-range lanes
// read zeros) plus a 32-bit per-lane byte offset.  Measured 7-11 % faster in the wgrad GEMM than
// global_load_lds with 64-bit per-lane addresses (profiles/r3_wgrad_stamps.md).  Inline asm so
// hipcc's waitcnt pass does not drain the prefetch before unrelated LDS reads: the caller retires
// these loads with vm_wait_all() ahead of the barrier that publishes the data.
typedef int i32x4v __attribute__((ext_vector_type(4)));
PL_DEV i32x4v srd_of(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  i32x4v r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)((uint32_t)(a >> 32) & 0xffffu));
  r[2] = __builtin_amdgcn_readfirstlane((int)bytes);
  r[3] = 0x00020000;
  return r;
}
PL_DEV void blds16(const i32x4v& srd, uint32_t voff, unsigned lds_byte) {
  asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(srd),
               "s"(__builtin_amdgcn_readfirstlane(lds_byte))
               : "memory", "m0");
}
// ... 4 B per lane into [m0 + 4 * lane] (buffer_load_dword ... lds), e.g. a row of 64 fp32 statistics
PL_DEV void blds4(const i32x4v& srd, uint32_t voff, unsigned lds_byte) {
  asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dword %0, %1, 0 offen lds" ::"v"(voff), "s"(srd),
               "s"(__builtin_amdgcn_readfirstlane(lds_byte))
               : "memory", "m0");
}
#define PL_CHECK_LAUNCH() (void)hipGetLastError()

// Debug builds (python -m pretraining_llm_amd.build --debug): report a violated device-side
// contract with printf and carry on (the kernels stay defensive; no trap, which would fault).
#ifdef PLLM_DEBUG
#define PL_DCHECK(cond, what, val)                                                              \
  do {                                                                                            \
    if (!(cond)) printf("[pllm debug] %s: %s violated (value %lld)\n", __func__, what, (long long)(val)); \
  } while (0)
#else
#define PL_DCHECK(cond, what, val) \
  do {                               \
  } while (0)
#endif

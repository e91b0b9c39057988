// Shared device helpers of the attention kernels (attention.hip, attn_bwd_ks.hip): MFMA / transposed-read
// wrappers, accumulator layout, RoPE rotation, the row-per-lane epilogue store and the swizzled LDS
// images.  Header-only, internal linkage (each translation unit gets its own copy).
#pragma once
#include "common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

PL_DEV f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
PL_DEV s16x4 ds_tr(const uint16_t* p) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p); }
PL_DEV bf16x8 cat_tr(const s16x4& lo, const s16x4& hi) {
  s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}
PL_DEV bf16x8 as_frag(const u32x4& v) { return __builtin_bit_cast(bf16x8, v); }
PL_DEV bf16x8 zero_frag() { return __builtin_bit_cast(bf16x8, u32x4{0u, 0u, 0u, 0u}); }
PL_DEV f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}
// element i of a 32x32 accumulator lives at row (i&3) + 8*(i>>2) + 4*half, column lane&31
PL_DEV int acc_row(int i, int half) { return (i & 3) + 8 * (i >> 2) + 4 * half; }
PL_DEV bf16x8 pack_frag(const f32x16& x, int s) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (bf16)x[8 * s + j];
  return f;
}

// ---------------------------------------------------------------------------
// Fused RoPE (rotate-half convention, ops/reference.py rope): element i < D/2 of a head row
// pairs with i + D/2; a' = a cos - b sin, b' = b cos + a sin at the row's position.  The kernels
// rotate q and k while staging them (registers / LDS images) and un-rotate dq and dk before
// the final stores, so the packed QKV tensor and its gradient stay unrotated and no separate
// RoPE pass over [B, T, H, D] exists in forward or backward.
// Rotates 8 + 8 bf16 values (a = elements i0..i0+7, b = i0+D/2..) held as two 16-B chunks.
PL_DEV void rope8(u32x4& lo, u32x4& hi, const float* cosr, const float* sinr, float dir) {
  float a[8], b[8], c[8], sn[8];
  unpack8(lo, a);
  unpack8(hi, b);
  const f32x4* cp = reinterpret_cast<const f32x4*>(cosr);
  const f32x4* sp = reinterpret_cast<const f32x4*>(sinr);
  const f32x4 c0 = cp[0], c1 = cp[1], s0 = sp[0], s1 = sp[1];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    c[e] = c0[e];
    c[4 + e] = c1[e];
    sn[e] = s0[e] * dir;
    sn[4 + e] = s1[e] * dir;
  }
  float o1[8], o2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    o1[e] = a[e] * c[e] - b[e] * sn[e];
    o2[e] = b[e] * c[e] + a[e] * sn[e];
  }
  lo = pack8(o1);
  hi = pack8(o2);
}

// Row-per-lane epilogue of 32x32 accumulator tiles (guide T21): acc[db] holds, for the lane's
// row, columns db*32 + 8g + 4hh + e (e < 4), the two half-waves sharing each row.  Packs to
// bf16 (times sc), swaps group pairs (k, k+1) across the half-waves with v_permlane32_swap and
// stores one contiguous 16-B chunk per pair: 2*NDB dwordx4 stores instead of 4*NDB dwordx2 (the
// store tail is issue-bound, per instruction).  row: 16-B aligned.
template <int NDB>
PL_DEV void store_row_bf16(uint16_t* row, const f32x16 (&acc)[NDB], float sc, int hh) {
  u32x2 pk[4 * NDB];
#pragma unroll
  for (int db = 0; db < NDB; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      pk[4 * db + g][0] = pack_bf16x2(acc[db][4 * g] * sc, acc[db][4 * g + 1] * sc);
      pk[4 * db + g][1] = pack_bf16x2(acc[db][4 * g + 2] * sc, acc[db][4 * g + 3] * sc);
    }
#pragma unroll
  for (int k = 0; k < 4 * NDB; k += 2) {
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      const auto sw = __builtin_amdgcn_permlane32_swap(pk[k][d], pk[k + 1][d], false, false);
      pk[k][d] = sw[0];
      pk[k + 1][d] = sw[1];
    }
    *reinterpret_cast<u32x4*>(row + 8 * k + 8 * hh) = u32x4{pk[k][0], pk[k][1], pk[k + 1][0], pk[k + 1][1]};
  }
}

// ---------------------------------------------------------------------------
// Swizzled LDS image of a [rows][W] bf16 tile (W = 32, 64 or 128 elements).
// Chunk ch (16 B) of row r lives at chunk position ch ^ f(r):
//   W=128 (256 B rows): f = ((r&3)<<2) | ((r>>2)&3)       (guide T10 layout (b))
//   W=64  (128 B rows): f = bitrev3((r>>1)&7)
//   W=32  ( 64 B rows): f = (r>>2)&3
// For the 16-lane groups of ds_read_b128 (16 distinct rows, same chunk) and the
// 32-lane halves of ds_read_b64_tr_b16 (4 consecutive rows x 64 contiguous bytes)
// every f above maps the accesses to distinct 16-B bank slots.
// ---------------------------------------------------------------------------
template <int W>
struct Img {
  static PL_DEV int f(int r) {
    if constexpr (W == 128) return ((r & 3) << 2) | ((r >> 2) & 3);
    else if constexpr (W == 64) {
      const int b = (r >> 1) & 7;
      return ((b & 1) << 2) | (b & 2) | ((b >> 2) & 1);
    } else return (r >> 2) & 3;
  }
  // element offset of (row, col); col's 8-aligned chunk is swizzled, col&7 kept
  static PL_DEV int off(int r, int col) { return r * W + (((col >> 3) ^ f(r)) << 3) + (col & 7); }
  // a row's two RoPE-partner halves (chunks c and c + W/16) stored so that every 8-lane group
  // of ds_write_b128 (bank = byte address mod 128) covers 128 distinct bytes: at W = 64 rows 2k
  // and 2k+1 share f, so an odd row stores its upper half first (same image, same reads)
  static PL_DEV void st_pair(uint16_t* base, int r, int c, const u32x4& lo, const u32x4& hi) {
    constexpr int H = W / 16;
    const bool sw = W == 64 && (r & 1);
    st16(base + off(r, (sw ? c + H : c) * 8), sw ? hi : lo);
    st16(base + off(r, (sw ? c : c + H) * 8), sw ? lo : hi);
  }
};

// The fused-role backward's dS^T image [keys][128 queries] (256-B rows): chunk ch of row r at
// ch ^ fs(r), fs linear in r's bits 0..2 (4, 9, 2).  Conflict-free both for the dQ task's
// ds_read_b64_tr_b16 (4 consecutive rows x 4 aligned chunks -> 16 distinct positions) and for the
// 16-B dS stores, whose 8-lane ds_write_b128 groups are 8 consecutive rows at one chunk (bank =
// address mod 128 B: fs mod 8 is a permutation over any 8 aligned rows).  Img<128>'s swizzle gave
// the former 8-B dS stores a 2-way conflict on every store (16 rows per ds_write_b64 group onto
// 8 slots mod 128 B): ~64 conflict cycles per wave and iteration (profiles/r3_pmc_attn_*_bwd.md).
struct ImgS {
  static PL_DEV int f(int r) { return ((r & 1) ? 4 : 0) ^ ((r & 2) ? 9 : 0) ^ ((r & 4) ? 2 : 0); }
  static PL_DEV int off(int r, int col) { return r * 128 + (((col >> 3) ^ f(r)) << 3) + (col & 7); }
};

constexpr float kLog2e = 1.4426950408889634f;

// ---------------------------------------------------------------------------
// Inline-asm MFMAs with an explicit register class (attn_bwd_ks.hip): hipcc left to
// itself put the long-lived accumulators in whichever file it liked and copied them at branch joins.
// Hazards the compiler does not pad for asm (cdna_hip_programming.md §5.7) are the caller's: NOP
// variants open with s_nop 1 (a VALU-written operand), mfma_settle() precedes a non-MFMA reader.
// v_mfma_f32_32x32x16_bf16 with the accumulator in arch VGPRs: acc (+)= A B.  NOP: the statement opens
// with s_nop 1 (2 wait states) -- needed when A / B / C was just written by a VALU instruction (a chain's
// first MFMA after its VALU-initialised accumulator); A / B from LDS reads and C from the chain's
// previous MFMA need none (s_nop 1 on all 80 MFMAs of a slice cost ~160 issue cycles per wave)
template <bool NOP = false>
PL_DEV void mfma_v(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  if constexpr (NOP) asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
  else asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}
template <bool NOP = false>
PL_DEV void mfma_v0(f32x16& acc, const bf16x8& a, const bf16x8& b) {  // acc = A B
  if constexpr (NOP) asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "v"(b));
  else asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "v"(b));
}
// ... with the accumulator pinned to the accumulator file.  B (the packed P / dS fragments) was written
// by VALU at least one pipelined step (>= 2 MFMAs) earlier; the accumulators' zero init is far back
template <bool NOP = false>
PL_DEV void mfma_a(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  if constexpr (NOP) asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  else asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
// an MFMA result read by anything but the next MFMA of its chain: 16-pass XDL -> 18 wait states
PL_DEV void mfma_settle(f32x16& x) { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+v"(x)); }
PL_DEV void mfma_settle(f32x16& x, f32x16& y) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+v"(x), "+v"(y));
}


}  // namespace

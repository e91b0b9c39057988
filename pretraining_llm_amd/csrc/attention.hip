// Causal flash attention, forward and backward, on gfx950 MFMA (v_mfma_f32_32x32x16_bf16).
//
// Replaces the reference's per-head Python loop of materialised T x T score
// matrices (src/models/attention.py:47-57: q@k^T * hd^-1/2, masked_fill(tril==0,
// -inf), softmax, @v; concat at :95) with an O(T)-memory online-softmax kernel.
// Q/K/V are read in place out of the packed QKV GEMM output through strides and
// the gradients are written straight into the packed dQKV buffer.
//
// Layout choices (CDNA4, wave64):
//  * LDS tiles are [rows][D] bf16 with NO padding and an XOR swizzle of the
//    16-byte chunks (Img<D>): conflict-free both for ds_read_b128 row reads
//    (MFMA operands that sum over D) and for ds_read_b64_tr_b16 transposed reads
//    (operands that sum over rows), so one image serves both (guide §5.5 T2/T10).
//  * forward: one workgroup = 4 waves, each owning 2 (D <= 64) or 1 (D = 128)
//    blocks of 32 query rows, K/V tiles of 64 keys double-buffered in LDS through
//    registers (issue-early / write-late, T14).
//    S^T = K.Q^T is computed with the QUERY on the MFMA lane, so the softmax row
//    statistics (m, l) are per-lane scalars and the P^T accumulator is directly
//    the B operand of O^T += V^T.P^T (no LDS round trip for P).
//  * backward: one workgroup = NW waves = 32*NW keys of one (batch, kv-head)
//    (D<=64: 8 waves/256 keys, D=128: 4 waves/128 keys); each
//    wave keeps dK^T/dV^T for its 32 keys in registers across all query blocks
//    (and all query heads of a GQA group), so dK/dV need no cross-workgroup sum.
//    S and dP are computed with the KEY on the lane and initialised with
//    -LSE/scale and -delta, so P = exp2(c*S') and dS = P*dP' need no extra pass.
//    Under the causal mask a wave whose 32 keys all follow a 32-query sub-block
//    skips it outright (zeros into the dS^T image), and dQ k-steps past the
//    diagonal are skipped.  dQ per key block is summed over its keys on chip and written to a
//    per-key-block fp32 slab; a second kernel sums the slabs in a fixed order
//    (deterministic; the first version's fp32 atomics were its floor).  The key blocks run
//    in passes so the slab workspace is bounded independently of T (O(T) memory).
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "attn_common.h"
#include "common.h"
#include "kernels.h"

namespace {

// ============================================================================
// forward
// ============================================================================
// One workgroup = 4 waves.  A wave owns QB blocks of 32 query rows (QB = 2 for
// D <= 64, 1 for D = 128: register budget), so every K fragment read from LDS and
// every V transposed read feeds QB MFMAs instead of one, and the softmax of one
// block overlaps the other block's MFMAs.  With QB = 2 wave w takes blocks w and
// 7 - w of the workgroup's eight, which gives every wave the same share of the
// causal diagonal.  A block whose keys in a tile are all masked (or whose rows lie
// past T, e.g. decode) skips its MFMAs and softmax on a wave-uniform branch.
// lazy-max threshold of the forward's online softmax, log2 units (p <= 2^8)
constexpr float kLazyThr = 8.f;
#ifndef PLLM_FWD_STAMPS
#define PLLM_FWD_STAMPS 0  // diagnostic: per-phase s_memtime sums of the forward loop
#endif
#ifndef PL_BWD_DQ_KREG
#define PL_BWD_DQ_KREG 8  // D <= 64 backward: dQ-task K^T fragments held in registers (key steps 0..7 of 16)
#endif
#ifndef PLLM_BWD_STAMPS
#define PLLM_BWD_STAMPS 0  // diagnostic: per-phase s_memtime sums of the D <= 64 backward loop
#endif
// Measured and removed in round 5 (records kept in profiles/): a software-pipelined forward tile loop
// (no faster, r3_attn_fwd_experiments.md), an exponent-ready "V3" forward, the 8-wave D = 128 forward
// (neutral, r4_attn_experiments.md), register-staged K/V tiles instead of LDS DMA in the forward, and in
// the backward the spread / asymmetric Q-dO DMA issue and the wave-4-7 stagger (r4_attn_experiments.md).

template <int D>
struct FwdCfg {
  static constexpr int NW = 4;
  static constexpr int MINB = 2;  // launch bounds: 2 waves per SIMD
  static constexpr int QB = D <= 64 ? 2 : 1;
  static constexpr int BM = NW * 32 * QB, BN = 64;
  static constexpr int CPR = D / 8;   // 16 B chunks per row
  static constexpr int TILE = BN * D;  // elements per K (or V) tile
  static constexpr int LDS_ELEMS = 4 * TILE;
};

template <int D, bool ROPE>
__global__ __launch_bounds__(64 * FwdCfg<D>::NW, FwdCfg<D>::MINB) void attn_fwd_kernel(AttnFwdArgs a) {
  using C = FwdCfg<D>;
  using I = Img<D>;
  constexpr int BM = C::BM, BN = C::BN, CPR = C::CPR, TILE = C::TILE, QB = C::QB, NW = C::NW;
  constexpr int NKS = D / 16, NDB = D / 32;
  __shared__ __attribute__((aligned(16))) uint16_t smem[C::LDS_ELEMS];

  const int nqb = (a.T + BM - 1) / BM;
  // heaviest (last) query blocks of every head first.  A head-local order (a head's blocks
  // adjacent inside one XCD's range, for L2 reuse of its K/V) measured 0-38 % slower
  // (profiles/r2_attn_order_ab.txt)
  const int BH = a.B * a.H;
  const int id = blockIdx.x;
  const int qb = nqb - 1 - id / BH;
  const int bh = id % BH;
  const int b = bh / a.H, h = bh % a.H, hk = h / (a.H / a.Hkv);
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int q0 = qb * BM;
  const int off = a.S - a.T;
  const uint16_t* qp = a.q + b * a.q_sb + (int64_t)h * a.q_sh;
  const uint16_t* kp = a.k + b * a.k_sb + (int64_t)hk * a.k_sh;
  const uint16_t* vp = a.v + b * a.v_sb + (int64_t)hk * a.v_sh;

  // first query row of each of this wave's blocks, and the end of its (causal) key range
  int qw[QB], qend[QB];
#pragma unroll
  for (int j = 0; j < QB; ++j) {
    qw[j] = q0 + 32 * (j == 0 ? w : 2 * NW - 1 - w);
    qend[j] = qw[j] >= a.T ? 0 : (a.causal ? min(a.S, qw[j] + 32 + off) : a.S);
  }
  bf16x8 qf[QB][NKS];
#pragma unroll
  for (int j = 0; j < QB; ++j) {
    const int qi = qw[j] + r;
    u32x4 raw[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
      raw[ks] = qi < a.T ? ld16(qp + (int64_t)qi * a.q_st + 16 * ks + 8 * hh) : u32x4{0u, 0u, 0u, 0u};
    if (ROPE && qi < a.T) {
      // the lane's chunks ks and ks + NKS/2 hold head-dim elements i and i + D/2
      const int64_t tab = (int64_t)(qi + off) * (D / 2);
#pragma unroll
      for (int ks = 0; ks < NKS / 2; ++ks)
        rope8(raw[ks], raw[ks + NKS / 2], a.rope_cos + tab + 16 * ks + 8 * hh, a.rope_sin + tab + 16 * ks + 8 * hh,
              1.f);
    }
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) qf[j][ks] = as_frag(raw[ks]);
  }
  vm_wait_all();  // Q fragments ready before the tile loop (see common.h)

  int kv_end = a.S;
  if (a.causal) kv_end = min(a.S, q0 + BM + off);
  const int ntiles = (kv_end + BN - 1) / BN;

  // chunk i of this thread: row c / CPR, column chunk (c % CPR2) + (i odd ? CPR2 : 0) with
  // c = tid + NTH * (i / 2) and CPR2 = CPR / 2, so a thread holds both RoPE partners of a row
  constexpr int CPR2 = CPR / 2, NTH = 64 * NW;
  constexpr int NPAIR = (BN * CPR2 + NTH - 1) / NTH;
  u32x4 kr[2 * NPAIR], vr[2 * NPAIR];
  // K / V rows by buffer loads through a per-tile descriptor (scalar base = the tile's first
  // row): rows past S read as zeros (range check), per-lane offsets loop-invariant
  auto gload = [&](int t) {
    const int kv0 = t * BN;
    const auto krs = rows_rsrc(kp + (int64_t)kv0 * a.k_st, a.S - kv0, a.k_st, D);
    const auto vrs = rows_rsrc(vp + (int64_t)kv0 * a.v_st, a.S - kv0, a.v_st, D);
#pragma unroll
    for (int i = 0; i < 2 * NPAIR; ++i) {
      const int c = tid + NTH * (i / 2), row = c / CPR2, col = c % CPR2 + (i & 1) * CPR2;
      if (c < BN * CPR2) {
        kr[i] = buf_ld16(krs, (uint32_t)(row * (int)a.k_st + col * 8) * 2u);
        vr[i] = buf_ld16(vrs, (uint32_t)(row * (int)a.v_st + col * 8) * 2u);
      } else {
        kr[i] = u32x4{0u, 0u, 0u, 0u};
        vr[i] = u32x4{0u, 0u, 0u, 0u};
      }
    }
  };
  auto swrite = [&](int buf, int t, int vbuf) {
    uint16_t* Kb = smem + buf * TILE;
    uint16_t* Vb = smem + 2 * TILE + vbuf * TILE;
#pragma unroll
    for (int i = 0; i < 2 * NPAIR; i += 2) {
      const int c = tid + NTH * (i / 2), row = c / CPR2, col = c % CPR2;
      if (c >= BN * CPR2) continue;
      if (ROPE) {
        const int key = t * BN + row;
        const int64_t tab = (int64_t)min(key, a.S - 1) * (D / 2) + col * 8;
        rope8(kr[i], kr[i + 1], a.rope_cos + tab, a.rope_sin + tab, 1.f);
      }
      I::st_pair(Kb, row, col, kr[i], kr[i + 1]);
      I::st_pair(Vb, row, col, vr[i], vr[i + 1]);
    }
  };

  // LDS DMA of the plain loop (no fused RoPE): each wave moves PPW 1-KiB pieces of the K then V
  // tile straight into the swizzled image -- lane l of a piece fills LDS chunk 64 p + l, so it
  // loads the logical chunk that the image stores there (row g / CPR, chunk (g % CPR) ^ f(row)).
  // No staging registers, no ds_write restage; rows past S read as zeros (descriptor range).
  constexpr bool DMA = !ROPE;
  constexpr int PCS = BN * CPR / 64;  // pieces per tile
  constexpr int PPW = 2 * PCS / NW;   // K + V pieces per wave
  static_assert(2 * PCS % NW == 0 && PCS % PPW == 0, "a wave's pieces lie in one operand");
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const bool dv = (wu * PPW) / PCS != 0;  // this wave moves V pieces (else K)
  uint32_t doff[PPW];
#pragma unroll
  for (int k = 0; k < PPW; ++k) {
    const int g = ((wu * PPW + k) % PCS) * 64 + lane, row = g / CPR, cc = (g % CPR) ^ I::f(row);
    doff[k] = (uint32_t)(row * (int)(dv ? a.v_st : a.k_st) + cc * 8) * 2u;
  }
  const unsigned lds0 = (unsigned)(uintptr_t)smem;
  auto gdma = [&](int t, int buf) {
    const int kv0 = t * BN, rows = min(a.S - kv0, BN);
    const int64_t st = dv ? a.v_st : a.k_st;
    const uint16_t* base = (dv ? vp : kp) + (int64_t)kv0 * st;
    const i32x4v srd = srd_of(base, (uint32_t)(((int64_t)(rows - 1) * st + D) * 2));
    const unsigned dst = lds0 + 2u * (unsigned)((dv ? 2 * TILE : 0) + buf * TILE);
#pragma unroll
    for (int k = 0; k < PPW; ++k) blds16(srd, doff[k], dst + 1024u * (unsigned)((wu * PPW + k) % PCS));
  };

  // per-lane LDS element offsets with the swizzle applied once (see attn_bwd_kernel): K
  // fragment reads fk ^ (ks << 4) + 32 kb D, V transposed reads fv0 / fv8 ^ (db << 5) + 16 kst D
  const int g1 = (lane >> 4) & 1, tq = (lane & 15) >> 2, tp = lane & 3;
  const int fk = I::off(r, 8 * hh);
  const int fv0 = I::off(4 * hh + tq, 16 * g1 + 4 * tp), fv8 = I::off(4 * hh + tq + 8, 16 * g1 + 4 * tp);
  f32x16 o[QB][NDB];
  // m: the running max in log2 units (raw score x c2), the reference point of the exponent.  It is
  // moved LAZILY (guide T13): only when some row's tile max exceeds it by more than kLazyThr, so
  // p = exp2(s c2 - m) <= 2^kLazyThr and the O / l rescale runs on a few tiles instead of nearly
  // every one (with an eager max, any of a wave's 32 rows gaining a new maximum -- most tiles --
  // forced the whole O block through a rescale).  p up to 2^8 loses nothing in bf16 (same relative
  // precision) and O / l accumulate in fp32.
  float m[QB], l[QB];
#pragma unroll
  for (int j = 0; j < QB; ++j) {
#pragma unroll
    for (int db = 0; db < NDB; ++db) o[j][db] = zero16();
    m[j] = -INFINITY;
    l[j] = 0.f;
  }
  const float c2 = a.scale_log2;

#if PLLM_FWD_STAMPS
  uint64_t st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t st_start = __builtin_amdgcn_s_memtime();
#endif
  if (ntiles > 0) {
    if constexpr (DMA) {
      gdma(0, 0);
      vm_wait_all();
    } else {
      gload(0);
      swrite(0, 0, 0);
    }
  }
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
#if PLLM_FWD_STAMPS
    uint64_t ts_prev = __builtin_amdgcn_s_memtime();
    auto stamp = [&](int i) {
      const uint64_t now = __builtin_amdgcn_s_memtime();
      st_acc[i] += now - ts_prev;
      ts_prev = now;
    };
#define PL_STAMP(i) stamp(i)
#else
#define PL_STAMP(i)
#endif
    const int buf = t & 1;
    if (t + 1 < ntiles) {
      if constexpr (DMA) gdma(t + 1, buf ^ 1);
      else gload(t + 1);
    }
    PL_STAMP(0);
    const int kv0 = t * BN;
    // which of this wave's blocks see keys of this tile: a compile-time mask per code
    // path, so no MFMA is predicated (an if-converted MFMA keeps both results live)
    const int mask = (kv0 < qend[0] ? 1 : 0) | (QB > 1 && kv0 < qend[QB - 1] ? 2 : 0);
    auto tile = [&](auto mask_c) {
      constexpr int MASK = decltype(mask_c)::value;
      const uint16_t* Kb = smem + buf * TILE;
      const uint16_t* Vb = smem + 2 * TILE + buf * TILE;
      f32x16 s[QB][2];
#pragma unroll
      for (int j = 0; j < QB; ++j) s[j][0] = s[j][1] = zero16();
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          const bf16x8 kf = as_frag(ld16(Kb + kb * 32 * D + (fk ^ (ks << 4))));
#pragma unroll
          for (int j = 0; j < QB; ++j)
            if ((MASK >> j) & 1) s[j][kb] = mfma32(kf, qf[j][ks], s[j][kb]);
        }
      }
      if constexpr (MASK == 3 && QB == 2) {
        // K fragment reads issued ahead of the MFMA pairs that consume them (hipcc's own order
        // waited lgkmcnt(0) before every pair)
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 2);
#pragma unroll
        for (int i = 0; i < 2 * NKS - 2; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 2);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 2);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 2);
      }
      PL_STAMP(1);
      bf16x8 pf[QB][4];
#pragma unroll
      for (int j = 0; j < QB; ++j) {
        if (!((MASK >> j) & 1)) continue;
        const int qi = qw[j] + r;
        const bool need_mask = (kv0 + BN > a.S) || (a.causal && kv0 + BN - 1 > qw[j] + off);
        if (need_mask) {
          // element i of key half kb is key kv0 + 32 kb + 4 hh + acc_row(i, 0): dead past S or
          // after the lane's query -- one compare per element against a per-lane limit (a
          // per-element condition compiled to scalar-mask branches)
          const int lim0 = (a.causal ? min(a.S - 1, qi + off) : a.S - 1) - (kv0 + 4 * hh);
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
            for (int i = 0; i < 16; ++i)
              s[j][kb][i] = acc_row(i, 0) > lim0 - 32 * kb ? -INFINITY : s[j][kb][i];
          }
        }
        // two independent max / sum chains per lane (ILP), then the lane pair (r, r+32)
        float mx0 = -INFINITY, mx1 = -INFINITY;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          mx0 = fmaxf(mx0, s[j][0][i]);
          mx1 = fmaxf(mx1, s[j][1][i]);
        }
        float mx = fmaxf(mx0, mx1);
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float mx2 = mx * c2;  // this tile's row max in log2 units (-inf: row fully masked)
        // (m = -inf: +inf > thr, the first visible tile always sets m; mx2 = m = -inf: NaN, false)
        if (__any(mx2 - m[j] > kLazyThr)) {
          const float mnew = fmaxf(m[j], mx2);
          const float alpha = mnew == -INFINITY ? 1.f : fast_exp2(m[j] - mnew);  // m = -inf -> 0
#pragma unroll
          for (int db = 0; db < NDB; ++db)
#pragma unroll
            for (int i = 0; i < 16; ++i) o[j][db][i] = o[j][db][i] * alpha;  // scalar multiplies
          l[j] *= alpha;
          m[j] = mnew;
        }
        const float mc = m[j] == -INFINITY ? 0.f : m[j];
        float ls0 = 0.f, ls1 = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p0 = fast_exp2(__builtin_fmaf(s[j][0][i], c2, -mc));
          const float p1 = fast_exp2(__builtin_fmaf(s[j][1][i], c2, -mc));
          s[j][0][i] = p0;
          s[j][1][i] = p1;
          ls0 += p0;
          ls1 += p1;
        }
        l[j] += ls0 + ls1;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          pf[j][2 * kb] = pack_frag(s[j][kb], 0);
          pf[j][2 * kb + 1] = pack_frag(s[j][kb], 1);
        }
      }
      PL_STAMP(2);
#pragma unroll
      for (int kst = 0; kst < 4; ++kst) {
#pragma unroll
        for (int db = 0; db < NDB; ++db) {
          const int rb = kst * 16 * D;
          const bf16x8 va = cat_tr(ds_tr(Vb + rb + (fv0 ^ (db << 5))), ds_tr(Vb + rb + (fv8 ^ (db << 5))));
#pragma unroll
          for (int j = 0; j < QB; ++j)
            if ((MASK >> j) & 1) o[j][db] = mfma32(va, pf[j][kst], o[j][db]);
        }
      }
      if constexpr (MASK == 3 && QB == 2) {
        // V transposed reads two steps (4 reads) ahead of their MFMA pairs
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 3);
#pragma unroll
        for (int i = 0; i < 4 * NDB - 2; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 3);
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 3);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 3);
      }
    };
    if (mask == 3) tile(std::integral_constant<int, 3>{});
    else if (mask == 1) tile(std::integral_constant<int, 1>{});
    else if (QB > 1 && mask == 2) tile(std::integral_constant<int, 2>{});
    PL_STAMP(3);
    if constexpr (DMA) vm_wait_all();
    else if (t + 1 < ntiles) swrite(buf ^ 1, t + 1, buf ^ 1);
    PL_STAMP(4);
    __syncthreads();
    PL_STAMP(5);
#if PLLM_FWD_STAMPS
    st_acc[6] += 1;
    st_acc[7] += (uint64_t)mask;
#endif
  }
#undef PL_STAMP

#if PLLM_FWD_STAMPS
  if (a.stamps && lane == 0) {
    unsigned long long* st = a.stamps + ((int64_t)blockIdx.x * NW + w) * 9;
#pragma unroll
    for (int i = 0; i < 8; ++i) st[i] = st_acc[i];
    st[8] = __builtin_amdgcn_s_memtime() - st_start;
  }
#endif
#pragma unroll
  for (int j = 0; j < QB; ++j) {
    const int qi = qw[j] + r;
    const float lt = l[j] + __shfl_xor(l[j], 32, 64);
    if (qi < a.T) {
      const float inv = lt > 0.f ? 1.f / lt : 0.f;
      store_row_bf16<NDB>(a.o + b * a.o_sb + (int64_t)qi * a.o_st + (int64_t)h * a.o_sh, o[j], inv, hh);
      if (hh == 0 && a.lse)
        a.lse[((int64_t)b * a.H + h) * a.T + qi] = (m[j] + log2f(lt)) * 0.69314718055994531f;
    }
  }
}

// ============================================================================
// backward
// ============================================================================
// delta[b,h,t] = sum_d dO[b,t,h,d] * O[b,t,h,d]
template <int D>
__global__ __launch_bounds__(256) void attn_bwd_pre_kernel(AttnBwdArgs a) {
  constexpr int CPR = D / 8;  // lanes per row
  const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t row = gid / CPR;  // row = (b*T + t)*H + h
  const int c = (int)(gid % CPR);
  const int64_t nrows = (int64_t)a.B * a.T * a.H;
  float acc = 0.f;
  int b = 0, t = 0, h = 0;
  if (row < nrows) {
    h = (int)(row % a.H);
    const int64_t bt = row / a.H;
    t = (int)(bt % a.T);
    b = (int)(bt / a.T);
    float x[8], y[8];
    unpack8(ld16(a.dO + b * a.do_sb + (int64_t)t * a.do_st + (int64_t)h * a.do_sh + c * 8), x);
    unpack8(ld16(a.o + b * a.o_sb + (int64_t)t * a.o_st + (int64_t)h * a.o_sh + c * 8), y);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += x[j] * y[j];
  }
#pragma unroll
  for (int o = CPR / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (row < nrows && c == 0) a.delta[((int64_t)b * a.H + h) * a.T + t] = acc;
}

// Fused-role backward tiling (D = 32 / 64; D = 128 runs the role-split kernel below): 8 waves
// (two per SIMD), each owning 32 keys (BK = 256 keys per workgroup); BQ = 128 query rows per
// iteration as NQB = 4 sub-blocks of 32.  KH (32-key halves per wave) stays a parameter of the
// code.  Measured and removed (same-box A/B, profiles/r2_attn_bwd_removed_variants_ab.jsonl):
//   * 4 waves x 64 keys (KH = 2, one wave per SIMD): 13-19 % slower at D = 64;
//   * 4 waves x 128 keys x 64 queries (48 KiB LDS, two workgroups per CU): 7-15 % slower;
//   * the role-split kernel at D = 64: 28-49 % slower;
//   * fused-role D = 128 (4 waves, one per SIMD, 64 / 128 queries): 19-26 % slower than role split;
//   * persistent grid (one workgroup per CU walking the items round-robin, next item's K/V loads
//     issued before the dK/dV stores, those stores deferred into the next item): 2-4 % slower
//     (profiles/r2_attn_bwd_persistent_negative.jsonl);
//   * delta = rowsum(dO O) formed in this kernel from O rows staged beside dO, instead of the
//     attn_bwd_pre_kernel pass: 3-4 % slower (profiles/r2_attn_delta_fused_negative.txt).

template <int D>
struct BwdCfg {
  static_assert(D == 32 || D == 64, "fused-role backward: D = 32 / 64");
  static constexpr int KH = 1;
  static constexpr int NW = 8;
  static constexpr int NT = 64 * NW;
  static constexpr int BK = 32 * KH * NW;
  static constexpr int BQ = 128;
  static constexpr int MIN_WAVES = 2;
  static constexpr int NQB = BQ / 32;
  static constexpr int CPR = D / 8;
  static constexpr int LDS_ELEMS = BK * D + 2 * BQ * D + BK * BQ;
};

// dQ: each key block's partial dQ (summed over its BK keys on chip, rounded once to bf16) goes
// to a slab of the current PASS: the host runs the key blocks in passes of at most
// ``nkb_pass`` blocks so the workspace is bounded independently of T; attn_dq_reduce_frag_kernel adds
// the slabs in fp32 in a fixed order (deterministic, no atomics) into an fp32 running sum / the
// bf16 dQ.  fp32 slabs (no partial rounding) measured +12 % (T 1024, D 64) to +34 % (T 4096)
// on the whole backward: the slab bytes are its second cost after the MFMAs.
// ROPE: q and k are rotated while staged, dk is rotated back before its store (dq in the reduce).
template <int D, int ROPE>
__global__ __launch_bounds__((BwdCfg<D>::NT), (BwdCfg<D>::MIN_WAVES)) void attn_bwd_kernel(AttnBwdArgs a) {
  using C = BwdCfg<D>;
  using I = Img<D>;
  static_assert(C::BQ == 128, "dS^T image");
  using IS = ImgS;  // dS^T image [keys][BQ]
  constexpr int NT = C::NT, BK = C::BK, BQ = C::BQ, NQB = C::NQB, CPR = C::CPR, KH = C::KH;
  constexpr int NKS = D / 16, NDB = D / 32;
  __shared__ __attribute__((aligned(16))) uint16_t smem[C::LDS_ELEMS];
  __shared__ __attribute__((aligned(16))) float rowc[2 * BQ];  // -lse/scale, -delta
  uint16_t* Kl = smem;
  uint16_t* Ql = smem + BK * D;
  uint16_t* Ol = Ql + BQ * D;             // dO tile
  uint16_t* Sl = Ol + BQ * D;             // dS^T image [key][q]

  // lowest key blocks (most query blocks under causal) of every head first; head-local order
  // measured 14-28 % slower (profiles/r2_attn_order_ab.txt)
  const int BH = a.B * a.Hkv;
  const int id = blockIdx.x;
  const int kb = a.kb0 + id / BH;
  const int bh = id % BH;
  const int b = bh / a.Hkv, hk = bh % a.Hkv;
  const int G = a.H / a.Hkv;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int k0 = kb * BK;
  const int kw0 = k0 + w * 32 * KH;       // first key of this wave
  const int off = a.S - a.T;
  const uint16_t* kp = a.k + b * a.k_sb + (int64_t)hk * a.k_sh;
  const uint16_t* vp = a.v + b * a.v_sb + (int64_t)hk * a.v_sh;

  // this lane's key rows (one per 32-key half) of V as B-operand fragments (k = head dim); the K
  // fragments are read back from the K image below (K crosses HBM / L2 once per workgroup)
  bf16x8 kf[KH][NKS], vf[KH][NKS];
#pragma unroll
  for (int kh = 0; kh < KH; ++kh) {
    const int key = kw0 + 32 * kh + r;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
      vf[kh][ks] = key < a.S ? as_frag(ld16(vp + (int64_t)key * a.v_st + 16 * ks + 8 * hh)) : zero_frag();
  }
  // whole (rotated) K block into LDS for the S and dQ products; a thread stages both RoPE partners
  constexpr int CPR2 = CPR / 2;
#pragma unroll
  for (int i = 0; i < (BK * CPR2 + NT - 1) / NT; ++i) {
    const int c = tid + NT * i, row = c / CPR2, col = c % CPR2, kk = k0 + row;
    if (c < BK * CPR2) {
      u32x4 lo = u32x4{0u, 0u, 0u, 0u}, hi = lo;
      if (kk < a.S) {
        lo = ld16(kp + (int64_t)kk * a.k_st + col * 8);
        hi = ld16(kp + (int64_t)kk * a.k_st + (col + CPR2) * 8);
        if (ROPE == 1) {
          const int64_t tab = (int64_t)kk * (D / 2) + col * 8;
          rope8(lo, hi, a.rope_cos + tab, a.rope_sin + tab, 1.f);
        }
      }
      I::st_pair(Kl, row, col, lo, hi);
    }
  }

  vm_wait_all();  // V fragments and the K image ready before the query loop (see common.h)
  __syncthreads();
  // K fragments of the lane's key rows from the (rotated) image: rows w*32*KH + 32 kh + r,
  // the Q-fragment read pattern (fq below)
#pragma unroll
  for (int kh = 0; kh < KH; ++kh)
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
      kf[kh][ks] = as_frag(ld16(Kl + (w * 32 * KH + 32 * kh) * D + (I::off(r, 8 * hh) ^ (ks << 4))));
  f32x16 dk[KH][NDB], dv[KH][NDB];
#pragma unroll
  for (int kh = 0; kh < KH; ++kh)
#pragma unroll
    for (int db = 0; db < NDB; ++db) {
      dk[kh][db] = zero16();
      dv[kh][db] = zero16();
    }
  const float c2 = a.scale_log2;
  const int g1 = (lane >> 4) & 1, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;
  const int nqb = (a.T + BQ - 1) / BQ;
  int qb_start = 0;
  if (a.causal) qb_start = max(0, k0 - off) / BQ;
  const int per_head = nqb - qb_start;
  const int total = per_head * G;

  // Q / dO tile chunks: as in the forward, chunk i of a thread is row c / CPR2, column chunk
  // (c % CPR2) + (i odd ? CPR2 : 0), c = tid + NT * (i / 2): both RoPE partners in one thread
  constexpr int QPAIR = (BQ * CPR2 + NT - 1) / NT;
  // QDMA (no in-kernel RoPE): the Q / dO tiles go HBM/L2 -> LDS by buffer_load ... lds, issued
  // right after the sub-block phase (the dQ task reads neither image) and waited at the next
  // iteration's top: no staging registers, no ds_write pass, one barrier less per iteration.
  // Pieces of 1 KiB = QRP rows; lane l fills row blk * QRP + l / CPR at chunk position l % CPR,
  // which holds logical chunk (l % CPR) ^ I::f(row) (the image's swizzle, applied to the source)
  constexpr bool QDMA = ROPE == 0;
  constexpr int QRP = 512 / D, QNP = BQ / QRP, QPPW = 2 * QNP / C::NW;
  static_assert(2 * QNP % C::NW == 0, "Q/dO pieces per wave");
  u32x4 qr[QDMA ? 1 : 2 * QPAIR], dor[QDMA ? 1 : 2 * QPAIR];
  uint32_t qvo[QPPW];
#pragma unroll
  for (int k = 0; k < QPPW; ++k) {
    const int pc = w * QPPW + k, img = pc / QNP, blk = pc % QNP;
    const int row = blk * QRP + lane / CPR, ch = (lane % CPR) ^ I::f(row);
    qvo[k] = (uint32_t)((row * (img == 0 ? a.q_st : a.do_st) + 8 * ch) * 2);
  }
  const unsigned lds_q = (unsigned)(uintptr_t)Ql, lds_o = (unsigned)(uintptr_t)Ol;
  // (head h, first query row q0) of an iteration come from the loop's incremental counters: an
  // it / per_head here was a run-time integer division (a long scalar chain) twice per iteration
  auto qdma_srd = [&](int h, int q0, i32x4v& qs, i32x4v& os) {
    const int rows = a.T - q0;
    qs = srd_of(a.q + b * a.q_sb + (int64_t)h * a.q_sh + (int64_t)q0 * a.q_st,
                (uint32_t)(((int64_t)(rows - 1) * a.q_st + D) * 2));
    os = srd_of(a.dO + b * a.do_sb + (int64_t)h * a.do_sh + (int64_t)q0 * a.do_st,
                (uint32_t)(((int64_t)(rows - 1) * a.do_st + D) * 2));
  };
  auto qdma_piece = [&](const i32x4v& qs, const i32x4v& os, int k) {
    const int wu = __builtin_amdgcn_readfirstlane(w);  // wave-uniform piece numbers: scalar descriptors
    const int pc = wu * QPPW + k, img = pc / QNP, blk = pc % QNP;
    blds16(img == 0 ? qs : os, qvo[k], (img == 0 ? lds_q : lds_o) + 1024u * blk);
  };
  auto qdma = [&](int h, int q0) {
    i32x4v qs, os;
    qdma_srd(h, q0, qs, os);
#pragma unroll
    for (int k = 0; k < QPPW; ++k) qdma_piece(qs, os, k);
  };
  float rc = 0.f;
  auto gload = [&](int h, int q0) {
    // Q / dO rows of head h by buffer loads through a per-tile descriptor (scalar base = row
    // q0): rows past T read as zeros (range check), per-lane offsets loop-invariant
    const auto qrs = rows_rsrc(a.q + b * a.q_sb + (int64_t)h * a.q_sh + (int64_t)q0 * a.q_st, a.T - q0, a.q_st, D);
    const auto ors = rows_rsrc(a.dO + b * a.do_sb + (int64_t)h * a.do_sh + (int64_t)q0 * a.do_st, a.T - q0, a.do_st, D);
    // per-lane offsets recomputed per iteration (a few VALU): hoisted out of the loop they are
    // spilled at D = 64's register pressure, and each reload's vmcnt(0) serialises the loads
    int tl = tid;
    asm volatile("" : "+v"(tl));
#pragma unroll
    for (int i = 0; i < (QDMA ? 0 : 2 * QPAIR); ++i) {
      const int c = tl + NT * (i / 2), row = c / CPR2, col = c % CPR2 + (i & 1) * CPR2;
      if (c < BQ * CPR2) {
        qr[i] = buf_ld16(qrs, (uint32_t)(row * (int)a.q_st + col * 8) * 2u);
        dor[i] = buf_ld16(ors, (uint32_t)(row * (int)a.do_st + col * 8) * 2u);
      } else {
        qr[i] = u32x4{0u, 0u, 0u, 0u};
        dor[i] = u32x4{0u, 0u, 0u, 0u};
      }
    }
    if (tid < 2 * BQ) {
      // unconditional load (clamped row) consumed only at the LDS write of the next iteration:
      // a use here, or a load under a branch, makes hipcc wait vmcnt(0) -- for the Q/dO
      // prefetch above too
      // waves [0, BQ/64) load -lse rows, the next BQ/64 waves -delta: a wave-uniform (scalar)
      // base, so no per-lane 64-bit pointer is kept live (it was spilled at D = 64)
      const float* base = __builtin_amdgcn_readfirstlane(tid >> 6) < BQ / 64 ? a.lse : a.delta;
      const int q = min(q0 + (tid & (BQ - 1)), a.T - 1);
      rc = base[((int64_t)b * a.H + h) * a.T + q];
    }
  };

  // dQ task of this wave in each iteration: (query sub-block, d-block)
  constexpr int NTASK = NQB * NDB;

  // dQ fragment blocks of an iteration are STORED one iteration late, right after the next
  // iteration's Q/dO staging: vmcnt counts stores too (gfx9 has no separate store counter), so
  // stores issued at the end of an iteration would make the next iteration's first wait (for the
  // prefetched Q/dO) wait out their latency as well (same-box A/B: neutral at the GPT-2 / llama
  // shapes, where that latency was already covered).
  constexpr int NTPW = (NTASK + C::NW - 1) / C::NW;
  // the dQ task's K^T fragments (A operand, key steps 0..KREG-1) in registers: the K block is fixed for
  // the workgroup and, with one task per wave (NTPW == 1), so is the wave's d-block -- the same reads
  // every iteration otherwise
  constexpr int KREG = NTPW == 1 ? PL_BWD_DQ_KREG : 0;
  bf16x8 kdq[KREG > 0 ? KREG : 1];
  if constexpr (KREG > 0) {
    const int tdb0 = __builtin_amdgcn_readfirstlane(w) % NDB;
    const int dc0 = tdb0 * 32 + 16 * g1 + 4 * tp;
    const int k0a = I::off(8 * hh + tq, dc0), k4a = I::off(8 * hh + tq + 4, dc0);
#pragma unroll
    for (int ks = 0; ks < KREG; ++ks)
      kdq[ks] = cat_tr(ds_tr(Kl + 16 * ks * D + k0a), ds_tr(Kl + 16 * ks * D + k4a));
  }
  u32x4 dqv[NTPW][2];
  uint16_t* dqp[NTPW];
#pragma unroll
  for (int i = 0; i < NTPW; ++i) dqp[i] = nullptr;
  auto flush_dq = [&]() {
#pragma unroll
    for (int i = 0; i < NTPW; ++i)
      if (dqp[i] != nullptr) {
        st16(dqp[i], dqv[i][0]);
        st16(dqp[i] + 8, dqv[i][1]);
        dqp[i] = nullptr;
      }
  };

  // Per-lane LDS element offsets with the swizzle applied once.  Every image's f(row) depends
  // only on row bits 0..3, so row steps of 16 / 32 are plain additions (instruction immediates),
  // and column-chunk steps are XORs into the chunk bits:
  //   fragment reads (32 j + r, 16 ks + 8 hh)        = fq ^ (ks << 4) + 32 j D
  //   transposed reads (32 j + 16 st + 4 hh + tq (+8), 32 db + 16 g1 + 4 tp)
  //                                                   = ft0 (ft8) ^ (db << 5) + (32 j + 16 st) D
  //   dS^T stores (key row, 32 j + 8 g + 4 hh)        = fs ^ ((4 j + g) << 3)
  // Left to itself hipcc hoisted one full address per (j, ks / g / db) out of the loop and spilled
  // them (scratch reloads with vmcnt(0) inside the sub-blocks, serialising the Q/dO prefetch).
  const int fq = I::off(r, 8 * hh);
  const int ft0 = I::off(4 * hh + tq, 16 * g1 + 4 * tp), ft8 = I::off(4 * hh + tq + 8, 16 * g1 + 4 * tp);
  const int fs0 = IS::off(w * 32 * KH + r, 8 * hh);

  // static priority for the second-dispatched half of an 8-wave workgroup: it loses every
  // VALU arbitration to its older SIMD partner otherwise (MI355X_MICROARCH.md, 'Two waves
  // per SIMD' item 4)
  if (C::NW == 8 && w >= 4) __builtin_amdgcn_s_setprio(1);
  if constexpr (QDMA) {
    if (total > 0) {
      // row constants of iteration 0 (their load retired by this write), then its Q / dO DMA
      gload(hk * G, qb_start * BQ);
      if (tid < 2 * BQ) {
        const bool live = qb_start * BQ + (tid & (BQ - 1)) < a.T;
        rowc[tid] = live ? (tid < BQ ? -rc * kLog2e : -rc) : 0.f;  // -lse*log2(e), -delta
      }
      qdma(hk * G, qb_start * BQ);
    }
  } else if (total > 0) {
    gload(hk * G, qb_start * BQ);
  }
  // (head, query block) of iteration it, advanced incrementally (no integer division per step)
  int h = hk * G, qbi = qb_start;
#if PLLM_BWD_STAMPS
  uint64_t st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t st_start = __builtin_amdgcn_s_memtime();
  uint64_t ts_prev = st_start;
  auto stamp = [&](int i) {
    const uint64_t now = __builtin_amdgcn_s_memtime();
    st_acc[i] += now - ts_prev;
    ts_prev = now;
  };
#define PL_BSTAMP(i) stamp(i)
#else
#define PL_BSTAMP(i)
#endif
  for (int it = 0; it < total; ++it, (++qbi == nqb) ? (qbi = qb_start, ++h) : 0) {
    const int q0 = qbi * BQ;
    // the next iteration's (head, first query row)
    const bool wrap = qbi + 1 == nqb;
    const int hn = wrap ? h + 1 : h, qn0 = (wrap ? qb_start : qbi + 1) * BQ;
    PL_BSTAMP(7);
    // opaque per iteration: the (j, g) store offsets derived from it are formed next to their
    // stores instead of being hoisted out of the loop as 16 live registers
    int fs = fs0;
    asm volatile("" : "+v"(fs));
    // every path waits here for the prefetch (and the previous dQ stores, an iteration old): a
    // wait left inside the staging branches made hipcc assume loads still in flight at the
    // join and wait vmcnt(0) again before the next prefetch -- on the fresh dQ stores
    vm_wait_all();
    __syncthreads();  // previous iteration's readers of Q/dO/dS are done (QDMA: this one's tiles landed)
    PL_BSTAMP(0);
    if constexpr (QDMA) {
      flush_dq();
      if (it + 1 < total) gload(hn, qn0);  // the next iteration's row constants
    }
#pragma unroll
    for (int i = 0; i < (QDMA ? 0 : 2 * QPAIR); i += 2) {
      const int c = tid + NT * (i / 2), row = c / CPR2, col = c % CPR2;
      if (c < BQ * CPR2) {
        if (ROPE == 1 && q0 + row < a.T) {
          const int64_t tab = (int64_t)(q0 + row + off) * (D / 2) + col * 8;
          rope8(qr[i], qr[i + 1], a.rope_cos + tab, a.rope_sin + tab, 1.f);
        }
        I::st_pair(Ql, row, col, qr[i], qr[i + 1]);
        I::st_pair(Ol, row, col, dor[i], dor[i + 1]);
      }
    }
    if constexpr (!QDMA) {
      if (tid < 2 * BQ) {
        const bool live = q0 + (tid & (BQ - 1)) < a.T;
        rowc[tid] = live ? (tid < BQ ? -rc * kLog2e : -rc) : 0.f;  // -lse*log2(e), -delta
      }
      flush_dq();
      __syncthreads();
      PL_BSTAMP(1);
      if (it + 1 < total) gload(hn, qn0);
    }
    PL_BSTAMP(2);

    // rows past T need no mask: their Q / dO rows are zero-filled, their row constants 0
    const bool need_mask = (k0 + BK > a.S) || (a.causal && k0 + BK - 1 > q0 + off);
#pragma unroll
    for (int j = 0; j < NQB; ++j) {
      const int qj0 = q0 + 32 * j;
      // causal: the key halves of this wave that lie after every query of the sub-block have
      // P = dS = 0; keys grow with kh, so the live halves are a prefix (a compile-time count per
      // code path: no MFMA is predicated)
      int live = KH;
      if (a.causal) {
        live = 0;
#pragma unroll
        for (int kh = 0; kh < KH; ++kh)
          if (kw0 + 32 * kh <= qj0 + 31 + off) live = kh + 1;
      }
#pragma unroll
      for (int kh = 0; kh < KH; ++kh) {
        if (kh < live) continue;
#pragma unroll
        for (int k = 0; k < 4; k += 2)
          *reinterpret_cast<u32x4*>(Sl + 32 * kh * BQ + (fs ^ ((4 * j + k) << 3))) = u32x4{0u, 0u, 0u, 0u};
      }
      // MASKED is a compile-time property of the code path: a uniform run-time test per
      // element made hipcc emit one basic block per exponential (16 scalar branches per
      // sub-block), which also kept the exponentials from interleaving with the MFMAs
      auto body = [&](auto live_c, auto mask_c) {
        constexpr int NL = decltype(live_c)::value;
        constexpr bool MASKED = decltype(mask_c)::value;
        // S = Q K^T ; dP = dO V^T   (query rows in registers, key on the lane; zero-initialised
        // accumulators: the row constants enter in the exponent / the subtraction below)
        f32x16 s[NL], dp[NL];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 rd = *reinterpret_cast<const f32x4*>(&rowc[BQ + 32 * j + 8 * g + 4 * hh]);
#pragma unroll
          for (int kh = 0; kh < NL; ++kh)
#pragma unroll
            for (int e = 0; e < 4; ++e) dp[kh][4 * g + e] = rd[e];
        }
#pragma unroll
        for (int kh = 0; kh < NL; ++kh) s[kh] = zero16();
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          const int fo = 32 * j * D + (fq ^ (ks << 4));
          const bf16x8 qa = as_frag(ld16(Ql + fo));
          const bf16x8 oa = as_frag(ld16(Ol + fo));
#pragma unroll
          for (int kh = 0; kh < NL; ++kh) {
            s[kh] = mfma32(qa, kf[kh][ks], s[kh]);
            dp[kh] = mfma32(oa, vf[kh][ks], dp[kh]);
          }
        }
        // P = exp2(S c2 - lse log2e) ; dS = P (dP - delta)   (unscaled).  Masked paths: the
        // lane's element i (query qb + acc_row(i)) is dead iff acc_row(i) < lo[kh] (causal:
        // key > query; keys past S: all).  Query rows past T need no test: their Q / dO rows
        // are zero-filled and their row constants 0, so P = 1 meets dO = 0 (dV) and dS = 0
        // (dK, dQ), and no dQ row past T is stored.
        int lo[NL];
        if constexpr (MASKED) {
#pragma unroll
          for (int kh = 0; kh < NL; ++kh) {
            const int key = kw0 + 32 * kh + r;
            lo[kh] = key >= a.S ? 64 : (a.causal ? key - off - (qj0 + 4 * hh) : -64);
          }
        }
        bf16x8 pf[NL][2], sf[NL][2];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          // accumulator rows 4g..4g+3 are 4 consecutive queries: one 16-B LDS read each
          const f32x4 rs = *reinterpret_cast<const f32x4*>(&rowc[32 * j + 8 * g + 4 * hh]);
#pragma unroll
          for (int kh = 0; kh < NL; ++kh)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int i = 4 * g + e;
              float p = fast_exp2(__builtin_fmaf(s[kh][i], c2, rs[e]));
              if constexpr (MASKED) p = acc_row(i, 0) < lo[kh] ? 0.f : p;
              s[kh][i] = p;               // P
              dp[kh][i] = p * dp[kh][i];  // dS (unscaled; dP accumulated onto -delta)
            }
        }
#pragma unroll
        for (int kh = 0; kh < NL; ++kh) {
          pf[kh][0] = pack_frag(s[kh], 0);
          pf[kh][1] = pack_frag(s[kh], 1);
          sf[kh][0] = pack_frag(dp[kh], 0);
          sf[kh][1] = pack_frag(dp[kh], 1);
        }
        // dV^T += dO^T P ; dK^T += Q^T dS   (A operands by transposed reads of the [q][d] images,
        // each shared by the wave's NL key halves)
#pragma unroll
        for (int db = 0; db < NDB; ++db) {
#pragma unroll
          for (int st = 0; st < 2; ++st) {
            const int rb = (32 * j + 16 * st) * D, o0 = rb + (ft0 ^ (db << 5)), o8 = rb + (ft8 ^ (db << 5));
            const bf16x8 oA = cat_tr(ds_tr(Ol + o0), ds_tr(Ol + o8));
            const bf16x8 qA = cat_tr(ds_tr(Ql + o0), ds_tr(Ql + o8));
#pragma unroll
            for (int kh = 0; kh < NL; ++kh) {
              dv[kh][db] = mfma32(oA, pf[kh][st], dv[kh][db]);
              dk[kh][db] = mfma32(qA, sf[kh][st], dk[kh][db]);
            }
          }
        }
        // dS^T image: the lane's key rows.  The lane holds queries 8g + 4hh + (0..3) (dwords
        // 2(g&1), 2(g&1)+1 of the packed fragment sf[g/2]); v_permlane32_swap of the group pairs
        // (g, g+1) across the half-waves gives each lane 8 consecutive queries (8g + 8hh .. +7, g
        // even): one 16-B store per pair on the ImgS swizzle, conflict-free
#pragma unroll
        for (int kh = 0; kh < NL; ++kh) {
          u32x2 v[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const u32x4 w4 = __builtin_bit_cast(u32x4, sf[kh][g >> 1]);
            v[g] = u32x2{w4[2 * (g & 1)], w4[2 * (g & 1) + 1]};
          }
#pragma unroll
          for (int k = 0; k < 4; k += 2) {
#pragma unroll
            for (int d = 0; d < 2; ++d) {
              const auto sw = __builtin_amdgcn_permlane32_swap(v[k][d], v[k + 1][d], false, false);
              v[k][d] = sw[0];
              v[k + 1][d] = sw[1];
            }
            *reinterpret_cast<u32x4*>(Sl + 32 * kh * BQ + (fs ^ ((4 * j + k) << 3))) =
                u32x4{v[k][0], v[k][1], v[k + 1][0], v[k + 1][1]};
          }
        }
        // keep the scheduler from overlapping consecutive sub-blocks (their live ranges
        // together exceed the 256 registers of two waves per SIMD)
        __builtin_amdgcn_sched_barrier(0);
      };
      using TT = std::true_type;
      using FF = std::false_type;
      // per wave and sub-block: only the sub-block whose 32 queries overlap the wave's keys
      // (the causal diagonal) or a ragged key end needs the masked path
      const bool mask_j = need_mask && ((kw0 + 32 * KH > a.S) || (a.causal && kw0 + 32 * KH - 1 > qj0 + off));
      if (live == KH) {
        if (mask_j) body(std::integral_constant<int, KH>{}, TT{});
        else body(std::integral_constant<int, KH>{}, FF{});
      } else if (KH > 1 && live == 1) {
        body(std::integral_constant<int, 1>{}, TT{});
      }
    }
    PL_BSTAMP(3);
    __syncthreads();
    if constexpr (QDMA) {
      if (it + 1 < total) {
        // every wave is past its Q / dO / row-constant reads: the next tile's row constants (their
        // load retired by this write, before the DMA below is in flight), then its Q / dO DMA
        if (tid < 2 * BQ) {
          const bool live = qn0 + (tid & (BQ - 1)) < a.T;
          rowc[tid] = live ? (tid < BQ ? -rc * kLog2e : -rc) : 0.f;
        }
        qdma(hn, qn0);
      }
    }
    PL_BSTAMP(4);
    // dQ partial of this key block: dQ_kb[q, d] = dS[q, keys] K[keys, d], one (q sub-block,
    // d-block) task per wave (NTASK / NW of them), summed over all BK keys on chip, stored into
    // this pass's fp32 slab of the key block.
#pragma unroll
    for (int ti = 0; ti < NTPW; ++ti) {
      const int task = __builtin_amdgcn_readfirstlane(w) + ti * C::NW;
      if (task >= NTASK) break;
      const int tq_blk = task / NDB, tdb = task % NDB;
      const int qt0 = q0 + 32 * tq_blk;
      if (qt0 >= a.T) continue;  // a query tile past T (ragged last block): no fragment block exists
      // dQ^T tile = K^T dS^T (query on the lane), dumped as a coalesced fragment-order block
      // (attn_dq_reduce_frag_kernel reads it back).  Every key step runs, also the causal ones
      // past the task's last query: their dS^T rows are zeros in the image (dead sub-blocks are
      // zero-filled, masked elements give p = 0), and with no data-dependent exit the LDS reads
      // pipeline ahead of the MFMAs (the early exit serialised read -> wait -> MFMA per step:
      // ~2.9k of a 13.4k-cycle iteration, profiles/r3_attn_bwd_stamps.md)
      f32x16 acc = zero16();
      // key rows 16 ks + 8 hh + tq (+4): the 16 ks steps are additions (see fq above)
      const int qc = 32 * tq_blk + 16 * g1 + 4 * tp, dc = tdb * 32 + 16 * g1 + 4 * tp;
      const int sa0 = IS::off(8 * hh + tq, qc), sa4 = IS::off(8 * hh + tq + 4, qc);
      const int ka0 = I::off(8 * hh + tq, dc), ka4 = I::off(8 * hh + tq + 4, dc);
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        const bf16x8 A = cat_tr(ds_tr(Sl + 16 * ks * BQ + sa0), ds_tr(Sl + 16 * ks * BQ + sa4));
        const bf16x8 Bf = ks < KREG ? kdq[ks < KREG ? ks : 0]
                                    : cat_tr(ds_tr(Kl + 16 * ks * D + ka0), ds_tr(Kl + 16 * ks * D + ka4));
        acc = mfma32(Bf, A, acc);
      }
      float lo[8], hi[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        lo[e] = acc[e];
        hi[e] = acc[8 + e];
      }
      dqv[ti][0] = pack8(lo);
      dqv[ti][1] = pack8(hi);
      dqp[ti] = a.dq_acc + (kb - a.kb0) * a.slab +
                ((((int64_t)b * a.H + h) * a.nqt + (qt0 >> 5)) * NDB + tdb) * 1024 + lane * 16;
    }
    PL_BSTAMP(5);
#if PLLM_BWD_STAMPS
    st_acc[6] += 1;
#endif
  }
#undef PL_BSTAMP
#if PLLM_BWD_STAMPS
  if (a.stamps && lane == 0) {
    unsigned long long* stp = a.stamps + ((int64_t)blockIdx.x * C::NW + w) * 9;
#pragma unroll
    for (int i = 0; i < 8; ++i) stp[i] = st_acc[i];
    stp[8] = __builtin_amdgcn_s_memtime() - st_start;
  }
#endif
  flush_dq();
  // write dK (scaled) and dV for this lane's keys; with RoPE, dK is rotated back (R^T): the
  // lane's d-blocks db and db + NDB/2 hold the partner elements i and i + D/2
#pragma unroll
  for (int kh = 0; kh < KH; ++kh) {
    const int key = kw0 + 32 * kh + r;
    if (key >= a.S) continue;
    if (ROPE != 0) {
      const float* cr = a.rope_cos + (int64_t)key * (D / 2);
      const float* sr = a.rope_sin + (int64_t)key * (D / 2);
      if constexpr (NDB >= 2) {
#pragma unroll
        for (int db = 0; db < NDB / 2; ++db)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int d = db * 32 + 8 * (i >> 2) + 4 * hh + (i & 3);
            const float c = cr[d], sn = sr[d];
            const float x = dk[kh][db][i], y = dk[kh][db + NDB / 2][i];
            dk[kh][db][i] = x * c + y * sn;
            dk[kh][db + NDB / 2][i] = y * c - x * sn;
          }
      } else {
        // D = 32: one d-block; element i (dim 8(i/4) + 4hh + i%4) pairs with element i + 8
        // (dim + 16) of the same lane
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int d = 8 * (i >> 2) + 4 * hh + (i & 3);
          const float c = cr[d], sn = sr[d];
          const float x = dk[kh][0][i], y = dk[kh][0][i + 8];
          dk[kh][0][i] = x * c + y * sn;
          dk[kh][0][i + 8] = y * c - x * sn;
        }
      }
    }
    store_row_bf16<NDB>(a.dk + b * a.dk_sb + (int64_t)key * a.dk_st + (int64_t)hk * a.dk_sh, dk[kh], a.scale, hh);
    store_row_bf16<NDB>(a.dv + b * a.dv_sb + (int64_t)key * a.dv_st + (int64_t)hk * a.dv_sh, dv[kh], 1.f, hh);
  }
}

// ---------------------------------------------------------------------------
// Role-split backward ("RS"): one workgroup = 8 waves = 128 keys of one (batch, kv-head) as 4
// key groups of 32, each group served by a PAIR of waves on one SIMD (w and w + 4):
//   wave A (w < 4): S = Q K^T -> P (the keys' K rows in registers), dV^T += dO^T P;
//   wave B (w >= 4): dP = dO V^T (V rows in registers), dS = P (dP - delta) with P handed over
//   through LDS in the accumulator's own layout (element-wise, fp32), dK^T += Q^T dS, dS^T image.
// Each wave keeps ONE operand matrix and ONE gradient accumulator (half the registers of the
// fused-role kernel: two waves per SIMD at D = 128 instead of one, no AGPR shuffling), the two
// waves of a SIMD overlap one's exp / pack VALU with the other's MFMAs, and the MFMA work per
// wave is balanced (S + dV vs dP + dK).  dQ as before: per-key-block bf16 slabs, one task per wave.
template <int D>
struct RsCfg {
  static_assert(D == 128, "role-split backward: D = 128");
  static constexpr int NW = 8, NT = 512, NG = 4;  // waves, threads, key groups (wave pairs)
  static constexpr int BK = 32 * NG;               // 128 keys per workgroup
  static constexpr int BQ = 128;                   // queries per iteration (LDS: 145 KiB)
  static constexpr int NQB = BQ / 32;              // 32-query sub-blocks
  static constexpr int CPR = D / 8;
  static constexpr int PX = 2 * NG * 2 * 64 * 4;   // P hand-off (dwords): [parity][group][half][lane] bf16x8
  static constexpr int LDS_ELEMS = BK * D + 2 * BQ * D + BK * BQ;  // bf16: K, Q, dO, dS^T images
};

template <int D, int ROPE>
__global__ __launch_bounds__(512, 1) void attn_bwd_rs_kernel(AttnBwdArgs a) {
  using C = RsCfg<D>;
  using I = Img<D>;
  static_assert(C::BQ == 128, "dS^T image");
  using IS = ImgS;  // dS^T image (16-B stores after a half-wave swap: conflict-free, see ImgS)
  constexpr int NT = C::NT, BK = C::BK, BQ = C::BQ, NQB = C::NQB, CPR = C::CPR;
  constexpr int NKS = D / 16, NDB = D / 32;
  __shared__ __attribute__((aligned(16))) uint16_t smem[C::LDS_ELEMS];
  __shared__ __attribute__((aligned(16))) uint32_t px[C::PX];
  __shared__ __attribute__((aligned(16))) float rowc[2 * BQ];  // -lse/scale, -delta
  uint16_t* Kl = smem;
  uint16_t* Ql = smem + BK * D;
  uint16_t* Ol = Ql + BQ * D;
  uint16_t* Sl = Ol + BQ * D;

  const int BH = a.B * a.Hkv;
  const int id = blockIdx.x;
  const int kb = a.kb0 + id / BH;
  const int bh = id % BH;
  const int b = bh / a.Hkv, hk = bh % a.Hkv;
  const int G = a.H / a.Hkv;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const bool roleA = w < C::NG;  // wave-uniform
  const int grp = w & (C::NG - 1);
  const int k0 = kb * BK;
  const int kw0 = k0 + grp * 32;
  const int off = a.S - a.T;
  const uint16_t* kp = a.k + b * a.k_sb + (int64_t)hk * a.k_sh;
  const uint16_t* vp = a.v + b * a.v_sb + (int64_t)hk * a.v_sh;

  // this lane's key row of V (wave B) as B-operand fragments; wave A reads its K fragments back
  // from the (rotated) K image below, so K crosses HBM / L2 once per workgroup
  bf16x8 kvf[NKS];
  if (!roleA) {
    const int key = kw0 + r;
    const uint16_t* src = vp + (int64_t)key * a.v_st;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) kvf[ks] = key < a.S ? as_frag(ld16(src + 16 * ks + 8 * hh)) : zero_frag();
  }
  // whole (rotated) K block into LDS for the S (wave A) and dQ products
  constexpr int CPR2 = CPR / 2;
#pragma unroll
  for (int i = 0; i < (BK * CPR2 + NT - 1) / NT; ++i) {
    const int c = tid + NT * i, row = c / CPR2, col = c % CPR2, kk = k0 + row;
    if (c < BK * CPR2) {
      u32x4 lo = u32x4{0u, 0u, 0u, 0u}, hi = lo;
      if (kk < a.S) {
        lo = ld16(kp + (int64_t)kk * a.k_st + col * 8);
        hi = ld16(kp + (int64_t)kk * a.k_st + (col + CPR2) * 8);
        if (ROPE == 1) {
          const int64_t tab = (int64_t)kk * (D / 2) + col * 8;
          rope8(lo, hi, a.rope_cos + tab, a.rope_sin + tab, 1.f);
        }
      }
      I::st_pair(Kl, row, col, lo, hi);
    }
  }
  vm_wait_all();
  __syncthreads();
  if (roleA) {
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) kvf[ks] = as_frag(ld16(Kl + grp * 32 * D + (I::off(r, 8 * hh) ^ (ks << 4))));
  }

  f32x16 acc[NDB];  // dV^T (wave A) or dK^T (wave B) of the group's 32 keys
#pragma unroll
  for (int db = 0; db < NDB; ++db) acc[db] = zero16();
  const float c2 = a.scale_log2;
  const int g1 = (lane >> 4) & 1, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;
  const int nqb = (a.T + BQ - 1) / BQ;
  int qb_start = 0;
  if (a.causal) qb_start = max(0, k0 - off) / BQ;
  const int per_head = nqb - qb_start;
  const int total = per_head * G;

  constexpr int QPAIR = (BQ * CPR2 + NT - 1) / NT;
  u32x4 qr[2 * QPAIR], dor[2 * QPAIR];
  float rc = 0.f;
  auto gload = [&](int it) {
    const int h = hk * G + it / per_head;
    const int q0 = (qb_start + it % per_head) * BQ;
    const auto qrs = rows_rsrc(a.q + b * a.q_sb + (int64_t)h * a.q_sh + (int64_t)q0 * a.q_st, a.T - q0, a.q_st, D);
    const auto ors = rows_rsrc(a.dO + b * a.do_sb + (int64_t)h * a.do_sh + (int64_t)q0 * a.do_st, a.T - q0, a.do_st, D);
    int tl = tid;
    asm volatile("" : "+v"(tl));
#pragma unroll
    for (int i = 0; i < 2 * QPAIR; ++i) {
      const int c = tl + NT * (i / 2), row = c / CPR2, col = c % CPR2 + (i & 1) * CPR2;
      if (c < BQ * CPR2) {
        qr[i] = buf_ld16(qrs, (uint32_t)(row * (int)a.q_st + col * 8) * 2u);
        dor[i] = buf_ld16(ors, (uint32_t)(row * (int)a.do_st + col * 8) * 2u);
      } else {
        qr[i] = u32x4{0u, 0u, 0u, 0u};
        dor[i] = u32x4{0u, 0u, 0u, 0u};
      }
    }
    if (tid < 2 * BQ) {
      const bool isl = __builtin_amdgcn_readfirstlane(tid >> 6) < BQ / 64;
      const float* base = isl ? a.lse : a.delta;
      const int q = min(q0 + (tid & (BQ - 1)), a.T - 1);
      rc = base[((int64_t)b * a.H + h) * a.T + q];
    }
  };

  constexpr int NTASK = NQB * NDB;
  // per-lane LDS element offsets, swizzle applied once (see attn_bwd_kernel): fragment reads
  // fq ^ (ks << 4) + 32 j D, transposed reads ft0 / ft8 ^ (db << 5) + (32 j + 16 st) D, dS^T
  // stores fs ^ ((4 j + g) << 3)
  const int fq = I::off(r, 8 * hh);
  const int ft0 = I::off(4 * hh + tq, 16 * g1 + 4 * tp), ft8 = I::off(4 * hh + tq + 8, 16 * g1 + 4 * tp);
  const int fs0 = IS::off(grp * 32 + r, 8 * hh);

  // dQ fragment blocks of an iteration are STORED one iteration late, right after the next
  // iteration's Q/dO staging: vmcnt counts stores too (gfx9 has no separate store counter), so
  // stores issued at the end of an iteration would make the next iteration's first wait (for the
  // prefetched Q/dO) wait out their latency as well (same-box A/B: neutral at the GPT-2 / llama
  // shapes, where that latency was already covered).
  constexpr int NTPW = (NTASK + C::NW - 1) / C::NW;
  u32x4 dqv[NTPW][2];
  uint16_t* dqp[NTPW];
#pragma unroll
  for (int i = 0; i < NTPW; ++i) dqp[i] = nullptr;
  auto flush_dq = [&]() {
#pragma unroll
    for (int i = 0; i < NTPW; ++i)
      if (dqp[i] != nullptr) {
        st16(dqp[i], dqv[i][0]);
        st16(dqp[i] + 8, dqv[i][1]);
        dqp[i] = nullptr;
      }
  };
  if (total > 0) gload(0);
  // (head, query block) of iteration it, advanced incrementally (no integer division per step)
  int h = hk * G, qbi = qb_start;
  for (int it = 0; it < total; ++it, (++qbi == nqb) ? (qbi = qb_start, ++h) : 0) {
    const int q0 = qbi * BQ;
    int fs = fs0;
    asm volatile("" : "+v"(fs));
    vm_wait_all();  // prefetch landed on every path (see attn_bwd_kernel)
    __syncthreads();  // previous iteration's readers of Q / dO / dS^T are done
#pragma unroll
    for (int i = 0; i < 2 * QPAIR; i += 2) {
      const int c = tid + NT * (i / 2), row = c / CPR2, col = c % CPR2;
      if (c < BQ * CPR2) {
        if (ROPE == 1 && q0 + row < a.T) {
          const int64_t tab = (int64_t)(q0 + row + off) * (D / 2) + col * 8;
          rope8(qr[i], qr[i + 1], a.rope_cos + tab, a.rope_sin + tab, 1.f);
        }
        I::st_pair(Ql, row, col, qr[i], qr[i + 1]);
        I::st_pair(Ol, row, col, dor[i], dor[i + 1]);
      }
    }
    if (tid < 2 * BQ) {
      const bool live = q0 + (tid & (BQ - 1)) < a.T;
      rowc[tid] = live ? (tid < BQ ? -rc * kLog2e : rc) : 0.f;  // -lse*log2(e), delta
    }
    flush_dq();
    __syncthreads();
    if (it + 1 < total) gload(it + 1);

    // rows past T need no mask (zero-filled Q / dO rows, row constants 0: see attn_bwd_kernel)
    const bool need_mask = (k0 + BK > a.S) || (a.causal && k0 + BK - 1 > q0 + off);
#pragma unroll
    for (int j = 0; j < NQB; ++j) {
      const int qj0 = q0 + 32 * j;
      // causal: the group's keys all after every query of the sub-block -> P = dS = 0
      const bool live = !a.causal || kw0 <= qj0 + 31 + off;
      f32x16 x;
      bf16x8 f0, f1;
      // the packed bf16 P fragments of this group ([half][lane] 16 B: coalesced b128 accesses);
      // buffers alternate by sub-block parity (wave B's reads of sub-block j finish before it
      // reaches barrier j + 1, after which A rewrites the buffer).  B forms dS from this bf16 P,
      // the same rounding of P that the dV product consumes.
      uint32_t* pxj = px + ((j & 1) * C::NG + grp) * 2 * 64 * 4;
      if (live) {
        // S = Q K^T (wave A) or dP = dO V^T (wave B), key on the lane
        const uint16_t* Al = roleA ? Ql : Ol;
        auto chain = [&]() {
          x = zero16();
#pragma unroll
          for (int ks = 0; ks < NKS; ++ks) x = mfma32(as_frag(ld16(Al + 32 * j * D + (fq ^ (ks << 4)))), kvf[ks], x);
        };
        if (!roleA) chain();
        if (roleA) {
          // P = exp2(S c2 - lse log2e); the mask is a compile-time property of the code path (a
          // uniform run-time test per element compiles to a branch per exponential) and each
          // path carries its own MFMA chain (small paths were if-converted into one that always
          // paid the compare + select)
          auto expo = [&](auto mask_c) {
            constexpr bool MASKED = decltype(mask_c)::value;
            chain();
            int lo = 0;
            if constexpr (MASKED) {
              const int key = kw0 + r;
              lo = key >= a.S ? 64 : (a.causal ? key - off - (qj0 + 4 * hh) : -64);
            }
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const f32x4 rs = *reinterpret_cast<const f32x4*>(&rowc[32 * j + 8 * g + 4 * hh]);
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const int i = 4 * g + e;
                float p = fast_exp2(__builtin_fmaf(x[i], c2, rs[e]));
                if constexpr (MASKED) p = acc_row(i, 0) < lo ? 0.f : p;
                x[i] = p;
              }
            }
          };
          // only the group's diagonal sub-block (or a ragged key end) needs the masked path
          if (need_mask && ((kw0 + 32 > a.S) || (a.causal && kw0 + 31 > qj0 + off))) expo(std::true_type{});
          else expo(std::false_type{});
          f0 = pack_frag(x, 0);
          f1 = pack_frag(x, 1);
          *reinterpret_cast<u32x4*>(pxj + lane * 4) = __builtin_bit_cast(u32x4, f0);
          *reinterpret_cast<u32x4*>(pxj + (64 + lane) * 4) = __builtin_bit_cast(u32x4, f1);
        }
      } else if (!roleA) {
#pragma unroll
        for (int k = 0; k < 4; k += 2)
          *reinterpret_cast<u32x4*>(Sl + (fs ^ ((4 * j + k) << 3))) = u32x4{0u, 0u, 0u, 0u};
      }
      __syncthreads();  // P of sub-block j handed over
      if (live) {
        if (!roleA) {
          // dS = P (dP - delta) (unscaled); P read back in the same accumulator layout
          const u32x4 pw[2] = {*reinterpret_cast<const u32x4*>(pxj + lane * 4),
                               *reinterpret_cast<const u32x4*>(pxj + (64 + lane) * 4)};
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4) {
            const f32x4 rd = *reinterpret_cast<const f32x4*>(&rowc[BQ + 32 * j + 8 * q4 + 4 * hh]);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int i = 4 * q4 + e;
              const uint32_t wd = pw[i >> 3][(i & 7) >> 1];
              x[i] = (x[i] - rd[e]) * ((i & 1) ? hi_bf(wd) : lo_bf(wd));
            }
          }
          f0 = pack_frag(x, 0);
          f1 = pack_frag(x, 1);
          // dS^T image from the packed fragments (dwords 2(g&1), 2(g&1)+1 of f[g/2]): group pairs
          // swapped across the half-waves, one 16-B store of 8 consecutive queries per pair
          u32x2 v[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const u32x4 w4 = __builtin_bit_cast(u32x4, g < 2 ? f0 : f1);
            v[g] = u32x2{w4[2 * (g & 1)], w4[2 * (g & 1) + 1]};
          }
#pragma unroll
          for (int k = 0; k < 4; k += 2) {
#pragma unroll
            for (int d = 0; d < 2; ++d) {
              const auto sw = __builtin_amdgcn_permlane32_swap(v[k][d], v[k + 1][d], false, false);
              v[k][d] = sw[0];
              v[k + 1][d] = sw[1];
            }
            *reinterpret_cast<u32x4*>(Sl + (fs ^ ((4 * j + k) << 3))) = u32x4{v[k][0], v[k][1], v[k + 1][0], v[k + 1][1]};
          }
        }
        // dV^T += dO^T P (A) / dK^T += Q^T dS (B): A operands by transposed reads
        const uint16_t* Tl = roleA ? Ol : Ql;
#pragma unroll
        for (int db = 0; db < NDB; ++db) {
#pragma unroll
          for (int st = 0; st < 2; ++st) {
            const int rb = (32 * j + 16 * st) * D;
            const bf16x8 tA = cat_tr(ds_tr(Tl + rb + (ft0 ^ (db << 5))), ds_tr(Tl + rb + (ft8 ^ (db << 5))));
            acc[db] = mfma32(tA, st == 0 ? f0 : f1, acc[db]);
          }
        }
      }
    }
    __syncthreads();
    // dQ partial of this key block: one (query sub-block, d-block) task per wave
#pragma unroll
    for (int ti = 0; ti < NTPW; ++ti) {
      const int task = __builtin_amdgcn_readfirstlane(w) + ti * C::NW;
      if (task >= NTASK) break;
      const int tq_blk = task / NDB, tdb = task % NDB;
      const int qt0 = q0 + 32 * tq_blk;
      if (qt0 >= a.T) continue;  // a query tile past T (ragged last block): no fragment block exists
      // dQ^T tile = K^T dS^T: the accumulator has the QUERY on the lane and 16 head-dim values
      // per lane, dumped as one contiguous 2-KiB fragment-order block (two 16-B stores per lane,
      // coalesced) that attn_dq_reduce_frag_kernel reads back by (query, head-dim) position.
      // Every key step runs (causal steps past the task's queries read zero dS^T rows: see the
      // fused-role kernel), so the LDS reads pipeline ahead of the MFMAs
      f32x16 dqa = zero16();
      const int qc = 32 * tq_blk + 16 * g1 + 4 * tp, dc = tdb * 32 + 16 * g1 + 4 * tp;
      const int sa0 = IS::off(8 * hh + tq, qc), sa4 = IS::off(8 * hh + tq + 4, qc);
      const int ka0 = I::off(8 * hh + tq, dc), ka4 = I::off(8 * hh + tq + 4, dc);
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        const bf16x8 A = cat_tr(ds_tr(Sl + 16 * ks * BQ + sa0), ds_tr(Sl + 16 * ks * BQ + sa4));
        const bf16x8 Bf = cat_tr(ds_tr(Kl + 16 * ks * D + ka0), ds_tr(Kl + 16 * ks * D + ka4));
        dqa = mfma32(Bf, A, dqa);
      }
      float lo[8], hi[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        lo[e] = dqa[e];
        hi[e] = dqa[8 + e];
      }
      dqv[ti][0] = pack8(lo);
      dqv[ti][1] = pack8(hi);
      dqp[ti] = a.dq_acc + (kb - a.kb0) * a.slab +
                ((((int64_t)b * a.H + h) * a.nqt + (qt0 >> 5)) * NDB + tdb) * 1024 + lane * 16;
    }
  }
  flush_dq();
  // dV (wave A) / dK scaled and rotated back (wave B) for this lane's key
  const int key = kw0 + r;
  if (key >= a.S) return;
  if (!roleA && ROPE != 0) {
    const float* cr = a.rope_cos + (int64_t)key * (D / 2);
    const float* sr = a.rope_sin + (int64_t)key * (D / 2);
#pragma unroll
    for (int db = 0; db < NDB / 2; ++db)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int d = db * 32 + 8 * (i >> 2) + 4 * hh + (i & 3);
        const float c = cr[d], sn = sr[d];
        const float x0 = acc[db][i], y0 = acc[db + NDB / 2][i];
        acc[db][i] = x0 * c + y0 * sn;
        acc[db + NDB / 2][i] = y0 * c - x0 * sn;
      }
  }
  const float sc = roleA ? 1.f : a.scale;
  uint16_t* dst = roleA ? a.dv + b * a.dv_sb + (int64_t)key * a.dv_st + (int64_t)hk * a.dv_sh
                        : a.dk + b * a.dk_sb + (int64_t)key * a.dk_st + (int64_t)hk * a.dk_sh;
  store_row_bf16<NDB>(dst, acc, sc, hh);
}

// Reduce of the backward kernels' fragment-order dQ slabs.  One workgroup (64 x D/32 threads) per
// 32-query tile of one (batch, head): thread (d-block blk, lane l) reads its 32 contiguous bytes of
// the tile's block blk from every slab of the pass (coalesced 2-KiB wave reads; lane l holds query
// l%32 and head dims blk*32 + acc_row(i, l/32), i < 16), sums them in key-block order
// (deterministic) into the fp32 running sum (kept in the same fragment order) or, on the last
// pass, transposes the tile through LDS and writes dq = scale * total as whole 16-B row chunks,
// rotated back with RoPE (each thread holds a dim chunk and its d + D/2 partner).
template <int D, int BK, int ROPE>
__global__ __launch_bounds__(256) void attn_dq_reduce_frag_kernel(AttnBwdArgs a) {
  constexpr int NDB = D / 32, NTH = 64 * NDB, LD = D + 4;  // LD: padded fp32 row of the LDS tile
  __shared__ float tile[32 * LD];
  const int tid = threadIdx.x, blk = tid >> 6, lane = tid & 63, hh = lane >> 5;
  const int64_t bhq = blockIdx.x;  // (b * H + h) * nqt + qt
  const int qt = (int)(bhq % a.nqt);
  const int64_t bh = bhq / a.nqt;
  const int h = (int)(bh % a.H), b = (int)(bh / a.H);
  const int q = qt * 32 + (lane & 31);
  const int nkb = (a.S + BK - 1) / BK;
  int kmax = min(nkb - 1, a.kb0 + a.nkb_pass - 1);
  if (a.causal) kmax = min(kmax, (min(q, a.T - 1) + a.S - a.T) / BK);
  const int64_t e0 = (bhq * NDB + blk) * 1024 + lane * 16;
  float f[16];
  if (a.kb0 > 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) f[i] = a.dq_sum[e0 + i];
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) f[i] = 0.f;
  }
  // four slabs' loads in flight before their adds (the adds keep key-block order: deterministic); one
  // slab per trip left each thread one memory round trip per key block (2.9 TB/s at the llama shape)
  int kb = a.kb0;
  for (; kb + 3 <= kmax; kb += 4) {
    u32x4 v[4][2];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint16_t* p = a.dq_acc + (kb + u - a.kb0) * a.slab + e0;
      v[u][0] = ld16(p);
      v[u][1] = ld16(p + 8);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float x[8], y[8];
      unpack8(v[u][0], x);
      unpack8(v[u][1], y);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        f[i] += x[i];
        f[8 + i] += y[i];
      }
    }
  }
  for (; kb <= kmax; ++kb) {
    const uint16_t* p = a.dq_acc + (kb - a.kb0) * a.slab + e0;
    float x[8], y[8];
    unpack8(ld16(p), x);
    unpack8(ld16(p + 8), y);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      f[i] += x[i];
      f[8 + i] += y[i];
    }
  }
  if (a.kb0 + a.nkb_pass < nkb) {  // more passes follow: running sum in fragment order
#pragma unroll
    for (int i = 0; i < 16; ++i) a.dq_sum[e0 + i] = f[i];
    return;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) tile[(lane & 31) * LD + blk * 32 + acc_row(i, hh)] = f[i] * a.scale;
  __syncthreads();
  // write-out: 32 rows x D/16 chunk pairs (chunk c and its RoPE partner c + D/16), 8 dims each
  constexpr int CP = D / 16;
  for (int it = tid; it < 32 * CP; it += NTH) {
    const int row = it / CP, c = it % CP, qq = qt * 32 + row;
    if (qq >= a.T) continue;
    float lo[8], hi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      lo[e] = tile[row * LD + 8 * c + e];
      hi[e] = tile[row * LD + D / 2 + 8 * c + e];
    }
    if (ROPE != 0) {  // R^T: (x, y) at dims (d, d + D/2) -> (x c + y s, y c - x s)
      const int64_t tab = (int64_t)(qq + a.S - a.T) * (D / 2) + 8 * c;
      const f32x4* cp = reinterpret_cast<const f32x4*>(a.rope_cos + tab);
      const f32x4* sp = reinterpret_cast<const f32x4*>(a.rope_sin + tab);
      const f32x4 c0 = cp[0], c1 = cp[1], s0 = sp[0], s1 = sp[1];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float cs = e < 4 ? c0[e & 3] : c1[e & 3], sn = e < 4 ? s0[e & 3] : s1[e & 3];
        const float x0 = lo[e], y0 = hi[e];
        lo[e] = x0 * cs + y0 * sn;
        hi[e] = y0 * cs - x0 * sn;
      }
    }
    uint16_t* dq = a.dq + b * a.dq_sb + (int64_t)qq * a.dq_st + (int64_t)h * a.dq_sh;
    st16(dq + 8 * c, pack8(lo));
    st16(dq + D / 2 + 8 * c, pack8(hi));
  }
}

}  // namespace

namespace pllm {

bool attn_supported_head_dim(int D) { return D == 32 || D == 64 || D == 128; }

// key-stationary backward (attn_bwd_ks.hip) per head dim, a bit mask (1: D = 64, 2: D = 128): initial
// value from PLLM_ATTN_BWD_KS (comma list of head dims, default "128"), runtime A/B via attn_bwd_set_ks
static int g_attn_ks = -1;
static bool attn_bwd_ks(int D) {
  if (g_attn_ks < 0) {
    const char* e = std::getenv("PLLM_ATTN_BWD_KS");
    const char* v = e ? e : "128";
    g_attn_ks = (std::strstr(v, "64") ? 1 : 0) | (std::strstr(v, "128") ? 2 : 0);
  }
  return (D == 64 && (g_attn_ks & 1)) || (D == 128 && (g_attn_ks & 2));
}
void attn_bwd_set_ks(int mask) { g_attn_ks = mask & 3; }

int attn_bwd_key_block(int D) {
  if (attn_bwd_ks(D)) return attn_bwd_ks_key_block();
  return D == 128 ? RsCfg<128>::BK : BwdCfg<64>::BK;
}
bool attn_bwd_uses_ks(int D) { return attn_bwd_ks(D); }

template <int D>
static void attn_fwd_t(const AttnFwdArgs& a, hipStream_t st) {
  const int nqb = (a.T + FwdCfg<D>::BM - 1) / FwdCfg<D>::BM;
  const dim3 grid(nqb * a.B * a.H), blk(64 * FwdCfg<D>::NW);
  if (a.rope_cos) hipLaunchKernelGGL((attn_fwd_kernel<D, true>), grid, blk, 0, st, a);
  else hipLaunchKernelGGL((attn_fwd_kernel<D, false>), grid, blk, 0, st, a);
}

template <int D, int ROPE>
static void attn_bwd_t(AttnBwdArgs a, hipStream_t st) {
  const int64_t nrows = (int64_t)a.B * a.T * a.H;
  const int pre_grid = (int)((nrows * (D / 8) + 255) / 256);
  const int nkb = (a.S + BwdCfg<D>::BK - 1) / BwdCfg<D>::BK;
  if (!a.delta_ready) hipLaunchKernelGGL(attn_bwd_pre_kernel<D>, dim3(pre_grid), dim3(256), 0, st, a);
  // key blocks in passes of at most a.nkb_pass (bounded slab workspace)
  const int per = a.nkb_pass;
  for (int kb0 = 0; kb0 < nkb; kb0 += per) {
    a.kb0 = kb0;
    a.nkb_pass = min(per, nkb - kb0);
    hipLaunchKernelGGL((attn_bwd_kernel<D, ROPE>), dim3(a.nkb_pass * a.B * a.Hkv), dim3(BwdCfg<D>::NT), 0, st,
                       a);
    hipLaunchKernelGGL((attn_dq_reduce_frag_kernel<D, BwdCfg<D>::BK, ROPE>), dim3(a.B * a.H * a.nqt),
                       dim3(64 * (D / 32)), 0, st, a);
    a.nkb_pass = per;
  }
}

// RoPE mode: 0 none, 1 rotate q / k inputs and dq / dk outputs, 2 inputs already rotated (the
// caller's pre-pass), rotate the outputs back only
template <int D>
static void attn_bwd_r(const AttnBwdArgs& a, hipStream_t st) {
  if (!a.rope_cos) attn_bwd_t<D, 0>(a, st);
  else if (a.rope_in) attn_bwd_t<D, 1>(a, st);
  else attn_bwd_t<D, 2>(a, st);
}

void attn_fwd(const AttnFwdArgs& a, hipStream_t st) {
  if (a.D == 32) attn_fwd_t<32>(a, st);
  else if (a.D == 64) attn_fwd_t<64>(a, st);
  else attn_fwd_t<128>(a, st);
}

template <int D, int ROPE>
static void attn_bwd_rs_t(AttnBwdArgs a, hipStream_t st) {
  using C = RsCfg<D>;
  const int64_t nrows = (int64_t)a.B * a.T * a.H;
  const int pre_grid = (int)((nrows * (D / 8) + 255) / 256);
  const int nkb = (a.S + C::BK - 1) / C::BK;
  const int red_grid = a.B * a.H * a.nqt;  // one workgroup per 32-query tile
  if (!a.delta_ready) hipLaunchKernelGGL(attn_bwd_pre_kernel<D>, dim3(pre_grid), dim3(256), 0, st, a);
  const int per = a.nkb_pass;
  for (int kb0 = 0; kb0 < nkb; kb0 += per) {
    a.kb0 = kb0;
    a.nkb_pass = min(per, nkb - kb0);
    hipLaunchKernelGGL((attn_bwd_rs_kernel<D, ROPE>), dim3(a.nkb_pass * a.B * a.Hkv), dim3(C::NT), 0, st, a);
    hipLaunchKernelGGL((attn_dq_reduce_frag_kernel<D, C::BK, ROPE>), dim3(red_grid), dim3(64 * (D / 32)), 0, st, a);
    a.nkb_pass = per;
  }
}

template <int D>
static void attn_bwd_rs_r(const AttnBwdArgs& a, hipStream_t st) {
  if (!a.rope_cos) attn_bwd_rs_t<D, 0>(a, st);
  else if (a.rope_in) attn_bwd_rs_t<D, 1>(a, st);
  else attn_bwd_rs_t<D, 2>(a, st);
}

// key-stationary backward (attn_bwd_ks.hip): per pass of key blocks the main kernel (delta formed
// inside it) and the ordered slab reduce
template <int D>
static void attn_bwd_ks_t(AttnBwdArgs a, hipStream_t st) {
  const int64_t nrows = (int64_t)a.B * a.T * a.H;
  const int pre_grid = (int)((nrows * (D / 8) + 255) / 256);
  const int BK = attn_bwd_ks_key_block();
  const int nkb = (a.S + BK - 1) / BK;
  const int red_grid = a.B * a.H * a.nqt;  // one workgroup per 32-query tile
  // delta = rowsum(dO O) pre-pass (skipped when the caller already holds it)
  if (!a.delta_ready)
    hipLaunchKernelGGL(attn_bwd_pre_kernel<D>, dim3(pre_grid), dim3(256), 0, st, a);
  const int per = a.nkb_pass;
  for (int kb0 = 0; kb0 < nkb; kb0 += per) {
    a.kb0 = kb0;
    a.nkb_pass = min(per, nkb - kb0);
    attn_bwd_ks_launch(a, st);
    if (a.rope_cos) hipLaunchKernelGGL((attn_dq_reduce_frag_kernel<D, 256, 2>), dim3(red_grid), dim3(64 * (D / 32)), 0, st, a);
    else hipLaunchKernelGGL((attn_dq_reduce_frag_kernel<D, 256, 0>), dim3(red_grid), dim3(64 * (D / 32)), 0, st, a);
    a.nkb_pass = per;
  }
}

// D = 32 / 64: fused-role kernel; D = 128: role-split kernel; the key-stationary kernel where
// attn_bwd_ks(D) (q / k pre-rotated: the binding rotates them first when rope_in is set)
void attn_bwd(const AttnBwdArgs& a, hipStream_t st) {
  if (attn_bwd_ks(a.D) && !(a.rope_cos && a.rope_in)) {
    if (a.D == 64) attn_bwd_ks_t<64>(a, st);
    else attn_bwd_ks_t<128>(a, st);
    return;
  }
  if (a.D == 32) attn_bwd_r<32>(a, st);
  else if (a.D == 64) attn_bwd_r<64>(a, st);
  else attn_bwd_rs_r<128>(a, st);
}

}  // namespace pllm

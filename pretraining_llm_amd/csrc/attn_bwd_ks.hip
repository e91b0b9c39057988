// Key-stationary causal flash-attention backward for gfx950 (round 5; D = 64 / 128), replacing the
// role-split D = 128 kernel of attention.hip.  Reference math: /root/reference/src/models/attention.py:47-57
// (q k^T * hd^-1/2, causal masked_fill, softmax, @ v), whose backward this is.
//
// Register-class discipline (the reason this file exists apart from attention.hip): every MFMA is an
// inline-asm statement with an explicit register class -- the dK^T / dV^T accumulators ("+a") own
// the 256 AGPRs, the S / dP / dQ chains ("+v") the arch VGPRs.  Left to itself hipcc put the S and dQ
// accumulators into AGPRs, pushed dK / dV into VGPRs and spilled 400-1000 registers at D = 128, or
// copied all 256 accumulators between the two files at every join of the per-case code paths.
// Hazards the compiler does not pad for asm (cdna_hip_programming.md §5.7): each MFMA statement opens
// with s_nop 1 (a VALU-written A / B / C operand; free while the previous MFMA occupies the pipe), an
// accumulate chain into the same C needs nothing, and mfma_settle() (18 wait states, taking the
// result as an operand so every consumer is ordered after it) precedes any non-MFMA reader.
#include <type_traits>

#ifndef PLLM_BWD_STAMPS
#define PLLM_BWD_STAMPS 0  // diagnostic: per-phase s_memtime sums (scripts/build_variant.py -DPLLM_BWD_STAMPS=1)
#endif

#include "attn_common.h"
#include "common.h"
#include "kernels.h"

#ifndef PL_KS_DQ_KREG
#define PL_KS_DQ_KREG 4  // dQ-task K^T fragments held in registers (key steps 0..PL_KS_DQ_KREG-1 of 16)
#endif

namespace {

// ---------------------------------------------------------------------------
// Key-stationary backward ("KS", round 5; D = 64 / 128): one workgroup = 4 waves, ONE per SIMD
// (512 registers each) = 256 keys of one (batch, kv-head).  Wave w owns keys k0 + 64 w + [0, 64) as
// two 32-key blocks and keeps, across the whole sweep over the query slices of every query head of
// the group, their dK^T / dV^T accumulators (D = 128: 256 registers) and their V rows as MFMA B
// fragments in registers; K lives in one LDS image (S's B fragments by row reads, dQ's A operand by
// transposed reads).  A slice is BQ = 128 / NDB queries (D = 128: 32, D = 64: 64), so the slice's dQ
// tile is exactly 4 tasks of 32 queries x 32 head dims: one per wave, summed over all 256 keys
// (16 MFMAs) from the slice's dS^T image and stored as one bf16 fragment block per key block (the
// same slab format as the other kernels, reduced by attn_dq_reduce_frag_kernel<D, 256>).
// vs the role-split kernel it replaces at D = 128 (128 keys, 8 waves, P handed between wave pairs
// through LDS behind a barrier per 32-query sub-block, Q / dO staged through registers): ONE barrier
// per slice (double-buffered Q / dO / dS^T images and row constants: the next slice's Q / dO DMA is
// issued right after the barrier and waited just before the next one), half the dQ slab bytes
// (256-key blocks), no P hand-off, and every Q / dO / K fragment read feeds both key blocks.
// Guide: cdna_hip_programming.md Appendix B 'Attention backward' (key on the lane, row constants as
// the initial accumulator, one LDS image per operand for row and transposed reads).
template <int D>
struct KsCfg {
  static_assert(D == 64 || D == 128, "key-stationary backward: D = 64 / 128");
  static constexpr int NW = 4, NT = 256, BK = 256;
  static constexpr int NDB = D / 32, NKS = D / 16;
  static constexpr int NQB = 4 / NDB;        // 32-query sub-blocks per slice (one dQ task per wave)
  static constexpr int BQ = 32 * NQB;        // queries per slice
  static constexpr int CPR = D / 8;          // 16-B chunks per row
  static constexpr int QRP = 512 / D;        // rows per 1-KiB DMA piece
  static constexpr int QNP = BQ / QRP;       // pieces per Q (or dO) tile
  static constexpr int PPI = QNP / NW;       // pieces per image and wave: wave w moves rows [w, w+1) BQ/4
  static constexpr int QPPW = 2 * PPI;      // Q + dO pieces per wave and slice
  static constexpr int KPPW = BK / QRP / NW; // K image pieces per wave
  static constexpr int TILE = BQ * D;        // elements of one Q (dO) tile
  static constexpr int SIMG = BK * BQ;       // elements of one dS^T image [keys][BQ]
  static constexpr int LDS_ELEMS = BK * D + 4 * TILE + 2 * SIMG;  // 136 KiB at D = 64 and 128
};

// dS^T image [256 keys][W = BQ queries] of the KS kernel: chunk ch (16 B) of row r at ch ^ f(r).
// Stores: 16 B per lane, 8 consecutive key rows per 8-lane group at one logical chunk -> f is a
// bijection on 8 consecutive rows modulo the 128-B bank window.  Transposed dQ reads: 4 consecutive
// rows x the sub-block's 64 B; W = 32: 4 rows = 256 contiguous bytes (any f); W = 64: rows r and r+2
// share banks, so f(r) ^ f(r + 2) has bit 2 set.  f depends on row bits 0..2 only: +16-row steps are
// plain additions.
template <int W>
struct ImgT {
  static PL_DEV int f(int r) {
    if constexpr (W == 32) return (r >> 1) & 3;
    else return (((r >> 1) & 1) << 2) | ((r & 1) << 1) | ((r >> 2) & 1);
  }
  static PL_DEV int off(int r, int col) { return r * W + (((col >> 3) ^ f(r)) << 3) + (col & 7); }
};

template <int D, int ROPE>
__global__ __launch_bounds__(256, 1) void attn_bwd_ks_kernel(AttnBwdArgs a) {
  static_assert(ROPE != 1, "KS backward: q / k pre-rotated (ROPE 0 or 2)");
  using C = KsCfg<D>;
  using I = Img<D>;
  using IT = ImgT<C::BQ>;
  constexpr int BK = C::BK, BQ = C::BQ, NQB = C::NQB, NKS = C::NKS, NDB = C::NDB, CPR = C::CPR;
  constexpr int TILE = C::TILE, SIMG = C::SIMG, QRP = C::QRP, QNP = C::QNP, QPPW = C::QPPW;
  __shared__ __attribute__((aligned(1024))) uint16_t smem[C::LDS_ELEMS];
  // row constants per slot, LDS-DMA'd (64 lanes x 4 B: padded to 64): raw lse and delta = rowsum(dO O)
  // of the slice's rows.  delta comes from attn_bwd_pre_kernel: forming it in this kernel (dO / O rows
  // DMA'd beside Q / dO, fp32 FMAs beside the dQ MFMAs) measured 1212 us vs 1106 us for pre-pass +
  // kernel at 16x16x2048x128 (r5 A/B) -- the unpack + FMA VALU work lands on the MFMA-bound phases
  __shared__ __attribute__((aligned(16))) float lsec[2][64];
  __shared__ __attribute__((aligned(16))) float rowc[2][64];
  uint16_t* const Kl = smem;
  uint16_t* const QOl = smem + BK * D;  // slot s: Q tile at QOl + 2 s TILE, dO tile right after
  uint16_t* const Sl = QOl + 4 * TILE;  // slot s: dS^T image at Sl + s SIMG

  const int BH = a.B * a.Hkv;
  const int id = blockIdx.x;
  const int kb = a.kb0 + id / BH;  // lowest key blocks (longest causal sweeps) of every head first
  const int bh = id % BH;
  const int b = bh / a.Hkv, hk = bh % a.Hkv;
  const int G = a.H / a.Hkv;
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int k0 = kb * BK, kw0 = k0 + 64 * w;
  const int off = a.S - a.T;
  const unsigned lds0 = (unsigned)(uintptr_t)smem;
  const uint16_t* kp = a.k + b * a.k_sb + (int64_t)hk * a.k_sh;
  const uint16_t* vp = a.v + b * a.v_sb + (int64_t)hk * a.v_sh;

  // ---- sweep bounds: (query head of the group, BQ-query slice), causal slices from the key block on
  const int nqs = (a.T + BQ - 1) / BQ;
  const int qs_start = a.causal ? max(0, k0 - off) / BQ : 0;
  const int per_head = max(0, nqs - qs_start);
  const int total = per_head * G;

  // ---- K image by LDS DMA (lane l of piece p fills row p QRP + l / CPR at chunk position l % CPR,
  // which holds logical chunk (l % CPR) ^ f(row): the swizzle applied to the source); keys past S
  // read zeros (descriptor range)
  {
    const int rows = min(BK, a.S - k0);
    const i32x4v ks = srd_of(kp + (int64_t)k0 * a.k_st, (uint32_t)(((int64_t)(rows - 1) * a.k_st + D) * 2));
#pragma unroll
    for (int k = 0; k < C::KPPW; ++k) {
      const int p = w * C::KPPW + k, row = p * QRP + lane / CPR, ch = (lane % CPR) ^ I::f(row);
      blds16(ks, (uint32_t)((row * a.k_st + 8 * ch) * 2), lds0 + 1024u * (unsigned)p);
    }
  }
  // ---- Q / dO DMA of slice it into slot sl (k = img PPI + m: image img = Q, dO, piece w PPI + m)
  uint32_t qvo[QPPW];
#pragma unroll
  for (int k = 0; k < QPPW; ++k) {
    const int img = k / C::PPI, blk = w * C::PPI + k % C::PPI;
    const int row = blk * QRP + lane / CPR, ch = (lane % CPR) ^ I::f(row);
    const int64_t st = img == 0 ? a.q_st : a.do_st;
    qvo[k] = (uint32_t)((row * st + 8 * ch) * 2);
  }
  auto slice_of = [&](int it, int& h, int& q0) {
    h = hk * G + it / per_head;
    q0 = (qs_start + it % per_head) * BQ;
  };
  auto qdma = [&](int it, int sl) {
    int h, q0;
    slice_of(it, h, q0);
    const int rows = a.T - q0;
    const i32x4v qs = srd_of(a.q + b * a.q_sb + (int64_t)h * a.q_sh + (int64_t)q0 * a.q_st,
                             (uint32_t)(((int64_t)(rows - 1) * a.q_st + D) * 2));
    const i32x4v os = srd_of(a.dO + b * a.do_sb + (int64_t)h * a.do_sh + (int64_t)q0 * a.do_st,
                             (uint32_t)(((int64_t)(rows - 1) * a.do_st + D) * 2));
#pragma unroll
    for (int k = 0; k < QPPW; ++k) {
      const int img = k / C::PPI, blk = w * C::PPI + k % C::PPI;  // wave-uniform
      const unsigned dst = (unsigned)(BK * D + 2 * sl * TILE + img * TILE);
      blds16(img == 0 ? qs : os, qvo[k], lds0 + 2u * dst + 1024u * blk);
    }
  };
  // row constants of slice it by LDS DMA (buffer_load_dword ... lds, one wave each, lane l -> row q0 + l;
  // rows past T read zeros): no register round trip, so no compiler-inserted vmcnt(0) in front of a
  // register use (it waited out the previous slice's dQ stores too)
  auto rload = [&](int it) {
    int h, q0;
    slice_of(it, h, q0);
    const int64_t row0 = ((int64_t)b * a.H + h) * a.T + q0;
    if (w == 0) {
      const i32x4v srd = srd_of(a.lse + row0, (uint32_t)(a.T - q0) * 4u);
      blds4(srd, (uint32_t)lane * 4u, (unsigned)(uintptr_t)&lsec[it & 1][0]);
    } else if (w == 1) {
      const i32x4v srd = srd_of(a.delta + row0, (uint32_t)(a.T - q0) * 4u);
      blds4(srd, (uint32_t)lane * 4u, (unsigned)(uintptr_t)&rowc[it & 1][0]);
    }
  };

  // ---- V rows of this wave's keys as B fragments (k = head dim), zero past S
  bf16x8 vf[2][NKS];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) {
    const int key = kw0 + 32 * kh + r;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
      vf[kh][ks] = key < a.S ? as_frag(ld16(vp + (int64_t)key * a.v_st + 16 * ks + 8 * hh)) : zero_frag();
  }
  if (total > 0) {
    qdma(0, 0);
    rload(0);
    if (total > 1) {
      qdma(1, 1);
      rload(1);  // before the wait below: the first hand-off's vmcnt(2) has no dQ stores to skip
    }
  }
  vm_wait_all();
  __syncthreads();  // K image, slice 0 (and its row constants) landed for every wave

  f32x16 dk[2][NDB], dv[2][NDB];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh)
#pragma unroll
    for (int db = 0; db < NDB; ++db) {
      dk[kh][db] = zero16();
      dv[kh][db] = zero16();
    }
  const float c2 = a.scale_log2;
  const int g1 = (lane >> 4) & 1, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;
  // per-lane LDS element offsets, swizzle applied once (see attn_bwd_kernel): row fragment reads
  // fq ^ (ks << 4) + row-block base, transposed reads ft0 / ft8 ^ (db << 5) + (32 j + 16 st) D
  const int fq0 = I::off(r, 8 * hh);
  const int ft00 = I::off(4 * hh + tq, 16 * g1 + 4 * tp), ft80 = I::off(4 * hh + tq + 8, 16 * g1 + 4 * tp);
  const bool aligned = (off & 31) == 0 && kw0 + 64 <= a.S;
  // dQ task of this wave: (32-query sub-block, 32-dim block)
  const int tq_blk = w / NDB, tdb = w % NDB;
  const int qc = 32 * tq_blk + 16 * g1 + 4 * tp, dc = 32 * tdb + 16 * g1 + 4 * tp;
  const int sa00 = IT::off(8 * hh + tq, qc), sa40 = IT::off(8 * hh + tq + 4, qc);
  const int ka00 = I::off(8 * hh + tq, dc), ka40 = I::off(8 * hh + tq + 4, dc);
  // the dQ task's K^T fragments of key steps 0..PL_KS_DQ_KREG-1 in registers: the K block and the wave's d-block
  // are fixed, so these reads would repeat every slice (the dQ phase runs at the LDS read roof)
  bf16x8 kdq[PL_KS_DQ_KREG > 0 ? PL_KS_DQ_KREG : 1];
#pragma unroll
  for (int ks = 0; ks < PL_KS_DQ_KREG; ++ks) kdq[ks] = cat_tr(ds_tr(Kl + 16 * ks * D + ka00), ds_tr(Kl + 16 * ks * D + ka40));

#if PLLM_BWD_STAMPS
  // diagnostic build: per-wave s_memtime sums of the slice phases (host: PLLM_BWD_STAMPS=1 prints them)
  uint64_t st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t st_start = __builtin_amdgcn_s_memtime();
  uint64_t ts_prev = st_start;
  auto stamp = [&](int i) {
    const uint64_t now = __builtin_amdgcn_s_memtime();
    st_acc[i] += now - ts_prev;
    ts_prev = now;
  };
#define KS_STAMP(i) stamp(i)
#else
#define KS_STAMP(i)
#endif
  int h = hk * G, qi = qs_start;  // (head, slice) of iteration it, advanced incrementally
  for (int it = 0; it < total; ++it, (++qi == nqs) ? (qi = qs_start, ++h) : 0) {
    const int sl = it & 1;
    const int q0 = qi * BQ;
    // per-lane offsets made opaque per slice: the XOR-swizzled addresses derived from them are then
    // formed next to their reads instead of being hoisted out of the loop as ~50 live registers
    int fq = fq0, ft0 = ft00, ft8 = ft80, sa0 = sa00, sa4 = sa40, ka0 = ka00, ka4 = ka40;
    asm volatile("" : "+v"(fq), "+v"(ft0), "+v"(ft8), "+v"(sa0), "+v"(sa4), "+v"(ka0), "+v"(ka4));
    const uint16_t* Ql = QOl + 2 * sl * TILE;
    const uint16_t* Ol = Ql + TILE;
    const float* rl = rowc[sl];
    const float* ll = lsec[sl];
    uint16_t* Sd = Sl + sl * SIMG;
#pragma unroll
    for (int j = 0; j < NQB; ++j) {
      const int qj0 = q0 + 32 * j;
      // Software-pipelined sub-block: the wave's two key blocks (kb 0, 1) run staggered so that each
      // MFMA chain has the other block's VALU work beside it -- with one wave per SIMD nothing else
      // would fill the matrix pipe during the softmax:
      //   A: S0 / dP0 chains (16 MFMAs)
      //   B: S1 / dP1 chains          || P0 = exp2(S0 c2 - lse log2 e), dS0 = P0 (dP0 - delta), packs
      //   C: dV0 / dK0 (16 MFMAs)     || P1, dS1, packs
      //   D: dV1 / dK1 (16 MFMAs)     || dS^T image rows of both blocks
      // Each step is a run of (LDS reads one step ahead, 2 MFMAs, a slice of the other block's VALU)
      // groups fenced by sched_barrier, so hipcc neither clusters the MFMAs nor hoists the reads.
      // Masking (causal diagonal, ragged key end, unaligned offset) is folded into the S chains'
      // initial accumulators (0 or -inf per element: p = exp2(-inf) = 0), set up behind ONE wave-uniform
      // branch before the straight-line steps; a sub-block whose keys all follow its queries is fully
      // masked rather than skipped (one wave per SIMD: a skip saves no wall time, and a branch around
      // the dK / dV updates made hipcc copy the 256 accumulators at the join).
      const bool mask_j = !aligned || (a.causal && kw0 + 63 > qj0 + off);  // wave-uniform
      f32x16 s0, s1, d0, d1;
      if (mask_j) {
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
          const int key = kw0 + 32 * kh + r;
          const int lo = key >= a.S ? 64 : (a.causal ? key - off - (qj0 + 4 * hh) : -64);
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float mv = acc_row(i, 0) < lo ? -INFINITY : 0.f;
            if (kh == 0) s0[i] = mv;
            else s1[i] = mv;
          }
        }
      } else {
        s0 = zero16();
        s1 = zero16();
      }
      float rs[16];  // -lse log2(e) of the lane's 16 query rows
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(&ll[32 * j + 8 * g + 4 * hh]);
        const f32x4 y = *reinterpret_cast<const f32x4*>(&rl[32 * j + 8 * g + 4 * hh]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          rs[4 * g + e] = -kLog2e * x[e];
          d0[4 * g + e] = -y[e];  // dP accumulated onto -delta
        }
      }
      d1 = d0;
      __builtin_amdgcn_sched_barrier(0);
      KS_STAMP(7);
      // fragment reads of the S / dP chains: Q, dO rows of the sub-block and K rows of key block KH
      auto rd_sd = [&](int KH, int ks, bf16x8& qa, bf16x8& oa, bf16x8& kf) {
        const int fo = fq ^ (ks << 4);
        qa = as_frag(ld16(Ql + 32 * j * D + fo));
        oa = as_frag(ld16(Ol + 32 * j * D + fo));
        kf = as_frag(ld16(Kl + (64 * w + 32 * KH) * D + fo));
      };
      // transposed A operands of the dV / dK updates, step t = (db, st)
      auto rd_tr = [&](int t, bf16x8& oA, bf16x8& qA) {
        const int db = t >> 1, st = t & 1;
        const int rb = (32 * j + 16 * st) * D, o0 = rb + (ft0 ^ (db << 5)), o8 = rb + (ft8 ^ (db << 5));
        oA = cat_tr(ds_tr(Ol + o0), ds_tr(Ol + o8));
        qA = cat_tr(ds_tr(Ql + o0), ds_tr(Ql + o8));
      };
      // softmax slice of one key block: elements [i0, i0 + n) of P = exp2(S c2 + rs), dS = P dP
      auto sm = [&](f32x16& sc, f32x16& dp, int i0, int n) {
#pragma unroll
        for (int i = i0; i < i0 + n; ++i) {
          const float pv = fast_exp2(__builtin_fmaf(sc[i], c2, rs[i]));
          sc[i] = pv;
          dp[i] = pv * dp[i];
        }
      };
      constexpr int NT2 = 2 * NDB;  // (db, st) steps of a dV / dK update
      constexpr int EPS = 16 / NKS;  // softmax elements per step of the S / dP chains
      constexpr int EPT = 16 / NT2;  // ... per step of the dV / dK updates
      // LDS reads run TWO steps ahead of their MFMAs (3-deep register rings; one step = 2 MFMAs = 64
      // cycles did not cover the read latency under load: WAIT_ANY 38 % of wave cycles)
      constexpr int RA = 2;
      bf16x8 qa[RA + 1], oa[RA + 1], kf[RA + 1];
      auto rd_u = [&](int u) {  // S / dP step u of the A-then-B sequence: key block u / NKS, ks u % NKS
        rd_sd(u / NKS, u % NKS, qa[u % (RA + 1)], oa[u % (RA + 1)], kf[u % (RA + 1)]);
      };
#pragma unroll
      for (int u = 0; u < RA; ++u) rd_u(u);
      // ---- A: S0 / dP0
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        rd_u(ks + RA);
        const int c = ks % (RA + 1);
        if (ks == 0) {
          mfma_v<true>(s0, qa[c], kf[c]);  // s0 / d0: VALU-initialised (mask / -delta)
          mfma_v<true>(d0, oa[c], vf[0][ks]);
        } else {
          mfma_v(s0, qa[c], kf[c]);
          mfma_v(d0, oa[c], vf[0][ks]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      KS_STAMP(0);
      // ---- B: S1 / dP1 || softmax of block 0
      bf16x8 pf0[2], sf0[2];
      bf16x8 oA[RA + 1], qA[RA + 1];
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const int u = NKS + ks;
        if (u + RA < 2 * NKS) rd_u(u + RA);
        else rd_tr((u + RA - 2 * NKS) % NT2, oA[(u + RA - 2 * NKS) % (RA + 1)], qA[(u + RA - 2 * NKS) % (RA + 1)]);
        const int c = u % (RA + 1);
        if (ks == 0) {
          mfma_v<true>(s1, qa[c], kf[c]);
          mfma_v<true>(d1, oa[c], vf[1][ks]);
        } else {
          mfma_v(s1, qa[c], kf[c]);
          mfma_v(d1, oa[c], vf[1][ks]);
        }
        if (ks == 0) mfma_settle(s0, d0);  // block 0's chains done (behind this step's MFMAs)
        sm(s0, d0, EPS * ks, EPS);
        if ((EPS * (ks + 1)) % 8 == 0) {  // 8 elements done: one packed fragment pair
          const int h8 = EPS * (ks + 1) / 8 - 1;
          pf0[h8] = pack_frag(s0, h8);
          sf0[h8] = pack_frag(d0, h8);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      KS_STAMP(1);
      // ---- C: dV0 / dK0 || softmax of block 1   (transposed-read step v of the C-then-D sequence)
      bf16x8 pf1[2], sf1[2];
#pragma unroll
      for (int t = 0; t < NT2; ++t) {
        const int v = t;
        rd_tr((v + RA) % NT2, oA[(v + RA) % (RA + 1)], qA[(v + RA) % (RA + 1)]);
        const int c = v % (RA + 1);
        mfma_a(dv[0][t >> 1], oA[c], pf0[t & 1]);
        mfma_a(dk[0][t >> 1], qA[c], sf0[t & 1]);
        if (t == 0) mfma_settle(s1, d1);
        sm(s1, d1, EPT * t, EPT);
        if ((EPT * (t + 1)) % 8 == 0) {
          const int h8 = EPT * (t + 1) / 8 - 1;
          pf1[h8] = pack_frag(s1, h8);
          sf1[h8] = pack_frag(d1, h8);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      KS_STAMP(2);
      // ---- D: dV1 / dK1 || dS^T image rows of both key blocks (group pairs of 4 queries swapped
      // across the half-waves by v_permlane32_swap: one 16-B store of 8 consecutive queries per pair)
      auto ds_store = [&](int KH, const bf16x8 (&sf)[2], int k) {
        u32x2 v0, v1;
        {
          const u32x4 w4 = __builtin_bit_cast(u32x4, sf[k >> 1]);
          v0 = u32x2{w4[0], w4[1]};
          v1 = u32x2{w4[2], w4[3]};
        }
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const auto sw = __builtin_amdgcn_permlane32_swap(v0[d], v1[d], false, false);
          v0[d] = sw[0];
          v1[d] = sw[1];
        }
        *reinterpret_cast<u32x4*>(Sd + IT::off(64 * w + 32 * KH + r, 32 * j + 8 * k + 8 * hh)) =
            u32x4{v0[0], v0[1], v1[0], v1[1]};
      };
#pragma unroll
      for (int t = 0; t < NT2; ++t) {
        const int v = NT2 + t;
        if (v + RA < 2 * NT2) rd_tr((v + RA) % NT2, oA[(v + RA) % (RA + 1)], qA[(v + RA) % (RA + 1)]);
        const int c = v % (RA + 1);
        mfma_a(dv[1][t >> 1], oA[c], pf1[t & 1]);
        mfma_a(dk[1][t >> 1], qA[c], sf1[t & 1]);
        if (t < 4) ds_store(t >> 1, t < 2 ? sf0 : sf1, 2 * (t & 1));
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    KS_STAMP(3);
    // ---- hand-off: this slice's dS^T image and the next slice's Q / dO / row constants
    // own DMA pieces of slice it + 1 and its row constants, issued right after the previous barrier; the
    // 2 dQ slab stores issued after them (the previous slice's dQ task) may stay in flight (counted wait:
    // vmcnt(0) here waited out their write latency, p4 ~1.8k cycles of ~7k per slice)
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    __syncthreads();
    if (it + 2 < total) {
      qdma(it + 2, sl);  // every wave is past its reads of slot sl (slice it)
      rload(it + 2);
    }
    KS_STAMP(4);
    // ---- dQ partial of this key block: dQ^T tile (32 dims x 32 queries) = K^T dS^T over 256 keys
    // (no branch on a ragged last slice: its tiles past T read zero dS^T columns, and their two stores
    // go out of the descriptor's range -- dropped -- so every wave issues exactly 2 stores per slice,
    // which the counted vmcnt(2) of the hand-off relies on)
    const int qt0 = q0 + 32 * tq_blk;
    {
      f32x16 acc;
      constexpr int QA = 3;  // transposed reads QA steps ahead of the MFMA chain
      bf16x8 fa[QA + 1], fb[QA + 1];
      auto rd_q = [&](int ks) {
        fa[ks % (QA + 1)] = cat_tr(ds_tr(Sd + 16 * ks * BQ + sa0), ds_tr(Sd + 16 * ks * BQ + sa4));
        if (ks >= PL_KS_DQ_KREG) fb[ks % (QA + 1)] = cat_tr(ds_tr(Kl + 16 * ks * D + ka0), ds_tr(Kl + 16 * ks * D + ka4));
      };
#pragma unroll
      for (int ks = 0; ks < QA; ++ks) rd_q(ks);
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        if (ks + QA < BK / 16) rd_q(ks + QA);
        const bf16x8& kb_ = ks < PL_KS_DQ_KREG ? kdq[ks < PL_KS_DQ_KREG ? ks : 0] : fb[ks % (QA + 1)];
        if (ks == 0) mfma_v0(acc, kb_, fa[0]);
        else mfma_v(acc, kb_, fa[ks % (QA + 1)]);
        __builtin_amdgcn_sched_barrier(0);
      }
      mfma_settle(acc);
      float lo[8], hi[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        lo[e] = acc[e];
        hi[e] = acc[8 + e];
      }
      // this (key block, batch, head)'s slab tiles: nqt x NDB fragment blocks of 1024 bf16
      const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(a.dq_acc + (kb - a.kb0) * a.slab + ((int64_t)b * a.H + h) * a.nqt * NDB * 1024), (short)0,
          a.nqt * NDB * 2048, 0x00020000);
      const uint32_t doff = qt0 < a.T ? (uint32_t)(((qt0 >> 5) * NDB + tdb) * 2048 + lane * 32) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b128(pack8(lo), drs, doff, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(pack8(hi), drs, doff + 16u, 0, 0);
    }
    KS_STAMP(5);
#if PLLM_BWD_STAMPS
    st_acc[6] += 1;
#endif
  }
#if PLLM_BWD_STAMPS
  if (a.stamps && lane == 0) {
    unsigned long long* stp = a.stamps + ((int64_t)blockIdx.x * 4 + w) * 9;
#pragma unroll
    for (int i = 0; i < 8; ++i) stp[i] = st_acc[i];
    stp[8] = __builtin_amdgcn_s_memtime() - st_start;
  }
#endif
#undef KS_STAMP
  // ---- dK (scaled; RoPE: rotated back, R^T) and dV of this lane's keys: the accumulators settle
  // (18 wait states after the last MFMA), then every one is pinned behind that statement
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
#pragma unroll
  for (int kh = 0; kh < 2; ++kh)
#pragma unroll
    for (int db = 0; db < NDB; ++db) asm volatile("" : "+a"(dk[kh][db]), "+a"(dv[kh][db]));
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) {
    const int key = kw0 + 32 * kh + r;
    if (key >= a.S) continue;
    if (ROPE != 0) {
      const float* cr = a.rope_cos + (int64_t)key * (D / 2);
      const float* sr = a.rope_sin + (int64_t)key * (D / 2);
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
    }
    store_row_bf16<NDB>(a.dk + b * a.dk_sb + (int64_t)key * a.dk_st + (int64_t)hk * a.dk_sh, dk[kh], a.scale, hh);
    store_row_bf16<NDB>(a.dv + b * a.dv_sb + (int64_t)key * a.dv_st + (int64_t)hk * a.dv_sh, dv[kh], 1.f, hh);
  }
}


}  // namespace

namespace pllm {

int attn_bwd_ks_key_block() { return KsCfg<128>::BK; }

// one pass of key blocks [a.kb0, a.kb0 + a.nkb_pass) (the caller runs the delta pre-pass before and the
// slab reduce after)
void attn_bwd_ks_launch(const AttnBwdArgs& a, hipStream_t st) {
  const dim3 grid(a.nkb_pass * a.B * a.Hkv), blk(256);
  if (a.D == 64) {
    if (a.rope_cos) hipLaunchKernelGGL((attn_bwd_ks_kernel<64, 2>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL((attn_bwd_ks_kernel<64, 0>), grid, blk, 0, st, a);
  } else {
    if (a.rope_cos) hipLaunchKernelGGL((attn_bwd_ks_kernel<128, 2>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL((attn_bwd_ks_kernel<128, 0>), grid, blk, 0, st, a);
  }
}

}  // namespace pllm

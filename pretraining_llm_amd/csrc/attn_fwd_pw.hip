// Causal flash-attention forward for gfx950, one wave per SIMD ("PW", round 5; D = 64 / 128).
// Reference math: /root/reference/src/models/attention.py:47-57 (q k^T * hd^-1/2, causal
// masked_fill, softmax, @ v) -- the same online-softmax algorithm as attention.hip's attn_fwd_kernel,
// re-laid out so the matrix pipe is never idle behind the softmax:
//
//  * one workgroup = 4 waves = 256 query rows; wave w owns the 32-row blocks w and 7 - w (equal
//    shares of the causal diagonal) and the whole 512-register file: both blocks' O^T accumulators
//    live in AGPRs (D = 128: 128 registers), Q fragments, S^T chains and packed P in arch VGPRs;
//  * per 64-key tile the wave runs four MFMA steps, each beside the VALU work of the OTHER block:
//        1: S(b0, t)            || softmax of (b1, t-1), second key half + packing
//        2: O(b1) += V(t-1) P   || softmax of (b0, t): row max, lazy rescale, first key half
//        3: S(b1, t)            || softmax of (b0, t), second key half + packing
//        4: O(b0) += V(t) P     || softmax of (b1, t): row max, lazy rescale, first key half
//    so block 1's softmax straddles the tile seam (its P.V runs in the next tile's step 2);
//  * K tiles in a 2-deep and V tiles in a 3-deep LDS ring (V of tile t-1 is still read in step 2 of
//    tile t), both by LDS-DMA issued early in the tile, ONE barrier per tile;
//  * every MFMA is inline asm with an explicit register class (attn_common.h), VALU slices fenced
//    between them with sched_barrier so hipcc neither clusters the MFMAs nor hoists the VALU;
//  * blocks past their causal end drop out by wave-uniform tile variants (no masked MFMAs).
// The kernel it replaces at D = 128 ran two waves per SIMD, each softmax serialised behind its own
// block's S chain (36 % MFMA-busy).  Masking is folded into the S chains' initial accumulators.
#include <type_traits>

#include "attn_common.h"
#include "common.h"
#include "kernels.h"

namespace {

constexpr float kPwLazyThr = 8.f;  // lazy-max threshold (log2 units), as attn_fwd_kernel

PLLM_DEV void pin(float& x) { asm volatile("" : "+v"(x)); }

template <int D>
struct PwCfg {
  static_assert(D == 64 || D == 128, "PW forward: D = 64 / 128");
  static constexpr int NW = 4, BM = 256, BN = 64;
  static constexpr int NKS = D / 16, NDB = D / 32, CPR = D / 8;
  static constexpr int TILE = BN * D;          // elements of one K (V) tile
  static constexpr int NKB = 2, NVB = 3;       // ring depths
  static constexpr int PCS = BN * CPR / 64;    // 1-KiB DMA pieces per tile
  static constexpr int PPW = PCS / NW;         // per wave and operand
  static constexpr int NS = 2 * NKS;           // MFMAs of one block's S step (2 key halves)
  static constexpr int NP = 4 * NDB;           // MFMAs of one block's P.V step
  static constexpr int LDS_ELEMS = (NKB + NVB) * TILE;  // D = 128: 80 KiB
};

template <int D>
__global__ __launch_bounds__(256, 1) void attn_fwd_pw_kernel(AttnFwdArgs a) {
  using C = PwCfg<D>;
  using I = Img<D>;
  constexpr int BM = C::BM, BN = C::BN, NKS = C::NKS, NDB = C::NDB, CPR = C::CPR, TILE = C::TILE;
  constexpr int PCS = C::PCS, PPW = C::PPW, NS = C::NS, NP = C::NP;
  __shared__ __attribute__((aligned(1024))) uint16_t smem[C::LDS_ELEMS];
  uint16_t* const Kl = smem;                  // K tile t at Kl + (t % 2) TILE
  uint16_t* const Vl = smem + C::NKB * TILE;  // V tile t at Vl + (t % 3) TILE

  const int nqb = (a.T + BM - 1) / BM;
  const int BH = a.B * a.H;
  const int id = blockIdx.x;
  const int qb = nqb - 1 - id / BH;  // heaviest query blocks first
  const int bh = id % BH;
  const int b = bh / a.H, h = bh % a.H, hk = h / (a.H / a.Hkv);
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q0 = qb * BM, off = a.S - a.T;
  const uint16_t* qp = a.q + b * a.q_sb + (int64_t)h * a.q_sh;
  const uint16_t* kp = a.k + b * a.k_sb + (int64_t)hk * a.k_sh;
  const uint16_t* vp = a.v + b * a.v_sb + (int64_t)hk * a.v_sh;
  const unsigned lds0 = (unsigned)(uintptr_t)smem;

  // the wave's two blocks and their (causal) tile counts; block 1 never ends before block 0
  const int qw0 = q0 + 32 * w, qw1 = q0 + 32 * (7 - w);
  auto ntiles_of = [&](int qw) {
    const int kend = qw >= a.T ? 0 : (a.causal ? min(a.S, qw + 32 + off) : a.S);
    return (kend + BN - 1) / BN;
  };
  const int n0 = ntiles_of(qw0), n1 = ntiles_of(qw1);
  const int kv_end = a.causal ? min(a.S, q0 + BM + off) : a.S;
  const int ntiles = max(0, (kv_end + BN - 1) / BN);

  // Q fragments of both blocks (rows past T: zeros)
  bf16x8 qf0[NKS], qf1[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    const int i0 = qw0 + r, i1 = qw1 + r;
    qf0[ks] = i0 < a.T ? as_frag(ld16(qp + (int64_t)i0 * a.q_st + 16 * ks + 8 * hh)) : zero_frag();
    qf1[ks] = i1 < a.T ? as_frag(ld16(qp + (int64_t)i1 * a.q_st + 16 * ks + 8 * hh)) : zero_frag();
  }

  // ---- K / V tile DMA: wave w moves pieces [w PPW, (w + 1) PPW) of each operand (lane l of piece p
  // fills image chunk 64 p + l: logical chunk (g % CPR) ^ f(row) of row g / CPR); rows past S read zeros
  uint32_t dko[PPW], dvo[PPW];
#pragma unroll
  for (int k = 0; k < PPW; ++k) {
    const int g = (w * PPW + k) * 64 + lane, row = g / CPR, cc = (g % CPR) ^ I::f(row);
    dko[k] = (uint32_t)(row * (int)a.k_st + cc * 8) * 2u;
    dvo[k] = (uint32_t)(row * (int)a.v_st + cc * 8) * 2u;
  }
  // (branch-free: past the last tile the descriptor has range 0 and the pieces land zeros in a ring slot
  // no one reads any more -- a branch per piece split the MFMA steps into separate scheduling regions)
  auto dma = [&](bool isv, int t, int k) {
    const int kv0 = t * BN, rows = min(a.S - kv0, BN);
    const int64_t st = isv ? a.v_st : a.k_st;
    const uint16_t* base = (isv ? vp : kp) + (int64_t)min(kv0, a.S - 1) * st;
    const i32x4v srd = srd_of(base, rows > 0 ? (uint32_t)(((int64_t)(rows - 1) * st + D) * 2) : 0u);
    const unsigned dst = lds0 + 2u * (unsigned)(isv ? C::NKB * TILE + (t % C::NVB) * TILE : (t % C::NKB) * TILE);
    blds16(srd, isv ? dvo[k] : dko[k], dst + 1024u * (unsigned)(w * PPW + k));
  };

  // per-lane LDS offsets (swizzle applied once): K row reads fk ^ (ks << 4) + 32 kb D, V transposed
  // reads fv0 / fv8 ^ (db << 5) + 16 kst D
  const int g1 = (lane >> 4) & 1, tq = (lane & 15) >> 2, tp = lane & 3;
  const int fk0 = I::off(r, 8 * hh);
  const int fv00 = I::off(4 * hh + tq, 16 * g1 + 4 * tp), fv80 = I::off(4 * hh + tq + 8, 16 * g1 + 4 * tp);
  const float c2 = a.scale_log2;

  f32x16 o0[NDB], o1[NDB];
#pragma unroll
  for (int db = 0; db < NDB; ++db) {
    o0[db] = zero16();
    o1[db] = zero16();
  }
  float m0 = -INFINITY, m1 = -INFINITY, l0 = 0.f, l1 = 0.f, lh0 = 0.f, lh1 = 0.f;
  f32x16 s0[2], s1[2];
  bf16x8 pf0[4], pf1[4];

  if (ntiles > 0) {
#pragma unroll
    for (int k = 0; k < PPW; ++k) {
      dma(false, 0, k);
      dma(true, 0, k);
    }
  }
  vm_wait_all();
  __syncthreads();

  // S chain initial accumulators of block (qw, tile t): 0, or -inf where the key is masked
  auto s_init = [&](f32x16 (&s)[2], int qw, int t) {
    const int kv0 = t * BN;
    const bool need = (kv0 + BN > a.S) || (a.causal && kv0 + BN - 1 > qw + off);  // wave-uniform
    if (need) {
      const int qi = qw + r;
      const int lim = (a.causal ? min(a.S - 1, qi + off) : a.S - 1) - (kv0 + 4 * hh);
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) s[kb][i] = acc_row(i, 0) > lim - 32 * kb ? -INFINITY : 0.f;
    } else {
      s[0] = zero16();
      s[1] = zero16();
    }
  };
  // softmax, first half: row max over both key halves, lazy rescale of O / l, P of key half 0
  // split into NPC pieces (one per MFMA of the step it rides in)
  // (every slice is pinned between the MFMA statements it rides with: empty asm on its inputs before and
  // its results after -- sched_barrier alone let hipcc hoist the exps of a whole step ahead of its MFMAs)
  auto sm_max = [&](f32x16 (&s)[2], int piece, int npieces, float& mx) {
    // pieces [0, npieces): the running max over the 32 elements
    constexpr int E = 32;
    const int e0 = E * piece / npieces, e1 = E * (piece + 1) / npieces;
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (e >= e0 && e < e1) mx = fmaxf(mx, s[e >> 4][e & 15]);
    pin(mx);
  };
  auto sm_rescale = [&](float mx, float& m, float& l, f32x16 (&o)[NDB]) {
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mx2 = mx * c2;
    if (__any(mx2 - m > kPwLazyThr)) {  // wave-uniform; m = -inf: the first visible tile always sets m
      const float mnew = fmaxf(m, mx2);
      const float alpha = mnew == -INFINITY ? 1.f : fast_exp2(m - mnew);
#pragma unroll
      for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[db][i] *= alpha;
      l *= alpha;
      m = mnew;
    }
  };
  // exps of elements [e0, e1) of key half kb, their sum into ls
  auto sm_exp = [&](f32x16& s, int e0, int e1, float mc, float& ls) {
#pragma unroll
    for (int e = 0; e < 16; ++e)
      if (e >= e0 && e < e1) {
        float x = s[e];
        pin(x);
        const float p = fast_exp2(__builtin_fmaf(x, c2, -mc));
        s[e] = p;
        ls += p;
      }
    pin(ls);
  };

  // ---- one tile: L0 (block 0 live at t), F1 (block 1's tile t-1 to finish), L1 (block 1 live at t)
  auto tile = [&](int t, auto l0c, auto f1c, auto l1c) {
    constexpr bool L0 = decltype(l0c)::value, F1 = decltype(f1c)::value, L1 = decltype(l1c)::value;
    const uint16_t* Kb = Kl + (t % C::NKB) * TILE;
    const uint16_t* Vb = Vl + (t % C::NVB) * TILE;
    const uint16_t* Vp = Vl + ((t + C::NVB - 1) % C::NVB) * TILE;  // tile t - 1
    int fk = fk0, fv0 = fv00, fv8 = fv80;
    asm volatile("" : "+v"(fk), "+v"(fv0), "+v"(fv8));
    auto rd_k = [&](int u) {  // K fragment of S step u: key half u / NKS, ks u % NKS
      return as_frag(ld16(Kb + (u / NKS) * 32 * D + (fk ^ ((u % NKS) << 4))));
    };
    auto rd_v = [&](const uint16_t* V, int u) {  // V^T fragment of P.V step u: kst u / NDB, db u % NDB
      const int kst = u / NDB, db = u % NDB, rb = kst * 16 * D;
      return cat_tr(ds_tr(V + rb + (fv0 ^ (db << 5))), ds_tr(V + rb + (fv8 ^ (db << 5))));
    };
    constexpr int RA = 2;  // LDS reads two MFMAs ahead
    float mc0 = m0 == -INFINITY ? 0.f : m0, mc1 = m1 == -INFINITY ? 0.f : m1;

    // ---- step 1: S(b0, t) || block 1 (t - 1): exps of key half 1, packs, l
    if constexpr (L0) s_init(s0, qw0, t);
    {
      bf16x8 kr[RA + 1];
      if constexpr (L0) {
#pragma unroll
        for (int u = 0; u < RA; ++u) kr[u] = rd_k(u);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        if constexpr (L0) {
          if (u + RA < NS) kr[(u + RA) % (RA + 1)] = rd_k(u + RA);
          if (u % NKS == 0) mfma_v<true>(s0[u / NKS], kr[u % (RA + 1)], qf0[u % NKS]);
          else mfma_v(s0[u / NKS], kr[u % (RA + 1)], qf0[u % NKS]);
        }
        if constexpr (F1) {
          sm_exp(s1[1], 16 * u / NS, 16 * (u + 1) / NS, mc1, lh1);
          if (u == NS - 1) {
            pf1[2] = pack_frag(s1[1], 0);
            pf1[3] = pack_frag(s1[1], 1);
            l1 += lh1;
          }
        }
        if (u < PPW) dma(false, t + 1, u);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // ---- step 2: O(b1) += V(t-1) P(b1, t-1) || block 0 (t): max, rescale, exps of key half 0
    {
      bf16x8 vr[RA + 1];
      if constexpr (F1) {
#pragma unroll
        for (int u = 0; u < RA; ++u) vr[u] = rd_v(Vp, u);
      }
      float mx = -INFINITY;
      constexpr int NM = NP / 4 > 0 ? NP / 4 : 1;  // pieces of the max
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < NP; ++u) {
        if constexpr (F1) {
          if (u + RA < NP) vr[(u + RA) % (RA + 1)] = rd_v(Vp, u + RA);
          if (u == 0) mfma_a<true>(o1[u % NDB], vr[u % (RA + 1)], pf1[u / NDB]);
          else mfma_a(o1[u % NDB], vr[u % (RA + 1)], pf1[u / NDB]);
        }
        if constexpr (L0) {
          if (u == 0) mfma_settle(s0[0], s0[1]);
          if (u < NM) sm_max(s0, u, NM, mx);
          if (u == NM) {
            sm_rescale(mx, m0, l0, o0);
            mc0 = m0 == -INFINITY ? 0.f : m0;
            lh0 = 0.f;
          }
          if (u > NM) sm_exp(s0[0], 16 * (u - NM - 1) / (NP - NM - 1), 16 * (u - NM) / (NP - NM - 1), mc0, lh0);
        }
        if (u < PPW) dma(true, t + 1, u);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (L0) {
        pf0[0] = pack_frag(s0[0], 0);
        pf0[1] = pack_frag(s0[0], 1);
      }
    }
    // ---- step 3: S(b1, t) || block 0 (t): exps of key half 1, packs, l
    if constexpr (L1) s_init(s1, qw1, t);
    {
      bf16x8 kr[RA + 1];
      if constexpr (L1) {
#pragma unroll
        for (int u = 0; u < RA; ++u) kr[u] = rd_k(u);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        if constexpr (L1) {
          if (u + RA < NS) kr[(u + RA) % (RA + 1)] = rd_k(u + RA);
          if (u % NKS == 0) mfma_v<true>(s1[u / NKS], kr[u % (RA + 1)], qf1[u % NKS]);
          else mfma_v(s1[u / NKS], kr[u % (RA + 1)], qf1[u % NKS]);
        }
        if constexpr (L0) {
          sm_exp(s0[1], 16 * u / NS, 16 * (u + 1) / NS, mc0, lh0);
          if (u == NS - 1) {
            pf0[2] = pack_frag(s0[1], 0);
            pf0[3] = pack_frag(s0[1], 1);
            l0 += lh0;
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // ---- step 4: O(b0) += V(t) P(b0, t) || block 1 (t): max, rescale, exps of key half 0
    {
      bf16x8 vr[RA + 1];
      if constexpr (L0) {
#pragma unroll
        for (int u = 0; u < RA; ++u) vr[u] = rd_v(Vb, u);
      }
      float mx = -INFINITY;
      constexpr int NM = NP / 4 > 0 ? NP / 4 : 1;
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < NP; ++u) {
        if constexpr (L0) {
          if (u + RA < NP) vr[(u + RA) % (RA + 1)] = rd_v(Vb, u + RA);
          if (u == 0) mfma_a<true>(o0[u % NDB], vr[u % (RA + 1)], pf0[u / NDB]);
          else mfma_a(o0[u % NDB], vr[u % (RA + 1)], pf0[u / NDB]);
        }
        if constexpr (L1) {
          if (u == 0) mfma_settle(s1[0], s1[1]);
          if (u < NM) sm_max(s1, u, NM, mx);
          if (u == NM) {
            sm_rescale(mx, m1, l1, o1);
            mc1 = m1 == -INFINITY ? 0.f : m1;
            lh1 = 0.f;
          }
          if (u > NM) sm_exp(s1[0], 16 * (u - NM - 1) / (NP - NM - 1), 16 * (u - NM) / (NP - NM - 1), mc1, lh1);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (L1) {
        pf1[0] = pack_frag(s1[0], 0);
        pf1[1] = pack_frag(s1[0], 1);
      }
    }
    vm_wait_all();
    __syncthreads();
  };

  // one loop per tile variant (a variant dispatch inside one loop made hipcc reconcile the 128 O
  // accumulators across the variants at every iteration): both blocks live, block 1 alone, then the
  // finishing / barrier-only tiles
  using T_ = std::true_type;
  using F_ = std::false_type;
  int t = 0;
  if (n0 > 0) {
    tile(0, T_{}, F_{}, T_{});
    for (t = 1; t < n0; ++t) tile(t, T_{}, T_{}, T_{});
  } else if (n1 > 0) {
    tile(0, F_{}, F_{}, T_{});
    t = 1;
  }
  for (; t < n1; ++t) tile(t, F_{}, T_{}, T_{});
  if (t < ntiles && n1 > 0) {
    tile(t, F_{}, T_{}, F_{});  // block 1's last tile finishes here
    ++t;
  }
  for (; t < ntiles; ++t) tile(t, F_{}, F_{}, F_{});
  // ---- drain: block 1's last tile (its tile index n1 - 1 == ntiles - 1 when it ran to the end)
  if (n1 > 0 && n1 == ntiles) {
    const int t = ntiles - 1;
    const float mc1 = m1 == -INFINITY ? 0.f : m1;
    sm_exp(s1[1], 0, 16, mc1, lh1);
    pf1[2] = pack_frag(s1[1], 0);
    pf1[3] = pack_frag(s1[1], 1);
    l1 += lh1;
    const uint16_t* Vb = Vl + (t % C::NVB) * TILE;
    int fv0 = fv00, fv8 = fv80;
    asm volatile("" : "+v"(fv0), "+v"(fv8));
#pragma unroll
    for (int u = 0; u < NP; ++u) {
      const int kst = u / NDB, db = u % NDB, rb = kst * 16 * D;
      const bf16x8 va = cat_tr(ds_tr(Vb + rb + (fv0 ^ (db << 5))), ds_tr(Vb + rb + (fv8 ^ (db << 5))));
      mfma_a<true>(o1[db], va, pf1[kst]);
    }
  }
  // ---- epilogue: the accumulators settle, then O / l row stores and the LSE
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
#pragma unroll
  for (int db = 0; db < NDB; ++db) asm volatile("" : "+a"(o0[db]), "+a"(o1[db]));
  auto fin = [&](int qw, f32x16 (&o)[NDB], float m, float l) {
    const int qi = qw + r;
    const float lt = l + __shfl_xor(l, 32, 64);
    if (qi < a.T) {
      const float inv = lt > 0.f ? 1.f / lt : 0.f;
      store_row_bf16<NDB>(a.o + b * a.o_sb + (int64_t)qi * a.o_st + (int64_t)h * a.o_sh, o, inv, hh);
      if (hh == 0 && a.lse) a.lse[((int64_t)b * a.H + h) * a.T + qi] = (m + log2f(lt)) * 0.69314718055994531f;
    }
  };
  fin(qw0, o0, m0, l0);
  fin(qw1, o1, m1, l1);
}

}  // namespace

namespace pllm {

bool attn_fwd_pw_supported(const AttnFwdArgs& a) {
  return (a.D == 64 || a.D == 128) && a.rope_cos == nullptr;
}

void attn_fwd_pw(const AttnFwdArgs& a, hipStream_t st) {
  const int nqb = (a.T + 255) / 256;
  const dim3 grid(nqb * a.B * a.H), blk(256);
  if (a.D == 128) hipLaunchKernelGGL(attn_fwd_pw_kernel<128>, grid, blk, 0, st, a);
  else hipLaunchKernelGGL(attn_fwd_pw_kernel<64>, grid, blk, 0, st, a);
}

}  // namespace pllm

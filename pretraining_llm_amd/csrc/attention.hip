// Causal flash attention, forward and backward, on gfx950 MFMA (v_mfma_f32_32x32x16_bf16).
//
// Replaces the reference's per-head Python loop of materialised T x T score
// matrices (src/models/attention.py:47-57: q@k^T * hd^-1/2, masked_fill(tril==0,
// -inf), softmax, @v; concat at :95) with an O(T)-memory online-softmax kernel.
// Q/K/V are read in place out of the packed QKV GEMM output through strides and
// the gradients are written straight into the packed dQKV buffer.
//
// Layout choices (CDNA4, wave64):
//  * forward: one workgroup = 4 waves = 128 query rows, K/V tiles of 64 keys
//    double-buffered in LDS through registers (issue-early / write-late).
//    S^T = K.Q^T is computed with the QUERY on the MFMA lane, so the softmax row
//    statistics (m, l) are per-lane scalars and the P^T accumulator is directly
//    the B operand of O^T += V^T.P^T (no LDS round trip for P).  V^T fragments
//    come from ds_read_b64_tr_b16 transposed reads of the row-major V tile.
//  * backward: one workgroup = 4 waves = 128 keys of one (batch, kv-head); each
//    wave keeps dK^T/dV^T for its 32 keys in registers across all query blocks
//    (and all query heads of a GQA group), so dK/dV need no cross-workgroup sum.
//    S and dP are computed with the KEY on the lane and initialised with
//    -LSE/scale and -delta, so P = exp2(c*S') and dS = P*dP' need no extra pass.
//    dQ is summed over key blocks with fp32 atomics into a [B,T,H,D] buffer.
#include "common.h"
#include "kernels.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

PLLM_DEV f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
PLLM_DEV s16x4 ds_tr(const uint16_t* p) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p); }
PLLM_DEV bf16x8 cat_tr(const s16x4& lo, const s16x4& hi) {
  s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}
PLLM_DEV bf16x8 as_frag(const u32x4& v) { return __builtin_bit_cast(bf16x8, v); }
PLLM_DEV bf16x8 zero_frag() { return __builtin_bit_cast(bf16x8, u32x4{0u, 0u, 0u, 0u}); }
PLLM_DEV f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}
// element i of a 32x32 accumulator lives at row (i&3) + 8*(i>>2) + 4*half, column lane&31
PLLM_DEV int acc_row(int i, int half) { return (i & 3) + 8 * (i >> 2) + 4 * half; }
PLLM_DEV bf16x8 pack_frag(const f32x16& x, int s) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (bf16)x[8 * s + j];
  return f;
}

// ============================================================================
// forward
// ============================================================================
template <int D>
struct FwdCfg {
  static constexpr int BM = 128, BN = 64;
  static constexpr int KS = D + 8;    // K row stride (elements): row reads conflict-free
  static constexpr int VS = D + 32;   // V row stride: transposed reads conflict-free
  static constexpr int CPR = D / 8;   // 16 B chunks per row
  static constexpr int LPT = BN * CPR / 256;
  static constexpr int LDS_ELEMS = 2 * BN * KS + 2 * BN * VS;
};

template <int D>
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(AttnFwdArgs a) {
  using C = FwdCfg<D>;
  constexpr int BM = C::BM, BN = C::BN, KS = C::KS, VS = C::VS, CPR = C::CPR, LPT = C::LPT;
  constexpr int NKS = D / 16, NDB = D / 32;
  __shared__ __attribute__((aligned(16))) uint16_t smem[C::LDS_ELEMS];

  const int nqb = (a.T + BM - 1) / BM;
  const int BH = a.B * a.H;
  const int id = blockIdx.x;
  const int qb = nqb - 1 - id / BH;  // heaviest (last) query blocks first
  const int bh = id % BH;
  const int b = bh / a.H, h = bh % a.H, hk = h / (a.H / a.Hkv);
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int q0 = qb * BM, qw0 = q0 + w * 32, qi = qw0 + r;
  const int off = a.S - a.T;
  const uint16_t* qp = a.q + b * a.q_sb + (int64_t)h * a.q_sh;
  const uint16_t* kp = a.k + b * a.k_sb + (int64_t)hk * a.k_sh;
  const uint16_t* vp = a.v + b * a.v_sb + (int64_t)hk * a.v_sh;

  bf16x8 qf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks)
    qf[ks] = qi < a.T ? as_frag(ld16(qp + (int64_t)qi * a.q_st + 16 * ks + 8 * hh)) : zero_frag();

  int kv_end = a.S;
  if (a.causal) kv_end = min(a.S, q0 + BM + off);
  const int ntiles = (kv_end + BN - 1) / BN;
  const int wave_kv_end = a.causal ? min(a.S, qw0 + 32 + off) : a.S;

  u32x4 kr[LPT], vr[LPT];
  auto gload = [&](int t) {
    const int kv0 = t * BN;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int c = tid + 256 * i, row = c / CPR, col = c % CPR, key = kv0 + row;
      if (key < a.S) {
        kr[i] = ld16(kp + (int64_t)key * a.k_st + col * 8);
        vr[i] = ld16(vp + (int64_t)key * a.v_st + col * 8);
      } else {
        kr[i] = u32x4{0u, 0u, 0u, 0u};
        vr[i] = u32x4{0u, 0u, 0u, 0u};
      }
    }
  };
  auto swrite = [&](int buf) {
    uint16_t* Kb = smem + buf * BN * KS;
    uint16_t* Vb = smem + 2 * BN * KS + buf * BN * VS;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int c = tid + 256 * i, row = c / CPR, col = c % CPR;
      st16(Kb + row * KS + col * 8, kr[i]);
      st16(Vb + row * VS + col * 8, vr[i]);
    }
  };

  f32x16 o[NDB];
#pragma unroll
  for (int db = 0; db < NDB; ++db) o[db] = zero16();
  float m = -INFINITY, l = 0.f;
  const float c2 = a.scale_log2;
  const int g1 = (lane >> 4) & 1, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;

  if (ntiles > 0) {
    gload(0);
    swrite(0);
  }
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) gload(t + 1);
    const int kv0 = t * BN;
    if (kv0 < wave_kv_end) {
      const uint16_t* Kb = smem + buf * BN * KS;
      const uint16_t* Vb = smem + 2 * BN * KS + buf * BN * VS;
      f32x16 s[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        s[kb] = zero16();
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          const bf16x8 kf = as_frag(ld16(Kb + (kb * 32 + r) * KS + 16 * ks + 8 * hh));
          s[kb] = mfma32(kf, qf[ks], s[kb]);
        }
      }
      const bool need_mask = (kv0 + BN > a.S) || (a.causal && kv0 + BN - 1 > qw0 + off);
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float x = s[kb][i] * c2;
          if (need_mask) {
            const int key = kv0 + kb * 32 + acc_row(i, hh);
            if (key >= a.S || (a.causal && key > qi + off)) x = -INFINITY;
          }
          s[kb][i] = x;
          mx = fmaxf(mx, x);
        }
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = fmaxf(m, mx);
      const float muse = mnew == -INFINITY ? 0.f : mnew;
      const float alpha = exp2f(m - muse);
      float ls = 0.f;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = exp2f(s[kb][i] - muse);
          s[kb][i] = p;
          ls += p;
        }
      }
      l = l * alpha + ls;
      m = mnew;
#pragma unroll
      for (int db = 0; db < NDB; ++db) o[db] *= alpha;
      bf16x8 pf[4];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        pf[2 * kb] = pack_frag(s[kb], 0);
        pf[2 * kb + 1] = pack_frag(s[kb], 1);
      }
#pragma unroll
      for (int kst = 0; kst < 4; ++kst) {
#pragma unroll
        for (int db = 0; db < NDB; ++db) {
          const uint16_t* vb = Vb + (kst * 16 + 4 * hh + tq) * VS + db * 32 + 16 * g1 + 4 * tp;
          const bf16x8 va = cat_tr(ds_tr(vb), ds_tr(vb + 8 * VS));
          o[db] = mfma32(va, pf[kst], o[db]);
        }
      }
    }
    if (t + 1 < ntiles) swrite(buf ^ 1);
    __syncthreads();
  }

  const float lt = l + __shfl_xor(l, 32, 64);
  if (qi < a.T) {
    const float inv = lt > 0.f ? 1.f / lt : 0.f;
    uint16_t* op = a.o + b * a.o_sb + (int64_t)qi * a.o_st + (int64_t)h * a.o_sh;
#pragma unroll
    for (int db = 0; db < NDB; ++db) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u32x2 v2;
        v2[0] = pack_bf16x2(o[db][4 * g] * inv, o[db][4 * g + 1] * inv);
        v2[1] = pack_bf16x2(o[db][4 * g + 2] * inv, o[db][4 * g + 3] * inv);
        *reinterpret_cast<u32x2*>(op + db * 32 + 8 * g + 4 * hh) = v2;
      }
    }
    if (hh == 0 && a.lse) a.lse[((int64_t)b * a.H + h) * a.T + qi] = (m + log2f(lt)) * 0.69314718055994531f;
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

template <int D>
struct BwdCfg {
  static constexpr int BK = 128, BQ = 32;
  static constexpr int QS = D + 8;    // Q / dO tile stride (row reads + tr reads)
  static constexpr int KS = D + 32;   // K tile stride (tr reads only)
  static constexpr int DSS = 32 + 8;  // dS^T image stride (keys x 32 queries)
  static constexpr int CPR = D / 8;
  static constexpr int QLPT = (BQ * CPR + 255) / 256;
  static constexpr int KLPT = BK * CPR / 256;
  static constexpr int LDS_ELEMS = BK * KS + 2 * BQ * QS + BK * DSS;
};

template <int D>
__global__ __launch_bounds__(256, 2) void attn_bwd_kernel(AttnBwdArgs a) {
  using C = BwdCfg<D>;
  constexpr int BK = C::BK, BQ = C::BQ, QS = C::QS, KS = C::KS, DSS = C::DSS, CPR = C::CPR;
  constexpr int QLPT = C::QLPT, KLPT = C::KLPT;
  constexpr int NKS = D / 16, NDB = D / 32;
  __shared__ __attribute__((aligned(16))) uint16_t smem[C::LDS_ELEMS];
  __shared__ float rowc[2 * BQ];          // -lse/scale, -delta
  uint16_t* Kl = smem;
  uint16_t* Ql = smem + BK * KS;
  uint16_t* Ol = Ql + BQ * QS;            // dO tile
  uint16_t* Sl = Ol + BQ * QS;            // dS^T image [key][q]

  const int nkb = (a.S + BK - 1) / BK;
  const int BH = a.B * a.Hkv;
  const int id = blockIdx.x;
  const int kb = id / BH;                 // key block 0 (most query blocks under causal) first
  const int bh = id % BH;
  const int b = bh / a.Hkv, hk = bh % a.Hkv;
  const int G = a.H / a.Hkv;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int k0 = kb * BK, key = k0 + w * 32 + r;
  const int off = a.S - a.T;
  (void)nkb;
  const uint16_t* kp = a.k + b * a.k_sb + (int64_t)hk * a.k_sh;
  const uint16_t* vp = a.v + b * a.v_sb + (int64_t)hk * a.v_sh;

  // this lane's key row of K and V as B-operand fragments (k = head dim)
  bf16x8 kf[NKS], vf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    kf[ks] = key < a.S ? as_frag(ld16(kp + (int64_t)key * a.k_st + 16 * ks + 8 * hh)) : zero_frag();
    vf[ks] = key < a.S ? as_frag(ld16(vp + (int64_t)key * a.v_st + 16 * ks + 8 * hh)) : zero_frag();
  }
  // whole K block into LDS for the dQ product
#pragma unroll
  for (int i = 0; i < KLPT; ++i) {
    const int c = tid + 256 * i, row = c / CPR, col = c % CPR, kk = k0 + row;
    u32x4 v = kk < a.S ? ld16(kp + (int64_t)kk * a.k_st + col * 8) : u32x4{0u, 0u, 0u, 0u};
    st16(Kl + row * KS + col * 8, v);
  }

  f32x16 dk[NDB], dv[NDB];
#pragma unroll
  for (int db = 0; db < NDB; ++db) {
    dk[db] = zero16();
    dv[db] = zero16();
  }
  const float inv_scale = 1.f / a.scale, c2 = a.scale_log2;
  const int g1 = (lane >> 4) & 1, i16 = lane & 15, tq = i16 >> 2, tp = i16 & 3;
  const int nqb = (a.T + BQ - 1) / BQ;
  int qb_start = 0;
  if (a.causal) qb_start = max(0, k0 - off) / BQ;
  const int per_head = nqb - qb_start;
  const int total = per_head * G;

  u32x4 qr[QLPT], dor[QLPT];
  float rc = 0.f;
  auto gload = [&](int it) {
    const int h = hk * G + it / per_head;
    const int q0 = (qb_start + it % per_head) * BQ;
    const uint16_t* qp = a.q + b * a.q_sb + (int64_t)h * a.q_sh;
    const uint16_t* dop = a.dO + b * a.do_sb + (int64_t)h * a.do_sh;
#pragma unroll
    for (int i = 0; i < QLPT; ++i) {
      const int c = tid + 256 * i, row = c / CPR, col = c % CPR, q = q0 + row;
      if (c < BQ * CPR && q < a.T) {
        qr[i] = ld16(qp + (int64_t)q * a.q_st + col * 8);
        dor[i] = ld16(dop + (int64_t)q * a.do_st + col * 8);
      } else {
        qr[i] = u32x4{0u, 0u, 0u, 0u};
        dor[i] = u32x4{0u, 0u, 0u, 0u};
      }
    }
    if (tid < 2 * BQ) {
      const int q = q0 + (tid & (BQ - 1));
      const int64_t idx = ((int64_t)b * a.H + h) * a.T + q;
      if (q < a.T) rc = tid < BQ ? -a.lse[idx] * inv_scale : -a.delta[idx];
      else rc = 0.f;
    }
  };

  if (total > 0) gload(0);
  for (int it = 0; it < total; ++it) {
    const int h = hk * G + it / per_head;
    const int q0 = (qb_start + it % per_head) * BQ;
    __syncthreads();  // previous iteration's readers of Q/dO/dS are done
#pragma unroll
    for (int i = 0; i < QLPT; ++i) {
      const int c = tid + 256 * i, row = c / CPR, col = c % CPR;
      if (c < BQ * CPR) {
        st16(Ql + row * QS + col * 8, qr[i]);
        st16(Ol + row * QS + col * 8, dor[i]);
      }
    }
    if (tid < 2 * BQ) rowc[tid] = rc;
    __syncthreads();
    if (it + 1 < total) gload(it + 1);

    // S' = Q K^T - lse/scale ; dP' = dO V^T - delta   (query rows in registers, key on the lane)
    f32x16 s, dp;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      s[i] = rowc[acc_row(i, hh)];
      dp[i] = rowc[BQ + acc_row(i, hh)];
    }
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const bf16x8 qa = as_frag(ld16(Ql + r * QS + 16 * ks + 8 * hh));
      s = mfma32(qa, kf[ks], s);
      const bf16x8 oa = as_frag(ld16(Ol + r * QS + 16 * ks + 8 * hh));
      dp = mfma32(oa, vf[ks], dp);
    }
    const bool need_mask = (q0 + BQ > a.T) || (k0 + BK > a.S) || (a.causal && k0 + BK - 1 > q0 + off);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float p = exp2f(c2 * s[i]);
      if (need_mask) {
        const int q = q0 + acc_row(i, hh);
        if (q >= a.T || key >= a.S || (a.causal && key > q + off)) p = 0.f;
      }
      s[i] = p;           // P
      dp[i] = p * dp[i];  // dS (unscaled)
    }
    const bf16x8 pf0 = pack_frag(s, 0), pf1 = pack_frag(s, 1);
    const bf16x8 sf0 = pack_frag(dp, 0), sf1 = pack_frag(dp, 1);
    // dV^T += dO^T P ; dK^T += Q^T dS   (A operands by transposed reads of the [q][d] tiles)
#pragma unroll
    for (int db = 0; db < NDB; ++db) {
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const int rowq = st * 16 + 4 * hh + tq, col = db * 32 + 16 * g1 + 4 * tp;
        const uint16_t* ob = Ol + rowq * QS + col;
        const uint16_t* qb2 = Ql + rowq * QS + col;
        const bf16x8 oA = cat_tr(ds_tr(ob), ds_tr(ob + 8 * QS));
        const bf16x8 qA = cat_tr(ds_tr(qb2), ds_tr(qb2 + 8 * QS));
        dv[db] = mfma32(oA, st ? pf1 : pf0, dv[db]);
        dk[db] = mfma32(qA, st ? sf1 : sf0, dk[db]);
      }
    }
    // dS^T image: lane's key row, 4 consecutive queries per 8-byte store
    {
      uint16_t* srow = Sl + (w * 32 + r) * DSS;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u32x2 v2;
        v2[0] = pack_bf16x2(dp[4 * g], dp[4 * g + 1]);
        v2[1] = pack_bf16x2(dp[4 * g + 2], dp[4 * g + 3]);
        *reinterpret_cast<u32x2*>(srow + 8 * g + 4 * hh) = v2;
      }
    }
    __syncthreads();
    // dQ partial of this key block: dQ_kb[q, d] = dS[q, keys] K[keys, d], one d-block per wave
    // (waves w < NDB), summed over all BK keys on chip and stored with plain stores into the
    // key block's slab; attn_dq_reduce_kernel sums the slabs in a fixed order (deterministic,
    // and no fp32 atomics: they were the floor of the first version of this kernel).
    if (w < NDB) {
      const int db = w;
      f32x16 acc = zero16();
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        const int kr0 = ks * 16 + 8 * hh + tq;
        const uint16_t* sa = Sl + kr0 * DSS + 16 * g1 + 4 * tp;
        const uint16_t* kbp = Kl + kr0 * KS + db * 32 + 16 * g1 + 4 * tp;
        const bf16x8 A = cat_tr(ds_tr(sa), ds_tr(sa + 4 * DSS));
        const bf16x8 Bf = cat_tr(ds_tr(kbp), ds_tr(kbp + 4 * KS));
        acc = mfma32(A, Bf, acc);
      }
      const int64_t slab = (int64_t)a.B * a.T * a.H * D;
      float* dq = a.dq_acc + kb * slab + (((int64_t)b * a.T) * a.H + h) * D + db * 32 + r;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int q = q0 + acc_row(i, hh);
        if (q < a.T) dq[(int64_t)q * a.H * D] = acc[i];
      }
    }
  }
  // write dK (scaled) and dV for this lane's key
  if (key < a.S) {
    uint16_t* dkp = a.dk + b * a.dk_sb + (int64_t)key * a.dk_st + (int64_t)hk * a.dk_sh;
    uint16_t* dvp = a.dv + b * a.dv_sb + (int64_t)key * a.dv_st + (int64_t)hk * a.dv_sh;
#pragma unroll
    for (int db = 0; db < NDB; ++db) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u32x2 k2, v2;
        k2[0] = pack_bf16x2(dk[db][4 * g] * a.scale, dk[db][4 * g + 1] * a.scale);
        k2[1] = pack_bf16x2(dk[db][4 * g + 2] * a.scale, dk[db][4 * g + 3] * a.scale);
        v2[0] = pack_bf16x2(dv[db][4 * g], dv[db][4 * g + 1]);
        v2[1] = pack_bf16x2(dv[db][4 * g + 2], dv[db][4 * g + 3]);
        *reinterpret_cast<u32x2*>(dkp + db * 32 + 8 * g + 4 * hh) = k2;
        *reinterpret_cast<u32x2*>(dvp + db * 32 + 8 * g + 4 * hh) = v2;
      }
    }
  }
}

// dq (bf16, strided) = scale * sum over contributing key blocks of the fp32 slabs
// [nkb][B,T,H,D]; under the causal mask row t only reads blocks kb <= (t+off)/BK
// (the others were never written for it).
template <int D>
__global__ __launch_bounds__(256) void attn_dq_reduce_kernel(AttnBwdArgs a) {
  constexpr int CPR = D / 8;
  constexpr int BK = BwdCfg<D>::BK;
  const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t row = gid / CPR;
  const int c = (int)(gid % CPR);
  const int64_t nrows = (int64_t)a.B * a.T * a.H;
  if (row >= nrows) return;
  const int h = (int)(row % a.H);
  const int64_t bt = row / a.H;
  const int t = (int)(bt % a.T);
  const int b = (int)(bt / a.T);
  const int nkb = (a.S + BK - 1) / BK;
  int kmax = nkb - 1;
  if (a.causal) kmax = min(kmax, (t + a.S - a.T) / BK);
  const int64_t slab = nrows * D;
  float f[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const float* src = a.dq_acc + row * D + c * 8;
  for (int kb = 0; kb <= kmax; ++kb) {
    const f32x4* p = reinterpret_cast<const f32x4*>(src + kb * slab);
    const f32x4 x0 = p[0], x1 = p[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f[j] += x0[j];
      f[4 + j] += x1[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] *= a.scale;
  st16(a.dq + b * a.dq_sb + (int64_t)t * a.dq_st + (int64_t)h * a.dq_sh + c * 8, pack8(f));
}

}  // namespace

namespace pllm {

bool attn_supported_head_dim(int D) { return D == 32 || D == 64 || D == 128; }

template <int D>
static void attn_fwd_t(const AttnFwdArgs& a, hipStream_t st) {
  const int nqb = (a.T + 127) / 128;
  hipLaunchKernelGGL(attn_fwd_kernel<D>, dim3(nqb * a.B * a.H), dim3(256), 0, st, a);
}

template <int D>
static void attn_bwd_t(const AttnBwdArgs& a, hipStream_t st) {
  const int64_t nrows = (int64_t)a.B * a.T * a.H;
  const int pre_grid = (int)((nrows * (D / 8) + 255) / 256);
  const int nkb = (a.S + 127) / 128;
  hipLaunchKernelGGL(attn_bwd_pre_kernel<D>, dim3(pre_grid), dim3(256), 0, st, a);
  hipLaunchKernelGGL(attn_bwd_kernel<D>, dim3(nkb * a.B * a.Hkv), dim3(256), 0, st, a);
  hipLaunchKernelGGL(attn_dq_reduce_kernel<D>, dim3(pre_grid), dim3(256), 0, st, a);
}

void attn_fwd(const AttnFwdArgs& a, hipStream_t st) {
  if (a.D == 32) attn_fwd_t<32>(a, st);
  else if (a.D == 64) attn_fwd_t<64>(a, st);
  else attn_fwd_t<128>(a, st);
}

void attn_bwd(const AttnBwdArgs& a, hipStream_t st) {
  if (a.D == 32) attn_bwd_t<32>(a, st);
  else if (a.D == 64) attn_bwd_t<64>(a, st);
  else attn_bwd_t<128>(a, st);
}

}  // namespace pllm

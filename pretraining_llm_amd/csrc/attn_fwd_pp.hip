// Ping-pong causal flash-attention forward for head dim 64 on gfx950 (round 6).
// Reference math: /root/reference/src/models/attention.py:47-57 (q k^T * hd^-1/2, causal mask, softmax, @ v),
// per head, concatenated at :95 -- here O(T) memory, online softmax, one pass.
//
// Why (profiles/r5_pmc_attn_d64.md, MI355X_MICROARCH.md "Two waves per SIMD"): at D = 64 one 64-key tile of
// a wave's 64 query rows is 32 MFMAs (1,024 cycles: S = K Q^T and O += V P^T) against ~1,300 cycles of
// softmax VALU issue; the 4-wave kernel of attention.hip (two workgroups per CU, uncoordinated) spends ~3,000
// cycles per wave-tile, i.e. most of the time one SIMD's two waves wait or compute the same kind of phase.
// Here the two waves of a SIMD belong to one workgroup and alternate roles at every barrier:
//  * 8 waves = two groups of four (waves 0-3 / 4-7, one of each on every SIMD); group 1 runs one barrier
//    behind group 0, so while a group issues its MFMA phase (S of tile t + the PV of tile t - 1, s_setprio 1)
//    the other group on the same SIMD runs its softmax phase (VALU) -- the matrix pipe and the VALU are fed
//    by different waves;
//  * PV is software-pipelined one tile behind S (P(t) is formed in the VALU phase and consumed by the next
//    MFMA phase), so each phase depends only on the previous phase of the same wave;
//  * K / V tiles (64 keys) in LDS rings of 3 / 4 slots, filled by LDS-DMA three tiles ahead by the four
//    trailing waves during their softmax phase, waited with a counted vmcnt (one tile in flight across the
//    barrier);
//  * each wave owns 2 blocks of 32 query rows, w and 15 - w of the workgroup's 512 (equal causal work per
//    wave); a block's fully-masked tiles skip their MFMAs and softmax on a wave-uniform branch.
// Layouts and math as attn_fwd_kernel (attention.hip): S^T = K Q^T with the query on the MFMA lane, lazy
// rescaling (kLazyThr), fp32 O / l, the same swizzled LDS image (Img<64>) and row-per-lane epilogue.
#include "attn_common.h"
#include "kernels.h"

namespace {

constexpr int PD = 64;                 // head dim
constexpr int PNW = 8;                 // waves
constexpr int PBN = 64;                // keys per tile
constexpr int PBM = PNW * 2 * 32;      // query rows per workgroup (2 blocks of 32 per wave)
constexpr int PTILE = PBN * PD;        // elements of a K / V tile (8 KiB)
constexpr int PKR = 3, PVR = 4;        // ring slots
constexpr int PNKS = PD / 16, PNDB = PD / 32;
constexpr float kPLazyThr = 8.f;       // lazy-max threshold (log2 units), as attention.hip

PL_DEV void pf_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
template <int N>
PL_DEV void pf_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__global__ __launch_bounds__(64 * PNW, 2) void attn_fwd_pp_kernel(AttnFwdArgs a) {
  using I = Img<PD>;
  __shared__ __attribute__((aligned(1024))) uint16_t smem[(PKR + PVR) * PTILE];
  const int nqb = (a.T + PBM - 1) / PBM;
  const int BH = a.B * a.H;
  const int id = blockIdx.x;
  const int qb = nqb - 1 - id / BH;  // heaviest query blocks first
  const int bh = id % BH;
  const int b = bh / a.H, h = bh % a.H, hk = h / (a.H / a.Hkv);
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int gp = w >> 2;  // 0: leading group, 1: trailing group (also the DMA issuers)
  const int q0 = qb * PBM;
  const int off = a.S - a.T;
  const uint16_t* qp = a.q + b * a.q_sb + (int64_t)h * a.q_sh;
  const uint16_t* kp = a.k + b * a.k_sb + (int64_t)hk * a.k_sh;
  const uint16_t* vp = a.v + b * a.v_sb + (int64_t)hk * a.v_sh;

  int qw[2], qend[2];
  qw[0] = q0 + 32 * w;
  qw[1] = q0 + 32 * (2 * PNW - 1 - w);
#pragma unroll
  for (int j = 0; j < 2; ++j) qend[j] = qw[j] >= a.T ? 0 : (a.causal ? min(a.S, qw[j] + 32 + off) : a.S);
  bf16x8 qf[2][PNKS];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int qi = qw[j] + r;
#pragma unroll
    for (int ks = 0; ks < PNKS; ++ks)
      qf[j][ks] = as_frag(qi < a.T ? ld16(qp + (int64_t)qi * a.q_st + 16 * ks + 8 * hh) : u32x4{0u, 0u, 0u, 0u});
  }
  vm_wait_all();
  int kv_end = a.S;
  if (a.causal) kv_end = min(a.S, q0 + PBM + off);
  const int nt = (kv_end + PBN - 1) / PBN;  // tiles of the workgroup (every wave runs all of them)

  // LDS-DMA: a 1-KiB piece is 8 rows of a tile; lane l fills row 8 p + l / 8 at chunk position l % 8, which
  // holds logical chunk (l % 8) ^ f(row) (f depends on row & 15: on p's parity)
  const unsigned lds0 = (unsigned)(uintptr_t)smem;
  auto piece_off = [&](int p, int64_t st) {
    const int row = 8 * p + (lane >> 3), ch = (lane & 7) ^ I::f(row);
    return (uint32_t)((row * st + 8 * ch) * 2);
  };
  auto tile_srd = [&](int t, bool isv) {
    const int kv0 = t * PBN, rows = t < nt ? min(a.S - kv0, PBN) : 0;
    const int64_t st = isv ? a.v_st : a.k_st;
    const uint16_t* base = (isv ? vp : kp) + (int64_t)(t < nt ? kv0 : 0) * st;
    return srd_of(base, rows > 0 ? (uint32_t)(((int64_t)(rows - 1) * st + PD) * 2) : 0u);
  };
  auto kslot = [&](int t) { return lds0 + (unsigned)((t % PKR) * PTILE * 2); };
  auto vslot = [&](int t) { return lds0 + (unsigned)((PKR + t % PVR) * PTILE * 2); };
  // loop DMA (trailing group): wave 4 + i moves K pieces 2i, 2i + 1 and V pieces 2i, 2i + 1 of a tile
  const int wi = w & 3;
  const uint32_t dk0 = piece_off(2 * wi, a.k_st), dk1 = piece_off(2 * wi + 1, a.k_st);
  const uint32_t dv0 = piece_off(2 * wi, a.v_st), dv1 = piece_off(2 * wi + 1, a.v_st);
  auto dma_tile = [&](int t) {
    const i32x4v ks = tile_srd(t, false), vs = tile_srd(t, true);
    blds16(ks, dk0, kslot(t) + 1024u * (unsigned)(2 * wi));
    blds16(ks, dk1, kslot(t) + 1024u * (unsigned)(2 * wi + 1));
    blds16(vs, dv0, vslot(t) + 1024u * (unsigned)(2 * wi));
    blds16(vs, dv1, vslot(t) + 1024u * (unsigned)(2 * wi + 1));
  };
  // prologue: tiles 0, 1, 2 by all eight waves (wave w: K piece w, V piece w of each), landed, published
  {
    const uint32_t pk = piece_off(w, a.k_st), pv = piece_off(w, a.v_st);
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      blds16(tile_srd(t, false), pk, kslot(t) + 1024u * (unsigned)w);
      blds16(tile_srd(t, true), pv, vslot(t) + 1024u * (unsigned)w);
    }
  }
  vm_wait_all();
  pf_barrier();
  if (gp == 1) pf_barrier();  // the trailing group runs one barrier behind

  const int g1 = (lane >> 4) & 1, tq = (lane & 15) >> 2, tp = lane & 3;
  const int fk = I::off(r, 8 * hh);
  const int fv0 = I::off(4 * hh + tq, 16 * g1 + 4 * tp), fv8 = I::off(4 * hh + tq + 8, 16 * g1 + 4 * tp);
  const float c2 = a.scale_log2;
  f32x16 o[2][PNDB], s[2][2];
  float m[2], l[2];
  bf16x8 pf[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
#pragma unroll
    for (int db = 0; db < PNDB; ++db) o[j][db] = zero16();
    m[j] = -INFINITY;
    l[j] = 0.f;
  }
  // ---- MFMA phase pieces
  auto s_part = [&](auto mask_c, int t) {
    constexpr int MASK = decltype(mask_c)::value;
    const uint16_t* Kb = smem + (t % PKR) * PTILE;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int ks = 0; ks < PNKS; ++ks) {
        const bf16x8 kf = as_frag(ld16(Kb + kb * 32 * PD + (fk ^ (ks << 4))));
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if ((MASK >> j) & 1) s[j][kb] = mfma32(kf, qf[j][ks], ks == 0 ? zero16() : s[j][kb]);
      }
    }
  };
  auto pv_part = [&](auto mask_c, int t) {  // O += V(t) P(t)^T
    constexpr int MASK = decltype(mask_c)::value;
    const uint16_t* Vb = smem + (PKR + t % PVR) * PTILE;
#pragma unroll
    for (int kst = 0; kst < 4; ++kst) {
#pragma unroll
      for (int db = 0; db < PNDB; ++db) {
        const int rb = kst * 16 * PD;
        const bf16x8 va = cat_tr(ds_tr(Vb + rb + (fv0 ^ (db << 5))), ds_tr(Vb + rb + (fv8 ^ (db << 5))));
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if ((MASK >> j) & 1) o[j][db] = mfma32(va, pf[j][kst], o[j][db]);
      }
    }
  };
  // ---- softmax phase: P(t) of the blocks that see tile t, into pf
  auto softmax_part = [&](auto mask_c, int t) {
    constexpr int MASK = decltype(mask_c)::value;
    const int kv0 = t * PBN;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (!((MASK >> j) & 1)) continue;
      const int qi = qw[j] + r;
      const bool need_mask = (kv0 + PBN > a.S) || (a.causal && kv0 + PBN - 1 > qw[j] + off);
      if (need_mask) {
        const int lim0 = (a.causal ? min(a.S - 1, qi + off) : a.S - 1) - (kv0 + 4 * hh);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int i = 0; i < 16; ++i) s[j][kb][i] = acc_row(i, 0) > lim0 - 32 * kb ? -INFINITY : s[j][kb][i];
      }
      float mx0 = -INFINITY, mx1 = -INFINITY;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        mx0 = fmaxf(mx0, s[j][0][i]);
        mx1 = fmaxf(mx1, s[j][1][i]);
      }
      float mx = fmaxf(mx0, mx1);
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mx2 = mx * c2;
      if (__any(mx2 - m[j] > kPLazyThr)) {
        const float mnew = fmaxf(m[j], mx2);
        const float alpha = mnew == -INFINITY ? 1.f : fast_exp2(m[j] - mnew);
#pragma unroll
        for (int db = 0; db < PNDB; ++db)
#pragma unroll
          for (int i = 0; i < 16; ++i) o[j][db][i] = o[j][db][i] * alpha;
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
  };
  // One tile step = MFMA phase (S of tile t for the blocks of MS, PV of tile t - 1 for those of MP), barrier,
  // softmax phase (trailing group: the DMA of tile t + 3 first, its counted wait last), barrier.  The block
  // masks are compile-time per step: a wave's tiles fall into segments of constant masks (both blocks, then
  // the late block only, then none -- blocks w and 15 - w end in that order), so each segment is a loop of
  // one instantiation and only the segment boundaries join (runtime mask branches inside one step made hipcc
  // keep every variant's registers live: 399 spills).
  auto step = [&](auto ms_c, auto mp_c, int t) {
    constexpr int MS = decltype(ms_c)::value, MP = decltype(mp_c)::value;
    __builtin_amdgcn_s_setprio(1);
    if constexpr (MS != 0) s_part(ms_c, t);
    if constexpr (MP != 0) pv_part(mp_c, t - 1);
    __builtin_amdgcn_s_setprio(0);
    pf_barrier();
    if (gp == 1) dma_tile(t + 3);  // into the slots of tiles t (K) and t - 1 (V): read by both groups by now
    if constexpr (MS != 0) softmax_part(ms_c, t);
    if (gp == 1) pf_vmwait<4>();   // tile t + 2 landed (this wave's pieces); published by the barrier
    pf_barrier();
  };
  using C0 = std::integral_constant<int, 0>;
  using C2 = std::integral_constant<int, 2>;
  using C3 = std::integral_constant<int, 3>;
  // tiles [0, t1): both blocks; [t1, t2): the late block; [t2, nt): none
  const int t1 = min(nt, (qend[0] + PBN - 1) / PBN), t2 = min(nt, (qend[1] + PBN - 1) / PBN);
  int t = 0;
  if (t < t1) {
    step(C3{}, C0{}, t++);
    for (; t < t1; ++t) step(C3{}, C3{}, t);
  }
  if (t < t2) {
    if (t == 0) step(C2{}, C0{}, t++);
    else step(C2{}, C3{}, t++);
    for (; t < t2; ++t) step(C2{}, C2{}, t);
  }
  if (t < nt) {
    if (t == 0) step(C0{}, C0{}, t++);
    else if (t == t1) step(C0{}, C3{}, t++);
    else step(C0{}, C2{}, t++);
    for (; t < nt; ++t) step(C0{}, C0{}, t);
  }
  // the last tile's PV (mask of tile nt - 1)
  __builtin_amdgcn_s_setprio(1);
  if (nt > 0 && nt - 1 < t1) pv_part(C3{}, nt - 1);
  else if (nt > 0 && nt - 1 < t2) pv_part(C2{}, nt - 1);
  __builtin_amdgcn_s_setprio(0);
  if (gp == 0) pf_barrier();  // balance the trailing group's extra barrier
  vm_wait_all();

#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int qi = qw[j] + r;
    const float lt = l[j] + __shfl_xor(l[j], 32, 64);
    if (qi < a.T) {
      const float inv = lt > 0.f ? 1.f / lt : 0.f;
      store_row_bf16<PNDB>(a.o + b * a.o_sb + (int64_t)qi * a.o_st + (int64_t)h * a.o_sh, o[j], inv, hh);
      if (hh == 0 && a.lse) a.lse[((int64_t)b * a.H + h) * a.T + qi] = (m[j] + log2f(lt)) * 0.69314718055994531f;
    }
  }
}

}  // namespace

namespace pllm {

static int g_attn_fwd_pp = 0;
void attn_fwd_set_pp(int on) { g_attn_fwd_pp = on; }
bool attn_fwd_pp_applies(const AttnFwdArgs& a) { return g_attn_fwd_pp && a.D == PD && a.rope_cos == nullptr; }

void attn_fwd_pp(const AttnFwdArgs& a, hipStream_t st) {
  const int nqb = (a.T + PBM - 1) / PBM;
  hipLaunchKernelGGL(attn_fwd_pp_kernel, dim3(nqb * a.B * a.H), dim3(64 * PNW), 0, st, a);
}

}  // namespace pllm

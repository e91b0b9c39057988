// Host-side launch API of the gfx950 kernels.  Plain pointers + hipStream_t only,
// so the kernel translation units never include torch headers; bindings.cpp is
// the only file that knows about at::Tensor.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

struct AttnFwdArgs {
  const uint16_t *q, *k, *v;
  uint16_t* o;
  float* lse;  // [B, H, T] natural-log LSE, may be null
  // optional fused RoPE (rotate-half) of q and k: fp32 tables [>= S, D/2]; query row t sits at
  // position t + S - T, key row j at position j
  const float *rope_cos, *rope_sin;
  int B, H, Hkv, T, S, D;
  int64_t q_sb, q_st, q_sh, k_sb, k_st, k_sh, v_sb, v_st, v_sh, o_sb, o_st, o_sh;
  float scale, scale_log2;
  int causal;
  unsigned long long* stamps;  // diagnostic builds only (PLLM_FWD_STAMPS): per-wave phase cycles
};

// q [B, H, D] (one query per sequence), k/v rows of a [B, S_max, Hkv, D]-strided cache
struct DecodeArgs {
  const uint16_t *q, *k, *v;
  uint16_t* o;
  float *part_o, *part_lse;  // [B, H, splits, D] / [B, H, splits] when splits > 1
  const int* seqlen;         // optional device key count (graph capture); else S
  int seqlen_per_row;        // seqlen holds B counts (one per sequence) instead of one
  int B, H, Hkv, S, D, splits;
  int64_t q_sb, q_sh, k_sb, k_st, k_sh, v_sb, v_st, v_sh, o_sb, o_sh;
  float scale_log2;
};

struct AttnBwdArgs {
  const uint16_t *q, *k, *v, *o, *dO;
  const float* lse;
  const float *rope_cos, *rope_sin;  // optional fused RoPE (as AttnFwdArgs); dq/dk un-rotated
  float* delta;   // [B, H, T] scratch
  uint16_t* dq_acc;  // [nkb_pass][B, T, H, D] bf16 per-key-block dQ partial slabs of one pass
  float* dq_sum;  // [B, T, H, D] fp32 running dQ sum across passes (null when one pass)
  int kb0, nkb_pass;  // first key block of the pass / key blocks per pass (set by the host)
  int rope_in;        // with rope tables: 1 = rotate q / k in-kernel, 0 = already rotated (outputs only)
  int64_t slab;       // elements per dQ slab (>= B * ceil32(T) * H * D)
  int nqt;            // ceil(T / 32): query tiles per head in the fragment-order slab (RS kernel)
  uint16_t *dq, *dk, *dv;
  int B, H, Hkv, T, S, D;
  int64_t q_sb, q_st, q_sh, k_sb, k_st, k_sh, v_sb, v_st, v_sh, o_sb, o_st, o_sh, do_sb, do_st, do_sh;
  int64_t dq_sb, dq_st, dq_sh, dk_sb, dk_st, dk_sh, dv_sb, dv_st, dv_sh;
  float scale, scale_log2;
  int causal;
  unsigned long long* stamps;  // diagnostic builds only (PLLM_BWD_STAMPS): per-wave phase cycles
  int delta_ready;             // 1: delta already holds rowsum(dO * O) (gemm_tn epilogue 6): no pre-pass
};

namespace pllm {

// norm.hip
void norm_fwd(const void* x, const void* res, const void* w, const void* b, void* y, void* s, float* mean,
              float* rstd, int N, int C, float eps, bool rms, hipStream_t st);
int norm_bwd_grid(int N, int C);
// xb_part/xb: optional column sums of dx (bias grad of the layer that produced x)
// Gradient outputs (dw, db, xb, bias grads, wgrad, embedding grads) are bf16 or fp32 (grad_f32 /
// out_f32: the optimizer's flat-gradient dtype); activations and their gradients are bf16.
void norm_bwd(const void* dy, const void* s, const void* w, const float* mean, const float* rstd, const void* ds,
              void* dx, float* dw_part, float* db_part, void* dw, void* db, bool grad_f32, int N, int C, bool rms,
              bool accumulate, float* xb_part, void* xb, bool xb_accumulate, hipStream_t st);
// fp32 [G, C] slab -> [C] column sums (bf16 or fp32 out; optionally added into out)
void col_reduce(const float* part, int G, int C, void* out, bool out_f32, bool accumulate, hipStream_t st);
// bias gradient = column sums of a bf16 [N, C] matrix; part: fp32 [colsum_groups(N), C] workspace
int colsum_groups(int N);
void bias_grad(const void* x, int N, int C, float* part, void* out, bool out_f32, bool accumulate, hipStream_t st);

// elementwise.hip (op: 0 relu, 1 gelu-tanh)
void act_fwd(int op, const void* x, void* y, size_t n, hipStream_t st);
void act_bwd(int op, const void* dy, const void* xin, void* dx, size_t n, hipStream_t st);
// activation backward + fused bias gradient (column sums of dx) of the producing linear layer
void act_bwd_bias(int op, const void* dy, const void* xin, void* dx, int N, int C, float* part, void* bias_grad,
                  bool grad_f32, bool accumulate, hipStream_t st);
void swiglu_fwd(const void* gu, void* y, size_t rows, int F, hipStream_t st);
void swiglu_bwd(const void* dy, const void* gu, void* dgu, size_t rows, int F, hipStream_t st);
void rope(const void* in, void* out, const float* cosb, const float* sinb, size_t rows, int T, int n_heads_total,
          int n_rot, int D, int pos_offset, bool inverse, hipStream_t st, int out_heads = 0);
void scale_inplace(void* x, bool f32, const float* s, size_t n, hipStream_t st);  // x *= s[0] (no-op when 1)
// ring-attention LSE merge; st: element strides of o_acc (b, t, h), lse_acc (b, h, t), o (b, t, h), lse (b, h, t)
// zero n byte ranges of buf (desc int64 [n][3] on the device = start, end, bytes of the ranges before; 16-B
// aligned); total_bytes: all ranges together
void zero_ranges(void* buf, const int64_t* desc, int n, int64_t total_bytes, hipStream_t st);
void lse_merge(float* o_acc, float* lse_acc, const void* o, const float* lse, const int64_t* st, int B, int T, int H,
               int D, hipStream_t stream);

// cross_entropy.hip
void cross_entropy(const void* logits, int64_t ld, const int64_t* targets, int N, int V, int ignore_index,
                   float* loss, void* dlogits, const float* inv_n, hipStream_t st);
int cross_entropy_max_vocab();

// adamw.hip
void adamw_flat(void* param_bf16, float* master, float* m, float* v, const void* grad, bool grad_f32, size_t n,
                float lr, float b1, float b2, float eps, float wd, int step, float grad_scale,
                const float* scale_ptr, const uint8_t* wd_blocks, const float* hyper, hipStream_t st);
int sumsq_blocks(size_t n);
void sumsq(const void* x, bool f32, size_t n, float* part, hipStream_t st);
// out[0] = sqrt(sum(part[0..G))) * grad_scale (the gradient norm), out[1] = min(max_norm / (out[0] + 1e-6), 1)
void clip_coef(const float* part, int G, float grad_scale, float max_norm, float* out, hipStream_t st);

// embedding.hip
void embedding_fwd(const int64_t* idx, const void* wte, const void* wpe, void* out, int64_t N, int T, int C,
                   int pos_offset, int64_t V, hipStream_t st);
int64_t embedding_bwd_chunks(int64_t N);  // fp32 workspace: 2 * chunks * C floats
void embedding_bwd(const void* dx, const int32_t* sorted, const int32_t* perm, void* dwte, void* dwpe, bool grad_f32,
                   float* part, int64_t N, int Bn, int T, int C, int64_t V, hipStream_t st);

// gemm.hip: C[M,N] = epi(A[M,K] B[N,K]^T); epi 0 plain (+bias), 1 GELU (aux <- pre-activation),
// 2 ReLU, 3 GELU backward (aux = pre-activation in), 4 ReLU backward (aux = ReLU output in);
// 3 / 4 write column sums of C to colpart [gemm_colsum_groups(M)][N] (fp32)
struct GemmArgs {
  const uint16_t* A;
  const uint16_t* B;
  uint16_t* C;
  const uint16_t* bias;
  uint16_t* aux;
  float* colpart;
  int64_t lda, ldb, ldc, ldaux;
  int M, N, K;
  int group_m;  // set by gemm_tn
  float* delta;  // epilogue 6: [M / T, N / 64, T] row sums of C * aux per 64-column head
  int T;         // epilogue 6: rows per sequence
};
void gemm_tn(const GemmArgs& a, int epi, hipStream_t st);
// phased: 0 single-phase, 2 asym DMA, 4 ping-pong kernel (gemm_pp.hip); reserve_cus >= 0: CUs left
// free by the persistent grids (collectives in flight), -1 keeps the current setting
void gemm_set_config(int mfma, int group_m, int phased, int reserve_cus = -1, int persistent = -1);
// workgroup cap of the persistent GEMM grids (CUs minus reserve_cus; 2^30 when non-persistent)
int gemm_grid_cap();
void gemm_tn_pp(const GemmArgs& a, int epi, int ctas, hipStream_t st);  // gemm_pp.hip
int gemm_pp_colsum_groups(int M, int K);
bool gemm_pp_quad_epilogue(int K, int epi);
int gemm_colsum_groups(int M, int K);  // column-sum partial rows (epi 3 / 4) of the kernel serving K
bool gemm_uses_pp(int K, int epi, int T);
// gemm_wgrad.hip: dW[P,Q] (+)= dY[M,P]^T X[M,Q]; part: fp32 [S, P, Q] workspace (wgrad_plan)
void wgrad_plan(int M, int P, int Q, int* S, int* slice);
void wgrad_set_mfma(int mf);
void wgrad_force_slices(int s);
// bpart / bout (optional): also the bias gradient db[P] (+)= column sums of dY, through an fp32 [S][P]
// workspace (S = wgrad_bias_slices); returns whether it was computed (16x16x32 kernel only)
int wgrad_bias_slices(int M, int P, int Q);
// wgrad_pp.hip: the ping-pong weight-gradient kernel (fp32 targets; wgrad() dispatches to it)
bool wgrad_pp_supported(int M, int P, int Q, int S, int slice);
void wgrad_pp(const void* dy, int64_t lda, const void* x, int64_t ldb, int M, int P, int Q, int S, int slice,
              float* part, float* out, bool accumulate, float* bpart, int ctas, hipStream_t st);
// hybrid form (no bias, more tiles than workgroups): whole tiles for the grid's whole rounds, slices for
// the last one, finished by an ordered fix-up; part: wgrad_pp_hy_ws_floats floats
bool wgrad_hy_plan(int M, int P, int Q, int ctas, int* full, int* rem, int* S, int* slice_kt);
int64_t wgrad_pp_hy_ws_floats(int M, int P, int Q, int ctas);
void wgrad_pp_hy(const void* dy, int64_t lda, const void* x, int64_t ldb, int M, int P, int Q, float* part,
                 float* out, bool accumulate, int ctas, hipStream_t st);
void wgrad_set_hy(int on);  // A/B: hybrid weight gradients where they apply
// workspace floats wgrad() needs for this call (slice slabs or stream-K pieces)
int64_t wgrad_ws_floats(int M, int P, int Q, bool out_f32, bool bias);
bool wgrad(const void* dy, int64_t lda, const void* x, int64_t ldb, int M, int P, int Q, float* part, void* out,
           bool out_f32, bool accumulate, hipStream_t st, float* bpart = nullptr, void* bout = nullptr,
           bool bout_f32 = false);

// transpose.hip: desc int64 [n][6] = (src, dst, rows, cols, first tile, tiles per row band)
int transpose_tiles(int R, int C);
void transpose_batch(const int64_t* desc, int n, int total_tiles, hipStream_t st);

// sampling.hip: Gumbel-max draw of one token per row of logits [B, V] (temperature <= 0: argmax)
void sample_tokens(const void* logits, bool bf16_in, int64_t ld, int B, int V, float temperature, uint64_t seed,
                   int64_t* out, hipStream_t st);

// gemv.hip: y[M, N] = act(in[M, K] W[N, K]^T + bias) for M <= gemv_max_rows() (decode projections),
// in = x, or norm(x + res) with the residual stream x + res written to s_out when gamma is set
struct GemvArgs {
  const uint16_t* x;
  int64_t ldx;
  const uint16_t* res;    // nullable (NORM only)
  int64_t ldr;
  const uint16_t* gamma;  // nullable: no norm prologue
  const uint16_t* beta;   // nullable: RMSNorm / no shift
  uint16_t* s_out;        // nullable: x + res
  int64_t lds;
  float eps;
  int rms;
  const uint16_t* w;
  int64_t ldw;
  const uint16_t* bias;   // nullable
  uint16_t* y;
  int64_t ldy;
  int N, K, Mr;
  int act;  // 0 none, 1 GELU (tanh), 2 ReLU
  // decode KV-cache append (nullable kc): output columns [q_cols, q_cols + kv_cols) of row m
  // also go to kc[m, *pos, :], the next kv_cols to vc[m, *pos, :] (caches [B, S_max, kv_cols])
  uint16_t* kc;
  uint16_t* vc;
  const int64_t* pos;
  int pos_per_row;  // pos holds one position per row (continuous batching) instead of one
  int64_t kv_ldb;
  int q_cols, kv_cols, kv_smax;  // positions outside [0, kv_smax) are dropped, never written
};
int gemv_max_rows();
void gemv(const GemvArgs& a, hipStream_t st);

// attention.hip
bool attn_supported_head_dim(int D);
int attn_bwd_key_block(int D);  // keys per backward workgroup = dq_acc slab count divisor
bool attn_bwd_uses_ks(int D);    // the key-stationary backward serves head dim D (q / k must be pre-rotated)
// attn_bwd_ks.hip: keys per workgroup; one pass of the key-stationary main kernel (AttnBwdArgs as attn_bwd)
int attn_bwd_ks_key_block();

void attn_bwd_set_ks(int mask);  // A/B: bit 0 = D 64, bit 1 = D 128 on the key-stationary kernel
void attn_bwd_ks_launch(const AttnBwdArgs& a, hipStream_t st);
// attn_decode.hip: split-KV single-query attention over a KV cache
bool attn_decode_supported(int D, int group);
int attn_decode_splits(int B, int Hkv, int S_max);
void attn_decode(const DecodeArgs& a, hipStream_t st);
void attn_fwd(const AttnFwdArgs& a, hipStream_t st);
void attn_bwd(const AttnBwdArgs& a, hipStream_t st);

}  // namespace pllm

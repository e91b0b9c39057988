// torch op registration for the gfx950 kernels (namespace torch.ops.pllm).
//
// Every op checks device/dtype/shape contracts on the host BEFORE launching
// (a wrong shape must fail here, never fault on the GPU) and launches on the
// current HIP stream, so the ops compose with torch streams and hipGraph capture.
#include <ATen/ATen.h>
#include <cstdio>
#include <cstdlib>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "kernels.h"

using at::Tensor;

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_gpu(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
}
void check_bf16(const Tensor& t, const char* name) {
  check_gpu(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bfloat16, got ", t.scalar_type());
}
void check_contig(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
void check_aligned16(const Tensor& t, const char* name) {
  TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0, name, " must be 16-byte aligned");
}
const void* opt_ptr(const std::optional<Tensor>& t) { return t.has_value() ? t->data_ptr() : nullptr; }
// gradient accumulation targets (views of the optimizer's flat gradient): bf16 or fp32;
// returns true for fp32
bool check_grad(const Tensor& t, const char* name) {
  check_gpu(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kFloat, name,
              " must be bfloat16 or float32, got ", t.scalar_type());
  return t.scalar_type() == at::kFloat;
}

// ---------------------------------------------------------------- norms
std::vector<Tensor> norm_fwd(const Tensor& x, const std::optional<Tensor>& res, const Tensor& w,
                             const std::optional<Tensor>& b, double eps, bool rms) {
  check_bf16(x, "x");
  check_contig(x, "x");
  TORCH_CHECK(x.dim() == 2, "norm_fwd expects [N, C]");
  const int64_t N = x.size(0), C = x.size(1);
  TORCH_CHECK(C % 8 == 0 && C <= 4096, "norm: C must be a multiple of 8 and <= 4096, got ", C);
  check_bf16(w, "weight");
  TORCH_CHECK(w.numel() == C && w.is_contiguous(), "norm weight shape");
  if (b) {
    check_bf16(*b, "bias");
    TORCH_CHECK(b->numel() == C && b->is_contiguous(), "norm bias shape");
  }
  Tensor s;
  if (res) {
    check_bf16(*res, "residual");
    check_contig(*res, "residual");
    TORCH_CHECK(res->sizes() == x.sizes(), "residual shape");
    s = at::empty_like(x);
  } else {
    s = at::empty({0}, x.options());  // no residual: the residual stream is x itself (never aliased)
  }
  Tensor y = at::empty_like(x);
  auto f32 = x.options().dtype(at::kFloat);
  Tensor mean = at::empty({N}, f32), rstd = at::empty({N}, f32);
  if (N > 0)
    pllm::norm_fwd(x.data_ptr(), opt_ptr(res), w.data_ptr(), opt_ptr(b), y.data_ptr(), res ? s.data_ptr() : nullptr,
                   mean.data_ptr<float>(), rstd.data_ptr<float>(), (int)N, (int)C, (float)eps, rms, cur_stream());
  return {y, s, mean, rstd};
}

// dw_acc/db_acc: if given, the weight/bias gradients are ADDED into these (e.g. views of
// the optimizer's flat gradient buffer) and only dx is returned.
std::vector<Tensor> norm_bwd(const Tensor& dy, const Tensor& s, const Tensor& w, const Tensor& mean,
                             const Tensor& rstd, const std::optional<Tensor>& ds, bool has_bias, bool rms,
                             const std::optional<Tensor>& dw_acc, const std::optional<Tensor>& db_acc,
                             const std::optional<Tensor>& xb_acc) {
  check_bf16(dy, "dy");
  check_bf16(s, "s");
  check_contig(dy, "dy");
  check_contig(s, "s");
  TORCH_CHECK(dy.sizes() == s.sizes() && dy.dim() == 2, "norm_bwd shapes");
  const int64_t N = dy.size(0), C = dy.size(1);
  if (ds) {
    check_bf16(*ds, "ds");
    check_contig(*ds, "ds");
    TORCH_CHECK(ds->sizes() == dy.sizes(), "ds shape");
  }
  const bool acc = dw_acc.has_value();
  TORCH_CHECK(!has_bias || acc == db_acc.has_value(), "norm_bwd: dw_acc and db_acc must be given together");
  bool gf32 = false;
  if (acc) {
    gf32 = check_grad(*dw_acc, "dw_acc");
    TORCH_CHECK(dw_acc->numel() == C && dw_acc->is_contiguous(), "dw_acc shape");
    if (has_bias) {
      TORCH_CHECK(check_grad(*db_acc, "db_acc") == gf32, "db_acc dtype must match dw_acc");
      TORCH_CHECK(db_acc->numel() == C && db_acc->is_contiguous(), "db_acc shape");
    }
  } else {
    TORCH_CHECK(w.scalar_type() == at::kBFloat16, "norm_bwd: bf16 weight");
  }
  Tensor dx = at::empty_like(dy);
  Tensor dw = acc ? *dw_acc : at::zeros({C}, w.options());
  Tensor db = has_bias ? (acc ? *db_acc : at::zeros({C}, w.options())) : Tensor();
  const int G = pllm::norm_bwd_grid((int)N, (int)C);
  auto f32 = dy.options().dtype(at::kFloat);
  Tensor dwp = at::empty({G, C}, f32);
  Tensor dbp = has_bias ? at::empty({G, C}, f32) : Tensor();
  Tensor xbp;
  if (xb_acc) {  // fused bias gradient of the producer of x: accumulated into xb_acc
    TORCH_CHECK(acc && check_grad(*xb_acc, "xb_acc") == gf32, "xb_acc needs dw_acc targets of the same dtype");
    TORCH_CHECK(xb_acc->numel() == C && xb_acc->is_contiguous(), "xb_acc shape");
    xbp = at::empty({G, C}, f32);
  }
  if (N > 0) {
    pllm::norm_bwd(dy.data_ptr(), s.data_ptr(), w.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                   opt_ptr(ds), dx.data_ptr(), dwp.data_ptr<float>(), has_bias ? dbp.data_ptr<float>() : nullptr,
                   dw.data_ptr(), has_bias ? db.data_ptr() : nullptr, gf32, (int)N, (int)C, rms, acc,
                   xb_acc ? xbp.data_ptr<float>() : nullptr, xb_acc ? xb_acc->data_ptr() : nullptr, true,
                   cur_stream());
  }
  if (acc) return {dx};
  if (!has_bias) return {dx, dw};
  return {dx, dw, db};
}

// Op entry points (a mutable custom op may not return a Tensor list: torch.compile's
// auto-functionalisation only handles single-Tensor returns).
// norm_bwd: pure -> (dx, dw, db) (db empty without bias);  norm_bwd_acc: adds into the targets,
// returns dx.
std::tuple<Tensor, Tensor, Tensor> norm_bwd_op(const Tensor& dy, const Tensor& s, const Tensor& w, const Tensor& mean,
                                               const Tensor& rstd, const std::optional<Tensor>& ds, bool has_bias,
                                               bool rms) {
  auto o = norm_bwd(dy, s, w, mean, rstd, ds, has_bias, rms, std::nullopt, std::nullopt, std::nullopt);
  return {o[0], o[1], has_bias ? o[2] : at::empty({0}, w.options())};
}
Tensor norm_bwd_acc_op(const Tensor& dy, const Tensor& s, const Tensor& w, const Tensor& mean, const Tensor& rstd,
                       const std::optional<Tensor>& ds, bool has_bias, bool rms, Tensor& dw_acc,
                       const std::optional<Tensor>& db_acc, const std::optional<Tensor>& xb_acc) {
  return norm_bwd(dy, s, w, mean, rstd, ds, has_bias, rms, dw_acc, db_acc, xb_acc)[0];
}

// column sums of dy [..., C] (bias gradient); added into out_acc if given, else returned
Tensor bias_grad(const Tensor& dy, const std::optional<Tensor>& out_acc) {
  check_bf16(dy, "dy");
  check_contig(dy, "dy");
  const int64_t C = dy.size(-1);
  const int64_t N = C ? dy.numel() / C : 0;
  TORCH_CHECK(C % 8 == 0, "bias_grad: C % 8");
  Tensor out;
  bool of32 = false;
  if (out_acc) {
    of32 = check_grad(*out_acc, "out_acc");
    TORCH_CHECK(out_acc->numel() == C && out_acc->is_contiguous(), "out_acc shape");
    out = *out_acc;
  } else {
    out = at::zeros({C}, dy.options());
  }
  if (N > 0) {
    Tensor part = at::empty({pllm::colsum_groups((int)N), C}, dy.options().dtype(at::kFloat));
    pllm::bias_grad(dy.data_ptr(), (int)N, (int)C, part.data_ptr<float>(), out.data_ptr(), of32, true, cur_stream());
  }
  // accumulate mode returns an empty tensor: a custom op's output must not alias an input
  return out_acc ? at::empty({0}, dy.options()) : out;
}

// ---------------------------------------------------------------- weight-gradient GEMM
// out[P, Q] (+)= dy[M, P]^T @ x[M, Q]; accumulates into out_acc if given, else returns a new tensor.
// bias_acc (requires out_acc): the bias gradient column sums of dy are added into it too -- inside the
// GEMM when its kernel can (wgrad_kernel's all-ones MFMAs), else by the bias_grad kernels
Tensor bias_grad(const Tensor& dy, const std::optional<Tensor>& out_acc);
// overwrite (with out_acc): store dW into out_acc instead of adding (its first write of a step)
Tensor wgrad(const Tensor& dy, const Tensor& x, const std::optional<Tensor>& out_acc,
             const std::optional<Tensor>& bias_acc, bool overwrite) {
  check_bf16(dy, "dy");
  check_bf16(x, "x");
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && dy.size(0) == x.size(0), "wgrad: dy [M,P], x [M,Q]");
  TORCH_CHECK(dy.stride(1) == 1 && x.stride(1) == 1, "wgrad: unit column stride");
  const int64_t M = dy.size(0), P = dy.size(1), Q = x.size(1);
  TORCH_CHECK(P % 8 == 0 && Q % 8 == 0 && dy.stride(0) % 8 == 0 && x.stride(0) % 8 == 0, "wgrad: dims % 8");
  TORCH_CHECK(M % 64 == 0, "wgrad: M (tokens) must be a multiple of 64");
  check_aligned16(dy, "dy");
  check_aligned16(x, "x");
  Tensor out;
  bool of32 = false;
  if (out_acc) {
    of32 = check_grad(*out_acc, "out_acc");
    TORCH_CHECK(out_acc->numel() == P * Q && out_acc->is_contiguous(), "wgrad: out_acc shape");
    check_aligned16(*out_acc, "out_acc");
    out = *out_acc;
  } else {
    out = at::empty({P, Q}, dy.options());
  }
  int S = 1, slice = 1;
  pllm::wgrad_plan((int)M, (int)P, (int)Q, &S, &slice);
  const bool of32_pre = out_acc && out_acc->scalar_type() == at::kFloat;
  Tensor part = at::empty({std::max<int64_t>(pllm::wgrad_ws_floats((int)M, (int)P, (int)Q, of32_pre,
                                                                   bias_acc.has_value()), 1)},
                          dy.options().dtype(at::kFloat));
  bool bf32 = false;
  Tensor bpart;
  if (bias_acc) {
    TORCH_CHECK(out_acc.has_value(), "wgrad: bias_acc needs out_acc");
    bf32 = check_grad(*bias_acc, "bias_acc");
    TORCH_CHECK(bias_acc->numel() == P && bias_acc->is_contiguous(), "wgrad: bias_acc [P]");
    check_aligned16(*bias_acc, "bias_acc");
    bpart = at::empty({S, P}, dy.options().dtype(at::kFloat));
  }
  bool fused_b = false;
  if (M > 0)
    fused_b = pllm::wgrad(dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), (int)M, (int)P, (int)Q,
                          part.data_ptr<float>(), out.data_ptr(), of32, out_acc.has_value() && !overwrite,
                          cur_stream(), bias_acc ? bpart.data_ptr<float>() : nullptr,
                          bias_acc ? bias_acc->data_ptr() : nullptr, bf32);
  else if (!out_acc || overwrite)
    out.zero_();
  if (bias_acc && M > 0 && !fused_b) bias_grad(dy.is_contiguous() ? dy : dy.contiguous(), bias_acc);
  return out_acc ? at::empty({0}, dy.options()) : out;
}

// ---------------------------------------------------------------- fused-epilogue GEMM
// a [M, K] (row stride lda), b [N, K] contiguous -> [out [M, N], aux]:
// epi 0: out = a b^T (+ bias); 1: out = gelu(pre), aux = pre = a b^T + bias; 2: out = relu(a b^T + bias);
// 3 / 4: out = (a b^T) * gelu'(aux) / * (aux > 0), and when bias_acc is given its column sums are
// added into it (the producing layer's bias gradient, bf16 or fp32); 5: aux = [gate | up] [M, 2N],
// out = [dgate | dup] [M, 2N] with d = a b^T the SwiGLU output's gradient (swiglu_bwd fused)
std::tuple<Tensor, Tensor> gemm_tn(const Tensor& a, const Tensor& b, const std::optional<Tensor>& bias, int64_t epi,
                            const std::optional<Tensor>& aux, const std::optional<Tensor>& bias_acc, int64_t T) {
  check_bf16(a, "a");
  check_bf16(b, "b");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.size(1) == b.size(1), "gemm_tn: a [M, K], b [N, K]");
  TORCH_CHECK(a.stride(1) == 1 && b.is_contiguous(), "gemm_tn: K-contiguous operands");
  TORCH_CHECK(epi >= 0 && epi <= 7, "gemm_tn: epi 0..7");
  const int64_t M = a.size(0), K = a.size(1), N = epi == 7 ? b.size(0) / 2 : b.size(0);
  // epi 7: b = [gate | up] rows [2F, K] -> out = silu(gate) * up [M, F], aux = [gate | up] [M, 2F]
  // (the llama up-projection with its SwiGLU; ping-pong kernel only)
  TORCH_CHECK(epi != 7 || (b.size(0) % 16 == 0 && pllm::gemm_uses_pp((int)K, 7, 0)),
              "gemm_tn: epi 7 needs 2F % 16 == 0, K >= 128 and the ping-pong kernel");
  TORCH_CHECK(K % 64 == 0 && K > 0, "gemm_tn: K must be a positive multiple of 64, got ", K);
  TORCH_CHECK(N % 8 == 0 && a.stride(0) % 8 == 0, "gemm_tn: N and lda must be multiples of 8");
  TORCH_CHECK(M < (1 << 30) && N < (1 << 30), "gemm_tn: dims");
  TORCH_CHECK((int64_t)(std::min<int64_t>(M, 256) - 1) * a.stride(0) * 2 + K * 2 < (1ll << 31) &&
                  (int64_t)(std::min<int64_t>(N, 256) - 1) * K * 2 + K * 2 < (1ll << 31),
              "gemm_tn: a 256-row panel must span < 2 GiB");
  check_aligned16(a, "a");
  check_aligned16(b, "b");
  if (bias) {
    check_bf16(*bias, "bias");
    TORCH_CHECK(bias->numel() == N && bias->is_contiguous(), "gemm_tn: bias [N]");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(bias->data_ptr()) & 7) == 0, "gemm_tn: bias 8-byte aligned");
    TORCH_CHECK(epi <= 2, "gemm_tn: bias only in the forward epilogues");
  }
  Tensor out = at::empty({M, epi == 5 ? 2 * N : N}, a.options());
  Tensor aux_out = epi == 6   ? at::empty({T > 0 ? M / T : 0, N / 64, T}, a.options().dtype(at::kFloat))
                   : epi == 7 ? at::empty({M, 2 * N}, a.options())
                              : at::empty({epi == 1 ? M : 0, N}, a.options());
  pllm::GemmArgs g{};
  g.A = (const uint16_t*)a.data_ptr();
  g.B = (const uint16_t*)b.data_ptr();
  g.C = (uint16_t*)out.data_ptr();
  g.bias = bias ? (const uint16_t*)bias->data_ptr() : nullptr;
  g.lda = a.stride(0);
  g.ldb = K;
  g.ldc = epi == 5 ? 2 * N : N;
  g.M = (int)M;
  g.N = (int)N;
  g.K = (int)K;
  Tensor part;
  if (epi == 1) {
    g.aux = (uint16_t*)aux_out.data_ptr();
    g.ldaux = N;
  } else if (epi == 7) {
    TORCH_CHECK(!bias, "gemm_tn: epi 7 has no bias");
    g.aux = (uint16_t*)aux_out.data_ptr();
    g.ldaux = 2 * N;
  } else if (epi == 6) {
    TORCH_CHECK(aux.has_value(), "gemm_tn: epi 6 needs aux = the attention output [M, N]");
    check_bf16(*aux, "aux");
    TORCH_CHECK(aux->dim() == 2 && aux->size(0) == M && aux->size(1) == N && aux->stride(1) == 1 &&
                    aux->stride(0) % 8 == 0, "gemm_tn: aux [M, N]");
    TORCH_CHECK(T > 0 && M % T == 0 && N % 64 == 0, "gemm_tn: epi 6 needs T | M and 64 | N (head dim 64)");
    check_aligned16(*aux, "aux");
    g.aux = (uint16_t*)aux->data_ptr();
    g.ldaux = aux->stride(0);
    g.delta = aux_out.data_ptr<float>();
    g.T = (int)T;
  } else if (epi == 5) {
    TORCH_CHECK(aux.has_value(), "gemm_tn: epi 5 needs aux = [gate | up]");
    check_bf16(*aux, "aux");
    TORCH_CHECK(aux->dim() == 2 && aux->size(0) == M && aux->size(1) == 2 * N && aux->stride(1) == 1 &&
                    aux->stride(0) % 8 == 0, "gemm_tn: aux [M, 2N]");
    check_aligned16(*aux, "aux");
    g.aux = (uint16_t*)aux->data_ptr();
    g.ldaux = aux->stride(0);
  } else if (epi >= 3) {
    TORCH_CHECK(aux.has_value(), "gemm_tn: epi 3 / 4 need aux");
    check_bf16(*aux, "aux");
    TORCH_CHECK(aux->dim() == 2 && aux->size(0) == M && aux->size(1) == N && aux->stride(1) == 1 &&
                    aux->stride(0) % 8 == 0, "gemm_tn: aux [M, N]");
    check_aligned16(*aux, "aux");
    g.aux = (uint16_t*)aux->data_ptr();
    g.ldaux = aux->stride(0);
    part = at::empty({pllm::gemm_colsum_groups((int)M, (int)K), N}, a.options().dtype(at::kFloat));
    g.colpart = part.data_ptr<float>();
  }
  bool of32 = false;
  if (bias_acc) {
    TORCH_CHECK(epi == 3 || epi == 4, "gemm_tn: bias_acc only with epi 3 / 4");
    of32 = check_grad(*bias_acc, "bias_acc");
    TORCH_CHECK(bias_acc->numel() == N && bias_acc->is_contiguous(), "gemm_tn: bias_acc [N]");
  }
  if (M > 0) {
    pllm::gemm_tn(g, (int)epi, cur_stream());
    if (bias_acc)
      pllm::col_reduce(g.colpart, pllm::gemm_colsum_groups((int)M, (int)K), (int)N, bias_acc->data_ptr(), of32, true,
                       cur_stream());
  }
  return {out, aux_out};  // a (Tensor, Tensor) tuple: functionalization rejects Tensor[] beside an (a!) arg
}

// ---------------------------------------------------------------- skinny GEMM (decode)
// y[M, N] = act(in[M, K] w[N, K]^T (+ bias)) for M <= 8 token rows; in = x, or (gamma given)
// norm(x (+ res)) -- then also returns the residual stream s = x + res when res is given
std::tuple<Tensor, Tensor> gemv(const Tensor& x, const Tensor& w, const std::optional<Tensor>& bias,
                         const std::optional<Tensor>& res, const std::optional<Tensor>& gamma,
                         const std::optional<Tensor>& beta, double eps, int64_t rms, int64_t act,
                         const std::optional<Tensor>& kc, const std::optional<Tensor>& vc,
                         const std::optional<Tensor>& pos, int64_t q_cols) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "gemv: x [M,K], w [N,K]");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(M <= pllm::gemv_max_rows(), "gemv: at most ", pllm::gemv_max_rows(), " rows");
  TORCH_CHECK(K % 8 == 0 && x.stride(1) == 1 && w.stride(1) == 1 && x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0,
              "gemv: K % 8 == 0, unit column stride, row strides % 8");
  TORCH_CHECK(act >= 0 && act <= 2, "gemv: act 0 (none), 1 (gelu), 2 (relu)");
  check_aligned16(x, "x");
  check_aligned16(w, "w");
  if (bias) {
    check_bf16(*bias, "bias");
    TORCH_CHECK(bias->numel() == N && bias->is_contiguous(), "gemv: bias [N]");
  }
  TORCH_CHECK(!res || gamma, "gemv: res requires the norm prologue (gamma)");
  if (gamma) {
    check_bf16(*gamma, "gamma");
    TORCH_CHECK(gamma->numel() == K && gamma->is_contiguous(), "gemv: gamma [K]");
    check_aligned16(*gamma, "gamma");
    if (beta) {
      check_bf16(*beta, "beta");
      TORCH_CHECK(beta->numel() == K && beta->is_contiguous(), "gemv: beta [K]");
      check_aligned16(*beta, "beta");
    }
  }
  if (res) {
    check_bf16(*res, "res");
    TORCH_CHECK(res->dim() == 2 && res->size(0) == M && res->size(1) == K && res->stride(1) == 1 &&
                    res->stride(0) % 8 == 0,
                "gemv: res [M,K], unit column stride");
    check_aligned16(*res, "res");
  }
  int64_t kv_cols = 0, kv_ldb = 0;
  if (kc) {
    TORCH_CHECK(vc && pos, "gemv: kc needs vc and pos");
    check_bf16(*kc, "kc");
    check_bf16(*vc, "vc");
    TORCH_CHECK(kc->is_contiguous() && vc->is_contiguous() && kc->sizes() == vc->sizes() && kc->dim() >= 3 &&
                    kc->size(0) == M,
                "gemv: kc/vc contiguous [B = rows, S_max, ...] of equal shape");
    kv_ldb = kc->stride(0);
    kv_cols = kc->stride(1);
    TORCH_CHECK(q_cols >= 0 && q_cols + 2 * kv_cols == N, "gemv: q_cols + 2 * kv_cols must equal N");
    TORCH_CHECK(pos->scalar_type() == at::kLong && (pos->numel() == 1 || pos->numel() == M) &&
                    pos->is_contiguous() && pos->device() == x.device(),
                "gemv: pos int64 [1] or [M] (one position per row) on the device");
    // the position itself stays on the device (hipGraph replay); the caller bounds it by S_max
  }
  Tensor y = at::empty({M, N}, x.options());
  Tensor s;
  if (res) s = at::empty({M, K}, x.options());
  if (M > 0 && N > 0) {
    pllm::GemvArgs a{};
    a.x = (const uint16_t*)x.data_ptr();
    a.ldx = x.stride(0);
    a.res = res ? (const uint16_t*)res->data_ptr() : nullptr;
    a.ldr = res ? res->stride(0) : 0;
    a.gamma = gamma ? (const uint16_t*)gamma->data_ptr() : nullptr;
    a.beta = (gamma && beta) ? (const uint16_t*)beta->data_ptr() : nullptr;
    a.s_out = res ? (uint16_t*)s.data_ptr() : nullptr;
    a.lds = K;
    a.eps = (float)eps;
    a.rms = (int)rms;
    a.w = (const uint16_t*)w.data_ptr();
    a.ldw = w.stride(0);
    a.bias = bias ? (const uint16_t*)bias->data_ptr() : nullptr;
    a.y = (uint16_t*)y.data_ptr();
    a.ldy = N;
    a.N = (int)N;
    a.K = (int)K;
    a.Mr = (int)M;
    a.act = (int)act;
    a.kc = kc ? (uint16_t*)kc->data_ptr() : nullptr;
    a.vc = kc ? (uint16_t*)vc->data_ptr() : nullptr;
    a.pos = kc ? (const int64_t*)pos->data_ptr() : nullptr;
    a.pos_per_row = kc && pos->numel() == M && M > 1;
    a.kv_ldb = kv_ldb;
    a.q_cols = (int)q_cols;
    a.kv_cols = (int)kv_cols;
    a.kv_smax = kc ? (int)kc->size(1) : 0;
    TORCH_CHECK(!a.kc || a.act == 0, "gemv: KV-cache append takes no activation");
    pllm::gemv(a, cur_stream());
  }
  if (!res) s = at::empty({0}, x.options());
  return {y, s};
}

// ---------------------------------------------------------------- activations
Tensor act_fwd(const Tensor& x, int64_t op) {
  check_bf16(x, "x");
  check_contig(x, "x");
  TORCH_CHECK(x.numel() % 8 == 0, "activation numel must be a multiple of 8");
  Tensor y = at::empty_like(x);
  if (x.numel()) pllm::act_fwd((int)op, x.data_ptr(), y.data_ptr(), x.numel(), cur_stream());
  return y;
}
Tensor act_bwd(const Tensor& dy, const Tensor& xin, int64_t op) {
  check_bf16(dy, "dy");
  check_bf16(xin, "x");
  check_contig(dy, "dy");
  check_contig(xin, "x");
  TORCH_CHECK(dy.numel() == xin.numel() && dy.numel() % 8 == 0, "activation bwd shapes");
  Tensor dx = at::empty_like(dy);
  if (dy.numel()) pllm::act_bwd((int)op, dy.data_ptr(), xin.data_ptr(), dx.data_ptr(), dy.numel(), cur_stream());
  return dx;
}
// activation backward + bias gradient of the producing linear layer (column sums of dx),
// added into bias_acc; returns dx
Tensor act_bwd_bias(const Tensor& dy, const Tensor& xin, int64_t op, Tensor& bias_acc) {
  check_bf16(dy, "dy");
  check_bf16(xin, "x");
  check_contig(dy, "dy");
  check_contig(xin, "x");
  const bool gf32 = check_grad(bias_acc, "bias_acc");
  const int64_t C = dy.size(-1);
  TORCH_CHECK(dy.sizes() == xin.sizes() && C % 8 == 0, "act_bwd_bias shapes");
  TORCH_CHECK(bias_acc.numel() == C && bias_acc.is_contiguous(), "bias_acc shape");
  const int64_t N = dy.numel() / C;
  Tensor dx = at::empty_like(dy);
  if (N > 0) {
    Tensor part = at::empty({pllm::colsum_groups((int)N), C}, dy.options().dtype(at::kFloat));
    pllm::act_bwd_bias((int)op, dy.data_ptr(), xin.data_ptr(), dx.data_ptr(), (int)N, (int)C, part.data_ptr<float>(),
                       bias_acc.data_ptr(), gf32, true, cur_stream());
  }
  return dx;
}

Tensor swiglu_fwd(const Tensor& gu) {
  check_bf16(gu, "gate_up");
  check_contig(gu, "gate_up");
  const int64_t F2 = gu.size(-1);
  TORCH_CHECK(F2 % 16 == 0, "swiglu: last dim must be 2F with F % 8 == 0");
  auto sizes = gu.sizes().vec();
  sizes.back() = F2 / 2;
  Tensor y = at::empty(sizes, gu.options());
  const int64_t rows = gu.numel() / F2;
  if (rows) pllm::swiglu_fwd(gu.data_ptr(), y.data_ptr(), rows, (int)(F2 / 2), cur_stream());
  return y;
}
Tensor swiglu_bwd(const Tensor& dy, const Tensor& gu) {
  check_bf16(dy, "dy");
  check_bf16(gu, "gate_up");
  check_contig(dy, "dy");
  check_contig(gu, "gate_up");
  const int64_t F2 = gu.size(-1);
  TORCH_CHECK(dy.size(-1) * 2 == F2 && dy.numel() * 2 == gu.numel(), "swiglu bwd shapes");
  Tensor dgu = at::empty_like(gu);
  const int64_t rows = gu.numel() / F2;
  if (rows) pllm::swiglu_bwd(dy.data_ptr(), gu.data_ptr(), dgu.data_ptr(), rows, (int)(F2 / 2), cur_stream());
  return dgu;
}

// packed rows [..., n_heads_total * D]; rotates the first n_rot heads; T = positions per sequence
// attention pre-pass: the rotated q and k heads of a packed [.., (H + 2 Hkv) D] qkv tensor as one
// contiguous [.., (H + Hkv) D] buffer (v is not copied)
Tensor rope_qk(const Tensor& x, const Tensor& cos, const Tensor& sin, int64_t n_heads_total, int64_t n_rot, int64_t T) {
  check_bf16(x, "x");
  check_contig(x, "x");
  TORCH_CHECK(cos.scalar_type() == at::kFloat && sin.scalar_type() == at::kFloat, "rope tables must be fp32");
  TORCH_CHECK(cos.is_contiguous() && sin.is_contiguous(), "rope tables contiguous");
  const int64_t W = x.size(-1);
  TORCH_CHECK(W % n_heads_total == 0 && n_rot > 0 && n_rot <= n_heads_total, "rope_qk: heads");
  const int64_t D = W / n_heads_total;
  TORCH_CHECK(D % 16 == 0, "rope_qk: head dim must be a multiple of 16");
  TORCH_CHECK(cos.size(-1) == D / 2 && cos.size(0) >= T, "rope_qk: table shape");
  const int64_t rows = x.numel() / W;
  TORCH_CHECK(rows % T == 0, "rope_qk: rows must be a multiple of T");
  auto sizes = x.sizes().vec();
  sizes.back() = n_rot * D;
  Tensor out = at::empty(sizes, x.options());
  if (rows)
    pllm::rope(x.data_ptr(), out.data_ptr(), cos.data_ptr<float>(), sin.data_ptr<float>(), rows, (int)T,
               (int)n_heads_total, (int)n_rot, (int)D, 0, false, cur_stream(), (int)n_rot);
  return out;
}

Tensor rope(const Tensor& x, const Tensor& cos, const Tensor& sin, int64_t n_heads_total, int64_t n_rot, int64_t T,
            int64_t pos_offset, bool inverse) {
  check_bf16(x, "x");
  check_contig(x, "x");
  TORCH_CHECK(cos.scalar_type() == at::kFloat && sin.scalar_type() == at::kFloat, "rope tables must be fp32");
  TORCH_CHECK(cos.is_contiguous() && sin.is_contiguous(), "rope tables contiguous");
  const int64_t W = x.size(-1);
  TORCH_CHECK(W % n_heads_total == 0, "rope: width not divisible by heads");
  const int64_t D = W / n_heads_total;
  TORCH_CHECK(D % 16 == 0, "rope: head dim must be a multiple of 16");
  TORCH_CHECK(cos.size(-1) == D / 2 && cos.size(0) >= T + pos_offset, "rope: table shape");
  const int64_t rows = x.numel() / W;
  TORCH_CHECK(rows % T == 0, "rope: rows must be a multiple of T");
  Tensor out = at::empty_like(x);
  if (rows)
    pllm::rope(x.data_ptr(), out.data_ptr(), cos.data_ptr<float>(), sin.data_ptr<float>(), rows, (int)T,
               (int)n_heads_total, (int)n_rot, (int)D, (int)pos_offset, inverse, cur_stream());
  return out;
}

// x *= s in place (x bf16 or fp32, contiguous; s a 1-element fp32 GPU tensor); no pass at all when s == 1
void scale_(Tensor& x, const Tensor& s) {
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat, "scale_: x bf16 or fp32");
  check_contig(x, "x");
  TORCH_CHECK(s.scalar_type() == at::kFloat && s.numel() == 1 && s.is_cuda(), "scale must be a 1-element fp32 GPU tensor");
  TORCH_CHECK(x.numel() % 8 == 0, "scale_: numel % 8");
  check_aligned16(x, "x");
  if (x.numel())
    pllm::scale_inplace(x.data_ptr(), x.scalar_type() == at::kFloat, s.data_ptr<float>(), x.numel(), cur_stream());
}

// ring attention: fold a partial block result (o [B, T, H, D] bf16, lse [B, H, T] fp32) into the
// fp32 accumulators o_acc [B, T, H, D] / lse_acc [B, H, T] in place (views with any row strides)
// ranges: int64 [n, 2] element ranges [start, end) of buf, every bound 16-B aligned, ascending;
// total_len: their summed length (host-known, sizes the grid)
void zero_ranges_(Tensor& buf, const Tensor& ranges, int64_t total_len) {
  check_gpu(buf, "buf");
  check_contig(buf, "buf");
  TORCH_CHECK(ranges.is_cuda() && ranges.scalar_type() == at::kLong && ranges.dim() == 2 && ranges.size(1) == 2 &&
                  ranges.is_contiguous(), "zero_ranges_: ranges int64 [n, 2] on the GPU");
  const int64_t es = buf.element_size();
  TORCH_CHECK((total_len * es) % 16 == 0, "zero_ranges_: 16-B multiples");
  if (ranges.size(0) == 0 || total_len == 0) return;
  // descriptors (start, end, bytes before) in bytes, built on the device (the host never syncs)
  Tensor b = ranges * es;
  Tensor len = b.select(1, 1) - b.select(1, 0);
  Tensor desc = at::cat({b, (at::cumsum(len, 0) - len).unsqueeze(1)}, 1).contiguous();
  pllm::zero_ranges(buf.data_ptr(), desc.data_ptr<int64_t>(), (int)ranges.size(0), total_len * es, cur_stream());
}

void lse_merge_(Tensor& o_acc, Tensor& lse_acc, const Tensor& o, const Tensor& lse) {
  TORCH_CHECK(o_acc.scalar_type() == at::kFloat && lse_acc.scalar_type() == at::kFloat && lse.scalar_type() == at::kFloat,
              "lse_merge_: o_acc / lse_acc / lse fp32");
  check_bf16(o, "o");
  TORCH_CHECK(o_acc.dim() == 4 && o.sizes() == o_acc.sizes(), "lse_merge_: o_acc / o [B, T, H, D]");
  const int64_t B = o.size(0), T = o.size(1), H = o.size(2), D = o.size(3);
  TORCH_CHECK(lse_acc.dim() == 3 && lse_acc.size(0) == B && lse_acc.size(1) == H && lse_acc.size(2) == T &&
                  lse.sizes() == lse_acc.sizes(), "lse_merge_: lse_acc / lse [B, H, T]");
  // a row's D / 8 lanes must sit in ONE wave (64 % (D / 8) == 0): every lane reads lse_acc before lane 0
  // of the row writes the merged value (D = 48 / 80 / 96 would straddle two waves and race)
  TORCH_CHECK(D % 8 == 0 && D <= 128 && 64 % (D / 8) == 0 && o_acc.stride(3) == 1 && o.stride(3) == 1,
              "lse_merge_: D in {8, 16, 32, 64, 128}, unit head stride");
  for (int d = 0; d < 3; ++d)
    TORCH_CHECK(o_acc.stride(d) % 4 == 0 && o.stride(d) % 8 == 0, "lse_merge_: 16-B aligned rows");
  check_aligned16(o_acc, "o_acc");
  check_aligned16(o, "o");
  const int64_t st[12] = {o_acc.stride(0), o_acc.stride(1), o_acc.stride(2), lse_acc.stride(0), lse_acc.stride(1),
                          lse_acc.stride(2), o.stride(0), o.stride(1), o.stride(2), lse.stride(0), lse.stride(1),
                          lse.stride(2)};
  if (o.numel())
    pllm::lse_merge(o_acc.data_ptr<float>(), lse_acc.data_ptr<float>(), o.data_ptr(), lse.data_ptr<float>(), st,
                    (int)B, (int)T, (int)H, (int)D, cur_stream());
}

// ---------------------------------------------------------------- cross entropy
// returns per-row losses (fp32, 0 for ignored rows); if dlogits is given it is
// overwritten with d(mean loss)/dlogits (it may alias logits).
// ``inv_n``: optional fp32 [1] device scalar scaling dlogits (1 / #valid targets of the WHOLE
// batch when the rows are processed in chunks); default 1 / #valid targets of these rows.
Tensor cross_entropy(const Tensor& logits, const Tensor& targets, const std::optional<Tensor>& dlogits,
                     int64_t ignore_index, const std::optional<Tensor>& inv_n_opt) {
  check_bf16(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits must be [N, V] with unit column stride");
  const int64_t N = logits.size(0), V = logits.size(1);
  TORCH_CHECK(logits.stride(0) % 8 == 0 && V % 8 == 0, "cross_entropy: V and row stride must be multiples of 8");
  TORCH_CHECK(V <= pllm::cross_entropy_max_vocab(), "cross_entropy: vocab too large for the register-resident kernel");
  check_aligned16(logits, "logits");
  TORCH_CHECK(targets.is_cuda() && targets.numel() == N, "targets shape");
  Tensor tg = targets.reshape({N}).to(at::kLong).contiguous();
  if (dlogits) {
    check_bf16(*dlogits, "dlogits");
    TORCH_CHECK(dlogits->sizes() == logits.sizes() && dlogits->strides() == logits.strides(), "dlogits layout");
  }
  Tensor loss = at::empty({N}, logits.options().dtype(at::kFloat));
  Tensor inv_n;
  if (inv_n_opt) {
    TORCH_CHECK(inv_n_opt->is_cuda() && inv_n_opt->scalar_type() == at::kFloat && inv_n_opt->numel() == 1,
                "cross_entropy: inv_n must be a 1-element fp32 device tensor");
    inv_n = inv_n_opt->reshape({1});
  } else {
    inv_n = (tg != ignore_index).sum().to(at::kFloat).clamp_min(1.0).reciprocal().reshape({1});
  }
  if (N)
    pllm::cross_entropy(logits.data_ptr(), logits.stride(0), tg.data_ptr<int64_t>(), (int)N, (int)V, (int)ignore_index,
                        loss.data_ptr<float>(), dlogits ? dlogits->data_ptr() : nullptr, inv_n.data_ptr<float>(),
                        cur_stream());
  return loss;
}

// ---------------------------------------------------------------- optimizer
void adamw_(Tensor& param, Tensor& master, Tensor& m, Tensor& v, const Tensor& grad, double lr, double b1, double b2,
            double eps, double wd, int64_t step, double grad_scale, const std::optional<Tensor>& scale,
            const std::optional<Tensor>& wd_mask, const std::optional<Tensor>& hyper) {
  const int64_t n = master.numel();
  TORCH_CHECK(master.scalar_type() == at::kFloat && m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat,
              "adamw: master/m/v must be fp32");
  TORCH_CHECK(m.numel() == n && v.numel() == n && grad.numel() == n, "adamw: sizes");
  TORCH_CHECK(master.is_contiguous() && m.is_contiguous() && v.is_contiguous() && grad.is_contiguous(), "adamw: contiguous");
  TORCH_CHECK(n % 8 == 0, "adamw: flat size must be a multiple of 8");
  const bool gf32 = grad.scalar_type() == at::kFloat;
  TORCH_CHECK(gf32 || grad.scalar_type() == at::kBFloat16, "adamw: grad must be fp32 or bf16");
  void* pp = nullptr;
  if (param.defined() && param.numel()) {
    check_bf16(param, "param");
    TORCH_CHECK(param.numel() == n && param.is_contiguous(), "adamw: param size");
    pp = param.data_ptr();
  }
  for (auto* t : {&master, &m, &v}) check_aligned16(*t, "adamw buffer");
  check_aligned16(grad, "grad");
  const float* sp = nullptr;
  if (scale) {
    TORCH_CHECK(scale->scalar_type() == at::kFloat && scale->numel() == 1 && scale->is_cuda(), "adamw scale");
    sp = scale->data_ptr<float>();
  }
  const uint8_t* wm = nullptr;
  if (wd_mask) {
    TORCH_CHECK(wd_mask->scalar_type() == at::kByte && wd_mask->is_cuda() && wd_mask->is_contiguous(), "wd_mask: uint8 GPU");
    TORCH_CHECK(wd_mask->numel() * 64 >= n, "wd_mask: one byte per 64 elements");
    wm = wd_mask->data_ptr<uint8_t>();
  }
  const float* hp = nullptr;
  if (hyper) {  // device-side [lr, 1/bc1, 1/sqrt(bc2)] (graph-capturable step)
    TORCH_CHECK(hyper->scalar_type() == at::kFloat && hyper->is_cuda() && hyper->numel() >= 3, "adamw: hyper");
    hp = hyper->data_ptr<float>();
  }
  if (n)
    pllm::adamw_flat(pp, master.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), grad.data_ptr(), gf32, n,
                     (float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (int)step, (float)grad_scale, sp, wm, hp,
                     cur_stream());
}

Tensor sumsq(const Tensor& x) {
  check_gpu(x, "x");
  TORCH_CHECK(x.is_contiguous() && x.numel() % 8 == 0, "sumsq: contiguous, numel % 8");
  const bool f32 = x.scalar_type() == at::kFloat;
  TORCH_CHECK(f32 || x.scalar_type() == at::kBFloat16, "sumsq dtype");
  const int G = pllm::sumsq_blocks(x.numel());
  Tensor part = at::empty({G}, x.options().dtype(at::kFloat));
  if (x.numel()) pllm::sumsq(x.data_ptr(), f32, x.numel(), part.data_ptr<float>(), cur_stream());
  else part.zero_();
  return part.sum();
}

// gradient norm and clip coefficient of a flat gradient in two launches (partial sums of squares, then one
// single-block finish): returns [norm * grad_scale, min(max_norm / (norm * grad_scale + 1e-6), 1)] (fp32, GPU)
Tensor grad_norm_clip(const Tensor& x, double grad_scale, double max_norm) {
  check_gpu(x, "x");
  TORCH_CHECK(x.is_contiguous() && x.numel() % 8 == 0, "grad_norm_clip: contiguous, numel % 8");
  const bool f32 = x.scalar_type() == at::kFloat;
  TORCH_CHECK(f32 || x.scalar_type() == at::kBFloat16, "grad_norm_clip dtype");
  const int G = pllm::sumsq_blocks(x.numel());
  Tensor part = at::empty({G}, x.options().dtype(at::kFloat));
  Tensor out = at::empty({2}, x.options().dtype(at::kFloat));
  if (x.numel()) pllm::sumsq(x.data_ptr(), f32, x.numel(), part.data_ptr<float>(), cur_stream());
  else part.zero_();
  pllm::clip_coef(part.data_ptr<float>(), G, (float)grad_scale, (float)max_norm, out.data_ptr<float>(), cur_stream());
  return out;
}

// ---------------------------------------------------------------- embedding
Tensor embedding_fwd(const Tensor& idx, const Tensor& wte, const std::optional<Tensor>& wpe, int64_t pos_offset) {
  check_bf16(wte, "wte");
  TORCH_CHECK(idx.is_cuda() && idx.dim() == 2, "idx must be [B, T] on GPU");
  const int64_t C = wte.size(1), T = idx.size(1);
  TORCH_CHECK(C % 8 == 0 && wte.is_contiguous(), "embedding: C % 8");
  if (wpe) {
    check_bf16(*wpe, "wpe");
    TORCH_CHECK(wpe->size(1) == C && wpe->size(0) >= T + pos_offset && wpe->is_contiguous(), "wpe shape");
  }
  Tensor ix = idx.to(at::kLong).contiguous();
  Tensor out = at::empty({idx.size(0), T, C}, wte.options());
  if (ix.numel())
    pllm::embedding_fwd(ix.data_ptr<int64_t>(), wte.data_ptr(), opt_ptr(wpe), out.data_ptr(), ix.numel(), (int)T, (int)C,
                        (int)pos_offset, wte.size(0), cur_stream());
  return out;
}

// dwte_acc/dwpe_acc: if given, gradients are ADDED into them (flat-buffer views) and
// nothing is returned; otherwise fresh zero-initialised gradients are returned.
std::vector<Tensor> embedding_bwd(const Tensor& dx, const Tensor& idx, int64_t V, int64_t n_pos, bool has_wpe,
                                  const std::optional<Tensor>& dwte_acc, const std::optional<Tensor>& dwpe_acc) {
  check_bf16(dx, "dx");
  check_contig(dx, "dx");
  const int64_t Bn = idx.size(0), T = idx.size(1), C = dx.size(-1);
  TORCH_CHECK(dx.numel() == Bn * T * C, "embedding bwd shape");
  TORCH_CHECK(!has_wpe || n_pos >= T, "embedding bwd: n_pos < T");
  const bool acc = dwte_acc.has_value();
  TORCH_CHECK(!has_wpe || acc == dwpe_acc.has_value(), "embedding_bwd: both or neither accumulation targets");
  bool gf32 = false;
  if (acc) {
    gf32 = check_grad(*dwte_acc, "dwte_acc");
    check_aligned16(*dwte_acc, "dwte_acc");
    TORCH_CHECK(dwte_acc->numel() == V * C && dwte_acc->is_contiguous(), "dwte_acc shape");
    if (has_wpe) {
      TORCH_CHECK(check_grad(*dwpe_acc, "dwpe_acc") == gf32, "dwpe_acc dtype must match dwte_acc");
      check_aligned16(*dwpe_acc, "dwpe_acc");
      TORCH_CHECK(dwpe_acc->numel() == n_pos * C && dwpe_acc->is_contiguous(), "dwpe_acc shape");
    }
  }
  TORCH_CHECK(idx.is_cuda(), "idx on GPU");
  auto flat = idx.reshape({-1}).to(at::kInt);
  auto sr = flat.sort(/*stable=*/true, 0, false);
  Tensor sorted = std::get<0>(sr).contiguous(), perm = std::get<1>(sr).to(at::kInt).contiguous();
  Tensor dwte = acc ? *dwte_acc : at::zeros({V, C}, dx.options());
  Tensor dwpe = has_wpe ? (acc ? *dwpe_acc : at::zeros({n_pos, C}, dx.options())) : Tensor();
  Tensor part = at::empty({2 * pllm::embedding_bwd_chunks(Bn * T) * C}, dx.options().dtype(at::kFloat));
  if (Bn * T)
    pllm::embedding_bwd(dx.data_ptr(), sorted.data_ptr<int32_t>(), perm.data_ptr<int32_t>(), dwte.data_ptr(),
                        has_wpe ? dwpe.data_ptr() : nullptr, gf32, part.data_ptr<float>(), Bn * T, (int)Bn, (int)T,
                        (int)C, V, cur_stream());
  if (acc) return {};
  if (!has_wpe) return {dwte};
  return {dwte, dwpe};
}

// embedding_bwd: pure -> (dwte, dwpe) (dwpe empty without positions); embedding_bwd_acc: adds
// into the targets
std::tuple<Tensor, Tensor> embedding_bwd_op(const Tensor& dx, const Tensor& idx, int64_t V, int64_t n_pos,
                                            bool has_wpe) {
  auto o = embedding_bwd(dx, idx, V, n_pos, has_wpe, std::nullopt, std::nullopt);
  return {o[0], has_wpe ? o[1] : at::empty({0}, dx.options())};
}
void embedding_bwd_acc_op(const Tensor& dx, const Tensor& idx, int64_t V, int64_t n_pos, bool has_wpe,
                          Tensor& dwte_acc, const std::optional<Tensor>& dwpe_acc) {
  embedding_bwd(dx, idx, V, n_pos, has_wpe, dwte_acc, dwpe_acc);
}

// ---------------------------------------------------------------- batched transpose
// Builds the descriptor table for dst[i] = src[i]^T (bf16 2-D, dims % 8 == 0, 16-B aligned);
// returns it as a device int64 tensor [n, 6] whose last row-count column is the tile total.
Tensor transpose_plan(const std::vector<Tensor>& src, const std::vector<Tensor>& dst) {
  TORCH_CHECK(src.size() == dst.size() && !src.empty(), "transpose_plan: matching non-empty lists");
  const int64_t n = (int64_t)src.size();
  Tensor desc = at::empty({n, 6}, at::TensorOptions().dtype(at::kLong));
  int64_t* d = desc.data_ptr<int64_t>();
  int64_t tiles = 0;
  for (int64_t i = 0; i < n; ++i) {
    const Tensor &s = src[i], &t = dst[i];
    check_bf16(s, "src");
    check_bf16(t, "dst");
    check_contig(s, "src");
    check_contig(t, "dst");
    TORCH_CHECK(s.dim() == 2 && t.dim() == 2 && t.size(0) == s.size(1) && t.size(1) == s.size(0),
                "transpose_plan: dst must be [cols, rows] of src");
    TORCH_CHECK(s.size(0) % 8 == 0 && s.size(1) % 8 == 0, "transpose_plan: dims must be multiples of 8");
    check_aligned16(s, "src");
    check_aligned16(t, "dst");
    const int R = (int)s.size(0), C = (int)s.size(1);
    d[i * 6 + 0] = (int64_t)(uintptr_t)s.data_ptr();
    d[i * 6 + 1] = (int64_t)(uintptr_t)t.data_ptr();
    d[i * 6 + 2] = R;
    d[i * 6 + 3] = C;
    d[i * 6 + 4] = tiles;
    d[i * 6 + 5] = (C + 63) / 64;
    tiles += pllm::transpose_tiles(R, C);
  }
  TORCH_CHECK(tiles < (1ll << 31), "transpose_plan: too many tiles");
  return desc.to(src[0].device());
}

// total_tiles = sum over matrices of ceil(rows/64) * ceil(cols/64) (tiles past the table's
// last matrix are guarded in the kernel: they load and store nothing)
void transpose_run(const Tensor& desc, int64_t total_tiles) {
  TORCH_CHECK(desc.is_cuda() && desc.scalar_type() == at::kLong && desc.dim() == 2 && desc.size(1) == 6 &&
                  desc.is_contiguous(), "transpose_run: desc from transpose_plan");
  pllm::transpose_batch(desc.data_ptr<int64_t>(), (int)desc.size(0), (int)total_tiles, cur_stream());
}

// ---------------------------------------------------------------- sampling
// logits [B, V] (fp32 or bf16, unit column stride) -> int64 [B, 1] token ids
Tensor sample(const Tensor& logits, double temperature, int64_t seed) {
  check_gpu(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "sample: logits [B, V] with unit column stride");
  TORCH_CHECK(logits.scalar_type() == at::kFloat || logits.scalar_type() == at::kBFloat16,
              "sample: logits must be float32 or bfloat16");
  const int64_t B = logits.size(0), V = logits.size(1);
  TORCH_CHECK(V > 0 && V < (1ll << 31), "sample: vocabulary size");
  Tensor out = at::empty({B, 1}, logits.options().dtype(at::kLong));
  if (B > 0)
    pllm::sample_tokens(logits.data_ptr(), logits.scalar_type() == at::kBFloat16, logits.stride(0), (int)B, (int)V,
                        (float)temperature, (uint64_t)seed, out.data_ptr<int64_t>(), cur_stream());
  return out;
}

// ---------------------------------------------------------------- attention
void check_head_view(const Tensor& t, const char* name, int64_t D) {
  check_bf16(t, name);
  TORCH_CHECK(t.dim() == 4, name, " must be [B, T, H, D]");
  TORCH_CHECK(t.size(3) == D && t.stride(3) == 1, name, ": head dim must be innermost/contiguous");
  TORCH_CHECK(t.stride(2) % 8 == 0 && t.stride(1) % 8 == 0 && t.stride(0) % 8 == 0, name, ": strides must be multiples of 8");
  check_aligned16(t, name);
}

// the attention kernels read a head's rows through a buffer descriptor with 32-bit byte offsets
// (common.h rows_rsrc): the last row must start below 2 GiB of that head's slice
void check_rows_span(const Tensor& t, const char* name) {
  const int64_t D = t.size(3), rows = t.size(1);
  TORCH_CHECK(rows == 0 || ((rows - 1) * t.stride(1) + D) * 2 < (int64_t(1) << 31), "attention: ", name,
              " spans >= 2 GiB within one head (sequence x row stride too large for 32-bit offsets)");
}

// fused RoPE tables: fp32 contiguous [>= S, D/2] on the device (both or neither)
void check_rope(const std::optional<Tensor>& c, const std::optional<Tensor>& sn, int64_t S, int64_t D) {
  TORCH_CHECK(c.has_value() == sn.has_value(), "attention: rope_cos and rope_sin go together");
  if (!c) return;
  for (const Tensor* t : {&*c, &*sn}) {
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->dim() == 2,
                "attention: rope tables must be contiguous fp32 [positions, D/2] GPU tensors");
    TORCH_CHECK(t->size(1) == D / 2 && t->size(0) >= S, "attention: rope table shape [>= S, D/2]");
    check_aligned16(*t, "rope table");
  }
}

std::vector<Tensor> attn_fwd(const Tensor& q, const Tensor& k, const Tensor& v, bool causal, double scale,
                             const std::optional<Tensor>& rope_cos, const std::optional<Tensor>& rope_sin) {
  const int64_t D = q.size(3);
  TORCH_CHECK(pllm::attn_supported_head_dim((int)D), "attention: head dim must be 32, 64 or 128, got ", D);
  check_head_view(q, "q", D);
  check_head_view(k, "k", D);
  check_head_view(v, "v", D);
  const int64_t B = q.size(0), T = q.size(1), H = q.size(2), S = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(k.size(0) == B && v.size(0) == B && v.size(1) == S && v.size(2) == Hkv, "k/v shape");
  TORCH_CHECK(H % Hkv == 0, "H % Hkv");
  TORCH_CHECK(!causal || S >= T, "causal attention needs S >= T");
  check_rope(rope_cos, rope_sin, S, D);
  check_rows_span(k, "k");
  check_rows_span(v, "v");
  Tensor o = at::empty({B, T, H, D}, q.options());
  Tensor lse = at::empty({B, H, T}, q.options().dtype(at::kFloat));
  AttnFwdArgs a{};
  a.q = (const uint16_t*)q.data_ptr();
  a.k = (const uint16_t*)k.data_ptr();
  a.v = (const uint16_t*)v.data_ptr();
  a.o = (uint16_t*)o.data_ptr();
  a.lse = lse.data_ptr<float>();
  a.rope_cos = rope_cos ? rope_cos->data_ptr<float>() : nullptr;
  a.rope_sin = rope_sin ? rope_sin->data_ptr<float>() : nullptr;
  a.B = B; a.H = H; a.Hkv = Hkv; a.T = T; a.S = S; a.D = D;
  a.q_sb = q.stride(0); a.q_st = q.stride(1); a.q_sh = q.stride(2);
  a.k_sb = k.stride(0); a.k_st = k.stride(1); a.k_sh = k.stride(2);
  a.v_sb = v.stride(0); a.v_st = v.stride(1); a.v_sh = v.stride(2);
  a.o_sb = o.stride(0); a.o_st = o.stride(1); a.o_sh = o.stride(2);
  a.scale = (float)scale;
  a.scale_log2 = (float)(scale * 1.4426950408889634);
  a.causal = causal ? 1 : 0;
  // diagnostic (a PLLM_FWD_STAMPS=1 build of attention.hip + this env): per-wave phase cycles of
  // the forward's tile loop, summed and printed to stderr after the launch
  static const bool stamps = std::getenv("PLLM_FWD_STAMPS") != nullptr;
  Tensor st;
  if (stamps) {
    const int64_t nqb = (T + 127) / 128;  // >= the workgroups of every forward kernel
    st = at::zeros({nqb * B * H * 4 * 9}, q.options().dtype(at::kLong));
    a.stamps = (unsigned long long*)st.data_ptr();
  }
  if (B * T * H > 0 && S > 0) pllm::attn_fwd(a, cur_stream());
  if (st.defined()) {
    auto h = st.view({-1, 9}).to(at::kCPU).to(at::kDouble);
    auto tot = h.sum(0);
    const double tiles = tot[6].item<double>();
    fprintf(stderr, "[fwd stamps] waves %lld tiles %.0f | per tile: p0 %.0f p1 %.0f p2 %.0f p3 %.0f p4 %.0f p5 %.0f | per wave total %.0f (p7 sum %.0f)\n",
            (long long)h.size(0), tiles, tot[0].item<double>() / tiles, tot[1].item<double>() / tiles,
            tot[2].item<double>() / tiles, tot[3].item<double>() / tiles, tot[4].item<double>() / tiles,
            tot[5].item<double>() / tiles, tot[8].item<double>() / h.size(0), tot[7].item<double>());
  }
  return {o, lse};
}

// single-query decode attention: q [B, 1, H, D], k/v [B, S, Hkv, D] views of a KV cache
// (any batch/row strides).  ``seqlen``: optional int32 device scalar overriding S (the
// number of valid cache rows) so a captured decode step replays at every position.
Tensor attn_decode(const Tensor& q, const Tensor& k, const Tensor& v, double scale, const c10::optional<Tensor>& seqlen) {
  const int64_t D = q.size(3);
  check_head_view(q, "q", D);
  check_head_view(k, "k", D);
  check_head_view(v, "v", D);
  const int64_t B = q.size(0), H = q.size(2), S = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(q.size(1) == 1, "attn_decode: one query per sequence");
  TORCH_CHECK(k.size(0) == B && v.size(0) == B && v.size(1) == S && v.size(2) == Hkv && k.size(3) == D && v.size(3) == D,
              "attn_decode: k/v shape");
  TORCH_CHECK(H % Hkv == 0 && pllm::attn_decode_supported((int)D, (int)(H / Hkv)),
              "attn_decode: head dim 32/64/128 and group size 1/2/4/8 supported");
  Tensor o = at::empty({B, 1, H, D}, q.options());
  DecodeArgs a{};
  a.q = (const uint16_t*)q.data_ptr();
  a.k = (const uint16_t*)k.data_ptr();
  a.v = (const uint16_t*)v.data_ptr();
  a.o = (uint16_t*)o.data_ptr();
  a.B = B; a.H = H; a.Hkv = Hkv; a.S = S; a.D = D;
  a.q_sb = q.stride(0); a.q_sh = q.stride(2);
  a.k_sb = k.stride(0); a.k_st = k.stride(1); a.k_sh = k.stride(2);
  a.v_sb = v.stride(0); a.v_st = v.stride(1); a.v_sh = v.stride(2);
  a.o_sb = o.stride(0); a.o_sh = o.stride(2);
  a.scale_log2 = (float)(scale * 1.4426950408889634);
  if (seqlen.has_value()) {
    TORCH_CHECK(seqlen->is_cuda() && seqlen->scalar_type() == at::kInt && seqlen->is_contiguous() &&
                    (seqlen->numel() == 1 || seqlen->numel() == B),
                "attn_decode: seqlen must be an int32 device tensor of 1 or B elements");
    a.seqlen = seqlen->data_ptr<int>();
    a.seqlen_per_row = seqlen->numel() == B && B > 1;
  }
  a.splits = pllm::attn_decode_splits((int)B, (int)Hkv, (int)S);
  Tensor part_o, part_lse;
  if (a.splits > 1) {
    part_o = at::empty({B, H, a.splits, D}, q.options().dtype(at::kFloat));
    part_lse = at::empty({B, H, a.splits}, q.options().dtype(at::kFloat));
    a.part_o = part_o.data_ptr<float>();
    a.part_lse = part_lse.data_ptr<float>();
  }
  if (B > 0 && S > 0) pllm::attn_decode(a, cur_stream());
  return o;
}

// dQ slab workspace budget of the attention backward (bytes); PLLM_ATTN_BWD_WS_MB or the
// attn_bwd_set_workspace_mb op (tests force multi-pass runs with it)
int64_t g_attn_ws_bytes = -1;
int64_t attn_bwd_ws_bytes() {
  if (g_attn_ws_bytes < 0) {
    const char* e = std::getenv("PLLM_ATTN_BWD_WS_MB");
    g_attn_ws_bytes = (int64_t)((e ? std::atof(e) : 4096.0) * (1 << 20));
  }
  return g_attn_ws_bytes;
}

// dq/dk/dv are written into caller-provided views (e.g. slices of a packed dQKV buffer)
void attn_bwd(const Tensor& dout, const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o, const Tensor& lse,
              Tensor& dq, Tensor& dk, Tensor& dv, bool causal, double scale, const std::optional<Tensor>& rope_cos,
              const std::optional<Tensor>& rope_sin, bool rope_in, const std::optional<Tensor>& delta_in) {
  const int64_t D = q.size(3);
  TORCH_CHECK(pllm::attn_supported_head_dim((int)D), "attention: head dim must be 32, 64 or 128");
  for (auto& pr : std::vector<std::pair<const Tensor*, const char*>>{
           {&dout, "dout"}, {&q, "q"}, {&k, "k"}, {&v, "v"}, {&o, "o"}, {&dq, "dq"}, {&dk, "dk"}, {&dv, "dv"}})
    check_head_view(*pr.first, pr.second, D);
  const int64_t B = q.size(0), T = q.size(1), H = q.size(2), S = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(dout.sizes() == q.sizes() && o.sizes() == q.sizes() && dq.sizes() == q.sizes(), "attn bwd q-side shapes");
  TORCH_CHECK(dk.sizes() == k.sizes() && dv.sizes() == v.sizes() && v.sizes() == k.sizes(), "attn bwd kv-side shapes");
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == B * H * T, "lse shape");
  check_rope(rope_cos, rope_sin, S, D);
  auto f32 = q.options().dtype(at::kFloat);
  // delta_in: rowsum(dO * O) already computed (the output projection's gemm_tn epilogue 6)
  if (delta_in)
    TORCH_CHECK(delta_in->scalar_type() == at::kFloat && delta_in->is_contiguous() && delta_in->numel() == B * H * T,
                "attn_bwd: delta [B, H, T] fp32");
  Tensor delta = delta_in ? *delta_in : at::empty({B, H, T}, f32);
  // per-key-block bf16 dQ partial slabs (attention.hip: plain stores + ordered fp32 reduce, no
  // atomics), run in passes of at most `per` key blocks: the workspace is bounded by
  // PLLM_ATTN_BWD_WS_MB (default 4096 MiB: one pass for every shipped config -- passes split the
  // causal work unevenly, 2 passes cost llama-1.3B +20 %) however long the sequence, plus one fp32 running
  // sum when more than one pass is needed
  check_rows_span(q, "q");
  check_rows_span(dout, "dout");
  const int64_t kbk = pllm::attn_bwd_key_block((int)D);
  const int64_t nkb = (S + kbk - 1) / kbk;
  const int64_t nqt = (T + 31) / 32;
  const int64_t slab_elems = B * H * nqt * 32 * D;  // T rounded up to the 32-row fragment tiles
  const int64_t slab_bytes = slab_elems * 2;
  const int64_t ws_budget = attn_bwd_ws_bytes();
  const int64_t per = std::max<int64_t>(1, std::min<int64_t>(nkb, ws_budget / std::max<int64_t>(1, slab_bytes)));
  Tensor dq_acc = at::empty({per, slab_elems}, q.options());  // bf16 partial slabs
  Tensor dq_sum = per < nkb ? at::empty({slab_elems}, q.options().dtype(at::kFloat)) : Tensor();
  // the key-stationary backward stages q / k by LDS DMA: with in-kernel RoPE requested, rotate them
  // here once (positions t + S - T for queries, s for keys) and run it on the rotated copies
  Tensor qrot, krot;
  const bool ks_rot = rope_cos && rope_in && pllm::attn_bwd_uses_ks((int)D);
  if (ks_rot) {
    const Tensor qc = q.contiguous(), kc = k.contiguous();
    qrot = at::empty_like(qc);
    krot = at::empty_like(kc);
    if (B * T > 0)
      pllm::rope(qc.data_ptr(), qrot.data_ptr(), rope_cos->data_ptr<float>(), rope_sin->data_ptr<float>(), B * T,
                 (int)T, (int)H, (int)H, (int)D, (int)(S - T), false, cur_stream());
    if (B * S > 0)
      pllm::rope(kc.data_ptr(), krot.data_ptr(), rope_cos->data_ptr<float>(), rope_sin->data_ptr<float>(), B * S,
                 (int)S, (int)Hkv, (int)Hkv, (int)D, 0, false, cur_stream());
  }
  const Tensor& qx = ks_rot ? qrot : q;
  const Tensor& kx = ks_rot ? krot : k;
  AttnBwdArgs a{};
  a.q = (const uint16_t*)qx.data_ptr();
  a.k = (const uint16_t*)kx.data_ptr();
  a.v = (const uint16_t*)v.data_ptr();
  a.o = (const uint16_t*)o.data_ptr();
  a.dO = (const uint16_t*)dout.data_ptr();
  a.lse = lse.data_ptr<float>();
  a.rope_cos = rope_cos ? rope_cos->data_ptr<float>() : nullptr;
  a.rope_sin = rope_sin ? rope_sin->data_ptr<float>() : nullptr;
  a.delta = delta.data_ptr<float>();
  a.dq_acc = (uint16_t*)dq_acc.data_ptr();
  a.dq_sum = dq_sum.defined() ? dq_sum.data_ptr<float>() : nullptr;
  a.kb0 = 0;
  a.rope_in = rope_in && !ks_rot ? 1 : 0;
  a.slab = slab_elems;
  a.nqt = (int)nqt;
  a.nkb_pass = (int)per;
  a.dq = (uint16_t*)dq.data_ptr();
  a.dk = (uint16_t*)dk.data_ptr();
  a.dv = (uint16_t*)dv.data_ptr();
  a.B = B; a.H = H; a.Hkv = Hkv; a.T = T; a.S = S; a.D = D;
  a.q_sb = qx.stride(0); a.q_st = qx.stride(1); a.q_sh = qx.stride(2);
  a.k_sb = kx.stride(0); a.k_st = kx.stride(1); a.k_sh = kx.stride(2);
  a.v_sb = v.stride(0); a.v_st = v.stride(1); a.v_sh = v.stride(2);
  a.o_sb = o.stride(0); a.o_st = o.stride(1); a.o_sh = o.stride(2);
  a.do_sb = dout.stride(0); a.do_st = dout.stride(1); a.do_sh = dout.stride(2);
  a.dq_sb = dq.stride(0); a.dq_st = dq.stride(1); a.dq_sh = dq.stride(2);
  a.dk_sb = dk.stride(0); a.dk_st = dk.stride(1); a.dk_sh = dk.stride(2);
  a.dv_sb = dv.stride(0); a.dv_st = dv.stride(1); a.dv_sh = dv.stride(2);
  a.scale = (float)scale;
  a.scale_log2 = (float)(scale * 1.4426950408889634);
  a.causal = causal ? 1 : 0;
  a.delta_ready = delta_in ? 1 : 0;
  static const bool bstamps = std::getenv("PLLM_BWD_STAMPS") != nullptr;
  Tensor bst;
  if (bstamps) {  // diagnostic, with a PLLM_BWD_STAMPS=1 build of attention.hip / attn_bwd_ks.hip
    bst = at::zeros({nkb * B * Hkv * 8 * 9}, q.options().dtype(at::kLong));
    a.stamps = (unsigned long long*)bst.data_ptr();
  }
  if (B * T * H > 0 && S > 0) pllm::attn_bwd(a, cur_stream());
  if (bst.defined()) {
    auto hs = bst.view({-1, 9}).to(at::kCPU).to(at::kDouble);
    auto tot = hs.sum(0);
    const double its = tot[6].item<double>();
    // fused-role kernel: wait+barrier, stage+barrier, gload, subblocks, barrier, dq, -, loop-top;
    // key-stationary kernel: A (S0/dP0), B (S1/dP1 | softmax 0), C (dV0/dK0 | softmax 1), D (dV1/dK1 | dS^T),
    // wait + barrier + DMA issue, dQ task, -, init
    fprintf(stderr, "[bwd stamps] waves %lld iters %.0f | per iter (cycles): p0 %.0f p1 %.0f p2 %.0f p3 %.0f p4 %.0f p5 %.0f p7 %.0f | per wave %.0f\n",
            (long long)hs.size(0), its, tot[0].item<double>() / its, tot[1].item<double>() / its,
            tot[2].item<double>() / its, tot[3].item<double>() / its, tot[4].item<double>() / its,
            tot[5].item<double>() / its, tot[7].item<double>() / its, tot[8].item<double>() / hs.size(0));
  }
}

}  // namespace

TORCH_LIBRARY(pllm, m) {
  m.def("norm_fwd(Tensor x, Tensor? residual, Tensor weight, Tensor? bias, float eps, bool rms) -> Tensor[]");
  m.def("norm_bwd(Tensor dy, Tensor s, Tensor weight, Tensor mean, Tensor rstd, Tensor? ds, bool has_bias, bool rms) -> (Tensor, Tensor, Tensor)");
  m.def("norm_bwd_acc(Tensor dy, Tensor s, Tensor weight, Tensor mean, Tensor rstd, Tensor? ds, bool has_bias, bool rms, Tensor(a!) dw_acc, Tensor(b!)? db_acc=None, Tensor(c!)? xb_acc=None) -> Tensor");
  m.def("bias_grad(Tensor dy, Tensor(a!)? out_acc=None) -> Tensor");
  m.def("wgrad(Tensor dy, Tensor x, Tensor(a!)? out_acc=None, Tensor(b!)? bias_acc=None, bool overwrite=False) -> Tensor");
  m.def("gemm_tn(Tensor a, Tensor b, Tensor? bias, int epi, Tensor? aux=None, Tensor(a!)? bias_acc=None, int T=0) -> (Tensor, Tensor)");
  m.def("gemm_uses_pp(int K, int epi) -> bool", [](int64_t K, int64_t epi) { return pllm::gemm_uses_pp((int)K, (int)epi, 16); });
  m.def("gemm_set_config(int mfma, int group_m, int phased=-1, int reserve_cus=-1, int persistent=-1) -> ()",
        [](int64_t mf, int64_t gm, int64_t ph, int64_t rc, int64_t pe) {
          pllm::gemm_set_config((int)mf, (int)gm, (int)ph, (int)rc, (int)pe);
        });
  m.def("wgrad_set_mfma(int mf) -> ()", [](int64_t mf) { pllm::wgrad_set_mfma((int)mf); });
  m.def("wgrad_set_hy(int on) -> ()", [](int64_t on) { pllm::wgrad_set_hy((int)on); });
  m.def("attn_bwd_set_ks(int mask) -> ()", [](int64_t m) { pllm::attn_bwd_set_ks((int)m); });
  m.def("wgrad_force_slices(int s) -> ()", [](int64_t s) { pllm::wgrad_force_slices((int)s); });
  m.def("attn_bwd_set_workspace_mb(float mb) -> ()", [](double mb) { g_attn_ws_bytes = (int64_t)(mb * (1 << 20)); });
  m.def("gemv(Tensor x, Tensor w, Tensor? bias, Tensor? res=None, Tensor? gamma=None, Tensor? beta=None, float eps=1e-5, int rms=0, int act=0, Tensor(a!)? kc=None, Tensor(b!)? vc=None, Tensor? pos=None, int q_cols=0) -> (Tensor, Tensor)");
  m.def("act_fwd(Tensor x, int op) -> Tensor");
  m.def("act_bwd(Tensor dy, Tensor x, int op) -> Tensor");
  m.def("act_bwd_bias(Tensor dy, Tensor x, int op, Tensor(a!) bias_acc) -> Tensor");
  m.def("swiglu_fwd(Tensor gate_up) -> Tensor");
  m.def("swiglu_bwd(Tensor dy, Tensor gate_up) -> Tensor");
  m.def("rope(Tensor x, Tensor cos, Tensor sin, int n_heads_total, int n_rot, int T, int pos_offset, bool inverse) -> Tensor");
  m.def("rope_qk(Tensor x, Tensor cos, Tensor sin, int n_heads_total, int n_rot, int T) -> Tensor");
  m.def("scale_(Tensor(a!) x, Tensor s) -> ()");
  m.def("lse_merge_(Tensor(a!) o_acc, Tensor(b!) lse_acc, Tensor o, Tensor lse) -> ()");
  m.def("zero_ranges_(Tensor(a!) buf, Tensor ranges, int total_len) -> ()");
  m.def("cross_entropy(Tensor logits, Tensor targets, Tensor(a!)? dlogits, int ignore_index, Tensor? inv_n=None) -> Tensor");
  m.def("adamw_(Tensor(a!) param, Tensor(b!) master, Tensor(c!) m, Tensor(d!) v, Tensor grad, float lr, float b1, float b2, float eps, float wd, int step, float grad_scale, Tensor? scale, Tensor? wd_mask, Tensor? hyper=None) -> ()");
  m.def("sumsq(Tensor x) -> Tensor");
  m.def("grad_norm_clip(Tensor x, float grad_scale, float max_norm) -> Tensor");
  m.def("embedding_fwd(Tensor idx, Tensor wte, Tensor? wpe, int pos_offset) -> Tensor");
  m.def("embedding_bwd(Tensor dx, Tensor idx, int V, int n_pos, bool has_wpe) -> (Tensor, Tensor)");
  m.def("embedding_bwd_acc(Tensor dx, Tensor idx, int V, int n_pos, bool has_wpe, Tensor(a!) dwte_acc, Tensor(b!)? dwpe_acc=None) -> ()");
  m.def("transpose_plan(Tensor[] src, Tensor[] dst) -> Tensor");
  m.def("transpose_run(Tensor desc, int total_tiles) -> ()");
  m.def("sample(Tensor logits, float temperature, int seed) -> Tensor");
  m.def("attn_fwd(Tensor q, Tensor k, Tensor v, bool causal, float scale, Tensor? rope_cos=None, Tensor? rope_sin=None) -> Tensor[]");
  m.def("attn_decode(Tensor q, Tensor k, Tensor v, float scale, Tensor? seqlen=None) -> Tensor");
  m.def("attn_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, Tensor(a!) dq, Tensor(b!) dk, Tensor(c!) dv, bool causal, float scale, Tensor? rope_cos=None, Tensor? rope_sin=None, bool rope_in=True, Tensor? delta=None) -> ()");
}

TORCH_LIBRARY_IMPL(pllm, CUDA, m) {
  m.impl("norm_fwd", norm_fwd);
  m.impl("norm_bwd", norm_bwd_op);
  m.impl("norm_bwd_acc", norm_bwd_acc_op);
  m.impl("bias_grad", bias_grad);
  m.impl("wgrad", wgrad);
  m.impl("gemm_tn", gemm_tn);
  m.impl("act_fwd", act_fwd);
  m.impl("act_bwd", act_bwd);
  m.impl("act_bwd_bias", act_bwd_bias);
  m.impl("swiglu_fwd", swiglu_fwd);
  m.impl("swiglu_bwd", swiglu_bwd);
  m.impl("rope", rope);
  m.impl("rope_qk", rope_qk);
  m.impl("scale_", scale_);
  m.impl("lse_merge_", lse_merge_);
  m.impl("zero_ranges_", zero_ranges_);
  m.impl("cross_entropy", cross_entropy);
  m.impl("adamw_", adamw_);
  m.impl("sumsq", sumsq);
  m.impl("grad_norm_clip", grad_norm_clip);
  m.impl("embedding_fwd", embedding_fwd);
  m.impl("embedding_bwd", embedding_bwd_op);
  m.impl("embedding_bwd_acc", embedding_bwd_acc_op);
  m.impl("transpose_plan", transpose_plan);
  m.impl("transpose_run", transpose_run);
  m.impl("sample", sample);
  m.impl("attn_fwd", attn_fwd);
  m.impl("attn_decode", attn_decode);
  m.impl("gemv", gemv);
  m.impl("attn_bwd", attn_bwd);
}

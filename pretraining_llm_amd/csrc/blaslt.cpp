// Library GEMMs with hipBLASLt's own activation epilogues (torch.ops.pllm.gemm_lt).
//
// The forward up-projection of a GELU / ReLU MLP is a plain TN GEMM at K = C (768-2048) where
// hipBLASLt's main loop still beats the hand-written ping-pong kernel (profiles/r4_gemm_pp.md), but
// through torch it needs a second pass for the activation (act_fwd: read + write of the whole
// [tokens, 4C] pre-activation).  hipBLASLt can apply bias + GELU in its store epilogue and write the
// pre-activation as an auxiliary output in the same pass (HIPBLASLT_EPILOGUE_GELU_AUX_BIAS: the
// backward's GELU' epilogue reads it) -- or bias + ReLU with no auxiliary output (the ReLU
// backward needs only the activation's sign).  Reference MLP: /root/reference/src/models/mlp.py:24-26.
//
// Row-major y[M, N] = x[M, K] w[N, K]^T + b is the column-major product y^T = w^T(op T) x (op N):
// m = N, n = M, k = K; the bias is per column-major row (per output feature).
//
// Workspace: each launch takes the bytes its algorithm asks for from torch's caching allocator on the
// current stream (so concurrent streams and graph captures never share one).
//
// Algorithm choice: the heuristic's candidates for each (M, N, K, epilogue) are timed once on the
// first eager call (hipEvents on the current stream, 3 launches each) and the fastest is cached; a
// call inside a hipGraph capture or with tune=false takes the heuristic's first candidate (without
// caching it, unless tune=false: deterministic runs pin the heuristic's choice).
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include "ab.h"
#include <torch/library.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

using at::Tensor;

namespace {

#define LT_CHECK(expr)                                                                         \
  do {                                                                                         \
    hipblasStatus_t st_ = (expr);                                                              \
    TORCH_CHECK(st_ == HIPBLAS_STATUS_SUCCESS, "hipBLASLt: ", #expr, " failed with status ", \
                (int)st_);                                                                     \
  } while (0)

constexpr size_t kWorkspaceBytes = 64ull << 20;
constexpr int kCandidates = 16;

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, d = nullptr;
  std::vector<hipblasLtMatmulHeuristicResult_t> cands;
  int64_t M = 0, N = 0, K = 0;
  int chosen = -1;  // index into cands once timed (or pinned)
};

struct DevState {
  hipblasLtHandle_t handle = nullptr;
  std::map<std::tuple<int64_t, int64_t, int64_t, int, bool>, Plan> plans;
};

std::mutex g_mu;
std::map<int, DevState> g_dev;

// epi: 0 = none, 1 = GELU with the pre-activation as aux output, 2 = ReLU
hipblasLtEpilogue_t lt_epilogue(int epi, bool bias) {
  switch (epi) {
    case 1: return bias ? HIPBLASLT_EPILOGUE_GELU_AUX_BIAS : HIPBLASLT_EPILOGUE_GELU_AUX;
    case 2: return bias ? HIPBLASLT_EPILOGUE_RELU_BIAS : HIPBLASLT_EPILOGUE_RELU;
    default: return bias ? HIPBLASLT_EPILOGUE_BIAS : HIPBLASLT_EPILOGUE_DEFAULT;
  }
}

Plan make_plan(DevState& ds, int64_t M, int64_t N, int64_t K, int epi, bool bias) {
  Plan p;
  p.M = M, p.N = N, p.K = K;
  LT_CHECK(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  int32_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  uint32_t e = lt_epilogue(epi, bias);
  LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e)));
  if (bias) {
    int32_t bt = HIP_R_16BF;
    LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  }
  if (epi == 1) {
    int64_t ld = N;
    int32_t at = HIP_R_16BF;
    LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld)));
    LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at, sizeof(at)));
  }
  LT_CHECK(hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16BF, K, N, K));  // w: column-major [K, N]
  LT_CHECK(hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16BF, K, M, K));  // x: column-major [K, M]
  LT_CHECK(hipblasLtMatrixLayoutCreate(&p.d, HIP_R_16BF, N, M, N));  // y: column-major [N, M]
  hipblasLtMatmulPreference_t pref;
  LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t ws = kWorkspaceBytes;
  LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws)));
  p.cands.resize(kCandidates);
  int got = 0;
  hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(ds.handle, p.desc, p.a, p.b, p.d, p.d, pref, kCandidates,
                                                       p.cands.data(), &got);
  hipblasLtMatmulPreferenceDestroy(pref);
  p.cands.resize(st == HIPBLAS_STATUS_SUCCESS ? got : 0);
  return p;
}

// D = w^T x (+ bias) (+ C when c != nullptr: beta = 1, C laid out as D)
void run(DevState& ds, Plan& p, int idx, const void* w, const void* x, void* y, const void* c, void* ws,
         hipStream_t s) {
  const float one = 1.f, zero = 0.f;
  LT_CHECK(hipblasLtMatmul(ds.handle, p.desc, &one, w, p.a, x, p.b, c ? &one : &zero, c ? c : y, p.d, y, p.d,
                           &p.cands[idx].algo, ws, p.cands[idx].workspaceSize, s));
}

void set_ptrs(Plan& p, const void* bias, void* aux) {
  if (bias) LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
  if (aux) LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux, sizeof(aux)));
}

// the workspace comes from torch's caching allocator on the current stream, so concurrent streams
// and graph captures each get their own
Tensor workspace(size_t bytes, const Tensor& like) {
  return at::empty({(int64_t)std::max<size_t>(bytes, 1)}, like.options().dtype(at::kByte));
}

// times every candidate (3 launches each after one untimed) on the live operands; returns the fastest
int autotune(DevState& ds, Plan& p, const Tensor& w, const Tensor& x, void* y, const void* c, hipStream_t s) {
  size_t wmax = 0;
  for (auto& c : p.cands) wmax = std::max(wmax, c.workspaceSize);
  Tensor ws = workspace(wmax, x);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  int best = 0;
  float best_ms = 1e30f;
  for (int i = 0; i < (int)p.cands.size(); ++i) {
    run(ds, p, i, w.data_ptr(), x.data_ptr(), y, c, ws.data_ptr(), s);
    (void)hipEventRecord(e0, s);
    for (int r = 0; r < 3; ++r) run(ds, p, i, w.data_ptr(), x.data_ptr(), y, c, ws.data_ptr(), s);
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (pllm::ab_int("lt_verbose", 0) != 0)
      fprintf(stderr, "gemm_lt autotune M=%lld N=%lld K=%lld candidate %d: %.1f us\n", (long long)p.M,
              (long long)p.N, (long long)p.K, i, ms * 1e3f / 3);
    if (ms < best_ms) best_ms = ms, best = i;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return best;
}

void check_operands(const Tensor& x, const Tensor& w, const std::optional<Tensor>& bias, int64_t epi) {
  TORCH_CHECK(x.is_cuda() && w.is_cuda(), "gemm_lt: GPU tensors");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "gemm_lt: bf16 operands");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "gemm_lt: x [M, K], w [N, K]");
  TORCH_CHECK(x.is_contiguous() && w.is_contiguous(), "gemm_lt: contiguous operands");
  TORCH_CHECK(epi >= 0 && epi <= 2, "gemm_lt: epi 0 (none), 1 (GELU + aux), 2 (ReLU)");
  if (bias) {
    TORCH_CHECK(bias->scalar_type() == at::kBFloat16 && bias->is_contiguous() && bias->numel() == w.size(0),
                "gemm_lt: bias [N] bf16");
  }
}

// y = act(x w^T + b (+ c)) into y [M, N] (row stride N); pre (epi 1): the pre-activation; c: an
// [M, N] addend (the residual stream: y = residual + x w^T + b in one rounding)
void lt_matmul(const Tensor& x, const Tensor& w, const std::optional<Tensor>& bias, int64_t epi, bool tune,
               const Tensor& y, void* pre, const void* c = nullptr) {
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  if (M == 0 || N == 0) return;
  const c10::DeviceGuard guard(x.device());  // handle, stream and workspace of x's device
  const int dev = x.get_device();
  hipStream_t s = c10::hip::getCurrentHIPStream().stream();
  std::lock_guard<std::mutex> lk(g_mu);
  DevState& ds = g_dev[dev];
  if (!ds.handle) LT_CHECK(hipblasLtCreate(&ds.handle));
  auto key = std::make_tuple(M, N, K, (int)epi + (c ? 16 : 0), bias.has_value());
  auto it = ds.plans.find(key);
  if (it == ds.plans.end()) it = ds.plans.emplace(key, make_plan(ds, M, N, K, (int)epi, bias.has_value())).first;
  Plan& p = it->second;
  TORCH_CHECK(!p.cands.empty(), "gemm_lt: hipBLASLt has no solution for M=", M, " N=", N, " K=", K, " epi=", epi);
  set_ptrs(p, bias ? bias->data_ptr() : nullptr, pre);
  int idx = p.chosen;
  if (idx < 0) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(s, &cs);
    if (!tune) {
      idx = p.chosen = 0;
    } else if (cs == hipStreamCaptureStatusNone) {
      idx = p.chosen = autotune(ds, p, w, x, y.data_ptr(), c, s);
    } else {
      idx = 0;
    }
  }
  Tensor ws = workspace(p.cands[idx].workspaceSize, x);
  run(ds, p, idx, w.data_ptr(), x.data_ptr(), y.data_ptr(), c, ws.data_ptr(), s);
}

// y = act(x w^T + b): x [M, K], w [N, K], bias [N] (all bf16, contiguous); epi 1 also returns the
// pre-activation x w^T + b (the GELU backward's input), else an empty tensor
std::tuple<Tensor, Tensor> gemm_lt(const Tensor& x, const Tensor& w, const std::optional<Tensor>& bias, int64_t epi,
                                   bool tune, const std::optional<Tensor>& residual) {
  check_operands(x, w, bias, epi);
  if (residual) {
    TORCH_CHECK(epi == 0, "gemm_lt: a residual addend only with epi 0");
    TORCH_CHECK(residual->is_cuda() && residual->scalar_type() == at::kBFloat16 && residual->is_contiguous() &&
                    residual->dim() == 2 && residual->size(0) == x.size(0) && residual->size(1) == w.size(0),
                "gemm_lt: residual [M, N] contiguous bf16");
  }
  Tensor y = at::empty({x.size(0), w.size(0)}, x.options());
  Tensor pre = epi == 1 ? at::empty({x.size(0), w.size(0)}, x.options()) : at::empty({0}, x.options());
  lt_matmul(x, w, bias, epi, tune, y, epi == 1 ? pre.data_ptr() : nullptr,
            residual ? residual->data_ptr() : nullptr);
  return {y, pre};
}

// the same into a caller's contiguous [M, N] bf16 tensor (the chunked LM head's logits buffer)
void gemm_lt_out(const Tensor& x, const Tensor& w, const std::optional<Tensor>& bias, const Tensor& out, bool tune) {
  check_operands(x, w, bias, 0);
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kBFloat16 && out.is_contiguous() && out.dim() == 2 &&
                  out.size(0) == x.size(0) && out.size(1) == w.size(0),
              "gemm_lt_out: out [M, N] contiguous bf16");
  lt_matmul(x, w, bias, 0, tune, out, nullptr);
}

// number of heuristic candidates for a raw hipBLASLt epilogue / bias type / aux type (-1: attribute
// left unset): support probing (bench/gelu_epi_bench.py --probe)
int64_t gemm_lt_probe(int64_t M, int64_t N, int64_t K, int64_t epilogue, int64_t bias_type, int64_t aux_type) {
  std::lock_guard<std::mutex> lk(g_mu);
  DevState& ds = g_dev[0];
  if (!ds.handle) LT_CHECK(hipblasLtCreate(&ds.handle));
  hipblasLtMatmulDesc_t desc;
  hipblasLtMatrixLayout_t a, b, d;
  LT_CHECK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  int32_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  uint32_t e = (uint32_t)epilogue;
  LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e)));
  if (bias_type >= 0) {
    int32_t bt = (int32_t)bias_type;
    LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  }
  int64_t ld = N;
  LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld)));
  if (aux_type >= 0) {
    int32_t at = (int32_t)aux_type;
    LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at, sizeof(at)));
  }
  LT_CHECK(hipblasLtMatrixLayoutCreate(&a, HIP_R_16BF, K, N, K));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&b, HIP_R_16BF, K, M, K));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&d, HIP_R_16BF, N, M, N));
  hipblasLtMatmulPreference_t pref;
  LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t ws = kWorkspaceBytes;
  LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws)));
  std::vector<hipblasLtMatmulHeuristicResult_t> r(kCandidates);
  int got = 0;
  hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(ds.handle, desc, a, b, d, d, pref, kCandidates, r.data(), &got);
  hipblasLtMatmulPreferenceDestroy(pref);
  hipblasLtMatrixLayoutDestroy(a);
  hipblasLtMatrixLayoutDestroy(b);
  hipblasLtMatrixLayoutDestroy(d);
  hipblasLtMatmulDescDestroy(desc);
  return st == HIPBLAS_STATUS_SUCCESS ? got : -(int64_t)st;
}

// (M, N, K, epi, has_bias, candidates, chosen) for every plan made so far: bench / test introspection
std::vector<int64_t> gemm_lt_plans() {
  std::lock_guard<std::mutex> lk(g_mu);
  std::vector<int64_t> out;
  for (auto& [dev, ds] : g_dev)
    for (auto& [k, p] : ds.plans) {
      out.insert(out.end(), {std::get<0>(k), std::get<1>(k), std::get<2>(k), std::get<3>(k), (int64_t)std::get<4>(k),
                             (int64_t)p.cands.size(), (int64_t)p.chosen});
    }
  return out;
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(pllm, m) {
  m.def("gemm_lt(Tensor x, Tensor w, Tensor? bias, int epi, bool tune=True, Tensor? residual=None) -> (Tensor, Tensor)");
  m.def("gemm_lt_out(Tensor x, Tensor w, Tensor? bias, Tensor(a!) out, bool tune=True) -> ()");
  m.def("gemm_lt_plans() -> int[]", &gemm_lt_plans);
  m.def("gemm_lt_probe(int M, int N, int K, int epilogue, int bias_type, int aux_type) -> int", &gemm_lt_probe);
}

TORCH_LIBRARY_IMPL(pllm, CUDA, m) {
  m.impl("gemm_lt", gemm_lt);
  m.impl("gemm_lt_out", gemm_lt_out);
}

// Probe: do hipBLASLt's fused activation epilogues have fast gfx950 solutions at the GPT-2 MLP shapes?
//   fwd  : H^T[F,M] = W1^T . X^T (+bias)            BIAS            (current: + separate act_fwd kernel)
//          G = gelu(H), aux = H                      GELU_AUX_BIAS   (fuses act_fwd)
//   bwd  : dG^T[F,M] = Wp^T . dY^T                   DEFAULT         (current: + act_bwd_colsum kernel)
//          dH = dgelu(dG, aux), db = rowsum(dH)      DGELU_BGRAD     (fuses act_bwd + bias grad)
// Build: hipcc -O2 --offload-arch=gfx950 bench/hipblaslt_epilogue_probe.cpp -lhipblaslt -o /tmp/probe
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    auto _s = (x);                                                                    \
    if ((int)_s != 0) { fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, (int)_s); exit(1); } \
  } while (0)

static hipblasLtHandle_t H;
static void* ws;
static const size_t WS = 64 << 20;

struct Case {
  const char* name;
  hipblasOperation_t ta, tb;
  int m, n, k;  // column-major D[m,n] = op(A)[m,k] op(B)[k,n]
  hipblasLtEpilogue_t epi;
  bool bias, aux;
};

static float run(const Case& c, int iters) {
  hipblasLtMatmulDesc_t d;
  CK(hipblasLtMatmulDescCreate(&d, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  CK(hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_TRANSA, &c.ta, sizeof(c.ta)));
  CK(hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_TRANSB, &c.tb, sizeof(c.tb)));
  CK(hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE, &c.epi, sizeof(c.epi)));
  void *A, *B, *D, *bias = nullptr, *aux = nullptr;
  CK(hipMalloc(&A, (size_t)c.m * c.k * 2));
  CK(hipMalloc(&B, (size_t)c.k * c.n * 2));
  CK(hipMalloc(&D, (size_t)c.m * c.n * 2));
  CK(hipMemset(A, 0, (size_t)c.m * c.k * 2));
  CK(hipMemset(B, 0, (size_t)c.k * c.n * 2));
  if (c.bias) {
    CK(hipMalloc(&bias, (size_t)c.m * 4));
    CK(hipMemset(bias, 0, (size_t)c.m * 4));
    hipDataType bt = c.epi == HIPBLASLT_EPILOGUE_DGELU_BGRAD ? HIP_R_32F : HIP_R_16BF;
    CK(hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
    CK(hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  }
  if (c.aux) {
    CK(hipMalloc(&aux, (size_t)c.m * c.n * 2));
    CK(hipMemset(aux, 0, (size_t)c.m * c.n * 2));
    int64_t ld = c.m;
    hipDataType at = HIP_R_16BF;
    CK(hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux, sizeof(aux)));
    CK(hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld)));
    CK(hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at, sizeof(at)));
  }
  hipblasLtMatrixLayout_t la, lb, ld;
  const int ar = c.ta == HIPBLAS_OP_N ? c.m : c.k, ac = c.ta == HIPBLAS_OP_N ? c.k : c.m;
  const int br = c.tb == HIPBLAS_OP_N ? c.k : c.n, bc = c.tb == HIPBLAS_OP_N ? c.n : c.k;
  CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, ar, ac, ar));
  CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, br, bc, br));
  CK(hipblasLtMatrixLayoutCreate(&ld, HIP_R_16BF, c.m, c.n, c.m));
  hipblasLtMatmulPreference_t pref;
  CK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t wsz = WS;
  CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsz, sizeof(wsz)));
  hipblasLtMatmulHeuristicResult_t res[16];
  int n = 0;
  auto st = hipblasLtMatmulAlgoGetHeuristic(H, d, la, lb, ld, ld, pref, 16, res, &n);
  float best = -1.f;
  int besti = -1;
  if (st == HIPBLAS_STATUS_SUCCESS && n > 0) {
    float alpha = 1.f, beta = 0.f;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < n; ++i) {
      if (hipblasLtMatmul(H, d, &alpha, A, la, B, lb, &beta, D, ld, D, ld, &res[i].algo, ws, WS, 0) != 0) continue;
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, 0));
      for (int it = 0; it < iters; ++it)
        hipblasLtMatmul(H, d, &alpha, A, la, B, lb, &beta, D, ld, D, ld, &res[i].algo, ws, WS, 0);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const float us = 1000.f * ms / iters;
      if (best < 0 || us < best) best = us, besti = i;
    }
  }
  const double fl = 2.0 * c.m * c.n * c.k;
  printf("{\"case\": \"%s\", \"m\": %d, \"n\": %d, \"k\": %d, \"heuristic_status\": %d, \"n_algos\": %d, \"best_us\": %.1f, "
         "\"tflops\": %.1f, \"best_idx\": %d}\n",
         c.name, c.m, c.n, c.k, (int)st, n, best, best > 0 ? fl / (best * 1e-6) / 1e12 : 0.0, besti);
  fflush(stdout);
  hipFree(A); hipFree(B); hipFree(D);
  if (bias) hipFree(bias);
  if (aux) hipFree(aux);
  hipblasLtMatrixLayoutDestroy(la); hipblasLtMatrixLayoutDestroy(lb); hipblasLtMatrixLayoutDestroy(ld);
  hipblasLtMatmulPreferenceDestroy(pref);
  hipblasLtMatmulDescDestroy(d);
  return best;
}

int main() {
  CK(hipblasLtCreate(&H));
  CK(hipMalloc(&ws, WS));
  const int M = 65536, C = 768, F = 3072;
  std::vector<Case> cs = {
      // forward up-projection: D[F, M] = W1(K=C x F, stored [F][C] -> transA) . X^T
      {"fwd_up_bias", HIPBLAS_OP_T, HIPBLAS_OP_N, F, M, C, HIPBLASLT_EPILOGUE_BIAS, true, false},
      {"fwd_up_gelu_bias", HIPBLAS_OP_T, HIPBLAS_OP_N, F, M, C, HIPBLASLT_EPILOGUE_GELU_BIAS, true, false},
      {"fwd_up_gelu_aux_bias", HIPBLAS_OP_T, HIPBLAS_OP_N, F, M, C, HIPBLASLT_EPILOGUE_GELU_AUX_BIAS, true, true},
      // backward: dG^T[F, M] = Wp(stored [C][F] -> col-major F x C, N) . dY^T (C x M, N)
      {"bwd_dgrad_nn", HIPBLAS_OP_N, HIPBLAS_OP_N, F, M, C, HIPBLASLT_EPILOGUE_DEFAULT, false, false},
      {"bwd_dgrad_nt", HIPBLAS_OP_T, HIPBLAS_OP_N, F, M, C, HIPBLASLT_EPILOGUE_DEFAULT, false, false},
      {"bwd_dgelu", HIPBLAS_OP_N, HIPBLAS_OP_N, F, M, C, HIPBLASLT_EPILOGUE_DGELU, false, true},
      {"bwd_dgelu_bgrad", HIPBLAS_OP_N, HIPBLAS_OP_N, F, M, C, HIPBLASLT_EPILOGUE_DGELU_BGRAD, true, true},
      {"bwd_dgelu_bgrad_nt", HIPBLAS_OP_T, HIPBLAS_OP_N, F, M, C, HIPBLASLT_EPILOGUE_DGELU_BGRAD, true, true},
  };
  for (auto& c : cs) run(c, 20);
  return 0;
}

// hipBLASLt plans with fused epilogues; see blaslt.h.
#include "blaslt.h"

#include <hipblaslt/hipblaslt.h>
#include <hipblaslt/hipblaslt-ext.hpp>

#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <tuple>
#include <vector>

namespace ffk {
namespace lt {
namespace {

#define LT_CHECK(x)                                                                        \
  do {                                                                                     \
    hipblasStatus_t s_ = (x);                                                              \
    if (s_ != HIPBLAS_STATUS_SUCCESS)                                                      \
      throw std::runtime_error(std::string("hipBLASLt: ") + #x + " -> " + std::to_string((int)s_)); \
  } while (0)

hipblasLtHandle_t handle() {
  static hipblasLtHandle_t h = nullptr;
  static std::once_flag once;
  std::call_once(once, [] { LT_CHECK(hipblasLtCreate(&h)); });
  return h;
}

struct Plan {
  PlanKey key;
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasOperation_t opA, opB;
  std::vector<hipblasLtMatmulHeuristicResult_t> algos;
  hipblasLtEpilogue_t epi;
};

std::vector<std::unique_ptr<Plan>>& plans() {
  static std::vector<std::unique_ptr<Plan>> p;
  return p;
}
std::map<std::tuple<int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int,
                    int, int64_t>,
         int64_t>&
plan_index() {
  static std::map<std::tuple<int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t,
                             int, int, int64_t>,
                  int64_t>
      m;
  return m;
}
std::mutex mu;

hipblasLtEpilogue_t to_lt(int e) {
  switch (e) {
    case EPI_NONE: return HIPBLASLT_EPILOGUE_DEFAULT;
    case EPI_BIAS: return HIPBLASLT_EPILOGUE_BIAS;
    case EPI_GELU_AUX_BIAS: return HIPBLASLT_EPILOGUE_GELU_AUX_BIAS;
    case EPI_DGELU_BGRAD: return HIPBLASLT_EPILOGUE_DGELU_BGRAD;
    case EPI_BGRADB: return HIPBLASLT_EPILOGUE_BGRADB;
    case EPI_RELU_BIAS: return HIPBLASLT_EPILOGUE_RELU_BIAS;
    case EPI_GELU_BIAS: return HIPBLASLT_EPILOGUE_GELU_BIAS;
    case EPI_DGELU: return HIPBLASLT_EPILOGUE_DGELU;
    case EPI_RELU_AUX_BIAS: return HIPBLASLT_EPILOGUE_RELU_AUX_BIAS;
    case EPI_GELU_AUX: return HIPBLASLT_EPILOGUE_GELU_AUX;
  }
  throw std::runtime_error("hipBLASLt: unknown epilogue " + std::to_string(e));
}

bool has_bias(int e) {
  return e == EPI_BIAS || e == EPI_GELU_AUX_BIAS || e == EPI_DGELU_BGRAD || e == EPI_BGRADB || e == EPI_RELU_BIAS ||
         e == EPI_GELU_BIAS || e == EPI_RELU_AUX_BIAS;
}
bool has_aux(int e) {
  return e == EPI_GELU_AUX_BIAS || e == EPI_DGELU_BGRAD || e == EPI_DGELU || e == EPI_RELU_AUX_BIAS ||
         e == EPI_GELU_AUX;
}

hipblasLtMatrixLayout_t layout(hipDataType t, int64_t rows, int64_t cols, int64_t ld, int64_t batch, int64_t stride) {
  hipblasLtMatrixLayout_t l;
  LT_CHECK(hipblasLtMatrixLayoutCreate(&l, t, rows, cols, ld));
  if (batch > 1) {
    int32_t b = (int32_t)batch;
    LT_CHECK(hipblasLtMatrixLayoutSetAttribute(l, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &b, sizeof(b)));
    LT_CHECK(hipblasLtMatrixLayoutSetAttribute(l, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &stride,
                                               sizeof(stride)));
  }
  return l;
}

Plan* get(int64_t id) {
  if (id < 0 || id >= (int64_t)plans().size()) throw std::runtime_error("hipBLASLt: bad plan id");
  return plans()[id].get();
}

}  // namespace

int64_t plan(const PlanKey& k, int max_algos, bool all_algos, size_t max_ws, const void* bias, const void* aux,
             int* n_algos) {
  std::lock_guard<std::mutex> g(mu);
  int flags = (k.a_k ? 1 : 0) | (k.b_k ? 2 : 0) | (k.out_f32 ? 4 : 0) | (k.bias_f32 ? 8 : 0) | (k.beta_nz ? 16 : 0) |
              (all_algos ? 32 : 0);
  auto key = std::make_tuple(k.M, k.N, k.K, k.lda, k.ldb, k.ldc, k.batch, k.sA, k.sB, k.sC, flags, k.epi, k.aux_ld);
  auto it = plan_index().find(key);
  if (it != plan_index().end()) {
    *n_algos = (int)plans()[it->second]->algos.size();
    return it->second;
  }
  auto p = std::make_unique<Plan>();
  p->key = k;
  p->epi = to_lt(k.epi);
  hipDataType bf = HIP_R_16BF, outT = k.out_f32 ? HIP_R_32F : HIP_R_16BF;
  // column-major view: D^T[N, M] = op(B)[N, K] . op(A)[K, M]
  p->opA = k.b_k ? HIPBLAS_OP_T : HIPBLAS_OP_N;  // library "A" = our B
  p->opB = k.a_k ? HIPBLAS_OP_N : HIPBLAS_OP_T;  // library "B" = our A
  p->la = k.b_k ? layout(bf, k.K, k.N, k.ldb, k.batch, k.sB) : layout(bf, k.N, k.K, k.ldb, k.batch, k.sB);
  p->lb = k.a_k ? layout(bf, k.K, k.M, k.lda, k.batch, k.sA) : layout(bf, k.M, k.K, k.lda, k.batch, k.sA);
  p->lc = layout(outT, k.N, k.M, k.ldc, k.batch, k.sC);
  LT_CHECK(hipblasLtMatmulDescCreate(&p->desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  int32_t ta = p->opA, tb = p->opB;
  LT_CHECK(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  LT_CHECK(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  uint32_t epi = p->epi;
  LT_CHECK(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
  if (has_bias(k.epi)) {
    int32_t bt = k.bias_f32 ? HIP_R_32F : HIP_R_16BF;
    LT_CHECK(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
    LT_CHECK(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
  }
  if (has_aux(k.epi)) {
    int64_t ld = k.aux_ld;
    LT_CHECK(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld)));
    int32_t at = HIP_R_16BF;
    LT_CHECK(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at, sizeof(at)));
    LT_CHECK(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux, sizeof(aux)));
  }
  if (all_algos) {
    std::vector<hipblasLtMatmulHeuristicResult_t> all;
    LT_CHECK(hipblaslt_ext::getAllAlgos(handle(), hipblaslt_ext::GemmType::HIPBLASLT_GEMM, p->opA, p->opB, bf, bf, outT,
                                        outT, HIPBLAS_COMPUTE_32F, all));
    float one = 1.f, beta = k.beta_nz ? 1.f : 0.f;
    for (auto& r : all) {
      size_t ws = 0;
      if (hipblaslt_ext::matmulIsAlgoSupported(handle(), p->desc, &one, p->la, p->lb, &beta, p->lc, p->lc, r.algo, ws) ==
              HIPBLAS_STATUS_SUCCESS &&
          ws <= max_ws) {
        r.workspaceSize = ws;
        p->algos.push_back(r);
        if ((int)p->algos.size() >= max_algos) break;
      }
    }
  } else {
    hipblasLtMatmulPreference_t pref;
    LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
    uint64_t wsb = max_ws;
    LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
    std::vector<hipblasLtMatmulHeuristicResult_t> res(max_algos);
    int got = 0;
    hipblasStatus_t s = hipblasLtMatmulAlgoGetHeuristic(handle(), p->desc, p->la, p->lb, p->lc, p->lc, pref, max_algos,
                                                        res.data(), &got);
    hipblasLtMatmulPreferenceDestroy(pref);
    if (s == HIPBLAS_STATUS_SUCCESS)
      for (int i = 0; i < got; ++i)
        if (res[i].state == HIPBLAS_STATUS_SUCCESS) p->algos.push_back(res[i]);
  }
  *n_algos = (int)p->algos.size();
  int64_t id = (int64_t)plans().size();
  plans().push_back(std::move(p));
  plan_index()[key] = id;
  return id;
}

int num_algos(int64_t id) { return (int)get(id)->algos.size(); }

int algo_index(int64_t id, int a) {
  Plan* p = get(id);
  if (a < 0 || a >= (int)p->algos.size()) return -1;
  return hipblaslt_ext::getIndexFromAlgo(p->algos[a].algo);
}

int find_algo(int64_t id, int sol, size_t max_ws) {
  Plan* p = get(id);
  for (int i = 0; i < (int)p->algos.size(); ++i)
    if (hipblaslt_ext::getIndexFromAlgo(p->algos[i].algo) == sol) return i;
  std::vector<int> idx{sol};
  std::vector<hipblasLtMatmulHeuristicResult_t> r;
  if (hipblaslt_ext::getAlgosFromIndex(handle(), idx, r) != HIPBLAS_STATUS_SUCCESS || r.empty()) return -1;
  float one = 1.f, beta = p->key.beta_nz ? 1.f : 0.f;
  size_t ws = 0;
  if (hipblaslt_ext::matmulIsAlgoSupported(handle(), p->desc, &one, p->la, p->lb, &beta, p->lc, p->lc, r[0].algo, ws) !=
          HIPBLAS_STATUS_SUCCESS ||
      ws > max_ws)
    return -1;
  r[0].workspaceSize = ws;
  p->algos.push_back(r[0]);
  return (int)p->algos.size() - 1;
}

size_t algo_ws(int64_t id, int a) { return get(id)->algos.at(a).workspaceSize; }

std::string algo_name(int64_t id, int a) {
  Plan* p = get(id);
  return hipblaslt_ext::getKernelNameFromAlgo(handle(), p->algos.at(a).algo);
}

int run(int64_t id, int a, const void* A, const void* B, void* C, const void* bias, void* aux, float alpha, float beta,
        void* ws, size_t ws_bytes, hipStream_t st) {
  Plan* p = get(id);
  if (a < 0 || a >= (int)p->algos.size()) return (int)HIPBLAS_STATUS_INVALID_VALUE;
  auto& r = p->algos[a];
  if (r.workspaceSize > ws_bytes) return (int)HIPBLAS_STATUS_INVALID_VALUE;
  if (has_bias(p->key.epi)) {
    LT_CHECK(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
  }
  if (has_aux(p->key.epi)) {
    LT_CHECK(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux, sizeof(aux)));
  }
  // library "A" = our B, library "B" = our A
  return (int)hipblasLtMatmul(handle(), p->desc, &alpha, B, p->la, A, p->lb, &beta, C, p->lc, C, p->lc, &r.algo, ws,
                              r.workspaceSize, st);
}

}  // namespace lt
}  // namespace ffk

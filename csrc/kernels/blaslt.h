// hipBLASLt GEMMs with fused epilogues (bias, GELU + pre-activation store, dGELU + bias gradient).
//
// The plain library GEMM already beats our MFMA kernels on BERT-sized shapes (profiles/
// gemm_probe_r1_v5.txt); what it lacked through torch.mm was the epilogue, so every GELU linear
// paid a separate elementwise pass over [tokens, 4096] in forward and another in backward. Here
// the library's own epilogues do that work inside the GEMM:
//   EPI_BIAS           D = A.B + bias
//   EPI_GELU_AUX_BIAS  Z = A.B + bias (aux store), D = gelu_tanh(Z)      (Linear fwd, GELU)
//   EPI_DGELU_BGRAD    D = (A.B) * gelu_tanh'(Z), dbias = colsum(D)       (dgrad of the NEXT
//                      linear, producing dZ of this one: cross-op fusion done by the executor)
//   EPI_BGRADB         D = A.B, dbias = sums of B's reduction rows        (wgrad + bias grad)
// Row-major [M,N] outputs are column-major [N,M] to the library, so the call is D^T = B^T A^T.
// Plans (descriptors + candidate algorithms) are cached per call site; the Python side times the
// candidates once (autotune) and replays the winner by index.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <string>

namespace ffk {
namespace lt {

enum Epi : int {
  EPI_NONE = 0,
  EPI_BIAS = 1,
  EPI_GELU_AUX_BIAS = 2,
  EPI_DGELU_BGRAD = 3,
  EPI_BGRADB = 4,
  EPI_RELU_BIAS = 5,
  EPI_GELU_BIAS = 6,
  EPI_DGELU = 7,
  EPI_RELU_AUX_BIAS = 8,
  EPI_GELU_AUX = 9,
};

struct PlanKey {
  int64_t M, N, K, lda, ldb, ldc, batch, sA, sB, sC;
  bool a_k, b_k, out_f32, bias_f32, beta_nz;
  int epi;
  int64_t aux_ld;
};

// Creates (or returns the cached) plan; returns its id. n_algos receives the number of candidate
// algorithms (heuristic top-k, or every supported solution when all_algos).
// bias / aux: the call site's buffers (the library checks epilogue support with them set).
int64_t plan(const PlanKey& k, int max_algos, bool all_algos, size_t max_ws, const void* bias, const void* aux,
             int* n_algos);
int num_algos(int64_t plan_id);
// Solution index of candidate `algo` (stable across processes for one library build), -1 if none.
int algo_index(int64_t plan_id, int algo);
// Candidate position of a solution index inside the plan (adds it if the library accepts it for
// this problem); -1 if unsupported.
int find_algo(int64_t plan_id, int solution_index, size_t max_ws);
size_t algo_ws(int64_t plan_id, int algo);
std::string algo_name(int64_t plan_id, int algo);
// D = epilogue(alpha * op(A).op(B) + beta * C); C == D. Returns the hipblasStatus_t.
int run(int64_t plan_id, int algo, const void* A, const void* B, void* C, const void* bias, void* aux, float alpha,
        float beta, void* ws, size_t ws_bytes, hipStream_t st);

}  // namespace lt
}  // namespace ffk

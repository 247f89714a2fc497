#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ffk {

struct GemmArgs {
  const uint16_t* A = nullptr;  // bf16
  const uint16_t* B = nullptr;  // bf16
  void* C = nullptr;            // bf16 or fp32 (out_f32)
  void* Z = nullptr;            // optional bf16 pre-activation output (same layout as C)
  const void* bias = nullptr;   // optional [N], fp32 or bf16 (bias_bf16)
  float* ws = nullptr;          // split-K workspace
  int M = 0, N = 0, K = 0;
  int64_t lda = 0, ldb = 0, ldc = 0;
  int64_t sA = 0, sB = 0, sC = 0;  // batch strides in elements
  int batch = 1;
  float alpha = 1.f, beta = 0.f;
  int act = 10;  // ACT_NONE
  bool a_kcontig = true, b_kcontig = true;
  bool out_f32 = false;
  bool bias_bf16 = false;
  bool vec_ok = false;
  bool vec8_ok = false;  // 16-B row chunks of C/Z (and of the split-K slab) can be stored whole
  int splitk = 1;
  int kchunk = 0;
  int64_t a_bytes = 0, b_bytes = 0;  // operand storage sizes (range checks of the DMA path)
  // 6: persistent 8-wave ping-pong (gemm_pp.hip; falls back to 2 for what it refuses), 2: 256-row
  // kernel with the fused epilogues (gemm256.hip), 1: 256x128 kernel (gemm_big.hip), 0: 128x128
  // (this file). Round 5 removed the 4-wave kernels 3 / 4 / 5 (gemm_w4{,p,q}.hip): the ping-pong
  // kernel matched or beat them at every zoo call site they won (profiles/gemm_zoo_tune_r5.txt).
  int impl = 2;
  // Backward-activation epilogue (gemm256 only, see gemm_dact_bf16): C = (alpha*A.B) * act'(zin),
  // zin the producer's bf16 pre-activation in C's layout; colpart (optional) receives per-128-row
  // fp32 column sums of that product, [2 * ceil(M / 256)][N], for the producer's bias gradient.
  const void* zin = nullptr;
  float* colpart = nullptr;
  bool dact = false;
  int ablate = 0;  // measurement builds only (impl 61: gemm_pp without its loop DMA)
  bool skip_reduce = false;  // split-K: write the slabs only (the caller runs slab_sum, e.g. on a side stream)
};

void gemm_bf16(GemmArgs p, hipStream_t stream);
int64_t gemm_workspace_bytes(int M, int N, int K, int batch, int splitk);
int gemm_pick_splitk(int M, int N, int K, int batch, int impl = 2);
bool gemm_big_bf16(const GemmArgs& p, int64_t a_bytes, int64_t b_bytes, hipStream_t stream);
bool gemm256_bf16(const GemmArgs& p, int64_t a_bytes, int64_t b_bytes, hipStream_t stream);
// persistent 8-wave ping-pong 256x256x64 kernel, two waves per SIMD alternating MFMA and memory
// phases (gemm_pp.hip); batch 1, no beta / split-K / activation, K % 64 == 0
bool gemm_pp_bf16(const GemmArgs& p, int64_t a_bytes, int64_t b_bytes, hipStream_t stream);
int gemm256_bn(int M, int N, int batch, int splitk);
// fp32 operands and output on the f32-input MFMA (gemm_f32.hip): any shape / layout, batch strides,
// alpha / beta / bias / activation / pre-activation epilogue (A, B, C, Z reinterpreted as float)
void gemm_f32(const GemmArgs& p, hipStream_t stream);
// fp32 attention path: -inf above the causal diagonal of [rows][Sk] scores (rows = batch * Sq)
void causal_mask_f32(float* s, int64_t rows, int Sq, int Sk, hipStream_t st);
// dgrad GEMM of a consumer Linear fused with the producer Linear's activation backward:
// C[M,N] bf16 = (A.B) * act'(zin), colpart as above. False when the shape / alignment does not
// fit the 256-row kernel's coalesced epilogue (the caller then runs GEMM + bias_act_bwd).
bool gemm_dact_bf16(GemmArgs p, hipStream_t stream);

}  // namespace ffk

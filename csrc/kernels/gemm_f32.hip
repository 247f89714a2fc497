// fp32 GEMM on the f32-input MFMA (v_mfma_f32_32x32x2_f32: exact f32 products, one rounding per
// fmaf, 1/16 of the bf16 rate = the f32 VALU peak) for the --dtype fp32 path (the reference trains
// in fp32: src/ops/kernels/linear_kernels.cu:213, cublasGemmEx).
//
// C[b][m][n] = act(alpha * sum_k op(A)[m][k] op(B)[k][n] + beta * C + bias[n]) (Z: pre-activation).
// 128 x 128 x 32 block tile, 256 threads as 2 x 2 waves of 64 x 64 (2 x 2 MFMA tiles of 32 x 32).
// Operands stage k-major in LDS ([32][128 + 4] floats per operand) so that a fragment read (32
// consecutive rows or columns at one k) is one conflict-free ds_read_b32 per lane; the next K-tile's
// global loads (float4 along the contiguous dimension when aligned) are in registers while the
// current one computes (register double buffering, one barrier pair per K-tile). Any M / N / K,
// either operand K- or MN-contiguous, strided batches (blockIdx.z).
#include "common.h"
#include "gemm.h"
#include "ops.h"

namespace ffk {
namespace f32g {

constexpr int BM = 128, BN = 128, BK = 32, NT = 256, LDP = BM + 4;
typedef float f32x16 __attribute__((ext_vector_type(16)));

// 16 floats of one operand per thread per K-tile: rows/cols r of [128][32] (K-contig: 8 float4 along
// k per row chunk) or k-rows of [32][128] (MN-contig: float4 along m/n)
template <bool KCONT, bool VEC>
__device__ __forceinline__ void load_tile(const float* __restrict__ P, int64_t ld, int mn0, int k0, int MN, int K,
                                          int tid, float (&r)[16]) {
  if (KCONT) {  // element (mn, k) at P[mn * ld + k]; thread: row = tid / 2 (0..127), k half = tid % 2
    const int row = tid >> 1, kh = (tid & 1) * 16;
    const int mn = mn0 + row;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = k0 + kh + q * 4;
      if (VEC && mn < MN && k + 3 < K) {
        const float4 v = *reinterpret_cast<const float4*>(P + (int64_t)mn * ld + k);
        r[q * 4 + 0] = v.x; r[q * 4 + 1] = v.y; r[q * 4 + 2] = v.z; r[q * 4 + 3] = v.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) r[q * 4 + e] = (mn < MN && k + e < K) ? P[(int64_t)mn * ld + k + e] : 0.f;
      }
    }
  } else {  // element (mn, k) at P[k * ld + mn]; thread: k row = tid / 8, 16 columns at (tid % 8) * 16
    const int kr = tid >> 3, c0 = (tid & 7) * 16;
    const int k = k0 + kr;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int mn = mn0 + c0 + q * 4;
      if (VEC && k < K && mn + 3 < MN) {
        const float4 v = *reinterpret_cast<const float4*>(P + (int64_t)k * ld + mn);
        r[q * 4 + 0] = v.x; r[q * 4 + 1] = v.y; r[q * 4 + 2] = v.z; r[q * 4 + 3] = v.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) r[q * 4 + e] = (k < K && mn + e < MN) ? P[(int64_t)k * ld + mn + e] : 0.f;
      }
    }
  }
}

// registers -> k-major LDS image s[k][mn]
template <bool KCONT>
__device__ __forceinline__ void store_tile(float* s, int tid, const float (&r)[16]) {
  if (KCONT) {
    const int row = tid >> 1, kh = (tid & 1) * 16;
#pragma unroll
    for (int e = 0; e < 16; ++e) s[(kh + e) * LDP + row] = r[e];
  } else {
    const int kr = tid >> 3, c0 = (tid & 7) * 16;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<float4*>(s + kr * LDP + c0 + q * 4) = make_float4(r[q * 4], r[q * 4 + 1], r[q * 4 + 2], r[q * 4 + 3]);
  }
}

template <bool A_K, bool B_K, bool VA, bool VB>
__global__ void __launch_bounds__(NT) gemm_f32_kernel(GemmArgs p) {
  __shared__ float sA[BK * LDP], sB[BK * LDP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tm = (p.M + BM - 1) / BM, tn = (p.N + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, tm * tn);
  const int m0 = (bid / tn) * BM, n0 = (bid % tn) * BN;
  const int b = blockIdx.z;
  const float* A = reinterpret_cast<const float*>(p.A) + (int64_t)b * p.sA;
  const float* B = reinterpret_cast<const float*>(p.B) + (int64_t)b * p.sB;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  float ra[16], rb[16];
  load_tile<A_K, VA>(A, p.lda, m0, 0, p.M, p.K, tid, ra);
  load_tile<B_K, VB>(B, p.ldb, n0, 0, p.N, p.K, tid, rb);
  const int nk = (p.K + BK - 1) / BK;
  for (int t = 0; t < nk; ++t) {
    store_tile<A_K>(sA, tid, ra);
    store_tile<B_K>(sB, tid, rb);
    __syncthreads();
    if (t + 1 < nk) {  // next K-tile's loads in flight during this tile's MFMAs
      load_tile<A_K, VA>(A, p.lda, m0, (t + 1) * BK, p.M, p.K, tid, ra);
      load_tile<B_K, VB>(B, p.ldb, n0, (t + 1) * BK, p.N, p.K, tid, rb);
    }
#pragma unroll
    for (int ks = 0; ks < BK / 2; ++ks) {
      const int k = 2 * ks + (lane >> 5);
      float a[2], bv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = sA[k * LDP + wm * 64 + i * 32 + (lane & 31)];
#pragma unroll
      for (int j = 0; j < 2; ++j) bv[j] = sB[k * LDP + wn * 64 + j * 32 + (lane & 31)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], bv[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  // epilogue: D layout of 32x32: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
  float* C = reinterpret_cast<float*>(p.C) + (int64_t)b * p.sC;
  float* Z = p.Z ? reinterpret_cast<float*>(p.Z) + (int64_t)b * p.sC : nullptr;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 64 + j * 32 + (lane & 31);
      if (n >= p.N) continue;
      const float bias = p.bias ? (p.bias_bf16 ? bf2f(reinterpret_cast<const bf16_t*>(p.bias)[n])
                                               : reinterpret_cast<const float*>(p.bias)[n])
                                : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m >= p.M) continue;
        float* dst = C + (int64_t)m * p.ldc + n;
        float x = acc[i][j][r] * p.alpha;
        if (p.beta != 0.f) x += p.beta * *dst;
        x += bias;
        if (Z) Z[(int64_t)m * p.ldc + n] = x;
        *dst = p.act != ACT_NONE ? act_fwd(p.act, x) : x;
      }
    }
}

template <bool A_K, bool B_K>
static void launch(const GemmArgs& p, dim3 g, hipStream_t s, bool va, bool vb) {
  if (va && vb) hipLaunchKernelGGL((gemm_f32_kernel<A_K, B_K, true, true>), g, dim3(NT), 0, s, p);
  else if (va) hipLaunchKernelGGL((gemm_f32_kernel<A_K, B_K, true, false>), g, dim3(NT), 0, s, p);
  else if (vb) hipLaunchKernelGGL((gemm_f32_kernel<A_K, B_K, false, true>), g, dim3(NT), 0, s, p);
  else hipLaunchKernelGGL((gemm_f32_kernel<A_K, B_K, false, false>), g, dim3(NT), 0, s, p);
}

}  // namespace f32g

void gemm_f32(const GemmArgs& p, hipStream_t stream) {
  using namespace f32g;
  if (p.M <= 0 || p.N <= 0 || p.batch <= 0) return;
  auto al = [](const void* q, int64_t ld, int64_t st) { return ((uintptr_t)q % 16) == 0 && ld % 4 == 0 && st % 4 == 0; };
  const bool va = al(p.A, p.lda, p.sA), vb = al(p.B, p.ldb, p.sB);
  dim3 grid(((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN), 1, p.batch);
  if (p.a_kcontig && p.b_kcontig) launch<true, true>(p, grid, stream, va, vb);
  else if (p.a_kcontig) launch<true, false>(p, grid, stream, va, vb);
  else if (p.b_kcontig) launch<false, true>(p, grid, stream, va, vb);
  else launch<false, false>(p, grid, stream, va, vb);
}

// scores[b][i][j] = -inf for j > i + (Sk - Sq): the causal mask of the fp32 attention path, before
// its softmax (row-major [rows = batch * Sq][Sk], fp32)
__global__ void causal_mask_kernel(float* __restrict__ s, int64_t rows, int Sq, int Sk) {
  const int64_t n = rows * Sk;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(e % Sk);
    const int i = (int)((e / Sk) % Sq);
    if (j > i + (Sk - Sq)) s[e] = -INFINITY;
  }
}
void causal_mask_f32(float* s, int64_t rows, int Sq, int Sk, hipStream_t st) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(causal_mask_kernel, dim3(ew_grid(rows * Sk, 256)), dim3(256), 0, st, s, rows, Sq, Sk);
}

}  // namespace ffk

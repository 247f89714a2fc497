// Embedding lookup (with optional bag aggregation SUM/AVG as in DLRM) and its backward.
// Forward: one wave per output row gathers `bag` table rows with 16-B loads and sums in fp32.
// Backward: fp32 atomic scatter-add into the gradient table, one 256-B-contiguous wave
// instruction per (row, 64-column chunk) — the atomic shape Guideline 12 / MI355X_MICROARCH
// 'Global float atomics' measures at full rate.
// Replaces reference src/ops/embedding.cu (embed_forward_with_aggr / embed_backward_with_aggr).
#include "common.h"
#include "ops.h"

namespace ffk {

template <typename T, typename I>
__global__ void emb_fwd_kernel(const I* __restrict__ idx, const T* __restrict__ table, T* __restrict__ out,
                               int64_t n_rows, int bag, int dim, int64_t num_rows, int avg) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const float scale = avg ? 1.f / bag : 1.f;
  for (int64_t r = wave; r < n_rows; r += nwaves) {
    for (int c = lane; c < dim; c += 64) {
      float s = 0.f;
      for (int b = 0; b < bag; ++b) {
        int64_t id = (int64_t)idx[r * bag + b];
        if (id < 0 || id >= num_rows) continue;
        s += Cvt<T>::to_f(table[id * dim + c]);
      }
      out[r * dim + c] = Cvt<T>::from_f(s * scale);
    }
  }
}

template <typename T, typename I>
__global__ void emb_bwd_kernel(const I* __restrict__ idx, const T* __restrict__ dout, float* __restrict__ dtable,
                               int64_t n_rows, int bag, int dim, int64_t num_rows, int avg) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const float scale = avg ? 1.f / bag : 1.f;
  for (int64_t r = wave; r < n_rows; r += nwaves) {
    for (int c = lane; c < dim; c += 64) {
      const float g = Cvt<T>::to_f(dout[r * dim + c]) * scale;
      for (int b = 0; b < bag; ++b) {
        int64_t id = (int64_t)idx[r * bag + b];
        if (id < 0 || id >= num_rows) continue;
        atomicAdd(dtable + id * dim + c, g);
      }
    }
  }
}

void embedding_fwd(int dt, int idx64, const void* idx, const void* table, void* out, int64_t n_out_rows, int bag,
                   int dim, int64_t num_rows, int aggr_avg, hipStream_t st) {
  if (n_out_rows == 0) return;
  const int blocks = (int)std::min<int64_t>((n_out_rows + 3) / 4, 16384);
#define EF(T, I) hipLaunchKernelGGL((emb_fwd_kernel<T, I>), dim3(blocks), dim3(256), 0, st, (const I*)idx, (const T*)table, \
                                    (T*)out, n_out_rows, bag, dim, num_rows, aggr_avg)
  if (dt == DT_BF16) { if (idx64) EF(bf16_t, int64_t); else EF(bf16_t, int); }
  else { if (idx64) EF(float, int64_t); else EF(float, int); }
#undef EF
}
void embedding_bwd(int dt, int idx64, const void* idx, const void* dout, float* dtable, int64_t n_out_rows, int bag,
                   int dim, int64_t num_rows, int aggr_avg, hipStream_t st) {
  if (n_out_rows == 0) return;
  const int blocks = (int)std::min<int64_t>((n_out_rows + 3) / 4, 16384);
#define EB(T, I) hipLaunchKernelGGL((emb_bwd_kernel<T, I>), dim3(blocks), dim3(256), 0, st, (const I*)idx, (const T*)dout, \
                                    dtable, n_out_rows, bag, dim, num_rows, aggr_avg)
  if (dt == DT_BF16) { if (idx64) EB(bf16_t, int64_t); else EB(bf16_t, int); }
  else { if (idx64) EB(float, int64_t); else EB(float, int); }
#undef EB
}

}  // namespace ffk

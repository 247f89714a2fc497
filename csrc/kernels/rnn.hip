// LSTM cell kernels (pointwise part of one timestep; the GEMMs run on the shared GEMM path).
//
// Reference: nmt/lstm.cu (cuDNN RNN LSTM over chunks of timesteps, the legacy Legion NMT app).
// Here the input projection X.W_ih^T + b for all timesteps is one GEMM, the recurrent projection
// h_{t-1}.W_hh^T is one GEMM per step accumulated (beta = 1) into that step's rows, and these
// kernels do everything else of a step in one pass:
//   forward : i,f,o = sigmoid, g = tanh of the four gate pre-activations; c = f*c_prev + i*g;
//             h = o*tanh(c). The activated gates overwrite the pre-activations (kept for the
//             backward), c is kept in fp32 for every step, h goes straight into y[:, t].
//   backward: dh = dy[:, t] + dh_rec; dc = dc_next + dh*o*(1 - tanh(c)^2); the four gate
//             gradients (pre-activation) land in dG[:, t] and dc_prev = dc*f.
// Layout: gates row b of step t at G + b*ldg + t*4H (ldg = L*4H), gate order i, f, g, o (torch).
#include "common.h"
#include "ops.h"

namespace ffk {

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

template <typename T>
__global__ void __launch_bounds__(256) lstm_fwd_cell_kernel(T* __restrict__ G, int64_t ldg, const float* __restrict__ c_prev,
                                                            float* __restrict__ c_out, T* __restrict__ h_out,
                                                            int64_t ldh, int B, int H) {
  const int64_t n = (int64_t)B * H;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(idx / H), j = (int)(idx % H);
    T* g = G + (int64_t)b * ldg;
    const float i = sigm(Cvt<T>::to_f(g[j]));
    const float f = sigm(Cvt<T>::to_f(g[H + j]));
    const float gg = tanhf(Cvt<T>::to_f(g[2 * H + j]));
    const float o = sigm(Cvt<T>::to_f(g[3 * H + j]));
    const float c = f * c_prev[idx] + i * gg;
    c_out[idx] = c;
    h_out[(int64_t)b * ldh + j] = Cvt<T>::from_f(o * tanhf(c));
    g[j] = Cvt<T>::from_f(i);
    g[H + j] = Cvt<T>::from_f(f);
    g[2 * H + j] = Cvt<T>::from_f(gg);
    g[3 * H + j] = Cvt<T>::from_f(o);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) lstm_bwd_cell_kernel(const T* G, int64_t ldg, const float* __restrict__ c,
                                                            const float* __restrict__ c_prev, const T* __restrict__ dy,
                                                            int64_t lddy, const T* __restrict__ dh_rec,
                                                            float* __restrict__ dc /* in: dc_next, out: dc_prev */,
                                                            T* dG /* may alias G: each lane reads then writes the
                                                                     same four gate slots */, int B, int H) {
  const int64_t n = (int64_t)B * H;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(idx / H), j = (int)(idx % H);
    const T* g = G + (int64_t)b * ldg;
    const float i = Cvt<T>::to_f(g[j]), f = Cvt<T>::to_f(g[H + j]);
    const float gg = Cvt<T>::to_f(g[2 * H + j]), o = Cvt<T>::to_f(g[3 * H + j]);
    float dh = dy ? Cvt<T>::to_f(dy[(int64_t)b * lddy + j]) : 0.f;
    if (dh_rec) dh += Cvt<T>::to_f(dh_rec[idx]);
    const float tc = tanhf(c[idx]);
    const float dcv = dc[idx] + dh * o * (1.f - tc * tc);
    T* d = dG + (int64_t)b * ldg;
    d[j] = Cvt<T>::from_f(dcv * gg * i * (1.f - i));
    d[H + j] = Cvt<T>::from_f(dcv * c_prev[idx] * f * (1.f - f));
    d[2 * H + j] = Cvt<T>::from_f(dcv * i * (1.f - gg * gg));
    d[3 * H + j] = Cvt<T>::from_f(dh * tc * o * (1.f - o));
    dc[idx] = dcv * f;
  }
}

void lstm_fwd_cell(int dt, void* G, int64_t ldg, const float* c_prev, float* c_out, void* h_out, int64_t ldh, int B,
                   int H, hipStream_t st) {
  if (B == 0 || H == 0) return;
  const dim3 grid(ew_grid((int64_t)B * H, 256));
  if (dt == DT_BF16)
    hipLaunchKernelGGL(lstm_fwd_cell_kernel<bf16_t>, grid, dim3(256), 0, st, (bf16_t*)G, ldg, c_prev, c_out,
                       (bf16_t*)h_out, ldh, B, H);
  else
    hipLaunchKernelGGL(lstm_fwd_cell_kernel<float>, grid, dim3(256), 0, st, (float*)G, ldg, c_prev, c_out,
                       (float*)h_out, ldh, B, H);
}

void lstm_bwd_cell(int dt, const void* G, int64_t ldg, const float* c, const float* c_prev, const void* dy,
                   int64_t lddy, const void* dh_rec, float* dc, void* dG, int B, int H, hipStream_t st) {
  if (B == 0 || H == 0) return;
  const dim3 grid(ew_grid((int64_t)B * H, 256));
  if (dt == DT_BF16)
    hipLaunchKernelGGL(lstm_bwd_cell_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)G, ldg, c, c_prev,
                       (const bf16_t*)dy, lddy, (const bf16_t*)dh_rec, dc, (bf16_t*)dG, B, H);
  else
    hipLaunchKernelGGL(lstm_bwd_cell_kernel<float>, grid, dim3(256), 0, st, (const float*)G, ldg, c, c_prev,
                       (const float*)dy, lddy, (const float*)dh_rec, dc, (float*)dG, B, H);
}

}  // namespace ffk

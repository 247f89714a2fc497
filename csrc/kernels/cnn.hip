// CNN support kernels (NCHW): batch normalization and 2-D pooling, forward and backward.
//
// Reference: src/ops/batch_norm.cu (cuDNN spatial batch norm, fused ReLU) and src/ops/pool_2d.cu
// (cuDNN max / average pooling). Here:
//   * BatchNorm statistics are a split reduction: grid (C, S) workgroups each fold a contiguous
//     slice of one channel's N*H*W elements with Welford (count, mean, M2) — stable where
//     sum / sum-of-squares cancels — and a finalize pass merges the S partials per channel, updates
//     the running statistics (momentum, unbiased variance as torch does) and saves mean / rstd.
//     The normalize(+ReLU) pass and the backward dx pass are elementwise; the backward's two
//     per-channel sums (dy, dy * xhat, with the ReLU mask recomputed from x) reuse the split
//     reduction.
//   * Max pooling records the winning window offset (one byte per output) so the backward is a
//     gather: each input element sums dy over the outputs whose window it won — no atomics, no
//     read of the whole window again. Average pooling follows torch's divisor rules
//     (count_include_pad, windows clipped at the padded border).
#include "common.h"
#include "ops.h"

namespace ffk {

// ------------------------------------------------------------------------------- batch norm
__device__ __forceinline__ void wf_merge(float& n, float& mean, float& m2, float n2, float mean2, float m22) {
  if (n2 == 0.f) return;
  if (n == 0.f) { n = n2; mean = mean2; m2 = m22; return; }
  const float nt = n + n2, d = mean2 - mean;
  mean += d * (n2 / nt);
  m2 += m22 + d * d * (n * n2 / nt);
  n = nt;
}

// Workgroup reduction of NV floats per thread through LDS (256 threads).
template <int NV, typename F>
__device__ __forceinline__ void block_fold(float* v, float (*sh)[4], F merge) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float w[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) w[i] = __shfl_xor(v[i], o, 64);
    merge(v, w);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < NV; ++i) sh[i][wave] = v[i];
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      float w[NV];
#pragma unroll
      for (int i = 0; i < NV; ++i) w[i] = sh[i][k];
      merge(v, w);
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) bn_stats_kernel(const T* __restrict__ x, float* __restrict__ part, int N, int C,
                                                       int HW, int S) {
  __shared__ float sh[3][4];
  const int c = blockIdx.x, s = blockIdx.y;
  const int64_t M = (int64_t)N * HW;
  const int64_t j0 = M * s / S, j1 = M * (s + 1) / S;
  float n = 0.f, mean = 0.f, m2 = 0.f;
  for (int64_t j = j0 + threadIdx.x; j < j1; j += 256) {
    const int64_t img = j / HW, hw = j - img * HW;
    const float v = Cvt<T>::to_f(x[(img * C + c) * HW + hw]);
    n += 1.f;
    const float d = v - mean;
    mean += d / n;
    m2 += d * (v - mean);
  }
  float v[3] = {n, mean, m2};
  block_fold<3>(v, sh, [](float* a, const float* b) { wf_merge(a[0], a[1], a[2], b[0], b[1], b[2]); });
  if (threadIdx.x == 0) {
    float* p = part + ((int64_t)c * S + s) * 3;
    p[0] = v[0]; p[1] = v[1]; p[2] = v[2];
  }
}

__global__ void bn_finalize_kernel(const float* __restrict__ part, int C, int S, float eps, float momentum,
                                   float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                   float* __restrict__ run_mean, float* __restrict__ run_var) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float n = 0.f, mean = 0.f, m2 = 0.f;
  for (int s = 0; s < S; ++s) {
    const float* p = part + ((int64_t)c * S + s) * 3;
    wf_merge(n, mean, m2, p[0], p[1], p[2]);
  }
  const float var = n > 0.f ? m2 / n : 0.f;
  mean_out[c] = mean;
  rstd_out[c] = rsqrtf(var + eps);
  if (run_mean) run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean;
  if (run_var) run_var[c] = (1.f - momentum) * run_var[c] + momentum * (n > 1.f ? m2 / (n - 1.f) : var);
}

// inference statistics: mean = running mean, rstd = 1/sqrt(running var + eps)
__global__ void bn_running_kernel(const float* __restrict__ run_mean, const float* __restrict__ run_var, int C,
                                  float eps, float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean_out[c] = run_mean[c];
  rstd_out[c] = rsqrtf(run_var[c] + eps);
}

template <typename T>
__global__ void __launch_bounds__(256) bn_apply_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                       const float* __restrict__ mean, const float* __restrict__ rstd,
                                                       const T* __restrict__ g, const T* __restrict__ b, int64_t total,
                                                       int C, int HW, int relu) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int c = (int)((i / HW) % C);
    float v = (Cvt<T>::to_f(x[i]) - mean[c]) * rstd[c] * Cvt<T>::to_f(g[c]) + Cvt<T>::to_f(b[c]);
    if (relu) v = fmaxf(v, 0.f);
    y[i] = Cvt<T>::from_f(v);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd, const T* __restrict__ g,
                                                            const T* __restrict__ b, float* __restrict__ part, int N,
                                                            int C, int HW, int S, int relu) {
  __shared__ float sh[2][4];
  const int c = blockIdx.x, s = blockIdx.y;
  const int64_t M = (int64_t)N * HW;
  const int64_t j0 = M * s / S, j1 = M * (s + 1) / S;
  const float mu = mean[c], rs = rstd[c], gc = Cvt<T>::to_f(g[c]), bc = Cvt<T>::to_f(b[c]);
  float s1 = 0.f, s2 = 0.f;
  for (int64_t j = j0 + threadIdx.x; j < j1; j += 256) {
    const int64_t img = j / HW, hw = j - img * HW;
    const int64_t i = (img * C + c) * HW + hw;
    const float xh = (Cvt<T>::to_f(x[i]) - mu) * rs;
    float d = Cvt<T>::to_f(dy[i]);
    if (relu && xh * gc + bc <= 0.f) d = 0.f;
    s1 += d;
    s2 += d * xh;
  }
  float v[2] = {s1, s2};
  block_fold<2>(v, sh, [](float* a, const float* bb) { a[0] += bb[0]; a[1] += bb[1]; });
  if (threadIdx.x == 0) {
    float* p = part + ((int64_t)c * S + s) * 2;
    p[0] = v[0]; p[1] = v[1];
  }
}

__global__ void bn_bwd_finalize_kernel(const float* __restrict__ part, int C, int S, float* __restrict__ sums,
                                       float* __restrict__ dg, float* __restrict__ db) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s1 = 0.f, s2 = 0.f;
  for (int s = 0; s < S; ++s) {
    s1 += part[((int64_t)c * S + s) * 2];
    s2 += part[((int64_t)c * S + s) * 2 + 1];
  }
  sums[2 * c] = s1;
  sums[2 * c + 1] = s2;
  if (dg) dg[c] += s2;
  if (db) db[c] += s1;
}

template <typename T>
__global__ void __launch_bounds__(256) bn_bwd_dx_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                        const float* __restrict__ mean, const float* __restrict__ rstd,
                                                        const T* __restrict__ g, const T* __restrict__ b,
                                                        const float* __restrict__ sums, T* __restrict__ dx,
                                                        int64_t total, int C, int HW, float inv_m, int relu) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int c = (int)((i / HW) % C);
    const float rs = rstd[c], gc = Cvt<T>::to_f(g[c]);
    const float xh = (Cvt<T>::to_f(x[i]) - mean[c]) * rs;
    float d = Cvt<T>::to_f(dy[i]);
    if (relu && xh * gc + Cvt<T>::to_f(b[c]) <= 0.f) d = 0.f;
    dx[i] = Cvt<T>::from_f(gc * rs * (d - sums[2 * c] * inv_m - xh * sums[2 * c + 1] * inv_m));
  }
}

// per-channel sum of dy over (n, h, w) — the bias gradient of a convolution — with the ReLU mask
// of the forward output applied on the way (dz = dy * (y > 0) written when requested)
template <typename T>
__global__ void __launch_bounds__(256) chan_sum_kernel(const T* __restrict__ dy, const T* __restrict__ y,
                                                       T* __restrict__ dz, float* __restrict__ part, int N, int C,
                                                       int HW, int S) {
  __shared__ float sh[1][4];
  const int c = blockIdx.x, s = blockIdx.y;
  const int64_t M = (int64_t)N * HW;
  const int64_t j0 = M * s / S, j1 = M * (s + 1) / S;
  float acc = 0.f;
  for (int64_t j = j0 + threadIdx.x; j < j1; j += 256) {
    const int64_t img = j / HW, hw = j - img * HW;
    const int64_t i = (img * C + c) * HW + hw;
    float d = Cvt<T>::to_f(dy[i]);
    if (y && !(Cvt<T>::to_f(y[i]) > 0.f)) d = 0.f;
    if (dz) dz[i] = Cvt<T>::from_f(d);
    acc += d;
  }
  float v[1] = {acc};
  block_fold<1>(v, sh, [](float* a, const float* b) { a[0] += b[0]; });
  if (threadIdx.x == 0) part[(int64_t)c * S + s] = v[0];
}

__global__ void chan_sum_finalize_kernel(const float* __restrict__ part, int C, int S, float* __restrict__ db) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s1 = 0.f;
  for (int s = 0; s < S; ++s) s1 += part[(int64_t)c * S + s];
  db[c] += s1;
}

static int bn_splits(int C, int64_t M) {
  int64_t s = (1024 + C - 1) / C;
  s = std::min<int64_t>(s, std::max<int64_t>(1, M / 2048));
  return (int)std::max<int64_t>(1, std::min<int64_t>(s, 1024));
}
int bn_partial_floats(int N, int C, int HW) { return C * bn_splits(C, (int64_t)N * HW) * 3 + 2 * C; }

#define DT_DISPATCH(dt, ...)                                        \
  do {                                                              \
    if (dt == DT_BF16) { using T = bf16_t; __VA_ARGS__; }           \
    else { using T = float; __VA_ARGS__; }                          \
  } while (0)

void batchnorm_fwd(int dt, const void* x, void* y, const void* g, const void* b, float* mean, float* rstd,
                   float* run_mean, float* run_var, float* ws, int N, int C, int HW, float eps, float momentum,
                   int training, int relu, hipStream_t st) {
  const int64_t total = (int64_t)N * C * HW;
  if (total == 0) return;
  if (training) {
    const int S = bn_splits(C, (int64_t)N * HW);
    DT_DISPATCH(dt, hipLaunchKernelGGL(bn_stats_kernel<T>, dim3(C, S), dim3(256), 0, st, (const T*)x, ws, N, C, HW, S));
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, st, ws, C, S, eps, momentum, mean, rstd,
                       run_mean, run_var);
  } else {
    hipLaunchKernelGGL(bn_running_kernel, dim3((C + 255) / 256), dim3(256), 0, st, run_mean, run_var, C, eps, mean,
                       rstd);
  }
  DT_DISPATCH(dt, hipLaunchKernelGGL(bn_apply_kernel<T>, dim3(ew_grid(total, 256)), dim3(256), 0, st, (const T*)x,
                                     (T*)y, mean, rstd, (const T*)g, (const T*)b, total, C, HW, relu));
}

void batchnorm_bwd(int dt, const void* x, const void* dy, const void* g, const void* b, const float* mean,
                   const float* rstd, void* dx, float* dg, float* db, float* ws, int N, int C, int HW, int relu,
                   hipStream_t st) {
  const int64_t total = (int64_t)N * C * HW;
  if (total == 0) return;
  const int S = bn_splits(C, (int64_t)N * HW);
  float* sums = ws + (int64_t)C * S * 3;  // after the (3-float) partial area sized by bn_partial_floats
  DT_DISPATCH(dt, hipLaunchKernelGGL(bn_bwd_reduce_kernel<T>, dim3(C, S), dim3(256), 0, st, (const T*)x, (const T*)dy,
                                     mean, rstd, (const T*)g, (const T*)b, ws, N, C, HW, S, relu));
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, st, ws, C, S, sums, dg, db);
  DT_DISPATCH(dt, hipLaunchKernelGGL(bn_bwd_dx_kernel<T>, dim3(ew_grid(total, 256)), dim3(256), 0, st, (const T*)x,
                                     (const T*)dy, mean, rstd, (const T*)g, (const T*)b, sums, (T*)dx, total, C, HW,
                                     1.f / (float)((int64_t)N * HW), relu));
}

void channel_sum(int dt, const void* dy, const void* y, void* dz, float* db, float* ws, int N, int C, int HW,
                 hipStream_t st) {
  if ((int64_t)N * C * HW == 0) return;
  const int S = bn_splits(C, (int64_t)N * HW);
  DT_DISPATCH(dt, hipLaunchKernelGGL(chan_sum_kernel<T>, dim3(C, S), dim3(256), 0, st, (const T*)dy, (const T*)y,
                                     (T*)dz, ws, N, C, HW, S));
  if (db) hipLaunchKernelGGL(chan_sum_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, st, ws, C, S, db);
}

// ------------------------------------------------------------------------------- pooling
// pads: ph / pw on the top / left, ph1 / pw1 on the bottom / right (asymmetric for a spatially
// split block: only the global edges are padded)
struct PoolGeom {
  int N, C, H, W, OH, OW, kh, kw, sh, sw, ph, ph1, pw, pw1;
};

__device__ __forceinline__ float pool_divisor(const PoolGeom& p, int oh, int ow, int include_pad) {
  int h0 = oh * p.sh - p.ph, w0 = ow * p.sw - p.pw;
  int h1 = min(h0 + p.kh, p.H + p.ph1), w1 = min(w0 + p.kw, p.W + p.pw1);
  const int full = (h1 - h0) * (w1 - w0);
  h0 = max(h0, 0); w0 = max(w0, 0);
  h1 = min(h1, p.H); w1 = min(w1, p.W);
  return (float)(include_pad ? full : (h1 - h0) * (w1 - w0));
}

template <typename T>
__global__ void __launch_bounds__(256) pool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                       uint8_t* __restrict__ idx, PoolGeom p, int is_max,
                                                       int include_pad, int relu) {
  const int64_t total = (int64_t)p.N * p.C * p.OH * p.OW;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += stride) {
    const int ow = (int)(o % p.OW), oh = (int)((o / p.OW) % p.OH);
    const int64_t nc = o / ((int64_t)p.OW * p.OH);
    const T* xp = x + nc * p.H * p.W;
    const int h0 = oh * p.sh - p.ph, w0 = ow * p.sw - p.pw;
    float r;
    if (is_max) {
      float best = -INFINITY;
      int bi = 0;
      for (int i = 0; i < p.kh; ++i) {
        const int ih = h0 + i;
        if (ih < 0 || ih >= p.H) continue;
        for (int j = 0; j < p.kw; ++j) {
          const int iw = w0 + j;
          if (iw < 0 || iw >= p.W) continue;
          const float v = Cvt<T>::to_f(xp[ih * p.W + iw]);
          if (v > best || v != v) { best = v; bi = i * p.kw + j; }
        }
      }
      r = best;
      if (idx) idx[o] = (uint8_t)bi;
    } else {
      float s = 0.f;
      for (int i = 0; i < p.kh; ++i) {
        const int ih = h0 + i;
        if (ih < 0 || ih >= p.H) continue;
        for (int j = 0; j < p.kw; ++j) {
          const int iw = w0 + j;
          if (iw >= 0 && iw < p.W) s += Cvt<T>::to_f(xp[ih * p.W + iw]);
        }
      }
      r = s / pool_divisor(p, oh, ow, include_pad);
    }
    if (relu) r = fmaxf(r, 0.f);
    y[o] = Cvt<T>::from_f(r);
  }
}

// one thread per input element: sum dy over the outputs whose window covers it (max: whose
// recorded winner it is); relu after the pool masks by the output (avg) or the winner itself (max)
template <typename T>
__global__ void __launch_bounds__(256) pool_bwd_kernel(const T* __restrict__ x, const T* __restrict__ y,
                                                       const T* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                       T* __restrict__ dx, PoolGeom p, int is_max, int include_pad,
                                                       int relu) {
  const int64_t total = (int64_t)p.N * p.C * p.H * p.W;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int iw = (int)(i % p.W), ih = (int)((i / p.W) % p.H);
    const int64_t nc = i / ((int64_t)p.W * p.H);
    const int64_t ob = nc * p.OH * p.OW;
    // outputs oh with oh*sh - ph <= ih < oh*sh - ph + kh
    const int oh0 = ih + p.ph - p.kh < 0 ? 0 : (ih + p.ph - p.kh) / p.sh + 1;
    const int oh1 = min((ih + p.ph) / p.sh, p.OH - 1);
    const int ow0 = iw + p.pw - p.kw < 0 ? 0 : (iw + p.pw - p.kw) / p.sw + 1;
    const int ow1 = min((iw + p.pw) / p.sw, p.OW - 1);
    float g = 0.f;
    if (is_max && relu && !(Cvt<T>::to_f(x[i]) > 0.f)) {
      g = 0.f;  // a window this element won has output relu(x) = 0
    } else {
      for (int oh = oh0; oh <= oh1; ++oh) {
        for (int ow = ow0; ow <= ow1; ++ow) {
          const int64_t o = ob + (int64_t)oh * p.OW + ow;
          if (is_max) {
            const int win = (ih - (oh * p.sh - p.ph)) * p.kw + (iw - (ow * p.sw - p.pw));
            if (idx[o] == win) g += Cvt<T>::to_f(dy[o]);
          } else {
            if (relu && !(Cvt<T>::to_f(y[o]) > 0.f)) continue;
            g += Cvt<T>::to_f(dy[o]) / pool_divisor(p, oh, ow, include_pad);
          }
        }
      }
    }
    dx[i] = Cvt<T>::from_f(g);
  }
}

void pool2d_fwd(int dt, const void* x, void* y, uint8_t* idx, const int* geom, int is_max, int include_pad, int relu,
                hipStream_t st) {
  const PoolGeom p{geom[0], geom[1], geom[2], geom[3], geom[4],  geom[5],  geom[6],
                   geom[7], geom[8], geom[9], geom[10], geom[11], geom[12], geom[13]};
  const int N = p.N, C = p.C, OH = p.OH, OW = p.OW;
  const int64_t total = (int64_t)N * C * OH * OW;
  if (total == 0) return;
  DT_DISPATCH(dt, hipLaunchKernelGGL(pool_fwd_kernel<T>, dim3(ew_grid(total, 256)), dim3(256), 0, st, (const T*)x,
                                     (T*)y, idx, p, is_max, include_pad, relu));
}

void pool2d_bwd(int dt, const void* x, const void* y, const void* dy, const uint8_t* idx, void* dx, const int* geom,
                int is_max, int include_pad, int relu, hipStream_t st) {
  const PoolGeom p{geom[0], geom[1], geom[2], geom[3], geom[4],  geom[5],  geom[6],
                   geom[7], geom[8], geom[9], geom[10], geom[11], geom[12], geom[13]};
  const int N = p.N, C = p.C, H = p.H, W = p.W;
  const int64_t total = (int64_t)N * C * H * W;
  if (total == 0) return;
  DT_DISPATCH(dt, hipLaunchKernelGGL(pool_bwd_kernel<T>, dim3(ew_grid(total, 256)), dim3(256), 0, st, (const T*)x,
                                     (const T*)y, (const T*)dy, idx, (T*)dx, p, is_max, include_pad, relu));
}

}  // namespace ffk

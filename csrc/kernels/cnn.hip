// CNN support kernels (NCHW and NHWC): batch normalization and 2-D pooling, forward and backward.
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
#include <algorithm>
#include <stdexcept>

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
  int64_t j = j0 + threadIdx.x;
  int img = (int)(j / HW), hw = (int)(j - (int64_t)img * HW);
  for (; j < j1; j += 256) {
    const float v = Cvt<T>::to_f(x[((int64_t)img * C + c) * HW + hw]);
    n += 1.f;
    const float d = v - mean;
    mean += d / n;
    m2 += d * (v - mean);
    hw += 256;
    if (hw >= HW) {
      img += hw / HW;
      hw %= HW;
    }
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

// IT: uint32_t below 2^32 elements (32-bit channel index math), else int64_t
template <typename T, typename IT>
__global__ void __launch_bounds__(256) bn_apply_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                       const float* __restrict__ mean, const float* __restrict__ rstd,
                                                       const T* __restrict__ g, const T* __restrict__ b, int64_t total,
                                                       int C, int HW, int relu) {
  const IT stride = (IT)gridDim.x * blockDim.x;
  for (IT i = (IT)blockIdx.x * blockDim.x + threadIdx.x; i < (IT)total; i += stride) {
    const int c = (int)((i / (IT)HW) % (IT)C);
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
  int64_t j = j0 + threadIdx.x;
  int img = (int)(j / HW), hw = (int)(j - (int64_t)img * HW);
  for (; j < j1; j += 256) {
    const int64_t i = ((int64_t)img * C + c) * HW + hw;
    const float xh = (Cvt<T>::to_f(x[i]) - mu) * rs;
    float d = Cvt<T>::to_f(dy[i]);
    if (relu && xh * gc + bc <= 0.f) d = 0.f;
    s1 += d;
    s2 += d * xh;
    hw += 256;
    if (hw >= HW) {
      img += hw / HW;
      hw %= HW;
    }
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
    const float* p = part + ((int64_t)c * S + s) * 2;
    s1 += p[0];
    s2 += p[1];
  }
  sums[2 * c] = s1;
  sums[2 * c + 1] = s2;
  if (dg) dg[c] += s2;
  if (db) db[c] += s1;
}

template <typename T, typename IT>
__global__ void __launch_bounds__(256) bn_bwd_dx_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                        const float* __restrict__ mean, const float* __restrict__ rstd,
                                                        const T* __restrict__ g, const T* __restrict__ b,
                                                        const float* __restrict__ sums, T* __restrict__ dx,
                                                        int64_t total, int C, int HW, float inv_m, int relu) {
  const IT stride = (IT)gridDim.x * blockDim.x;
  for (IT i = (IT)blockIdx.x * blockDim.x + threadIdx.x; i < (IT)total; i += stride) {
    const int c = (int)((i / (IT)HW) % (IT)C);
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
  // (image, pixel) of this thread's first element by one division, then advanced incrementally
  // (a 64-bit division per element was most of this kernel's time). U elements per lane are
  // loaded before any is used: the planes have odd H x W in most CNNs (Inception: 35 x 35,
  // 17 x 17), so 16-B vectors do not apply, and one 2-B load in flight per lane left the kernel
  // at ~1.4 TB/s.
  constexpr int U = 4;
  int64_t j = j0 + threadIdx.x;
  int img = (int)(j / HW), hw = (int)(j - (int64_t)img * HW);
  auto advance = [&]() {
    hw += 256;
    if (hw >= HW) {
      img += hw / HW;
      hw %= HW;
    }
  };
  for (; j + (U - 1) * 256 < j1; j += U * 256) {
    int64_t ii[U];
    float d[U], yv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      ii[u] = ((int64_t)img * C + c) * HW + hw;
      advance();
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      d[u] = Cvt<T>::to_f(dy[ii[u]]);
      yv[u] = y ? Cvt<T>::to_f(y[ii[u]]) : 1.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!(yv[u] > 0.f)) d[u] = 0.f;
      if (dz) dz[ii[u]] = Cvt<T>::from_f(d[u]);
      acc += d[u];
    }
  }
  for (; j < j1; j += 256) {
    const int64_t i = ((int64_t)img * C + c) * HW + hw;
    float d = Cvt<T>::to_f(dy[i]);
    if (y && !(Cvt<T>::to_f(y[i]) > 0.f)) d = 0.f;
    if (dz) dz[i] = Cvt<T>::from_f(d);
    acc += d;
    advance();
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

// ------------------------------------------------------------------------------- NHWC (bf16)
// Channel-last activations ([M = N*H*W rows][C], C % 8 == 0): a per-channel statistic is a column
// reduction. A workgroup owns up to 256 channels — L = min(32, C/8) lanes of 8 channels (one 16-B
// load) per row — and R = 256 / L rows at a time, U rows in flight per thread; the R row partials
// merge through LDS and each (split, channel) partial lands at part[s][c][NV], coalesced for the
// finalize pass. Elementwise passes read 8 channels per thread.
struct ColGeom {
  int64_t M;
  int C, C8, L, R, S;
};
enum { CR_STATS = 0, CR_BWD = 1, CR_SUM = 2 };

__device__ __forceinline__ void ld8(const bf16_t* p, float* v) {
  const uint4 raw = *reinterpret_cast<const uint4*>(p);
  const bf16_t* e = reinterpret_cast<const bf16_t*>(&raw);
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = bf2f(e[k]);
}
__device__ __forceinline__ void st8(bf16_t* p, const float* v) {
  uint4 raw;
  bf16_t* e = reinterpret_cast<bf16_t*>(&raw);
#pragma unroll
  for (int k = 0; k < 8; ++k) e[k] = f2bf(v[k]);
  *reinterpret_cast<uint4*>(p) = raw;
}

// STATS: a = x -> Welford (n, mean, M2); BWD: a = x, b = dy -> (sum d, sum d * xhat) with the ReLU
// mask recomputed; SUM: a = dy, b = y (optional ReLU mask) -> sum dz, dz written when requested.
// (Adding the SUM partials straight into the bias gradient by float atomics was slower: ~600
// splits' same-address atomics serialize, and capping the splits starves the reduction.)
template <int MODE>
__global__ void __launch_bounds__(256) nhwc_colred_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b,
                                                          bf16_t* __restrict__ dz, const float* __restrict__ mean,
                                                          const float* __restrict__ rstd, const bf16_t* __restrict__ g,
                                                          const bf16_t* __restrict__ bb, float* __restrict__ part,
                                                          ColGeom q, int relu) {
  constexpr int NV = MODE == CR_STATS ? 3 : MODE == CR_BWD ? 2 : 1, U = 4;
  __shared__ float sh[256 * 8 * NV];
  const int t = threadIdx.x, l = t % q.L, r = t / q.L;
  const int c8 = blockIdx.x * 32 + l, s = blockIdx.y;
  const bool act = r < q.R && c8 < q.C8;
  const int64_t j0 = q.M * s / q.S, j1 = q.M * (s + 1) / q.S;
  float n = 0.f, v0[8], v1[8];
  float mu[8], rs[8], gc[8], bc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { v0[k] = 0.f; v1[k] = 0.f; }
  if (MODE == CR_BWD && act) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = c8 * 8 + k;
      mu[k] = mean[c]; rs[k] = rstd[c]; gc[k] = bf2f(g[c]); bc[k] = bf2f(bb[c]);
    }
  }
  if (act) {
    for (int64_t j = j0 + r; j < j1; j += (int64_t)U * q.R) {
      float xa[U][8], xb[U][8];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t row = j + (int64_t)u * q.R;
        ok[u] = row < j1;
        const int64_t o = row * q.C + c8 * 8;
        if (ok[u]) {
          ld8(a + o, xa[u]);
          if (MODE == CR_BWD || (MODE == CR_SUM && b)) ld8(b + o, xb[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (!ok[u]) continue;
        if (MODE == CR_STATS) {
          n += 1.f;
          const float inv = 1.f / n;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float d = xa[u][k] - v0[k];
            v0[k] += d * inv;
            v1[k] += d * (xa[u][k] - v0[k]);
          }
        } else if (MODE == CR_BWD) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float xh = (xa[u][k] - mu[k]) * rs[k];
            float d = xb[u][k];
            if (relu && xh * gc[k] + bc[k] <= 0.f) d = 0.f;
            v0[k] += d;
            v1[k] += d * xh;
          }
        } else {
          float d[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            d[k] = (b && !(xb[u][k] > 0.f)) ? 0.f : xa[u][k];
            v0[k] += d[k];
          }
          if (dz) st8(dz + (j + (int64_t)u * q.R) * q.C + c8 * 8, d);
        }
      }
    }
  }
  float* my = sh + (size_t)t * 8 * NV;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (MODE == CR_STATS) {
      my[k * 3] = n;
      my[k * 3 + 1] = v0[k];
      my[k * 3 + 2] = v1[k];
    } else if (MODE == CR_BWD) {
      my[k * 2] = v0[k];
      my[k * 2 + 1] = v1[k];
    } else {
      my[k] = v0[k];
    }
  }
  __syncthreads();
  // thread t < 8 L folds channel t of this block over the R row partials
  if (t < 8 * q.L) {
    const int lc = t >> 3, k = t & 7;
    const int c = (blockIdx.x * 32 + lc) * 8 + k;
    if (c < q.C) {
      float f[3] = {0.f, 0.f, 0.f};
      for (int rr = 0; rr < q.R; ++rr) {
        const float* p = sh + ((size_t)(rr * q.L + lc) * 8 + k) * NV;
        if (MODE == CR_STATS) wf_merge(f[0], f[1], f[2], p[0], p[1], p[2]);
        else {
          f[0] += p[0];
          if (NV == 2) f[1] += p[1];
        }
      }
      float* o = part + ((int64_t)s * q.C + c) * NV;
#pragma unroll
      for (int v = 0; v < NV; ++v) o[v] = f[v];
    }
  }
}

// finalize of the NHWC partials part[S][C][NV]: a workgroup owns 8 channels, its 32
// thread groups fold strided subsets of the S splits (independent loads, 4 in flight: the partials
// sit in other XCDs' L2 or in HBM, so the fold is latency-bound) and merge through LDS
template <int MODE>
__global__ void __launch_bounds__(256) nhwc_finalize_kernel(const float* __restrict__ part, int C, int S, float eps,
                                                            float momentum, float* __restrict__ out0,
                                                            float* __restrict__ out1, float* __restrict__ run_mean,
                                                            float* __restrict__ run_var, float* __restrict__ dg,
                                                            float* __restrict__ db) {
  constexpr int NV = MODE == CR_STATS ? 3 : MODE == CR_BWD ? 2 : 1, CPB = 8, NG = 256 / CPB;
  __shared__ float sh[NG][CPB][NV];
  const int cl = threadIdx.x % CPB, sg = threadIdx.x / CPB;
  const int c = blockIdx.x * CPB + cl;
  float f[3] = {0.f, 0.f, 0.f};
  auto merge = [&](const float* v) {
    if (MODE == CR_STATS) wf_merge(f[0], f[1], f[2], v[0], v[1], v[2]);
    else
#pragma unroll
      for (int k = 0; k < NV; ++k) f[k] += v[k];
  };
  if (c < C) {
    int s = sg;
    for (; s + 3 * NG < S; s += 4 * NG) {
      float v[4][NV];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int k = 0; k < NV; ++k) v[u][k] = part[((int64_t)(s + NG * u) * C + c) * NV + k];
#pragma unroll
      for (int u = 0; u < 4; ++u) merge(v[u]);
    }
    for (; s < S; s += NG) merge(part + ((int64_t)s * C + c) * NV);
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) sh[sg][cl][k] = f[k];
  __syncthreads();
  if (sg != 0 || c >= C) return;
  for (int gi = 1; gi < NG; ++gi) merge(sh[gi][cl]);
  if (MODE == CR_STATS) {
    const float n = f[0], mean = f[1], m2 = f[2];
    const float var = n > 0.f ? m2 / n : 0.f;
    out0[c] = mean;
    out1[c] = rsqrtf(var + eps);
    if (run_mean) run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean;
    if (run_var) run_var[c] = (1.f - momentum) * run_var[c] + momentum * (n > 1.f ? m2 / (n - 1.f) : var);
  } else if (MODE == CR_BWD) {
    out0[2 * c] = f[0];
    out0[2 * c + 1] = f[1];
    if (dg) dg[c] += f[1];
    if (db) db[c] += f[0];
  } else {
    db[c] += f[0];
  }
}

__global__ void __launch_bounds__(256) bn_apply_nhwc_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd,
                                                            const bf16_t* __restrict__ g, const bf16_t* __restrict__ b,
                                                            uint32_t n8, int C8, int relu) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += gridDim.x * blockDim.x) {
    const int c0 = (int)(i % (uint32_t)C8) * 8;
    float v[8];
    ld8(x + (size_t)i * 8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = c0 + k;
      v[k] = (v[k] - mean[c]) * rstd[c] * bf2f(g[c]) + bf2f(b[c]);
      if (relu) v[k] = fmaxf(v[k], 0.f);
    }
    st8(y + (size_t)i * 8, v);
  }
}

__global__ void __launch_bounds__(256) bn_bwd_dx_nhwc_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ rstd,
                                                             const bf16_t* __restrict__ g,
                                                             const bf16_t* __restrict__ b,
                                                             const float* __restrict__ sums, bf16_t* __restrict__ dx,
                                                             uint32_t n8, int C8, float inv_m, int relu) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += gridDim.x * blockDim.x) {
    const int c0 = (int)(i % (uint32_t)C8) * 8;
    float xv[8], d[8];
    ld8(x + (size_t)i * 8, xv);
    ld8(dy + (size_t)i * 8, d);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = c0 + k;
      const float rs = rstd[c], gc = bf2f(g[c]);
      const float xh = (xv[k] - mean[c]) * rs;
      if (relu && xh * gc + bf2f(b[c]) <= 0.f) d[k] = 0.f;
      d[k] = gc * rs * (d[k] - sums[2 * c] * inv_m - xh * sums[2 * c + 1] * inv_m);
    }
    st8(dx + (size_t)i * 8, d);
  }
}

// splits of the NHWC column reduction: ~FF_BN_WG (default 1024) workgroups over (channel blocks x
// splits), each split at least one full trip of U x R rows. Fewer splits make each workgroup's
// share longer and the finalize's fold shorter.
static int bn_wg_target() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("FF_BN_WG");
    v = e ? std::max(1, atoi(e)) : 1024;
  }
  return v;
}
static ColGeom nhwc_geom(int64_t M, int C, int max_splits = 1024) {
  ColGeom q;
  q.M = M;
  q.C = C;
  q.C8 = C / 8;
  q.L = std::min(32, q.C8);
  q.R = 256 / q.L;
  const int ncb = (q.C8 + 31) / 32;
  const int64_t trips = (M + 4LL * q.R - 1) / (4LL * q.R);
  const int64_t wg = bn_wg_target();
  q.S = (int)std::max<int64_t>(1, std::min<int64_t>({(wg + ncb - 1) / ncb, trips, (int64_t)max_splits}));
  return q;
}

static int bn_splits(int C, int64_t M) {
  int64_t s = (1024 + C - 1) / C;
  s = std::min<int64_t>(s, std::max<int64_t>(1, M / 2048));
  return (int)std::max<int64_t>(1, std::min<int64_t>(s, 1024));
}
int bn_partial_floats(int N, int C, int HW) {
  const int64_t M = (int64_t)N * HW;
  int s = bn_splits(C, M);
  if (C % 8 == 0 && C > 0) s = std::max(s, nhwc_geom(M, C).S);
  return C * s * 3 + 2 * C;
}

#define DT_DISPATCH(dt, ...)                                        \
  do {                                                              \
    if (dt == DT_BF16) { using T = bf16_t; __VA_ARGS__; }           \
    else { using T = float; __VA_ARGS__; }                          \
  } while (0)

void batchnorm_fwd(int dt, const void* x, void* y, const void* g, const void* b, float* mean, float* rstd,
                   float* run_mean, float* run_var, float* ws, int N, int C, int HW, float eps, float momentum,
                   int training, int relu, int nhwc, hipStream_t st) {
  const int64_t total = (int64_t)N * C * HW;
  if (total == 0) return;
  if (nhwc) {  // bf16, C % 8 == 0 (checked by the binding)
    const ColGeom q = nhwc_geom((int64_t)N * HW, C);
    if (training) {
      hipLaunchKernelGGL(nhwc_colred_kernel<CR_STATS>, dim3((q.C8 + 31) / 32, q.S), dim3(256), 0, st, (const bf16_t*)x,
                         nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, ws, q, 0);
      hipLaunchKernelGGL(nhwc_finalize_kernel<CR_STATS>, dim3((C + 7) / 8), dim3(256), 0, st, ws, C, q.S, eps,
                         momentum, mean, rstd, run_mean, run_var, nullptr, nullptr);
    } else {
      hipLaunchKernelGGL(bn_running_kernel, dim3((C + 255) / 256), dim3(256), 0, st, run_mean, run_var, C, eps, mean,
                         rstd);
    }
    const uint32_t n8 = (uint32_t)(total / 8);
    hipLaunchKernelGGL(bn_apply_nhwc_kernel, dim3(ew_grid(n8, 256)), dim3(256), 0, st, (const bf16_t*)x, (bf16_t*)y,
                       mean, rstd, (const bf16_t*)g, (const bf16_t*)b, n8, C / 8, relu);
    return;
  }
  if (training) {
    const int S = bn_splits(C, (int64_t)N * HW);
    DT_DISPATCH(dt, hipLaunchKernelGGL(bn_stats_kernel<T>, dim3(C, S), dim3(256), 0, st, (const T*)x, ws, N, C, HW, S));
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, st, ws, C, S, eps, momentum, mean,
                       rstd,
                       run_mean, run_var);
  } else {
    hipLaunchKernelGGL(bn_running_kernel, dim3((C + 255) / 256), dim3(256), 0, st, run_mean, run_var, C, eps, mean,
                       rstd);
  }
  if (total < (1ll << 31))
    DT_DISPATCH(dt, hipLaunchKernelGGL((bn_apply_kernel<T, uint32_t>), dim3(ew_grid(total, 256)), dim3(256), 0, st,
                                       (const T*)x, (T*)y, mean, rstd, (const T*)g, (const T*)b, total, C, HW, relu));
  else
    DT_DISPATCH(dt, hipLaunchKernelGGL((bn_apply_kernel<T, int64_t>), dim3(ew_grid(total, 256)), dim3(256), 0, st,
                                       (const T*)x, (T*)y, mean, rstd, (const T*)g, (const T*)b, total, C, HW, relu));
}

void batchnorm_bwd(int dt, const void* x, const void* dy, const void* g, const void* b, const float* mean,
                   const float* rstd, void* dx, float* dg, float* db, float* ws, int N, int C, int HW, int relu,
                   int nhwc, hipStream_t st) {
  const int64_t total = (int64_t)N * C * HW;
  if (total == 0) return;
  if (nhwc) {
    const ColGeom q = nhwc_geom((int64_t)N * HW, C);
    float* sums = ws + (int64_t)C * q.S * 3;
    hipLaunchKernelGGL(nhwc_colred_kernel<CR_BWD>, dim3((q.C8 + 31) / 32, q.S), dim3(256), 0, st, (const bf16_t*)x,
                       (const bf16_t*)dy, nullptr, mean, rstd, (const bf16_t*)g, (const bf16_t*)b, ws, q, relu);
    hipLaunchKernelGGL(nhwc_finalize_kernel<CR_BWD>, dim3((C + 7) / 8), dim3(256), 0, st, ws, C, q.S, 0.f, 0.f, sums,
                       nullptr, nullptr, nullptr, dg, db);
    const uint32_t n8 = (uint32_t)(total / 8);
    hipLaunchKernelGGL(bn_bwd_dx_nhwc_kernel, dim3(ew_grid(n8, 256)), dim3(256), 0, st, (const bf16_t*)x,
                       (const bf16_t*)dy, mean, rstd, (const bf16_t*)g, (const bf16_t*)b, sums, (bf16_t*)dx, n8, C / 8,
                       1.f / (float)((int64_t)N * HW), relu);
    return;
  }
  const int S = bn_splits(C, (int64_t)N * HW);
  float* sums = ws + (int64_t)C * S * 3;  // after the (3-float) partial area sized by bn_partial_floats
  DT_DISPATCH(dt, hipLaunchKernelGGL(bn_bwd_reduce_kernel<T>, dim3(C, S), dim3(256), 0, st, (const T*)x, (const T*)dy,
                                     mean, rstd, (const T*)g, (const T*)b, ws, N, C, HW, S, relu));
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, st, ws, C, S, sums, dg, db);
  const float inv_m = 1.f / (float)((int64_t)N * HW);
  if (total < (1ll << 31))
    DT_DISPATCH(dt, hipLaunchKernelGGL((bn_bwd_dx_kernel<T, uint32_t>), dim3(ew_grid(total, 256)), dim3(256), 0, st,
                                       (const T*)x, (const T*)dy, mean, rstd, (const T*)g, (const T*)b, sums, (T*)dx,
                                       total, C, HW, inv_m, relu));
  else
    DT_DISPATCH(dt, hipLaunchKernelGGL((bn_bwd_dx_kernel<T, int64_t>), dim3(ew_grid(total, 256)), dim3(256), 0, st,
                                       (const T*)x, (const T*)dy, mean, rstd, (const T*)g, (const T*)b, sums, (T*)dx,
                                       total, C, HW, inv_m, relu));
}

void channel_sum(int dt, const void* dy, const void* y, void* dz, float* db, float* ws, int N, int C, int HW,
                 int nhwc, hipStream_t st) {
  if ((int64_t)N * C * HW == 0) return;
  if (nhwc) {
    const ColGeom q = nhwc_geom((int64_t)N * HW, C);
    hipLaunchKernelGGL(nhwc_colred_kernel<CR_SUM>, dim3((q.C8 + 31) / 32, q.S), dim3(256), 0, st, (const bf16_t*)dy,
                       (const bf16_t*)y, (bf16_t*)dz, nullptr, nullptr, nullptr, nullptr, ws, q, 0);
    // the [S][C] partials' fold into the bias gradient: queued with the other parameter-gradient
    // folds while the backward records them (fold_queue, elementwise.hip), else the finalize pass
    if (db && !fold_queue(ws, db, q.S, C, st))
      hipLaunchKernelGGL(nhwc_finalize_kernel<CR_SUM>, dim3((C + 7) / 8), dim3(256), 0, st, ws, C, q.S, 0.f, 0.f, nullptr,
                         nullptr, nullptr, nullptr, nullptr, db);
    return;
  }
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

// output-centric forward: one thread per output, 32-bit index math (64-bit division per element
// was the kernel's cost), the divisor once per output
template <typename T>
__global__ void __launch_bounds__(256) pool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                       uint8_t* __restrict__ idx, PoolGeom p, int is_max,
                                                       int include_pad, int relu) {
  const unsigned total = (unsigned)p.N * p.C * p.OH * p.OW;
  const unsigned ohw = (unsigned)p.OH * p.OW;
  for (unsigned o = blockIdx.x * blockDim.x + threadIdx.x; o < total; o += gridDim.x * blockDim.x) {
    const unsigned nc = o / ohw, r = o - nc * ohw;
    const int oh = (int)(r / (unsigned)p.OW), ow = (int)(r - (unsigned)oh * p.OW);
    const T* xp = x + (size_t)nc * p.H * p.W;
    const int h0 = oh * p.sh - p.ph, w0 = ow * p.sw - p.pw;
    const int i0 = max(0, -h0), i1 = min(p.kh, p.H - h0), j0 = max(0, -w0), j1 = min(p.kw, p.W - w0);
    float res;
    if (is_max) {
      float best = -INFINITY;
      int bi = 0;
      for (int i = i0; i < i1; ++i)
        for (int j = j0; j < j1; ++j) {
          const float v = Cvt<T>::to_f(xp[(h0 + i) * p.W + w0 + j]);
          if (v > best || v != v) { best = v; bi = i * p.kw + j; }
        }
      res = best;
      if (idx) idx[o] = (uint8_t)bi;
    } else {
      float sum = 0.f;
      for (int i = i0; i < i1; ++i)
        for (int j = j0; j < j1; ++j) sum += Cvt<T>::to_f(xp[(h0 + i) * p.W + w0 + j]);
      res = sum / pool_divisor(p, oh, ow, include_pad);
    }
    if (relu) res = fmaxf(res, 0.f);
    y[o] = Cvt<T>::from_f(res);
  }
}

// input-centric backward over whole planes: a workgroup stages P planes of dy (avg: pre-divided
// and ReLU-masked by y; max: dy and the winner bytes) in LDS, then every input element sums the
// outputs whose window covers it (max: whose recorded winner it is) from LDS
template <typename T, bool MAX>
__global__ void __launch_bounds__(256) pool_bwd_plane_kernel(const T* __restrict__ x, const T* __restrict__ y,
                                                             const T* __restrict__ dy,
                                                             const uint8_t* __restrict__ idx, T* __restrict__ dx,
                                                             PoolGeom p, int include_pad, int relu, int P) {
  extern __shared__ float sdy[];
  const int nplanes = p.N * p.C;
  const int pl0 = blockIdx.x * P, np = min(P, nplanes - pl0);
  const int nout = p.OH * p.OW, HW = p.H * p.W;
  uint8_t* sidx = reinterpret_cast<uint8_t*>(sdy + P * nout);
  const size_t obase = (size_t)pl0 * nout;
  for (int k = threadIdx.x; k < np * nout; k += 256) {
    float v = Cvt<T>::to_f(dy[obase + k]);
    if (MAX) {
      sidx[k] = idx[obase + k];
    } else {
      const int r = k % nout, oh = r / p.OW, ow = r - oh * p.OW;
      if (relu && !(Cvt<T>::to_f(y[obase + k]) > 0.f)) v = 0.f;
      v /= pool_divisor(p, oh, ow, include_pad);
    }
    sdy[k] = v;
  }
  __syncthreads();
  const size_t ibase = (size_t)pl0 * HW;
  for (int k = threadIdx.x; k < np * HW; k += 256) {
    const int pl = k / HW, r = k - pl * HW;
    const int ih = r / p.W, iw = r - ih * p.W;
    // outputs oh with oh*sh - ph <= ih < oh*sh - ph + kh
    const int oh0 = ih + p.ph - p.kh < 0 ? 0 : (ih + p.ph - p.kh) / p.sh + 1;
    const int oh1 = min((ih + p.ph) / p.sh, p.OH - 1);
    const int ow0 = iw + p.pw - p.kw < 0 ? 0 : (iw + p.pw - p.kw) / p.sw + 1;
    const int ow1 = min((iw + p.pw) / p.sw, p.OW - 1);
    const float* sp = sdy + pl * nout;
    float g = 0.f;
    if (MAX) {
      if (!(relu && !(Cvt<T>::to_f(x[ibase + k]) > 0.f))) {  // a window it won has output relu(x) = 0
        const uint8_t* ip = sidx + pl * nout;
        for (int oh = oh0; oh <= oh1; ++oh) {
          const int wi = (ih - (oh * p.sh - p.ph)) * p.kw + iw + p.pw;
          for (int ow = ow0; ow <= ow1; ++ow)
            if (ip[oh * p.OW + ow] == wi - ow * p.sw) g += sp[oh * p.OW + ow];
        }
      }
    } else {
      for (int oh = oh0; oh <= oh1; ++oh)
        for (int ow = ow0; ow <= ow1; ++ow) g += sp[oh * p.OW + ow];
    }
    dx[ibase + k] = Cvt<T>::from_f(g);
  }
}

// fallback for planes too large for LDS: one thread per input element, reading dy from memory
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
    const int oh0 = ih + p.ph - p.kh < 0 ? 0 : (ih + p.ph - p.kh) / p.sh + 1;
    const int oh1 = min((ih + p.ph) / p.sh, p.OH - 1);
    const int ow0 = iw + p.pw - p.kw < 0 ? 0 : (iw + p.pw - p.kw) / p.sw + 1;
    const int ow1 = min((iw + p.pw) / p.sw, p.OW - 1);
    float g = 0.f;
    if (!(is_max && relu && !(Cvt<T>::to_f(x[i]) > 0.f))) {
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


// NHWC (bf16, C % 8 == 0): one thread per (pixel, 8-channel chunk), 16-B loads of each window tap;
// consecutive lanes on consecutive chunks of one pixel, so every tap is a coalesced row read.
// The winner bytes are stored in the output's NHWC order (8 per thread, one 8-B store).
__global__ void __launch_bounds__(256) pool_fwd_nhwc_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                            uint8_t* __restrict__ idx, PoolGeom p, int is_max,
                                                            int include_pad, int relu) {
  const int C8 = p.C / 8;
  const unsigned total = (unsigned)p.N * p.OH * p.OW * C8;
  for (unsigned o = blockIdx.x * blockDim.x + threadIdx.x; o < total; o += gridDim.x * blockDim.x) {
    const unsigned pix = o / (unsigned)C8;
    const int c8 = (int)(o - pix * C8);
    const int ow = (int)(pix % (unsigned)p.OW);
    const unsigned t = pix / (unsigned)p.OW;
    const int oh = (int)(t % (unsigned)p.OH), n = (int)(t / (unsigned)p.OH);
    const int h0 = oh * p.sh - p.ph, w0 = ow * p.sw - p.pw;
    const int i0 = max(0, -h0), i1 = min(p.kh, p.H - h0), j0 = max(0, -w0), j1 = min(p.kw, p.W - w0);
    const bf16_t* xp = x + (size_t)n * p.H * p.W * p.C + c8 * 8;
    float res[8];
    if (is_max) {
      int bi[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) { res[k] = -INFINITY; bi[k] = 0; }
      for (int i = i0; i < i1; ++i)
        for (int j = j0; j < j1; ++j) {
          float v[8];
          ld8(xp + ((size_t)(h0 + i) * p.W + w0 + j) * p.C, v);
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (v[k] > res[k] || v[k] != v[k]) { res[k] = v[k]; bi[k] = i * p.kw + j; }
        }
      if (idx) {
        uint2 packed;
        packed.x = (uint32_t)bi[0] | ((uint32_t)bi[1] << 8) | ((uint32_t)bi[2] << 16) | ((uint32_t)bi[3] << 24);
        packed.y = (uint32_t)bi[4] | ((uint32_t)bi[5] << 8) | ((uint32_t)bi[6] << 16) | ((uint32_t)bi[7] << 24);
        *reinterpret_cast<uint2*>(idx + (size_t)o * 8) = packed;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) res[k] = 0.f;
      for (int i = i0; i < i1; ++i)
        for (int j = j0; j < j1; ++j) {
          float v[8];
          ld8(xp + ((size_t)(h0 + i) * p.W + w0 + j) * p.C, v);
#pragma unroll
          for (int k = 0; k < 8; ++k) res[k] += v[k];
        }
      const float inv = 1.f / pool_divisor(p, oh, ow, include_pad);
#pragma unroll
      for (int k = 0; k < 8; ++k) res[k] *= inv;
    }
    if (relu)
#pragma unroll
      for (int k = 0; k < 8; ++k) res[k] = fmaxf(res[k], 0.f);
    st8(y + (size_t)o * 8, res);
  }
}

// input-centric: every (input pixel, chunk) sums dy over the outputs whose window covers it (max:
// whose recorded winner it is), reading 16 B of dy (+ 8 winner bytes) per covering output
__global__ void __launch_bounds__(256) pool_bwd_nhwc_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ y,
                                                            const bf16_t* __restrict__ dy,
                                                            const uint8_t* __restrict__ idx, bf16_t* __restrict__ dx,
                                                            PoolGeom p, int is_max, int include_pad, int relu) {
  const int C8 = p.C / 8;
  const unsigned total = (unsigned)p.N * p.H * p.W * C8;
  for (unsigned e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const unsigned pix = e / (unsigned)C8;
    const int c8 = (int)(e - pix * C8);
    const int iw = (int)(pix % (unsigned)p.W);
    const unsigned t = pix / (unsigned)p.W;
    const int ih = (int)(t % (unsigned)p.H), n = (int)(t / (unsigned)p.H);
    const int oh0 = ih + p.ph - p.kh < 0 ? 0 : (ih + p.ph - p.kh) / p.sh + 1;
    const int oh1 = min((ih + p.ph) / p.sh, p.OH - 1);
    const int ow0 = iw + p.pw - p.kw < 0 ? 0 : (iw + p.pw - p.kw) / p.sw + 1;
    const int ow1 = min((iw + p.pw) / p.sw, p.OW - 1);
    float gsum[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) gsum[k] = 0.f;
    bool live[8];
    if (is_max && relu) {
      float xv[8];
      ld8(x + (size_t)e * 8, xv);
#pragma unroll
      for (int k = 0; k < 8; ++k) live[k] = xv[k] > 0.f;  // a window it won has output relu(x) = 0
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) live[k] = true;
    }
    for (int oh = oh0; oh <= oh1; ++oh)
      for (int ow = ow0; ow <= ow1; ++ow) {
        const size_t o8 = (((size_t)n * p.OH + oh) * p.OW + ow) * C8 + c8;
        float d[8];
        ld8(dy + o8 * 8, d);
        if (is_max) {
          const uint2 packed = *reinterpret_cast<const uint2*>(idx + o8 * 8);
          const int win = (ih - (oh * p.sh - p.ph)) * p.kw + (iw - (ow * p.sw - p.pw));
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const uint32_t word = k < 4 ? packed.x : packed.y;
            if ((int)((word >> (8 * (k & 3))) & 0xff) == win && live[k]) gsum[k] += d[k];
          }
        } else {
          const float inv = 1.f / pool_divisor(p, oh, ow, include_pad);
          float yv[8];
          if (relu) ld8(y + o8 * 8, yv);
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (!relu || yv[k] > 0.f) gsum[k] += d[k] * inv;
        }
      }
    st8(dx + (size_t)e * 8, gsum);
  }
}

// 3 x 3 / stride 1 / pad 1 average pooling, channel-last (Inception's branch pools): one thread
// per (image, column, 8-channel chunk) walks the rows with a sliding window of three row sums,
// so each input row is loaded once per thread (its 3 horizontal taps, neighbours' loads hitting
// the L1) instead of 9 taps per output from L2. Backward: the same window over dy / divisor
// (relu: dy only where the output was positive). Divisor = 9 with the pad counted, else
// (valid rows) x (valid columns).
__device__ __forceinline__ float avg3_cnt(int i, int n) { return (float)(3 - (i == 0) - (i == n - 1)); }

__global__ void __launch_bounds__(256) pool_avg3s1_fwd_nhwc_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                                   int N, int C, int H, int W, int include_pad,
                                                                   int relu) {
  const int C8 = C / 8;
  const unsigned total = (unsigned)N * W * C8;
  for (unsigned e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int c8 = (int)(e % (unsigned)C8);
    const unsigned t = e / (unsigned)C8;
    const int w = (int)(t % (unsigned)W), n = (int)(t / (unsigned)W);
    const bf16_t* xp = x + (size_t)n * H * W * C + c8 * 8;
    bf16_t* yp = y + (size_t)n * H * W * C + c8 * 8;
    auto rowsum = [&](int h, float* r) {
#pragma unroll
      for (int k = 0; k < 8; ++k) r[k] = 0.f;
#pragma unroll
      for (int dw = -1; dw <= 1; ++dw) {
        const int ww = w + dw;
        if (ww < 0 || ww >= W) continue;
        float v[8];
        ld8(xp + ((size_t)h * W + ww) * C, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] += v[k];
      }
    };
    float rm[8], r0[8], rp[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) rm[k] = 0.f;
    rowsum(0, r0);
    const float cw = include_pad ? 3.f : avg3_cnt(w, W);
    for (int h = 0; h < H; ++h) {
      if (h + 1 < H) rowsum(h + 1, rp);
      else {
#pragma unroll
        for (int k = 0; k < 8; ++k) rp[k] = 0.f;
      }
      const float inv = 1.f / ((include_pad ? 3.f : avg3_cnt(h, H)) * cw);
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        o[k] = (rm[k] + r0[k] + rp[k]) * inv;
        if (relu) o[k] = fmaxf(o[k], 0.f);
        rm[k] = r0[k];
        r0[k] = rp[k];
      }
      st8(yp + ((size_t)h * W + w) * C, o);
    }
  }
}

__global__ void __launch_bounds__(256) pool_avg3s1_bwd_nhwc_kernel(const bf16_t* __restrict__ y,
                                                                   const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx,
                                                                   int N, int C, int H, int W, int include_pad,
                                                                   int relu) {
  const int C8 = C / 8;
  const unsigned total = (unsigned)N * W * C8;
  for (unsigned e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int c8 = (int)(e % (unsigned)C8);
    const unsigned t = e / (unsigned)C8;
    const int w = (int)(t % (unsigned)W), n = (int)(t / (unsigned)W);
    const size_t base = (size_t)n * H * W * C + c8 * 8;
    // T(oh) = sum over the covering columns ow of dy(oh, ow) / div(oh, ow) (relu-masked)
    auto rowterm = [&](int oh, float* r) {
#pragma unroll
      for (int k = 0; k < 8; ++k) r[k] = 0.f;
      const float rh = include_pad ? 3.f : avg3_cnt(oh, H);
#pragma unroll
      for (int dw = -1; dw <= 1; ++dw) {
        const int ow = w + dw;
        if (ow < 0 || ow >= W) continue;
        const float inv = 1.f / (rh * (include_pad ? 3.f : avg3_cnt(ow, W)));
        float d[8];
        ld8(dy + base + ((size_t)oh * W + ow) * C, d);
        if (relu) {
          float yv[8];
          ld8(y + base + ((size_t)oh * W + ow) * C, yv);
#pragma unroll
          for (int k = 0; k < 8; ++k) r[k] += yv[k] > 0.f ? d[k] * inv : 0.f;
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) r[k] += d[k] * inv;
        }
      }
    };
    float rm[8], r0[8], rp[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) rm[k] = 0.f;
    rowterm(0, r0);
    for (int h = 0; h < H; ++h) {
      if (h + 1 < H) rowterm(h + 1, rp);
      else {
#pragma unroll
        for (int k = 0; k < 8; ++k) rp[k] = 0.f;
      }
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        o[k] = rm[k] + r0[k] + rp[k];
        rm[k] = r0[k];
        r0[k] = rp[k];
      }
      st8(dx + base + ((size_t)h * W + w) * C, o);
    }
  }
}

// FF_POOL_SLIDE=0: the generic channel-last pooling kernels for 3 x 3 / s1 / p1 average pools too
static bool pool_slide_on() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("FF_POOL_SLIDE");
    v = e ? atoi(e) : 1;
  }
  return v != 0;
}
static bool avg3s1(const PoolGeom& p, int is_max) {
  return !is_max && p.kh == 3 && p.kw == 3 && p.sh == 1 && p.sw == 1 && p.ph == 1 && p.pw == 1 && p.ph1 == 1 &&
         p.pw1 == 1 && p.OH == p.H && p.OW == p.W && p.C % 8 == 0 && pool_slide_on();
}

void pool2d_fwd(int dt, const void* x, void* y, uint8_t* idx, const int* geom, int is_max, int include_pad, int relu,
                int nhwc, hipStream_t st) {
  const PoolGeom p{geom[0], geom[1], geom[2], geom[3], geom[4],  geom[5],  geom[6],
                   geom[7], geom[8], geom[9], geom[10], geom[11], geom[12], geom[13]};
  const int64_t total = (int64_t)p.N * p.C * p.OH * p.OW;
  if (total == 0) return;
  if (total >= (1ll << 31) || (int64_t)p.N * p.C * p.H * p.W >= (1ll << 31))
    throw std::runtime_error("pool2d: tensors of 2^31 or more elements are not supported");
  if (nhwc) {
    if (avg3s1(p, is_max)) {
      const int64_t nt = (int64_t)p.N * p.W * (p.C / 8);
      hipLaunchKernelGGL(pool_avg3s1_fwd_nhwc_kernel, dim3((unsigned)std::min<int64_t>((nt + 255) / 256, 16384)),
                         dim3(256), 0, st, (const bf16_t*)x, (bf16_t*)y, p.N, p.C, p.H, p.W, include_pad, relu);
      return;
    }
    const int64_t n8 = total / 8;
    hipLaunchKernelGGL(pool_fwd_nhwc_kernel, dim3((unsigned)std::min<int64_t>((n8 + 255) / 256, 16384)), dim3(256), 0,
                       st, (const bf16_t*)x, (bf16_t*)y, idx, p, is_max, include_pad, relu);
    return;
  }
  DT_DISPATCH(dt, hipLaunchKernelGGL(pool_fwd_kernel<T>, dim3((unsigned)std::min<int64_t>((total + 255) / 256, 8192)),
                                     dim3(256), 0, st, (const T*)x, (T*)y, idx, p, is_max, include_pad, relu));
}

void pool2d_bwd(int dt, const void* x, const void* y, const void* dy, const uint8_t* idx, void* dx, const int* geom,
                int is_max, int include_pad, int relu, int nhwc, hipStream_t st) {
  const PoolGeom p{geom[0], geom[1], geom[2], geom[3], geom[4],  geom[5],  geom[6],
                   geom[7], geom[8], geom[9], geom[10], geom[11], geom[12], geom[13]};
  const int64_t total = (int64_t)p.N * p.C * p.H * p.W;
  if (total == 0) return;
  if (nhwc) {
    if (total >= (1ll << 31)) throw std::runtime_error("pool2d: tensors of 2^31 or more elements are not supported");
    if (avg3s1(p, is_max) && (!relu || y)) {
      const int64_t nt = (int64_t)p.N * p.W * (p.C / 8);
      hipLaunchKernelGGL(pool_avg3s1_bwd_nhwc_kernel, dim3((unsigned)std::min<int64_t>((nt + 255) / 256, 16384)),
                         dim3(256), 0, st, (const bf16_t*)y, (const bf16_t*)dy, (bf16_t*)dx, p.N, p.C, p.H, p.W,
                         include_pad, relu);
      return;
    }
    const int64_t n8 = total / 8;
    hipLaunchKernelGGL(pool_bwd_nhwc_kernel, dim3((unsigned)std::min<int64_t>((n8 + 255) / 256, 16384)), dim3(256), 0,
                       st, (const bf16_t*)x, (const bf16_t*)y, (const bf16_t*)dy, idx, (bf16_t*)dx, p, is_max,
                       include_pad, relu);
    return;
  }
  const int nout = p.OH * p.OW, HW = p.H * p.W, nplanes = p.N * p.C;
  constexpr int LDS_BYTES = 64 * 1024;
  if (total < (1ll << 31) && nout * 5 <= LDS_BYTES) {
    // planes per workgroup: ~2K input elements of work, within the LDS budget
    const int P = std::max(1, std::min({2048 / std::max(HW, 1), LDS_BYTES / (nout * 5), 64}));
    const unsigned grid = (unsigned)((nplanes + P - 1) / P);
    const size_t lds = (size_t)P * nout * (is_max ? 5 : 4);
    if (is_max)
      DT_DISPATCH(dt, hipLaunchKernelGGL((pool_bwd_plane_kernel<T, true>), dim3(grid), dim3(256), lds, st,
                                         (const T*)x, (const T*)y, (const T*)dy, idx, (T*)dx, p, include_pad, relu, P));
    else
      DT_DISPATCH(dt, hipLaunchKernelGGL((pool_bwd_plane_kernel<T, false>), dim3(grid), dim3(256), lds, st,
                                         (const T*)x, (const T*)y, (const T*)dy, idx, (T*)dx, p, include_pad, relu, P));
    return;
  }
  DT_DISPATCH(dt, hipLaunchKernelGGL(pool_bwd_kernel<T>, dim3(ew_grid(total, 256)), dim3(256), 0, st, (const T*)x,
                                     (const T*)y, (const T*)dy, idx, (T*)dx, p, is_max, include_pad, relu));
}

}  // namespace ffk

// LayerNorm forward (optionally fused with a residual add) and backward.
// One wave per row; the row stays in VGPRs between the statistics pass and the normalise pass
// (≤ 4096 columns at 16 B/lane), so HBM traffic is one read of x (+res) and one write of y.
// dgamma/dbeta: per-wave register partials across a grid-stride set of rows, then one fp32
// atomic per column per wave (Guideline 12).
// Replaces reference src/ops/layer_norm.cu (LayerNormForwardCUDAKernel / backward kernels).
#include "common.h"
#include "ops.h"

namespace ffk {

template <typename T, int NCH>
__global__ void __launch_bounds__(256) ln_fwd_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                     T* __restrict__ sum_out, const T* __restrict__ gamma,
                                                     const T* __restrict__ beta, T* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int rows, int cols, float eps) {
  constexpr int V = 16 / sizeof(T);
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  for (int row = wave; row < rows; row += nwaves) {
    const int64_t base = (int64_t)row * cols;
    float v[NCH][V];
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (c * 64 + lane) * V;
      if (col < cols) {
        load16(x + base + col, v[c]);
        if (res) {
          float r[V];
          load16(res + base + col, r);
#pragma unroll
          for (int j = 0; j < V; ++j) v[c][j] += r[j];
          if (sum_out) store16(sum_out + base + col, v[c]);
        }
#pragma unroll
        for (int j = 0; j < V; ++j) s += v[c][j];
      } else {
#pragma unroll
        for (int j = 0; j < V; ++j) v[c][j] = 0.f;
      }
    }
    const float mean = wave_sum(s) / cols;
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (c * 64 + lane) * V;
      if (col < cols) {
#pragma unroll
        for (int j = 0; j < V; ++j) { const float d = v[c][j] - mean; q += d * d; }
      }
    }
    const float rstd = rsqrtf(wave_sum(q) / cols + eps);
    if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (c * 64 + lane) * V;
      if (col < cols) {
        float g[V], bb[V], o[V];
        if (gamma) load16(gamma + col, g); else for (int j = 0; j < V; ++j) g[j] = 1.f;
        if (beta) load16(beta + col, bb); else for (int j = 0; j < V; ++j) bb[j] = 0.f;
#pragma unroll
        for (int j = 0; j < V; ++j) o[j] = (v[c][j] - mean) * rstd * g[j] + bb[j];
        store16(y + base + col, o);
      }
    }
  }
}

// Generic scalar path (any cols / alignment).
template <typename T>
__global__ void ln_fwd_generic(const T* __restrict__ x, const T* __restrict__ res, T* __restrict__ sum_out,
                               const T* __restrict__ gamma, const T* __restrict__ beta, T* __restrict__ y,
                               float* __restrict__ mean_out, float* __restrict__ rstd_out, int rows, int cols,
                               float eps) {
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  for (int row = wave; row < rows; row += nwaves) {
    const int64_t base = (int64_t)row * cols;
    float s = 0.f;
    for (int c = lane; c < cols; c += 64) {
      float v = Cvt<T>::to_f(x[base + c]);
      if (res) { v += Cvt<T>::to_f(res[base + c]); if (sum_out) sum_out[base + c] = Cvt<T>::from_f(v); }
      s += v;
    }
    const float mean = wave_sum(s) / cols;
    float q = 0.f;
    for (int c = lane; c < cols; c += 64) {
      float v = Cvt<T>::to_f(x[base + c]) + (res ? Cvt<T>::to_f(res[base + c]) : 0.f);
      q += (v - mean) * (v - mean);
    }
    const float rstd = rsqrtf(wave_sum(q) / cols + eps);
    if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
    for (int c = lane; c < cols; c += 64) {
      float v = Cvt<T>::to_f(x[base + c]) + (res ? Cvt<T>::to_f(res[base + c]) : 0.f);
      float g = gamma ? Cvt<T>::to_f(gamma[c]) : 1.f;
      float b = beta ? Cvt<T>::to_f(beta[c]) : 0.f;
      y[base + c] = Cvt<T>::from_f((v - mean) * rstd * g + b);
    }
  }
}

template <typename T, int NCH, int NT = 256>
__global__ void __launch_bounds__(NT) ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                     const T* __restrict__ gamma, const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in, T* __restrict__ dx,
                                                     const T* __restrict__ dres_in, float* __restrict__ pgam,
                                                     float* __restrict__ pbet, float* __restrict__ pdx, int rows,
                                                     int cols, int accumulate) {
  constexpr int V = 16 / sizeof(T);
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  float pg[NCH][V], pb[NCH][V], pd[NCH][V];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < V; ++j) { pg[c][j] = 0.f; pb[c][j] = 0.f; pd[c][j] = 0.f; }
  for (int row = wave; row < rows; row += nwaves) {
    const int64_t base = (int64_t)row * cols;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[NCH][V], gy[NCH][V];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (c * 64 + lane) * V;
      if (col < cols) {
        float xv[V], dv[V], g[V];
        load16(x + base + col, xv);
        load16(dy + base + col, dv);
        if (gamma) load16(gamma + col, g); else for (int j = 0; j < V; ++j) g[j] = 1.f;
#pragma unroll
        for (int j = 0; j < V; ++j) {
          xh[c][j] = (xv[j] - mean) * rstd;
          pg[c][j] += dv[j] * xh[c][j];
          pb[c][j] += dv[j];
          gy[c][j] = dv[j] * g[j];
          s1 += gy[c][j];
          s2 += gy[c][j] * xh[c][j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < V; ++j) { xh[c][j] = 0.f; gy[c][j] = 0.f; }
      }
    }
    s1 = wave_sum(s1) / cols;
    s2 = wave_sum(s2) / cols;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (c * 64 + lane) * V;
      if (col < cols) {
        float o[V];
#pragma unroll
        for (int j = 0; j < V; ++j) o[j] = rstd * (gy[c][j] - s1 - xh[c][j] * s2);
        if (dres_in) {
          float r[V];
          load16(dres_in + base + col, r);
#pragma unroll
          for (int j = 0; j < V; ++j) o[j] += r[j];
        }
        if (accumulate) {
          float r[V];
          load16(dx + base + col, r);
#pragma unroll
          for (int j = 0; j < V; ++j) o[j] += r[j];
        }
        // colsum of the input gradient: the bias gradient of the Linear producing this input,
        // fused here instead of a separate pass over the same [rows, cols] tensor
#pragma unroll
        for (int j = 0; j < V; ++j) pd[c][j] += o[j];
        store16(dx + base + col, o);
      }
    }
  }
  // per-wave partial column sums -> folded over the block's NT / 64 waves in LDS -> one
  // plain-stored slab row per block (reduced by col_reduce_add3); dynamic LDS = NT / 64 * cols
  // floats, reused for beta
  extern __shared__ float lds_red[];
  constexpr int NWB = NT / 64;
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int pass = 0; pass < 3; ++pass) {
    float* slab = pass == 2 ? pdx : (pass ? pbet : pgam);
    if (!slab) continue;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (c * 64 + lane) * V;
      if (col < cols)
#pragma unroll
        for (int j = 0; j < V; ++j) lds_red[w * cols + col + j] = pass == 2 ? pd[c][j] : (pass ? pb[c][j] : pg[c][j]);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < cols; k += NT) {
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < NWB; ++q) t += lds_red[q * cols + k];
      slab[(int64_t)blockIdx.x * cols + k] = t;
    }
    __syncthreads();
  }
}

template <typename T>
__global__ void ln_bwd_generic(const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ gamma,
                               const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
                               T* __restrict__ dx, const T* __restrict__ dres_in, float* __restrict__ dgamma,
                               float* __restrict__ dbeta, int rows, int cols, int accumulate) {
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  for (int row = wave; row < rows; row += nwaves) {
    const int64_t base = (int64_t)row * cols;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float s1 = 0.f, s2 = 0.f;
    for (int c = lane; c < cols; c += 64) {
      const float xh = (Cvt<T>::to_f(x[base + c]) - mean) * rstd;
      const float d = Cvt<T>::to_f(dy[base + c]);
      const float g = (gamma ? Cvt<T>::to_f(gamma[c]) : 1.f) * d;
      s1 += g; s2 += g * xh;
      if (dgamma) atomicAdd(dgamma + c, d * xh);
      if (dbeta) atomicAdd(dbeta + c, d);
    }
    s1 = wave_sum(s1) / cols;
    s2 = wave_sum(s2) / cols;
    for (int c = lane; c < cols; c += 64) {
      const float xh = (Cvt<T>::to_f(x[base + c]) - mean) * rstd;
      const float g = (gamma ? Cvt<T>::to_f(gamma[c]) : 1.f) * Cvt<T>::to_f(dy[base + c]);
      float o = rstd * (g - s1 - xh * s2);
      if (dres_in) o += Cvt<T>::to_f(dres_in[base + c]);
      if (accumulate) o += Cvt<T>::to_f(dx[base + c]);
      dx[base + c] = Cvt<T>::from_f(o);
    }
  }
}

static bool a16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// FF_LN_BWD_WIDE=1: the 1024-thread LayerNorm backward (256 partial rows). Opt-in: same-box A/B at
// BERT-Large b32 43.95 vs 43.94 ms/step (profiles/ln_bwd_wide_ab_r5.txt) — the shorter fold is
// paid back inside the kernel.
static bool ln_bwd_wide_on() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("FF_LN_BWD_WIDE");
    v = e ? atoi(e) : 0;
  }
  return v != 0;
}

void layernorm_fwd(int dt, const void* x, const void* res, void* sum_out, const void* gamma, const void* beta,
                   void* y, float* mean, float* rstd, int rows, int cols, float eps, hipStream_t st) {
  if (rows == 0) return;
  const int esz = dt == DT_BF16 ? 2 : 4;
  const int V = 16 / esz;
  const bool vec = (cols % V == 0) && a16(x) && a16(y) && (!res || a16(res)) && (!sum_out || a16(sum_out)) &&
                   (!gamma || a16(gamma)) && (!beta || a16(beta));
  const int nch = (cols + 64 * V - 1) / (64 * V);
  const int blocks = std::max(1, std::min((rows + 3) / 4, 4096));
#define LNF(T, N) hipLaunchKernelGGL((ln_fwd_kernel<T, N>), dim3(blocks), dim3(256), 0, st, (const T*)x, (const T*)res, \
                                     (T*)sum_out, (const T*)gamma, (const T*)beta, (T*)y, mean, rstd, rows, cols, eps)
  if (dt == DT_BF16) {
    using T = bf16_t;
    if (vec && nch <= 1) LNF(T, 1); else if (vec && nch <= 2) LNF(T, 2); else if (vec && nch <= 4) LNF(T, 4);
    else if (vec && nch <= 8) LNF(T, 8);
    else hipLaunchKernelGGL(ln_fwd_generic<T>, dim3(blocks), dim3(256), 0, st, (const T*)x, (const T*)res, (T*)sum_out,
                            (const T*)gamma, (const T*)beta, (T*)y, mean, rstd, rows, cols, eps);
  } else {
    using T = float;
    if (vec && nch <= 1) LNF(T, 1); else if (vec && nch <= 2) LNF(T, 2); else if (vec && nch <= 4) LNF(T, 4);
    else if (vec && nch <= 8) LNF(T, 8);
    else hipLaunchKernelGGL(ln_fwd_generic<T>, dim3(blocks), dim3(256), 0, st, (const T*)x, (const T*)res, (T*)sum_out,
                            (const T*)gamma, (const T*)beta, (T*)y, mean, rstd, rows, cols, eps);
  }
#undef LNF
}

// slab rows = blocks: 1024-thread blocks (16 waves, ~4 rows each) when the LDS fold fits (cols <=
// 1024): a quarter of the partial rows of the 256-thread form, so the fold reads 4x less and its
// serial per-column chain is 4x shorter. layernorm_bwd_waves(rows) bounds both (workspace size).
int layernorm_bwd_waves(int rows) { return std::max(1, std::min((rows + 15) / 16, 1024)); }
static bool ln_bwd_wide(int cols) { return cols <= 1024 && ln_bwd_wide_on(); }
static int ln_bwd_blocks(int rows, int cols) {
  return ln_bwd_wide(cols) ? std::max(1, std::min((rows + 63) / 64, 256)) : layernorm_bwd_waves(rows);
}

void layernorm_bwd(int dt, const void* dy, const void* x, const void* gamma, const float* mean, const float* rstd,
                   void* dx, const void* dres_in, float* dgamma, float* dbeta, float* dsum, float* ws, int rows,
                   int cols, int accumulate, hipStream_t st, int stage) {
  if (rows == 0) return;
  const int esz = dt == DT_BF16 ? 2 : 4;
  const int V = 16 / esz;
  const bool vec = (cols % V == 0) && a16(x) && a16(dy) && a16(dx) && (!dres_in || a16(dres_in)) &&
                   (!gamma || a16(gamma));
  const int nch = (cols + 64 * V - 1) / (64 * V);
  // ~4 rows per wave: enough waves in flight to cover HBM latency, slab partials stay small
  const bool wide = ln_bwd_wide(cols);
  const int blocks = ln_bwd_blocks(rows, cols);
  const int nw = blocks;
  // slab layout: [dgamma | dbeta | dsum] partials, nw rows each (absent ones skipped)
  float* pg = dgamma ? ws : nullptr;
  float* pb = dbeta ? ws + (int64_t)nw * cols : nullptr;
  float* pd = dsum ? ws + 2 * (int64_t)nw * cols : nullptr;
  bool used_slab = false;
  const bool fused_ok = vec && nch <= 4;
  if (stage == 2) {  // the slab folds only (bias_act_bwd's stage comment)
    if (fused_ok) col_reduce_add3(ws, dgamma, dbeta, dsum, nw, cols, st);
    else if (dsum) bias_act_bwd(dt, dx, nullptr, nullptr, dsum, ws + 2 * (int64_t)nw * cols, rows, cols, ACT_NONE, st, 2);
    return;
  }
#define LNB(T, N) do { used_slab = true; \
    if (wide) hipLaunchKernelGGL((ln_bwd_kernel<T, N, 1024>), dim3(blocks), dim3(1024), 16 * cols * sizeof(float), st, (const T*)dy, \
                                 (const T*)x, (const T*)gamma, mean, rstd, (T*)dx, (const T*)dres_in, pg, pb, pd, rows, cols, accumulate); \
    else hipLaunchKernelGGL((ln_bwd_kernel<T, N>), dim3(blocks), dim3(256), 4 * cols * sizeof(float), st, (const T*)dy, (const T*)x, \
                            (const T*)gamma, mean, rstd, (T*)dx, (const T*)dres_in, pg, pb, pd, rows, cols, accumulate); } while (0)
  if (dt == DT_BF16) {
    using T = bf16_t;
    if (vec && nch <= 1) LNB(T, 1); else if (vec && nch <= 2) LNB(T, 2); else if (vec && nch <= 4) LNB(T, 4);
    else hipLaunchKernelGGL(ln_bwd_generic<T>, dim3(blocks), dim3(256), 0, st, (const T*)dy, (const T*)x,
                            (const T*)gamma, mean, rstd, (T*)dx, (const T*)dres_in, dgamma, dbeta, rows, cols, accumulate);
  } else {
    using T = float;
    if (vec && nch <= 1) LNB(T, 1); else if (vec && nch <= 2) LNB(T, 2); else if (vec && nch <= 4) LNB(T, 4);
    else hipLaunchKernelGGL(ln_bwd_generic<T>, dim3(blocks), dim3(256), 0, st, (const T*)dy, (const T*)x,
                            (const T*)gamma, mean, rstd, (T*)dx, (const T*)dres_in, dgamma, dbeta, rows, cols, accumulate);
  }
#undef LNB
  if (used_slab) {
    if (stage == 0) col_reduce_add3(ws, dgamma, dbeta, dsum, nw, cols, st);
  } else if (dsum) {
    // generic path (unaligned / very wide rows): the colsum as its own pass over the written dx
    bias_act_bwd(dt, dx, nullptr, nullptr, dsum, ws + 2 * (int64_t)nw * cols, rows, cols, ACT_NONE, st, stage);
  }
  (void)fused_ok;
}

// ------------------------------------------------------------------------------- RMS norm
// y = x * rsqrt(mean(x^2) + eps) * w over the last dimension (T5 / LLaMA "LayerNorm" without
// centering). One 256-thread workgroup per row at a time, the row held in registers (MAXC
// columns per thread); the backward keeps each thread's column slice of dw in registers across
// all of its rows and adds it into the fp32 gradient with one atomic per column per workgroup.
__device__ __forceinline__ float block_sum256(float v, float* sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();  // sh is reused row after row
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  return sh[0] + sh[1] + sh[2] + sh[3];
}

template <typename T, int MAXC>
__global__ void __launch_bounds__(256) rms_fwd_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                      T* __restrict__ y, float* __restrict__ rstd, int rows, int d,
                                                      float eps) {
  __shared__ float sh[4];
  const int tid = threadIdx.x;
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const T* xr = x + (int64_t)row * d;
    float v[MAXC];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      const int c = tid + 256 * i;
      v[i] = c < d ? Cvt<T>::to_f(xr[c]) : 0.f;
      ss += v[i] * v[i];
    }
    const float r = rsqrtf(block_sum256(ss, sh) / (float)d + eps);
    if (tid == 0 && rstd) rstd[row] = r;
    T* yr = y + (int64_t)row * d;
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      const int c = tid + 256 * i;
      if (c < d) yr[c] = Cvt<T>::from_f(v[i] * r * Cvt<T>::to_f(w[c]));
    }
  }
}

template <typename T, int MAXC>
__global__ void __launch_bounds__(256) rms_bwd_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                      const T* __restrict__ dy, const float* __restrict__ rstd,
                                                      T* __restrict__ dx, float* __restrict__ dw, int rows, int d) {
  __shared__ float sh[4];
  const int tid = threadIdx.x;
  float dwp[MAXC];
#pragma unroll
  for (int i = 0; i < MAXC; ++i) dwp[i] = 0.f;
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const T* xr = x + (int64_t)row * d;
    const T* dyr = dy + (int64_t)row * d;
    const float r = rstd[row];
    float xv[MAXC], g[MAXC];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      const int c = tid + 256 * i;
      const float dv = c < d ? Cvt<T>::to_f(dyr[c]) : 0.f;
      xv[i] = c < d ? Cvt<T>::to_f(xr[c]) : 0.f;
      g[i] = c < d ? dv * Cvt<T>::to_f(w[c]) : 0.f;
      s += g[i] * xv[i];
      dwp[i] += dv * xv[i] * r;
    }
    const float k = r * r * r * block_sum256(s, sh) / (float)d;
    T* dxr = dx + (int64_t)row * d;
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      const int c = tid + 256 * i;
      if (c < d) dxr[c] = Cvt<T>::from_f(r * g[i] - k * xv[i]);
    }
  }
  if (dw) {
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      const int c = tid + 256 * i;
      if (c < d) atomicAdd(dw + c, dwp[i]);
    }
  }
}

void rmsnorm_fwd(int dt, const void* x, const void* w, void* y, float* rstd, int rows, int d, float eps,
                 hipStream_t st) {
  if (rows == 0) return;
  if (dt == DT_BF16) {
    const int g = std::max(1, std::min(rows, 1024));
    if (d <= 256 * 8) hipLaunchKernelGGL((rms_fwd_kernel<bf16_t, 8>), dim3(g), dim3(256), 0, st, (const bf16_t*)x,
                                         (const bf16_t*)w, (bf16_t*)y, rstd, rows, d, eps);
    else hipLaunchKernelGGL((rms_fwd_kernel<bf16_t, 32>), dim3(g), dim3(256), 0, st, (const bf16_t*)x,
                            (const bf16_t*)w, (bf16_t*)y, rstd, rows, d, eps);
  } else {
    const int g = std::max(1, std::min(rows, 1024));
    if (d <= 256 * 8) hipLaunchKernelGGL((rms_fwd_kernel<float, 8>), dim3(g), dim3(256), 0, st, (const float*)x,
                                         (const float*)w, (float*)y, rstd, rows, d, eps);
    else hipLaunchKernelGGL((rms_fwd_kernel<float, 32>), dim3(g), dim3(256), 0, st, (const float*)x,
                            (const float*)w, (float*)y, rstd, rows, d, eps);
  }
}

void rmsnorm_bwd(int dt, const void* x, const void* w, const void* dy, const float* rstd, void* dx, float* dw,
                 int rows, int d, hipStream_t st) {
  if (rows == 0) return;
  const int g = std::max(1, std::min(rows, 1024));
  if (dt == DT_BF16) {
    if (d <= 256 * 8) hipLaunchKernelGGL((rms_bwd_kernel<bf16_t, 8>), dim3(g), dim3(256), 0, st, (const bf16_t*)x,
                                         (const bf16_t*)w, (const bf16_t*)dy, rstd, (bf16_t*)dx, dw, rows, d);
    else hipLaunchKernelGGL((rms_bwd_kernel<bf16_t, 32>), dim3(g), dim3(256), 0, st, (const bf16_t*)x,
                            (const bf16_t*)w, (const bf16_t*)dy, rstd, (bf16_t*)dx, dw, rows, d);
  } else {
    if (d <= 256 * 8) hipLaunchKernelGGL((rms_bwd_kernel<float, 8>), dim3(g), dim3(256), 0, st, (const float*)x,
                                         (const float*)w, (const float*)dy, rstd, (float*)dx, dw, rows, d);
    else hipLaunchKernelGGL((rms_bwd_kernel<float, 32>), dim3(g), dim3(256), 0, st, (const float*)x,
                            (const float*)w, (const float*)dy, rstd, (float*)dx, dw, rows, d);
  }
}

}  // namespace ffk

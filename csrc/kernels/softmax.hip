// Row softmax fwd/bwd, fused softmax + sparse cross-entropy, CE/MSE loss gradients, metrics.
// One wave per row; pass 1 is an online max/sum (Appendix B 'Reduction': avoids the 3x re-read),
// pass 2 normalises. Replaces reference src/ops/kernels/softmax.cu,
// src/loss_functions/loss_functions.cu and src/metrics_functions/metrics_functions.cu.
#include "common.h"
#include "ops.h"

namespace ffk {

__device__ __forceinline__ void online_merge(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  if (mn == -INFINITY) { m = mn; s = 0.f; return; }
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

template <typename T>
__device__ __forceinline__ void row_stats(const T* __restrict__ xr, int cols, float scale, int lane, float& m,
                                          float& s) {
  m = -INFINITY;
  s = 0.f;
  for (int c = lane; c < cols; c += 64) {
    const float v = Cvt<T>::to_f(xr[c]) * scale;
    if (v > m) { s = s * __expf(m - v) + 1.f; m = v; }
    else s += __expf(v - m);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    online_merge(m, s, m2, s2);
  }
}

template <typename T>
__global__ void softmax_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int rows, int cols, float scale) {
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  for (int row = wave; row < rows; row += nwaves) {
    const T* xr = x + (int64_t)row * cols;
    T* yr = y + (int64_t)row * cols;
    float m, s;
    row_stats(xr, cols, scale, lane, m, s);
    const float inv = 1.f / s;
    for (int c = lane; c < cols; c += 64) yr[c] = Cvt<T>::from_f(__expf(Cvt<T>::to_f(xr[c]) * scale - m) * inv);
  }
}

template <typename T>
__global__ void softmax_bwd_kernel(const T* __restrict__ y, const T* __restrict__ dy, T* __restrict__ dx, int rows,
                                   int cols, float scale, int accumulate) {
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  for (int row = wave; row < rows; row += nwaves) {
    const int64_t base = (int64_t)row * cols;
    float d = 0.f;
    for (int c = lane; c < cols; c += 64) d += Cvt<T>::to_f(y[base + c]) * Cvt<T>::to_f(dy[base + c]);
    d = wave_sum(d);
    for (int c = lane; c < cols; c += 64) {
      float g = scale * Cvt<T>::to_f(y[base + c]) * (Cvt<T>::to_f(dy[base + c]) - d);
      if (accumulate) g += Cvt<T>::to_f(dx[base + c]);
      dx[base + c] = Cvt<T>::from_f(g);
    }
  }
}

// Visit one row with 16-B loads: a scalar head up to the first 16-B boundary (rows of an odd
// width such as BERT's 30522-entry vocabulary start at every 4-B offset), a vector body, a scalar tail.
template <typename T, typename F>
__device__ __forceinline__ void row_visit(const T* __restrict__ xr, int cols, int lane, F&& f) {
  constexpr int V = 16 / sizeof(T);
  const int head = min(cols, (int)(((16 - ((uintptr_t)xr & 15)) & 15) / sizeof(T)));
  if (lane < head) f(lane, Cvt<T>::to_f(xr[lane]));
  const int nvec = (cols - head) / V;
  const T* body = xr + head;
  int i = lane;
  // 4 x 16 B per lane in flight before the first use: one row per wave leaves each wave with a
  // single dependent load stream, which a one-load-per-iteration loop exposes to the full HBM /
  // Infinity-Cache latency
  for (; i + 192 < nvec; i += 256) {
    float v[4][V];
#pragma unroll
    for (int u = 0; u < 4; ++u) load16(body + (int64_t)(i + 64 * u) * V, v[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < V; ++j) f(head + (i + 64 * u) * V + j, v[u][j]);
  }
  for (; i < nvec; i += 64) {
    float v[V];
    load16(body + (int64_t)i * V, v);
#pragma unroll
    for (int j = 0; j < V; ++j) f(head + i * V + j, v[j]);
  }
  for (int c = head + nvec * V + lane; c < cols; c += 64) f(c, Cvt<T>::to_f(xr[c]));
}

// Fused softmax + sparse cross-entropy from the LOGITS (the [rows x classes] probabilities are
// never written): pass 1 = online max / sum-exp / argmax with 16-B loads, pass 2 = the gradient
// (p - onehot) * gscale.  Optional acc3 += {correct, sum CE, rows} folds the accuracy / CE metrics
// (reference metrics_functions.cu) into the same read of the logits.
template <typename T>
__global__ void __launch_bounds__(256) softmax_xent_kernel(const T* __restrict__ logits, const int* __restrict__ labels,
                                    float* __restrict__ loss, T* __restrict__ dlogits, int rows, int cols,
                                    float gscale, float* __restrict__ acc3) {
  constexpr int V = 16 / sizeof(T);
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  float correct = 0.f, ce = 0.f, cnt = 0.f;
  for (int row = wave; row < rows; row += nwaves) {
    const T* xr = logits + (int64_t)row * cols;
    float m = -INFINITY, s = 0.f;
    int bi = 0x7fffffff;
    row_visit(xr, cols, lane, [&](int c, float v) {
      if (v > m) { s = s * __expf(m - v) + 1.f; m = v; bi = c; }
      else s += __expf(v - m);
    });
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
      const int i2 = __shfl_xor(bi, o, 64);
      if (m2 > m || (m2 == m && i2 < bi)) bi = i2;
      online_merge(m, s, m2, s2);
    }
    const int lab = labels[row];
    const float lse = m + __logf(s);
    const bool valid = lab >= 0 && lab < cols;
    const float l = valid ? lse - Cvt<T>::to_f(xr[valid ? lab : 0]) : 0.f;
    if (lane == 0) {
      if (loss) loss[row] = l;
      correct += (bi == lab) ? 1.f : 0.f;
      ce += l;
      cnt += 1.f;
    }
    if (dlogits) {
      T* dr = dlogits + (int64_t)row * cols;
      if ((((uintptr_t)dr ^ (uintptr_t)xr) & 15) == 0) {
        const int head = min(cols, (int)(((16 - ((uintptr_t)xr & 15)) & 15) / sizeof(T)));
        if (lane < head) {
          const float p = __expf(Cvt<T>::to_f(xr[lane]) - lse);
          dr[lane] = Cvt<T>::from_f((p - (lane == lab ? 1.f : 0.f)) * gscale);
        }
        const int nvec = (cols - head) / V;
        int i = lane;
        for (; i + 192 < nvec; i += 256) {  // 4 loads in flight per lane (see row_visit)
          float v[4][V];
#pragma unroll
          for (int u = 0; u < 4; ++u) load16(xr + head + (i + 64 * u) * V, v[u]);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int c0 = head + (i + 64 * u) * V;
#pragma unroll
            for (int j = 0; j < V; ++j) v[u][j] = (__expf(v[u][j] - lse) - (c0 + j == lab ? 1.f : 0.f)) * gscale;
            store16(dr + c0, v[u]);
          }
        }
        for (; i < nvec; i += 64) {
          float v[V];
          const int c0 = head + i * V;
          load16(xr + c0, v);
#pragma unroll
          for (int j = 0; j < V; ++j) v[j] = (__expf(v[j] - lse) - (c0 + j == lab ? 1.f : 0.f)) * gscale;
          store16(dr + c0, v);
        }
        for (int c = head + nvec * V + lane; c < cols; c += 64) {
          const float p = __expf(Cvt<T>::to_f(xr[c]) - lse);
          dr[c] = Cvt<T>::from_f((p - (c == lab ? 1.f : 0.f)) * gscale);
        }
      } else {
        for (int c = lane; c < cols; c += 64) {
          const float p = __expf(Cvt<T>::to_f(xr[c]) - lse);
          dr[c] = Cvt<T>::from_f((p - (c == lab ? 1.f : 0.f)) * gscale);
        }
      }
    }
  }
  if (acc3 && lane == 0 && cnt > 0.f) {
    atomicAdd(acc3 + 0, correct);
    atomicAdd(acc3 + 1, ce);
    atomicAdd(acc3 + 2, cnt);
  }
}

// Register-resident variant for bf16 vocab-sized rows (2k..32k classes, even count): one 256-thread
// workgroup per row holds the whole row in registers (NPT packed bf16 pairs per thread), so the
// logits are read from HBM once instead of twice — the two-pass kernel above re-reads every row
// in its gradient pass, and with thousands of 61 KB rows in flight the re-read misses every cache
// (3.0 GB moved per call for 16384 x 30522 against 2.0 GB here; profiles/bert_large_hbm_bw_r1.txt).
template <int NPT>
__global__ void __launch_bounds__(256) softmax_xent_reg_kernel(const bf16_t* __restrict__ logits,
                                                               const int* __restrict__ labels,
                                                               float* __restrict__ loss, bf16_t* __restrict__ dlogits,
                                                               int rows, int cols, float gscale,
                                                               float* __restrict__ acc3) {
  __shared__ float red_m[4], red_s[4];
  __shared__ int red_i[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ndw = cols >> 1;
  float correct = 0.f, ce = 0.f, cnt = 0.f;
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const uint32_t* xr = reinterpret_cast<const uint32_t*>(logits + (int64_t)row * cols);
    uint32_t v[NPT];
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int d = tid + i * 256;
      v[i] = d < ndw ? xr[d] : 0u;
    }
    // pass 1 (registers): max with first-index argmax, then sum of exp
    float m = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int d = tid + i * 256;
      if (d < ndw) {
        const float lo = __uint_as_float(v[i] << 16), hi = __uint_as_float(v[i] & 0xffff0000u);
        if (lo > m) { m = lo; bi = 2 * d; }
        if (hi > m) { m = hi; bi = 2 * d + 1; }
      }
    }
    float sm = 0.f;
    if (m != -INFINITY) {
#pragma unroll
      for (int i = 0; i < NPT; ++i) {
        const int d = tid + i * 256;
        if (d < ndw) {
          sm += __expf(__uint_as_float(v[i] << 16) - m) + __expf(__uint_as_float(v[i] & 0xffff0000u) - m);
        }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(sm, o, 64);
      const int i2 = __shfl_xor(bi, o, 64);
      if (m2 > m || (m2 == m && i2 < bi)) bi = i2;
      online_merge(m, sm, m2, s2);
    }
    if (lane == 0) { red_m[w] = m; red_s[w] = sm; red_i[w] = bi; }
    __syncthreads();
    m = red_m[0]; sm = red_s[0]; bi = red_i[0];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      if (red_m[k] > m || (red_m[k] == m && red_i[k] < bi)) bi = red_i[k];
      online_merge(m, sm, red_m[k], red_s[k]);
    }
    __syncthreads();  // red_* is rewritten by the next row
    const int lab = labels[row];
    const float lse = m + __logf(sm);
    const bool valid = lab >= 0 && lab < cols;
    if (tid == 0) {
      const float xl = valid ? Cvt<bf16_t>::to_f(logits[(int64_t)row * cols + lab]) : 0.f;
      const float l = valid ? lse - xl : 0.f;
      if (loss) loss[row] = l;
      correct += (bi == lab) ? 1.f : 0.f;
      ce += l;
      cnt += 1.f;
    }
    if (dlogits) {  // pass 2 (registers): (softmax - onehot) * gscale, packed bf16 pairs
      uint32_t* dr = reinterpret_cast<uint32_t*>(dlogits + (int64_t)row * cols);
#pragma unroll
      for (int i = 0; i < NPT; ++i) {
        const int d = tid + i * 256;
        if (d < ndw) {
          const float p0 = (__expf(__uint_as_float(v[i] << 16) - lse) - (2 * d == lab ? 1.f : 0.f)) * gscale;
          const float p1 = (__expf(__uint_as_float(v[i] & 0xffff0000u) - lse) - (2 * d + 1 == lab ? 1.f : 0.f)) * gscale;
          dr[d] = (uint32_t)f2bf(p0) | ((uint32_t)f2bf(p1) << 16);
        }
      }
    }
  }
  if (acc3 && tid == 0 && cnt > 0.f) {
    atomicAdd(acc3 + 0, correct);
    atomicAdd(acc3 + 1, ce);
    atomicAdd(acc3 + 2, cnt);
  }
}

// Reference semantics (src/loss_functions/loss_functions.cu): the model ends in a Softmax op,
// the loss gradient w.r.t. the softmax INPUT is (p - y) * scale and Softmax::backward passes it
// through. dprobs here is that gradient.
template <typename T>
__global__ void xent_grad_kernel(const T* __restrict__ probs, const int* __restrict__ labels,
                                 const T* __restrict__ onehot, T* __restrict__ dprobs, float* __restrict__ loss,
                                 int rows, int cols, float gscale, int sparse) {
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  for (int row = wave; row < rows; row += nwaves) {
    const int64_t base = (int64_t)row * cols;
    float l = 0.f;
    const int lab = sparse ? labels[row] : -1;
    for (int c = lane; c < cols; c += 64) {
      const float p = Cvt<T>::to_f(probs[base + c]);
      const float t = sparse ? (c == lab ? 1.f : 0.f) : Cvt<T>::to_f(onehot[base + c]);
      dprobs[base + c] = Cvt<T>::from_f((p - t) * gscale);
      if (t != 0.f) l -= t * __logf(fmaxf(p, 1e-12f));
    }
    l = wave_sum(l);
    if (lane == 0 && loss) loss[row] = l;
  }
}

template <typename T>
__global__ void mse_grad_kernel(const T* __restrict__ pred, const T* __restrict__ label, T* __restrict__ dpred,
                                float* __restrict__ loss, int64_t n, float gscale) {
  __shared__ float red[4];
  float l = 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float d = Cvt<T>::to_f(pred[i]) - Cvt<T>::to_f(label[i]);
    dpred[i] = Cvt<T>::from_f(d * gscale);
    l += d * d;
  }
  l = block_sum<256>(l, red);
  if (threadIdx.x == 0 && loss) atomicAdd(loss, l);
}

// metrics: out[0] += #correct (argmax == label), out[1] += sum CE, out[2] += rows
template <typename T>
__global__ void metrics_kernel(const T* __restrict__ probs, const int* __restrict__ labels, int rows, int cols,
                               float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  float correct = 0.f, ce = 0.f, cnt = 0.f;
  for (int row = wave; row < rows; row += nwaves) {
    const int64_t base = (int64_t)row * cols;
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int c = lane; c < cols; c += 64) {
      const float v = Cvt<T>::to_f(probs[base + c]);
      if (v > best) { best = v; bi = c; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float b2 = __shfl_xor(best, o, 64);
      const int i2 = __shfl_xor(bi, o, 64);
      if (b2 > best || (b2 == best && i2 < bi)) { best = b2; bi = i2; }
    }
    if (lane == 0) {
      const int lab = labels[row];
      correct += (bi == lab) ? 1.f : 0.f;
      if (lab >= 0 && lab < cols) ce += -__logf(fmaxf(Cvt<T>::to_f(probs[base + lab]), 1e-12f));
      cnt += 1.f;
    }
  }
  if (lane == 0) {
    atomicAdd(out + 0, correct);
    atomicAdd(out + 1, ce);
    atomicAdd(out + 2, cnt);
  }
}

// Sum/mean over the middle axis of an [outer][red][inner] view.
template <typename T>
__global__ void reduce_mid_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t outer, int64_t red,
                                  int64_t inner, int mean) {
  const int64_t total = outer * inner;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int64_t o = i / inner, in = i % inner;
    const T* p = x + o * red * inner + in;
    float s = 0.f;
    for (int64_t r = 0; r < red; ++r) s += Cvt<T>::to_f(p[r * inner]);
    if (mean) s /= (float)red;
    y[i] = Cvt<T>::from_f(s);
  }
}

static int row_blocks(int rows) { return std::max(1, std::min((rows + 3) / 4, 8192)); }
// Two-pass row kernels (statistics pass, then a rewrite pass over the same row): at most 3
// workgroups (12 rows) per CU in flight so a row is still cache-resident for its second pass
// (see softmax_xent_fwd_bwd)
static int row_blocks_2pass(int rows) { return std::min(row_blocks(rows), 768); }

#define DT_DISPATCH(dt, ...)                                        \
  do {                                                              \
    if (dt == DT_BF16) { using T = bf16_t; __VA_ARGS__; }           \
    else { using T = float; __VA_ARGS__; }                          \
  } while (0)

void softmax_fwd(int dt, const void* x, void* y, int rows, int cols, float scale, hipStream_t st) {
  if (rows == 0) return;
  DT_DISPATCH(dt, hipLaunchKernelGGL(softmax_fwd_kernel<T>, dim3(row_blocks_2pass(rows)), dim3(256), 0, st, (const T*)x,
                                     (T*)y, rows, cols, scale));
}
void softmax_bwd(int dt, const void* y, const void* dy, void* dx, int rows, int cols, float scale, int accumulate,
                 hipStream_t st) {
  if (rows == 0) return;
  DT_DISPATCH(dt, hipLaunchKernelGGL(softmax_bwd_kernel<T>, dim3(row_blocks_2pass(rows)), dim3(256), 0, st, (const T*)y,
                                     (const T*)dy, (T*)dx, rows, cols, scale, accumulate));
}
void softmax_xent_fwd_bwd(int dt, const void* logits, const int* labels, float* loss, void* dlogits, int rows,
                          int cols, float gscale, float* acc3, hipStream_t st) {
  if (rows == 0) return;
  // opt-in (FF_XENT_REG=1): despite moving 1 GB less per call, the register-resident kernel measured
  // 0.6 ms/step SLOWER in a same-box A/B of the BERT-Large step (53.2 vs 52.6 ms, profiles/
  // softmax_xent_ab_r1.txt): one row per 256-thread workgroup with 4-B loads leaves too little
  // memory-level parallelism, which the two-pass kernel's 16-B x 4-deep loads have
  static const int reg_ok = getenv("FF_XENT_REG") ? atoi(getenv("FF_XENT_REG")) : 0;
  if (reg_ok && dt == DT_BF16 && cols % 2 == 0 && cols >= 4096 && cols <= 2 * 256 * 64) {
    const int g = std::min(rows, 2048);
    if (cols <= 2 * 256 * 32)
      hipLaunchKernelGGL(softmax_xent_reg_kernel<32>, dim3(g), dim3(256), 0, st, (const bf16_t*)logits, labels, loss,
                         (bf16_t*)dlogits, rows, cols, gscale, acc3);
    else
      hipLaunchKernelGGL(softmax_xent_reg_kernel<64>, dim3(g), dim3(256), 0, st, (const bf16_t*)logits, labels, loss,
                         (bf16_t*)dlogits, rows, cols, gscale, acc3);
    return;
  }
  // At most 3 workgroups (12 rows) per CU in flight: with every row of a 16384 x 30522 call in
  // flight at once (4096 workgroups) the ~500 MB between a row's two passes overflowed the 256 MB
  // Infinity Cache and the gradient pass re-read HBM; capped, the re-read hits the cache:
  // 795 -> 607 us per call (grid sweep 256..2048: 512..768 best; scripts/xent_probe.py,
  // profiles/softmax_xent_grid_r2.txt). FF_XENT_GRID overrides the cap.
  static const int grid_cap = getenv("FF_XENT_GRID") ? atoi(getenv("FF_XENT_GRID")) : 768;
  const int g = grid_cap > 0 ? std::min(row_blocks(rows), grid_cap) : row_blocks(rows);
  DT_DISPATCH(dt, hipLaunchKernelGGL(softmax_xent_kernel<T>, dim3(g), dim3(256), 0, st,
                                     (const T*)logits, labels, loss, (T*)dlogits, rows, cols, gscale, acc3));
}
void xent_grad(int dt, const void* probs, const int* labels, const void* onehot, void* dprobs, float* loss, int rows,
               int cols, float gscale, int sparse, hipStream_t st) {
  if (rows == 0) return;
  DT_DISPATCH(dt, hipLaunchKernelGGL(xent_grad_kernel<T>, dim3(row_blocks(rows)), dim3(256), 0, st,
                                     (const T*)probs, labels, (const T*)onehot, (T*)dprobs, loss, rows, cols, gscale,
                                     sparse));
}
void mse_grad(int dt, const void* pred, const void* label, void* dpred, float* loss, int64_t n, float gscale,
              hipStream_t st) {
  if (n == 0) return;
  DT_DISPATCH(dt, hipLaunchKernelGGL(mse_grad_kernel<T>, dim3(ew_grid(n, 256)), dim3(256), 0, st, (const T*)pred,
                                     (const T*)label, (T*)dpred, loss, n, gscale));
}
void metrics_classify(int dt, const void* probs, const int* labels, int rows, int cols, float* out,
                      hipStream_t st) {
  if (rows == 0) return;
  DT_DISPATCH(dt, hipLaunchKernelGGL(metrics_kernel<T>, dim3(std::min(row_blocks(rows), 1024)), dim3(256), 0, st,
                                     (const T*)probs, labels, rows, cols, out));
}
void reduce_rows(int dt, const void* x, void* y, int64_t outer, int64_t red, int64_t inner, int mean,
                 hipStream_t st) {
  const int64_t total = outer * inner;
  if (total == 0) return;
  DT_DISPATCH(dt, hipLaunchKernelGGL(reduce_mid_kernel<T>, dim3(ew_grid(total, 256)), dim3(256), 0, st, (const T*)x,
                                     (T*)y, outer, red, inner, mean));
}

}  // namespace ffk

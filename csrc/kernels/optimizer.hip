// Fused multi-tensor optimizers over flat parameter arenas.
// All trainable weights of one dtype live in ONE contiguous fp32 master buffer (plus an optional
// bf16 compute copy), gradients in ONE fp32 buffer: a single launch updates the whole model and
// writes the bf16 copy in the same pass (no separate cast kernel).
// Semantics follow reference src/runtime/optimizer_kernel.cu (sgd_update: momentum/nesterov/
// weight-decay; adam_update with bias-corrected alpha_t computed on the host, optimizer.cc:371).
#include "common.h"
#include "ops.h"

namespace ffk {

__global__ void sgd_kernel(float* __restrict__ w, const float* __restrict__ g, float* __restrict__ v,
                           bf16_t* __restrict__ wl, int64_t n, float lr, float momentum, int nesterov, float wd,
                           float gscale) {
  const int64_t nv = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    float4 wv = reinterpret_cast<float4*>(w)[i];
    float4 gv = reinterpret_cast<const float4*>(g)[i];
    float* wp = &wv.x;
    float* gp = &gv.x;
    float4 vv = make_float4(0, 0, 0, 0);
    if (momentum > 0.f) vv = reinterpret_cast<float4*>(v)[i];
    float* vp = &vv.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gt = gp[j] * gscale + wd * wp[j];
      if (momentum > 0.f) {
        vp[j] = vp[j] * momentum + gt;
        gt = nesterov ? gt + momentum * vp[j] : vp[j];
      }
      wp[j] -= lr * gt;
    }
    reinterpret_cast<float4*>(w)[i] = wv;
    if (momentum > 0.f) reinterpret_cast<float4*>(v)[i] = vv;
    if (wl) {
      ushort4 o;
      o.x = f2bf(wp[0]); o.y = f2bf(wp[1]); o.z = f2bf(wp[2]); o.w = f2bf(wp[3]);
      reinterpret_cast<ushort4*>(wl)[i] = o;
    }
  }
  for (int64_t i = nv * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float gt = g[i] * gscale + wd * w[i];
    if (momentum > 0.f) {
      v[i] = v[i] * momentum + gt;
      gt = nesterov ? gt + momentum * v[i] : v[i];
    }
    w[i] -= lr * gt;
    if (wl) wl[i] = f2bf(w[i]);
  }
}

// alpha_dev: the step size read from device memory instead of the argument (a captured hipGraph
// of the whole training step replays one launch whose alpha_t changes every step)
__global__ void adam_kernel(float* __restrict__ w, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, bf16_t* __restrict__ wl, int64_t n, float alpha_t, float b1,
                            float b2, float wd, float eps, float gscale, const float* __restrict__ alpha_dev) {
  if (alpha_dev) alpha_t = *alpha_dev;
  const int64_t nv = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    float4 wv = reinterpret_cast<float4*>(w)[i];
    float4 gv = reinterpret_cast<const float4*>(g)[i];
    float4 mv = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    float* wp = &wv.x; float* gp = &gv.x; float* mp = &mv.x; float* vp = &vv.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gt = gp[j] * gscale + wd * wp[j];
      mp[j] = b1 * mp[j] + (1.f - b1) * gt;
      vp[j] = b2 * vp[j] + (1.f - b2) * gt * gt;
      wp[j] -= alpha_t * mp[j] / (sqrtf(vp[j]) + eps);
    }
    reinterpret_cast<float4*>(w)[i] = wv;
    reinterpret_cast<float4*>(m)[i] = mv;
    reinterpret_cast<float4*>(v)[i] = vv;
    if (wl) {
      ushort4 o;
      o.x = f2bf(wp[0]); o.y = f2bf(wp[1]); o.z = f2bf(wp[2]); o.w = f2bf(wp[3]);
      reinterpret_cast<ushort4*>(wl)[i] = o;
    }
  }
  for (int64_t i = nv * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float gt = g[i] * gscale + wd * w[i];
    m[i] = b1 * m[i] + (1.f - b1) * gt;
    v[i] = b2 * v[i] + (1.f - b2) * gt * gt;
    w[i] -= alpha_t * m[i] / (sqrtf(v[i]) + eps);
    if (wl) wl[i] = f2bf(w[i]);
  }
}

// Row-sparse SGD for embedding tables (momentum 0, no weight decay: a row no id touched has a zero
// gradient, so skipping it is exact). Two passes, no sort: every occurrence i of row r stores i
// into mark[r] (one store wins), then only the occurrence that won applies w -= lr * g to the row
// (and refreshes its bf16 copy) — each touched row is updated exactly once whatever the
// duplicates, and clears the row's gradient (so zero_gradients can skip the table: only touched
// rows were ever non-zero). mark needs no clearing: pass 1 rewrites every row this step touches.
__global__ void sparse_rows_mark_kernel(const int64_t* __restrict__ idx, int n, int64_t rows, int* __restrict__ mark) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int64_t r = idx[i];
    if (r >= 0 && r < rows) mark[r] = i;
  }
}
__global__ void sparse_rows_sgd_kernel(const int64_t* __restrict__ idx, int n, int64_t rows, int dim,
                                       const int* __restrict__ mark, float* __restrict__ w,
                                       float* __restrict__ g, bf16_t* __restrict__ wl, float lr) {
  // one wave per occurrence, lanes over the row's columns
  const int i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  const int64_t r = idx[i];
  if (r < 0 || r >= rows || mark[r] != i) return;
  float* wr = w + r * dim;
  float* gr = g + r * dim;
  for (int d = lane; d < dim; d += 64) {
    const float v = wr[d] - lr * gr[d];
    wr[d] = v;
    gr[d] = 0.f;
    if (wl) wl[r * dim + d] = f2bf(v);
  }
}
void sgd_sparse_rows(const int64_t* idx, int n, int64_t rows, int dim, int* mark, float* master, float* grad,
                     void* lowp, float lr, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(sparse_rows_mark_kernel, dim3((n + 255) / 256), dim3(256), 0, st, idx, n, rows, mark);
  hipLaunchKernelGGL(sparse_rows_sgd_kernel, dim3((n + 3) / 4), dim3(256), 0, st, idx, n, rows, dim, mark, master,
                     grad, (bf16_t*)lowp, lr);
}

// max_blocks > 0 caps the grid (an update overlapped with the backward on a side stream leaves CU
// slots to the compute stream's kernels; the grid-stride loops keep enough bytes in flight).
// max_blocks < 0: short-lived workgroups instead of a grid-stride sweep — each thread updates about
// -max_blocks float4 groups and exits, so the CU slots of an overlapped update are handed back to
// the compute stream every few microseconds (a 2048-block sweep held every wave slot of every CU
// for its whole ~95 us and starved the backward's small-grid kernels, ~1.4 ms/step of BERT-Large).
static int opt_grid(int64_t n, int max_blocks) {
  if (max_blocks < 0) {
    const int64_t per = 256 * (int64_t)(-max_blocks);
    return (int)std::max<int64_t>(1, std::min<int64_t>((n / 4 + per - 1) / per, 1 << 30));
  }
  const int g = ew_grid(n / 4 + 1, 256);
  return max_blocks > 0 ? std::min(g, max_blocks) : g;
}
void sgd_update(float* master, const float* grad, float* mom, void* param_lowp, int64_t n, float lr, float momentum,
                int nesterov, float wd, float gscale, hipStream_t st, int max_blocks) {
  if (n == 0) return;
  hipLaunchKernelGGL(sgd_kernel, dim3(opt_grid(n, max_blocks)), dim3(256), 0, st, master, grad, mom,
                     (bf16_t*)param_lowp, n, lr, momentum, nesterov, wd, gscale);
}
void adam_update(float* master, const float* grad, float* m, float* v, void* param_lowp, int64_t n, float alpha_t,
                 float beta1, float beta2, float wd, float eps, float gscale, hipStream_t st, int max_blocks,
                 const float* alpha_dev) {
  if (n == 0) return;
  hipLaunchKernelGGL(adam_kernel, dim3(opt_grid(n, max_blocks)), dim3(256), 0, st, master, grad, m, v,
                     (bf16_t*)param_lowp, n, alpha_t, beta1, beta2, wd, eps, gscale, alpha_dev);
}

}  // namespace ffk

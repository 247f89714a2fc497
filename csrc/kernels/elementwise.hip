// Element-wise kernels (unary / scalar / binary with broadcast / cast / dropout / bias+act grad).
// Memory-bound: 16 B per lane vector path (Guideline 13), grid-stride, capped grid (Guideline 11).
// Replaces reference src/ops/element_unary.cu, src/ops/kernels/element_binary_kernels.cu,
// src/ops/kernels/dropout_kernels.cu, src/ops/kernels/cast_kernels.cu.
#include "common.h"
#include "ops.h"

#include <vector>

namespace ffk {

__device__ __forceinline__ float unary_f(int op, float x, float s) {
  switch (op) {
    case U_RELU: return fmaxf(x, 0.f);
    case U_SIGMOID: return 1.f / (1.f + __expf(-x));
    case U_TANH: return tanhf(x);
    case U_ELU: return x > 0.f ? x : (__expf(x) - 1.f);
    case U_GELU: return 0.5f * x * (1.f + fast_erf(x * 0.70710678118654752f));
    case U_EXP: return __expf(x);
    case U_SIN: return __sinf(x);
    case U_COS: return __cosf(x);
    case U_RSQRT: return rsqrtf(x);
    case U_POW: return powf(x, s);
    case U_IDENTITY: return x;
    case U_SCALAR_MUL: return x * s;
    case U_SCALAR_ADD: return x + s;
    case U_SCALAR_SUB: return x - s;
    case U_SCALAR_TRUEDIV: return x / s;
    case U_SCALAR_FLOORDIV: return floorf(x / s);
    case U_LOG: return __logf(x);
    case U_SQRT: return sqrtf(x);
    case U_NEG: return -x;
    case U_LEAKY_RELU: return x > 0.f ? x : x * s;
    default: return x;
  }
}
// d out / d in, given input x and output y
__device__ __forceinline__ float unary_df(int op, float x, float y, float s) {
  switch (op) {
    case U_RELU: return x > 0.f ? 1.f : 0.f;
    case U_SIGMOID: return y * (1.f - y);
    case U_TANH: return 1.f - y * y;
    case U_ELU: return x > 0.f ? 1.f : y + 1.f;
    case U_GELU: {
      float cdf = 0.5f * (1.f + fast_erf(x * 0.70710678118654752f));
      return cdf + x * 0.3989422804014327f * __expf(-0.5f * x * x);
    }
    case U_EXP: return y;
    case U_SIN: return __cosf(x);
    case U_COS: return -__sinf(x);
    case U_RSQRT: return -0.5f * y * y * y;
    case U_POW: return s * powf(x, s - 1.f);
    case U_IDENTITY: return 1.f;
    case U_SCALAR_MUL: return s;
    case U_SCALAR_ADD: return 1.f;
    case U_SCALAR_SUB: return 1.f;
    case U_SCALAR_TRUEDIV: return 1.f / s;
    case U_SCALAR_FLOORDIV: return 0.f;
    case U_LOG: return 1.f / x;
    case U_SQRT: return 0.5f / y;
    case U_NEG: return -1.f;
    case U_LEAKY_RELU: return x > 0.f ? 1.f : s;
    default: return 1.f;
  }
}

// OP >= 0: the op as a compile-time constant (ReLU, the CNN zoo's), -1: the run-time `op_rt` (a
// per-element switch over every op otherwise sits in the loop)
template <typename T, int OP = -1>
__global__ void unary_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n, int op_rt, float s) {
  const int op = OP >= 0 ? OP : op_rt;
  constexpr int V = 16 / sizeof(T);
  const int64_t nv = n / V;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    float v[V];
    load16(x + i * V, v);
#pragma unroll
    for (int j = 0; j < V; ++j) v[j] = unary_f(op, v[j], s);
    store16(y + i * V, v);
  }
  for (int64_t i = nv * V + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = Cvt<T>::from_f(unary_f(op, Cvt<T>::to_f(x[i]), s));
}

// OP = U_RELU: the gradient needs only y (y > 0 exactly where x > 0), so x is not read — a third
// less traffic than the generic form
template <typename T, int OP = -1>
__global__ void unary_bwd_kernel(const T* __restrict__ x, const T* __restrict__ y, const T* __restrict__ dy,
                                 T* __restrict__ dx, int64_t n, int op_rt, float s, int accumulate) {
  const int op = OP >= 0 ? OP : op_rt;
  constexpr int V = 16 / sizeof(T);
  const int64_t nv = n / V;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    float xv[V], yv[V], g[V], o[V];
    load16(y + i * V, yv);
    if constexpr (OP == U_RELU) {
#pragma unroll
      for (int j = 0; j < V; ++j) xv[j] = yv[j];
    } else {
      load16(x + i * V, xv);
    }
    load16(dy + i * V, g);
    if (accumulate) load16(dx + i * V, o);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      float d = g[j] * unary_df(op, xv[j], yv[j], s);
      o[j] = accumulate ? o[j] + d : d;
    }
    store16(dx + i * V, o);
  }
  for (int64_t i = nv * V + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float yi = Cvt<T>::to_f(y[i]);
    float d = Cvt<T>::to_f(dy[i]) * unary_df(op, OP == U_RELU ? yi : Cvt<T>::to_f(x[i]), yi, s);
    dx[i] = Cvt<T>::from_f(accumulate ? Cvt<T>::to_f(dx[i]) + d : d);
  }
}

__device__ __forceinline__ float binary_f(int op, float a, float b) {
  switch (op) {
    case B_ADD: return a + b;
    case B_SUB: return a - b;
    case B_MUL: return a * b;
    case B_DIV: return a / b;
    case B_MAX: return fmaxf(a, b);
    case B_MIN: return fminf(a, b);
    default: return a;
  }
}

// op | B_RELU: the consumer ReLU fused into the binary op (executor._plan_binary_relu: ResNet's
// residual add + ReLU in one pass instead of two)
constexpr int B_RELU = 0x100;
__device__ __forceinline__ float binary_act(int op, float a, float b) {
  const float r = binary_f(op & 0xff, a, b);
  return (op & B_RELU) ? fmaxf(r, 0.f) : r;
}

// Same-shape fast path.
template <typename T, int OP = -1>  // OP >= 0: compile-time op (B_ADD: residual adds), -1: run time
__global__ void binary_same_kernel(const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ c,
                                   int64_t n, int op_rt) {
  const int op = OP >= 0 ? OP : op_rt;
  constexpr int V = 16 / sizeof(T);
  const int64_t nv = n / V;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    float av[V], bv[V];
    load16(a + i * V, av);
    load16(b + i * V, bv);
#pragma unroll
    for (int j = 0; j < V; ++j) av[j] = binary_act(op, av[j], bv[j]);
    store16(c + i * V, av);
  }
  for (int64_t i = nv * V + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    c[i] = Cvt<T>::from_f(binary_act(op, Cvt<T>::to_f(a[i]), Cvt<T>::to_f(b[i])));
}

// General broadcast path: output shape `shape` (ndim <= 6), strides of a/b in elements
// (0 on broadcast dims).
struct BcastDesc {
  int ndim;
  int64_t shape[6];
  int64_t sa[6];
  int64_t sb[6];
};
template <typename T>
__global__ void binary_bcast_kernel(const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ c,
                                    int64_t n, int op, BcastDesc d) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    int64_t rem = i, oa = 0, ob = 0;
    for (int k = d.ndim - 1; k >= 0; --k) {
      const int64_t idx = rem % d.shape[k];
      rem /= d.shape[k];
      oa += idx * d.sa[k];
      ob += idx * d.sb[k];
    }
    c[i] = Cvt<T>::from_f(binary_act(op, Cvt<T>::to_f(a[oa]), Cvt<T>::to_f(b[ob])));
  }
}

// Binary backward at full output shape: da_full = dc * d(op)/da, db_full = dc * d(op)/db.
// (Reduction over broadcast dims is done by the caller.)
template <typename T>
__global__ void binary_bwd_kernel(const T* __restrict__ a, const T* __restrict__ b, const T* __restrict__ dc,
                                  T* __restrict__ da, T* __restrict__ db, int64_t n, int op, BcastDesc d,
                                  int same) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    int64_t oa = i, ob = i;
    if (!same) {
      int64_t rem = i;
      oa = 0; ob = 0;
      for (int k = d.ndim - 1; k >= 0; --k) {
        const int64_t idx = rem % d.shape[k];
        rem /= d.shape[k];
        oa += idx * d.sa[k];
        ob += idx * d.sb[k];
      }
    }
    const float g = Cvt<T>::to_f(dc[i]);
    const float av = Cvt<T>::to_f(a[oa]), bv = Cvt<T>::to_f(b[ob]);
    float ga, gb;
    switch (op) {
      case B_ADD: ga = g; gb = g; break;
      case B_SUB: ga = g; gb = -g; break;
      case B_MUL: ga = g * bv; gb = g * av; break;
      case B_DIV: ga = g / bv; gb = -g * av / (bv * bv); break;
      case B_MAX: ga = av >= bv ? g : 0.f; gb = av >= bv ? 0.f : g; break;
      case B_MIN: ga = av <= bv ? g : 0.f; gb = av <= bv ? 0.f : g; break;
      default: ga = g; gb = 0.f;
    }
    if (da) da[i] = Cvt<T>::from_f(ga);
    if (db) db[i] = Cvt<T>::from_f(gb);
  }
}

template <typename TI, typename TO>
__global__ void cast_kernel(const TI* __restrict__ x, TO* __restrict__ y, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = Cvt<TO>::from_f(Cvt<TI>::to_f(x[i]));
}

// Counter-based RNG (splitmix64 finaliser of (seed, offset, index)): deterministic per global
// element index, so every shard of a partitioned tensor draws the same mask as a 1-GPU run.
__device__ __forceinline__ float hash_uniform(uint64_t seed, uint64_t idx) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + idx + 0x632BE59BD9B4E019ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

template <typename T>
__global__ void dropout_kernel(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ mask, int64_t n,
                               float rate, uint64_t seed, uint64_t offset) {
  const float scale = 1.f / (1.f - rate);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const bool keep = hash_uniform(seed, offset + i) >= rate;
    mask[i] = keep;
    y[i] = Cvt<T>::from_f(keep ? Cvt<T>::to_f(x[i]) * scale : 0.f);
  }
}
template <typename T>
__global__ void dropout_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ mask, T* __restrict__ dx,
                                   int64_t n, float rate, int accumulate) {
  const float scale = 1.f / (1.f - rate);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float v = mask[i] ? Cvt<T>::to_f(dy[i]) * scale : 0.f;
    if (accumulate) v += Cvt<T>::to_f(dx[i]);
    dx[i] = Cvt<T>::from_f(v);
  }
}

// Fused activation-backward + bias-gradient for Linear/Conv epilogues:
//   dz[r][c] = dy[r][c] * act'(z[r][c]);   part[y][c] = sum_{r in chunk y} dz[r][c]
// A block = 4 waves x 512 columns (each lane 8 consecutive columns = one 16-B load per row, a wave
// reads 1 KiB contiguous per row); the waves interleave rows, 4 rows in flight per wave, and fold
// their sums through LDS so the fp32 slab has one row per block.  The slab is folded by
// col_reduce_add with <= 32 adders per address (the full-rate regime of MI355X_MICROARCH
// 'Global float atomics'; all blocks into one row is 14x slower, hence no direct atomics).
constexpr int BAB_COLS = 512;
// AK: the activation as a compile-time constant (GELU / ReLU, BERT's and the CNN zoo's), 0: the
// run-time `act` — a per-element switch over every activation left scalar branches around each
// element's act' in the loop (round 6: ~400 s_cbranch per 32-element group)
template <typename T, bool ACT, int AK = 0>
__global__ void __launch_bounds__(256) bias_act_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ z,
                                                           T* __restrict__ dz, float* __restrict__ part, int rows,
                                                           int cols, int act_rt, int rpb) {
  const int act = AK ? AK : act_rt;
  __shared__ float red[4][BAB_COLS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c0 = blockIdx.x * BAB_COLS + lane * 8;
  const int r0 = blockIdx.y * rpb, r1 = min(rows, r0 + rpb);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c0 < cols) {
    const bool vec = sizeof(T) == 2 && (cols & 7) == 0;
    int r = r0 + w;
    if (vec) {
      // U rows in flight per wave (U x 16 B per lane, plus z when ACT): the whole block's rows are
      // requested before the first add, which is what hides HBM latency on these short kernels
      constexpr int U = ACT ? 4 : 8;
      for (; r + 4 * (U - 1) < r1; r += 4 * U) {
        float g[U][8], zz[ACT ? U : 1][8];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          load16(dy + (int64_t)(r + 4 * u) * cols + c0, g[u]);
          if (ACT) load16(z + (int64_t)(r + 4 * u) * cols + c0, zz[ACT ? u : 0]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (ACT) {
#pragma unroll
            for (int j = 0; j < 8; ++j) g[u][j] *= act_grad(act, zz[ACT ? u : 0][j]);
            if (dz) store16(dz + (int64_t)(r + 4 * u) * cols + c0, g[u]);
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += g[u][j];
        }
      }
      for (; r < r1; r += 4) {
        float g[8], zz[8];
        load16(dy + (int64_t)r * cols + c0, g);
        if (ACT) {
          load16(z + (int64_t)r * cols + c0, zz);
#pragma unroll
          for (int j = 0; j < 8; ++j) g[j] *= act_grad(act, zz[j]);
          if (dz) store16(dz + (int64_t)r * cols + c0, g);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += g[j];
      }
    } else {
      for (; r < r1; r += 4) {
        const int64_t base = (int64_t)r * cols + c0;
        for (int j = 0; j < 8 && c0 + j < cols; ++j) {
          float g = Cvt<T>::to_f(dy[base + j]);
          if (ACT) {
            g *= act_grad(act, Cvt<T>::to_f(z[base + j]));
            if (dz) dz[base + j] = Cvt<T>::from_f(g);
          }
          acc[j] += g;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[w][lane * 8 + j] = acc[j];
  __syncthreads();
  if (part) {
    for (int k = threadIdx.x; k < BAB_COLS; k += 256) {
      const int c = blockIdx.x * BAB_COLS + k;
      if (c < cols) part[(int64_t)blockIdx.y * cols + c] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
    }
  }
}

// Column sums of a bf16 [rows, cols] matrix whose width is even but not a multiple of 8 (the MLM
// decoder's 30522-wide logit gradient: rows are only 4-byte aligned, so the 16-B path above does
// not apply and its scalar fallback ran at 1.3 TB/s). Each lane owns 2 adjacent columns (one 4-B
// load per row), a block 512 columns; 16 rows in flight per lane; one fp32 slab row per block.
__global__ void __launch_bounds__(256) colsum_pairs_kernel(const bf16_t* __restrict__ dy, float* __restrict__ part,
                                                           int rows, int cols, int rpb) {
  const int c0 = blockIdx.x * 512 + threadIdx.x * 2;
  const int r0 = blockIdx.y * rpb, r1 = min(rows, r0 + rpb);
  float a0 = 0.f, a1 = 0.f;
  if (c0 < cols) {
    constexpr int U = 16;
    int r = r0;
    for (; r + U <= r1; r += U) {
      uint32_t v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const uint32_t*>(dy + (int64_t)(r + u) * cols + c0);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        a0 += bf2f((bf16_t)(v[u] & 0xffffu));
        a1 += bf2f((bf16_t)(v[u] >> 16));
      }
    }
    for (; r < r1; ++r) {
      const uint32_t v = *reinterpret_cast<const uint32_t*>(dy + (int64_t)r * cols + c0);
      a0 += bf2f((bf16_t)(v & 0xffffu));
      a1 += bf2f((bf16_t)(v >> 16));
    }
    part[(int64_t)blockIdx.y * cols + c0] = a0;
    part[(int64_t)blockIdx.y * cols + c0 + 1] = a1;
  }
}

// out_k[c] += sum_{r < R} part[k*R*C + r*C + c] for the non-null outputs k < 3 (LN folds dgamma,
// dbeta and the fused bias-gradient colsum in one launch; gridDim.z = number of non-null outputs,
// mapped to their slab index through `which`). Block = 64 columns x 4 row lanes; gridDim.y row
// chunks (<= 32 adders per address).
struct Outs3 { float* p[3]; int which[3]; };
__global__ void col_reduce_add_kernel(const float* __restrict__ part, Outs3 o, int R, int C) {
  __shared__ float red[4][64];
  const int k = o.which[blockIdx.z];
  const float* p = part + (int64_t)k * R * C;
  float* out = o.p[k];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  const int per = (R + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * per, r1 = min(R, r0 + per);
  // four independent partial sums: the row loads of an unrolled iteration are all in flight
  // together (one dependent load per iteration left the ~100 launches per BERT step latency-bound)
  float s = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (c < C) {
    int r = r0 + rl;
    for (; r + 12 < r1; r += 16) {
      s += p[(int64_t)r * C + c];
      s1 += p[(int64_t)(r + 4) * C + c];
      s2 += p[(int64_t)(r + 8) * C + c];
      s3 += p[(int64_t)(r + 12) * C + c];
    }
    for (; r < r1; r += 4) s += p[(int64_t)r * C + c];
  }
  s = (s + s1) + (s2 + s3);
  red[rl][threadIdx.x & 63] = s;
  __syncthreads();
  if (rl == 0 && c < C) {
    s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    atomicAdd(out + c, s);
  }
}

// Deterministic variant (gy = 0): one 1024-thread block per 64 columns and output, 16 row lanes
// summed in a fixed order, a plain read-modify-write of the output (no float atomics: the atomic
// form's adds contended with the overlapped optimizer's traffic in the step, 6 us median but up to
// 150 us per call, and its sum order varied run to run).
// 32 columns (one 128-B line per row) x 32 row lanes per block, 8 independent loads in flight per
// lane: the fold of a 1024-row slab is 4 load round trips per lane. (64 columns x 16 lanes with 4 in
// flight took 16 round trips: 16 us per LayerNorm-backward fold, 1.6 ms of the BERT-Large step.)
__global__ void __launch_bounds__(1024) col_reduce_det_kernel(const float* __restrict__ part, Outs3 o, int R, int C) {
  constexpr int CW = 32, RL = 32, U = 8;
  __shared__ float red[RL][CW + 1];
  const int k = o.which[blockIdx.y];
  const float* p = part + (int64_t)k * R * C;
  float* out = o.p[k];
  const int c = blockIdx.x * CW + (threadIdx.x % CW);
  const int rl = threadIdx.x / CW;
  float acc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) acc[u] = 0.f;
  if (c < C) {
    int r = rl;
    for (; r + (U - 1) * RL < R; r += U * RL) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = p[(int64_t)(r + u * RL) * C + c];
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] += v[u];
    }
    for (; r < R; r += RL) acc[0] += p[(int64_t)r * C + c];
  }
  float t0 = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) t0 += acc[u];
  red[rl][threadIdx.x % CW] = t0;
  __syncthreads();
  if (rl == 0 && c < C) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < RL; ++i) t += red[i][threadIdx.x];
    out[c] += t;
  }
}

// row chunks per column block (atomic adders per output address); 0 = the deterministic kernel
// above (default); FF_COLRED_GY / col_reduce_set_gy
static int g_cr_gy = -1;
int col_reduce_gy() {
  if (g_cr_gy < 0) {
    const char* e = getenv("FF_COLRED_GY");
    g_cr_gy = e ? std::max(0, atoi(e)) : 0;
  }
  return g_cr_gy;
}
void col_reduce_set_gy(int g) { g_cr_gy = std::max(0, g); }

// Batched deterministic folds: up to FOLD_MAX (slab, output) pairs in one launch, each pair's
// column blocks a contiguous range of blockIdx.x; the per-pair arithmetic is col_reduce_det_kernel's
// (same order: bitwise equal results). Lets the ~76 parameter-gradient folds of a BERT-Large backward
// (LayerNorm gamma / beta, biases; 5-8 us each, latency-bound at 32-96 workgroups) run a few per
// launch, queued until a gradient bucket needs them (fold_record / fold_flush).
constexpr int FOLD_MAX = 24;
struct FoldRow { const float* part; float* out; int R, C, first, pad; };
struct FoldBatch { FoldRow r[FOLD_MAX]; int n; };
__global__ void __launch_bounds__(1024) col_reduce_batch_kernel(FoldBatch b) {
  constexpr int CW = 32, RL = 32, U = 8;
  __shared__ float red[RL][CW + 1];
  int i = 0;
  while (i + 1 < b.n && b.r[i + 1].first <= (int)blockIdx.x) ++i;  // uniform: scalar loop over <= 24 rows
  const float* p = b.r[i].part;
  float* out = b.r[i].out;
  const int R = b.r[i].R, C = b.r[i].C;
  const int c = ((int)blockIdx.x - b.r[i].first) * CW + (threadIdx.x % CW);
  const int rl = threadIdx.x / CW;
  float acc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) acc[u] = 0.f;
  if (c < C) {
    int r = rl;
    for (; r + (U - 1) * RL < R; r += U * RL) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = p[(int64_t)(r + u * RL) * C + c];
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] += v[u];
    }
    for (; r < R; r += RL) acc[0] += p[(int64_t)r * C + c];
  }
  float t0 = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) t0 += acc[u];
  red[rl][threadIdx.x % CW] = t0;
  __syncthreads();
  if (rl == 0 && c < C) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < RL; ++k) t += red[k][threadIdx.x];
    out[c] += t;
  }
}

// fold recorder: while on, col_reduce_add3's deterministic folds are queued instead of launched;
// fold_flush launches the queue. A second fold into an output already queued flushes first (two
// read-modify-writes of one output must not share a launch). Host-side state: one queue per
// process, used from the thread that runs the backward.
static bool g_fold_rec = false;
static std::vector<FoldRow> g_fold_q;
static hipStream_t g_fold_st = nullptr;
void fold_record(bool on) { g_fold_rec = on; }
int fold_pending() { return (int)g_fold_q.size(); }
void fold_flush(hipStream_t st) {
  size_t i = 0;
  while (i < g_fold_q.size()) {
    FoldBatch b;
    b.n = 0;
    int blocks = 0;
    for (; i < g_fold_q.size() && b.n < FOLD_MAX; ++i) {
      b.r[b.n] = g_fold_q[i];
      b.r[b.n].first = blocks;
      blocks += (g_fold_q[i].C + 31) / 32;
      ++b.n;
    }
    hipLaunchKernelGGL(col_reduce_batch_kernel, dim3(blocks), dim3(1024), 0, st, b);
  }
  g_fold_q.clear();
}

static void fold_push(const float* part, float* out, int R, int C, hipStream_t st) {
  if (!g_fold_q.empty() && st != g_fold_st) fold_flush(g_fold_st);
  g_fold_st = st;
  for (const FoldRow& q : g_fold_q)
    if (q.out == out) {
      fold_flush(st);
      break;
    }
  g_fold_q.push_back(FoldRow{part, out, R, C, 0, 0});
}
bool fold_queue(const float* part, float* out, int R, int C, hipStream_t st) {
  if (!g_fold_rec || col_reduce_gy() != 0 || R <= 0 || C <= 0) return false;
  fold_push(part, out, R, C, st);
  return true;
}

void col_reduce_add3(const float* part, float* out0, float* out1, float* out2, int R, int C, hipStream_t st) {
  if (R == 0 || C == 0) return;
  Outs3 o{{out0, out1, out2}, {0, 0, 0}};
  int nz = 0;
  for (int k = 0; k < 3; ++k)
    if (o.p[k]) o.which[nz++] = k;
  if (!nz) return;
  if (g_fold_rec && col_reduce_gy() == 0) {
    for (int z = 0; z < nz; ++z) fold_push(part + (int64_t)o.which[z] * R * C, o.p[o.which[z]], R, C, st);
    return;
  }
  if (col_reduce_gy() == 0) {
    hipLaunchKernelGGL(col_reduce_det_kernel, dim3((C + 31) / 32, nz), dim3(1024), 0, st, part, o, R, C);
    return;
  }
  const int gy = std::max(1, std::min(col_reduce_gy(), R / 8));
  hipLaunchKernelGGL(col_reduce_add_kernel, dim3((C + 63) / 64, gy, nz), dim3(256), 0, st, part, o, R, C);
}
void col_reduce_add2(const float* part, float* out0, float* out1, int R, int C, hipStream_t st) {
  col_reduce_add3(part, out0, out1, nullptr, R, C, st);
}
void col_reduce_add(const float* part, float* out, int R, int C, hipStream_t st) {
  col_reduce_add2(part, out, nullptr, R, C, st);
}

// out[i] = beta * out[i] + sum_s slabs[s][i] (fp32, n % 4 == 0, 16-B aligned): the reduction of a
// split-K GEMM whose S partial products were written as S slabs by one strided-batched GEMM.
__global__ void slab_sum_kernel(const float4* __restrict__ slabs, float4* __restrict__ out, int64_t nv, int S,
                                float beta) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    float4 a = slabs[i];
    for (int s = 1; s < S; ++s) {
      const float4 b = slabs[(int64_t)s * nv + i];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    if (beta != 0.f) {
      const float4 c = out[i];
      a.x += beta * c.x; a.y += beta * c.y; a.z += beta * c.z; a.w += beta * c.w;
    }
    out[i] = a;
  }
}
void slab_sum(const float* slabs, float* out, int64_t n, int S, float beta, hipStream_t st) {
  const int64_t nv = n / 4;
  hipLaunchKernelGGL(slab_sum_kernel, dim3(ew_grid(nv, 256)), dim3(256), 0, st, (const float4*)slabs, (float4*)out, nv,
                     S, beta);
}

static void bab_geometry(int rows, int cols, int& gx, int& gy, int& rpb) {
  gx = (cols + BAB_COLS - 1) / BAB_COLS;
  // >= ~1024 blocks where the shape allows (4+ per CU), >= 32 rows per block (one 8-row batch
  // per wave), slab rows = gy
  gy = std::max(1, std::min((1024 + gx - 1) / gx, (rows + 31) / 32));
  rpb = (((rows + gy - 1) / gy) + 31) / 32 * 32;
  gy = (rows + rpb - 1) / rpb;
}

int bias_act_bwd_chunks(int rows, int cols) {
  int gx, gy, rpb;
  bab_geometry(rows, cols, gx, gy, rpb);
  return gy;
}

// Epilogue pass for library GEMMs: zb = z + bias[col] (stored back if zout), y = act(zb).
// bf16, cols % 8 == 0: one 16-B vector per thread-step. In place (y == z) is allowed.
// Epilogue pass for library GEMMs: zb = z + bias[col] (stored back if zout), y = act(zb). With
// ACT_STORE_GRAD in act, zout receives act'(zb) instead (the consumer's dgrad epilogue then only
// multiplies by it; zout may alias z). bf16, cols % 8 == 0: one 16-B vector per thread-step. In
// place (y == z) is allowed.
template <int AK = 0>  // the activation as a compile-time constant (see bias_act_bwd_kernel), 0: run time
__global__ void bias_act_fwd_kernel(const bf16_t* __restrict__ z, const void* __restrict__ bias, int bias_bf16,
                                    bf16_t* zout, bf16_t* y, int64_t rows, int cols, int act_rt) {
  const bool sg = (act_rt & ACT_STORE_GRAD) != 0 && zout != nullptr;
  const int act = AK ? AK : (act_rt & 0xff);
  const int64_t nv = rows * (int64_t)cols / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // two 16-B vectors per lane in flight (the 2048-block grid alone leaves ~32 KB in flight per CU,
  // under what hides an HBM round trip); only the plain activation pass takes this path
  if (!bias) {
    for (; v + stride < nv; v += 2 * stride) {
      float x0[8], x1[8];
      load16(z + v * 8, x0);
      load16(z + (v + stride) * 8, x1);
      if (sg) {
        float g0[8], g1[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          act_fwd_grad(act, x0[j], x0[j], g0[j]);
          act_fwd_grad(act, x1[j], x1[j], g1[j]);
        }
        store16(zout + v * 8, g0);
        store16(zout + (v + stride) * 8, g1);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          x0[j] = act_fwd(act, x0[j]);
          x1[j] = act_fwd(act, x1[j]);
        }
      }
      store16(y + v * 8, x0);
      store16(y + (v + stride) * 8, x1);
    }
  }
  for (; v < nv; v += stride) {
    const int64_t e = v * 8;
    const int c = (int)(e % cols);
    float x[8];
    load16(z + e, x);
    if (bias) {
      if (bias_bf16) {
        float b[8];
        load16((const bf16_t*)bias + c, b);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] += b[j];
      } else {
        const float4 b0 = *reinterpret_cast<const float4*>((const float*)bias + c);
        const float4 b1 = *reinterpret_cast<const float4*>((const float*)bias + c + 4);
        x[0] += b0.x; x[1] += b0.y; x[2] += b0.z; x[3] += b0.w;
        x[4] += b1.x; x[5] += b1.y; x[6] += b1.z; x[7] += b1.w;
      }
      if (zout && !sg) store16(zout + e, x);
    }
    if (sg) {
      float g[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) act_fwd_grad(act, x[j], x[j], g[j]);
      store16(zout + e, g);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = act_fwd(act, x[j]);
    }
    store16(y + e, x);
  }
}

// ---------------------------------------------------------------- host launchers
#define FFK_DT_DISPATCH(dt, ...)                        \
  do {                                                  \
    if (dt == DT_BF16) { using T = bf16_t; __VA_ARGS__; } \
    else { using T = float; __VA_ARGS__; }              \
  } while (0)

void unary_fwd(int dt, const void* x, void* y, int64_t n, int op, float s, hipStream_t st) {
  if (n == 0) return;
  FFK_DT_DISPATCH(dt, {
    const dim3 grid(ew_grid(n / (16 / sizeof(T)) + 1, 256));
    if (op == U_RELU) hipLaunchKernelGGL((unary_fwd_kernel<T, U_RELU>), grid, dim3(256), 0, st, (const T*)x, (T*)y, n, op, s);
    else hipLaunchKernelGGL(unary_fwd_kernel<T>, grid, dim3(256), 0, st, (const T*)x, (T*)y, n, op, s);
  });
}
void unary_bwd(int dt, const void* x, const void* y, const void* dy, void* dx, int64_t n, int op, float s,
               int accumulate, hipStream_t st) {
  if (n == 0) return;
  FFK_DT_DISPATCH(dt, {
    const dim3 grid(ew_grid(n / (16 / sizeof(T)) + 1, 256));
    if (op == U_RELU)
      hipLaunchKernelGGL((unary_bwd_kernel<T, U_RELU>), grid, dim3(256), 0, st, (const T*)x, (const T*)y,
                         (const T*)dy, (T*)dx, n, op, s, accumulate);
    else
      hipLaunchKernelGGL(unary_bwd_kernel<T>, grid, dim3(256), 0, st, (const T*)x, (const T*)y, (const T*)dy,
                         (T*)dx, n, op, s, accumulate);
  });
}
void binary_fwd(int dt, const void* a, const void* b, void* c, int64_t n, int op, int ndim,
                const int64_t* shape, const int64_t* sa, const int64_t* sb, int same, hipStream_t st) {
  if (n == 0) return;
  BcastDesc d;
  d.ndim = ndim;
  for (int i = 0; i < ndim; ++i) { d.shape[i] = shape[i]; d.sa[i] = sa[i]; d.sb[i] = sb[i]; }
  FFK_DT_DISPATCH(dt, {
    if (same && ((uintptr_t)a % 16 == 0) && ((uintptr_t)b % 16 == 0) && ((uintptr_t)c % 16 == 0)) {
      const dim3 grid(ew_grid(n / (16 / sizeof(T)) + 1, 256));
      if (op == B_ADD)
        hipLaunchKernelGGL((binary_same_kernel<T, B_ADD>), grid, dim3(256), 0, st, (const T*)a, (const T*)b, (T*)c, n, op);
      else if (op == (B_ADD | B_RELU))
        hipLaunchKernelGGL((binary_same_kernel<T, B_ADD | B_RELU>), grid, dim3(256), 0, st, (const T*)a, (const T*)b,
                           (T*)c, n, op);
      else
        hipLaunchKernelGGL(binary_same_kernel<T>, grid, dim3(256), 0, st, (const T*)a, (const T*)b, (T*)c, n, op);
    }
    else {
      if (same) { d.ndim = 1; d.shape[0] = n; d.sa[0] = 1; d.sb[0] = 1; }
      hipLaunchKernelGGL(binary_bcast_kernel<T>, dim3(ew_grid(n, 256)), dim3(256), 0, st, (const T*)a,
                         (const T*)b, (T*)c, n, op, d);
    }
  });
}
void binary_bwd(int dt, const void* a, const void* b, const void* dc, void* da, void* db, int64_t n, int op,
                int ndim, const int64_t* shape, const int64_t* sa, const int64_t* sb, int same, hipStream_t st) {
  if (n == 0) return;
  BcastDesc d;
  d.ndim = ndim;
  for (int i = 0; i < ndim; ++i) { d.shape[i] = shape[i]; d.sa[i] = sa[i]; d.sb[i] = sb[i]; }
  FFK_DT_DISPATCH(dt, {
    hipLaunchKernelGGL(binary_bwd_kernel<T>, dim3(ew_grid(n, 256)), dim3(256), 0, st, (const T*)a,
                       (const T*)b, (const T*)dc, (T*)da, (T*)db, n, op, d, same);
  });
}
void cast(int dt_in, int dt_out, const void* x, void* y, int64_t n, hipStream_t st) {
  if (n == 0) return;
  dim3 g(ew_grid(n, 256));
  if (dt_in == DT_F32 && dt_out == DT_BF16)
    hipLaunchKernelGGL((cast_kernel<float, bf16_t>), g, dim3(256), 0, st, (const float*)x, (bf16_t*)y, n);
  else if (dt_in == DT_BF16 && dt_out == DT_F32)
    hipLaunchKernelGGL((cast_kernel<bf16_t, float>), g, dim3(256), 0, st, (const bf16_t*)x, (float*)y, n);
  else if (dt_in == DT_F32)
    hipLaunchKernelGGL((cast_kernel<float, float>), g, dim3(256), 0, st, (const float*)x, (float*)y, n);
  else
    hipLaunchKernelGGL((cast_kernel<bf16_t, bf16_t>), g, dim3(256), 0, st, (const bf16_t*)x, (bf16_t*)y, n);
}
void dropout_fwd(int dt, const void* x, void* y, uint8_t* mask, int64_t n, float rate, uint64_t seed,
                 uint64_t offset, hipStream_t st) {
  if (n == 0) return;
  FFK_DT_DISPATCH(dt, {
    hipLaunchKernelGGL(dropout_kernel<T>, dim3(ew_grid(n, 256)), dim3(256), 0, st, (const T*)x, (T*)y, mask, n,
                       rate, seed, offset);
  });
}
void dropout_bwd(int dt, const void* dy, const uint8_t* mask, void* dx, int64_t n, float rate, int accumulate,
                 hipStream_t st) {
  if (n == 0) return;
  FFK_DT_DISPATCH(dt, {
    hipLaunchKernelGGL(dropout_bwd_kernel<T>, dim3(ew_grid(n, 256)), dim3(256), 0, st, (const T*)dy, mask,
                       (T*)dx, n, rate, accumulate);
  });
}
void bias_act_fwd(const void* z, const void* bias, int bias_bf16, void* zout, void* y, int64_t rows, int cols,
                  int act, hipStream_t st) {
  if (rows == 0 || cols == 0) return;
  const dim3 grid(ew_grid(rows * cols / 8, 256));
  if ((act & 0xff) == ACT_GELU)
    hipLaunchKernelGGL(bias_act_fwd_kernel<ACT_GELU>, grid, dim3(256), 0, st, (const bf16_t*)z, bias, bias_bf16,
                       (bf16_t*)zout, (bf16_t*)y, rows, cols, act);
  else if ((act & 0xff) == ACT_RELU)
    hipLaunchKernelGGL(bias_act_fwd_kernel<ACT_RELU>, grid, dim3(256), 0, st, (const bf16_t*)z, bias, bias_bf16,
                       (bf16_t*)zout, (bf16_t*)y, rows, cols, act);
  else
    hipLaunchKernelGGL(bias_act_fwd_kernel<>, grid, dim3(256), 0, st, (const bf16_t*)z, bias, bias_bf16,
                       (bf16_t*)zout, (bf16_t*)y, rows, cols, act);
}

void bias_act_bwd(int dt, const void* dy, const void* z, void* dz, float* dbias, float* ws, int rows, int cols,
                  int act, hipStream_t st, int stage) {
  if (rows == 0 || cols == 0) return;
  int gx, gy, rpb;
  bab_geometry(rows, cols, gx, gy, rpb);
  // stage 0: both passes; 1: the row pass only (slab into ws); 2: the slab fold only (the caller
  // queues it on a side stream: the bias gradient is needed by the optimizer, not by the backward)
  if (stage == 2) {
    if (dbias) col_reduce_add(ws, dbias, gy, cols, st);
    return;
  }
  if (dt == DT_BF16 && act == ACT_NONE && dbias && (cols & 7) && !(cols & 1) && ((uintptr_t)dy & 3) == 0) {
    hipLaunchKernelGGL(colsum_pairs_kernel, dim3(gx, gy), dim3(256), 0, st, (const bf16_t*)dy, ws, rows, cols, rpb);
    if (stage == 0) col_reduce_add(ws, dbias, gy, cols, st);
    return;
  }
  FFK_DT_DISPATCH(dt, {
    if (act == ACT_GELU)
      hipLaunchKernelGGL((bias_act_bwd_kernel<T, true, ACT_GELU>), dim3(gx, gy), dim3(256), 0, st, (const T*)dy,
                         (const T*)z, (T*)dz, dbias ? ws : nullptr, rows, cols, act, rpb);
    else if (act == ACT_RELU)
      hipLaunchKernelGGL((bias_act_bwd_kernel<T, true, ACT_RELU>), dim3(gx, gy), dim3(256), 0, st, (const T*)dy,
                         (const T*)z, (T*)dz, dbias ? ws : nullptr, rows, cols, act, rpb);
    else if (act != ACT_NONE)
      hipLaunchKernelGGL((bias_act_bwd_kernel<T, true>), dim3(gx, gy), dim3(256), 0, st, (const T*)dy, (const T*)z,
                         (T*)dz, dbias ? ws : nullptr, rows, cols, act, rpb);
    else if (dbias)
      hipLaunchKernelGGL((bias_act_bwd_kernel<T, false>), dim3(gx, gy), dim3(256), 0, st, (const T*)dy, (const T*)z,
                         (T*)dz, ws, rows, cols, act, rpb);
  });
  if (dbias && stage == 0) col_reduce_add(ws, dbias, gy, cols, st);
}

}  // namespace ffk

// Mixture-of-experts routing on the device: TopK, GroupBy, Aggregate / AggregateSpec forward and
// backward without host synchronisation (capturable into a hipGraph).
//
// Reference: src/ops/topk.cu:336,445 (per-row heap top-k), group_by.cu:27,66, aggregate.cu:21,127,
// aggregate_spec.cu:21,143. The reference scans samples in order and gives each (sample, choice)
// the next free row of its expert, dropping overflow past the capacity; here that order is kept
// exactly, computed in parallel:
//   moe_count  : per 64-element chunk (one wave) and expert, how many (sample, choice) pairs
//   moe_scan   : exclusive scan over chunks per expert (one thread per expert) -> chunk bases
//                and the total load of every expert (the balance term of Aggregate's backward)
//   moe_rank   : rank inside the chunk (shuffle loop over the preceding lanes) + chunk base
//                = the row of the pair in its expert's tensor; valid = row < capacity
// GroupBy / Aggregate then move whole rows, one block per pair or per sample: no atomics (every
// expert row is written by exactly one pair, every sample row by one block).
#include "common.h"
#include "ops.h"

namespace ffk {

namespace {

template <typename T>
__device__ __forceinline__ float ld1(const T* p, int64_t i) {
  return Cvt<T>::to_f(p[i]);
}

// ---------------------------------------------------------------------------------------- top-k
// One wave per row; k passes of a wave arg-max (ties: lowest index), values descending.
template <typename T>
__global__ void __launch_bounds__(256) topk_fwd_kernel(const T* __restrict__ x, T* __restrict__ vals,
                                                       int* __restrict__ idx, int rows, int n, int k) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + (int64_t)row * n;
  int last_i = -1;
  float last_v = INFINITY;
  for (int j = 0; j < k; ++j) {
    // best among elements strictly after the previous pick in (value desc, index asc) order
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int c = lane; c < n; c += 64) {
      const float v = ld1(xr, c);
      const bool after = (v < last_v) || (v == last_v && c > last_i);
      const bool better = (v > bv) || (v == bv && c < bi);
      if (after && better) { bv = v; bi = c; }
    }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
      const float ov = __shfl_xor(bv, s);
      const int oi = __shfl_xor(bi, s);
      if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    if (lane == 0) {
      vals[(int64_t)row * k + j] = Cvt<T>::from_f(bv);
      idx[(int64_t)row * k + j] = bi;
    }
    last_v = bv;
    last_i = bi;
  }
}

// dx[row][c] = sum of dvals[row][j] over the picks j of column c (picks are distinct): each lane
// owns its columns, so every element is written once
template <typename T>
__global__ void __launch_bounds__(256) topk_bwd_kernel(const T* __restrict__ dvals, const int* __restrict__ idx,
                                                       T* __restrict__ dx, int rows, int n, int k) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  for (int c = lane; c < n; c += 64) {
    float s = 0.f;
    for (int j = 0; j < k; ++j)
      if (idx[(int64_t)row * k + j] == c) s += ld1(dvals, (int64_t)row * k + j);
    dx[(int64_t)row * n + c] = Cvt<T>::from_f(s);
  }
}

// --------------------------------------------------------------------------------------- routing
__device__ __forceinline__ int clamp_e(int e, int n) { return e < 0 ? 0 : (e >= n ? n - 1 : e); }

// counts[chunk][e]: pairs of chunk (64 consecutive flattened (sample, choice) pairs) per expert
__global__ void __launch_bounds__(256) moe_count_kernel(const int* __restrict__ assign, int L, int n,
                                                        int* __restrict__ counts) {
  const int lane = threadIdx.x & 63;
  const int chunk = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nchunks = (L + 63) / 64;
  if (chunk >= nchunks) return;
  const int i = chunk * 64 + lane;
  const int e = i < L ? clamp_e(assign[i], n) : -1;
  for (int x = lane; x < n; x += 64) counts[(int64_t)chunk * n + x] = 0;
  // one ballot per expert present in the wave (the lowest remaining expert each round)
  uint64_t todo = __ballot(e >= 0);
  while (todo) {
    const int first = __ffsll((unsigned long long)todo) - 1;
    const int ex = __shfl(e, first);
    const uint64_t m = __ballot(e == ex);
    if (lane == 0) counts[(int64_t)chunk * n + ex] = __popcll(m);
    todo &= ~m;
  }
}

// bases[chunk][e] = sum of counts over earlier chunks; total[e] = load of expert e
__global__ void moe_scan_kernel(const int* __restrict__ counts, int nchunks, int n, int* __restrict__ bases,
                                int* __restrict__ total) {
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    int run = 0;
    for (int c = 0; c < nchunks; ++c) {
      bases[(int64_t)c * n + e] = run;
      run += counts[(int64_t)c * n + e];
    }
    total[e] = run;
  }
}

// pos[i] = row of pair i in its expert's tensor (-1: dropped past the capacity)
__global__ void __launch_bounds__(256) moe_rank_kernel(const int* __restrict__ assign, int L, int n, int cap,
                                                       const int* __restrict__ bases, int* __restrict__ expert,
                                                       int* __restrict__ pos) {
  const int lane = threadIdx.x & 63;
  const int chunk = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nchunks = (L + 63) / 64;
  if (chunk >= nchunks) return;
  const int i = chunk * 64 + lane;
  const int raw = i < L ? assign[i] : -1;
  const int e = i < L ? clamp_e(raw, n) : -1;
  // rank among the earlier lanes of this chunk with the same expert
  int rank = 0;
  for (int s = 0; s < 64; ++s) {
    const int es = __shfl(e, s);
    if (s < lane && es == e) ++rank;
  }
  if (i < L) {
    const int p = bases[(int64_t)chunk * n + e] + rank;
    // out-of-range expert ids are routed nowhere (reference: valid requires 0 <= e < n)
    const bool ok = raw >= 0 && raw < n && p < cap;
    expert[i] = e;
    pos[i] = ok ? p : -1;
  }
}

// ------------------------------------------------------------------------------------- group-by
struct PtrTable {
  void* p[kMoeMaxExperts];
};

// zero every expert tensor [cap, D]
template <typename T>
__global__ void moe_zero_kernel(PtrTable outs, int n, int64_t elems) {
  const int e = blockIdx.y;
  T* o = reinterpret_cast<T*>(outs.p[e]);
  if (!o) return;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < elems; i += (int64_t)gridDim.x * blockDim.x)
    o[i] = Cvt<T>::from_f(0.f);
}

// out[expert[i]][pos[i]] = data[i / k] for the kept pairs; one block per pair, D columns
template <typename T>
__global__ void __launch_bounds__(256) groupby_fwd_kernel(const T* __restrict__ data, const int* __restrict__ expert,
                                                          const int* __restrict__ pos, PtrTable outs, int L, int k,
                                                          int D) {
  const int i = blockIdx.x;
  if (i >= L) return;
  const int p = pos[i];
  if (p < 0) return;
  T* o = reinterpret_cast<T*>(outs.p[expert[i]]) + (int64_t)p * D;
  const T* src = data + (int64_t)(i / k) * D;
  for (int c = threadIdx.x; c < D; c += blockDim.x) o[c] = src[c];
}

// dx[b] = sum over the kept choices j of dout[expert][pos] (null dout = zero gradient)
template <typename T>
__global__ void __launch_bounds__(256) groupby_bwd_kernel(PtrTable douts, const int* __restrict__ expert,
                                                          const int* __restrict__ pos, T* __restrict__ dx, int B,
                                                          int k, int D) {
  const int b = blockIdx.x;
  if (b >= B) return;
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    float s = 0.f;
    for (int j = 0; j < k; ++j) {
      const int i = b * k + j;
      const int p = pos[i];
      const T* d = reinterpret_cast<const T*>(douts.p[expert[i]]);
      if (p >= 0 && d) s += ld1(d, (int64_t)p * D + c);
    }
    dx[(int64_t)b * D + c] = Cvt<T>::from_f(s);
  }
}

// ------------------------------------------------------------------------------------ aggregate
// out[b] = sum_j w[b][j] * exp[expert][pos] (w = gate, or 1 for AggregateSpec)
template <typename T>
__global__ void __launch_bounds__(256) aggregate_fwd_kernel(const T* __restrict__ gate, PtrTable exps,
                                                            const int* __restrict__ expert,
                                                            const int* __restrict__ pos, T* __restrict__ out, int B,
                                                            int k, int D) {
  const int b = blockIdx.x;
  if (b >= B) return;
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    float s = 0.f;
    for (int j = 0; j < k; ++j) {
      const int i = b * k + j;
      const int p = pos[i];
      if (p < 0) continue;
      const float w = gate ? ld1(gate, i) : 1.f;
      s += w * ld1(reinterpret_cast<const T*>(exps.p[expert[i]]), (int64_t)p * D + c);
    }
    out[(int64_t)b * D + c] = Cvt<T>::from_f(s);
  }
}

// Backward, one block per sample b (4 waves; wave j handles choice j, looping when k > 4):
//   dexp[expert][pos] = w * dout[b]                       (rows no pair hits stay zero)
//   dgate[b][j]      = dout[b] . exp[expert][pos]         (0 for dropped pairs)
//   dfull[b][e]      = sum over j with expert e of dgate[b][j] * correct(b)
//                      + lambda * load(e), then minus its row mean
// (reference aggregate.cu: the gate gradient steers assignment towards correct experts and the
// balance term towards under-loaded ones; AggregateSpec: no gate product, no gate gradients)
template <typename T>
__global__ void __launch_bounds__(256) aggregate_bwd_kernel(const T* __restrict__ dout, const T* __restrict__ gate,
                                                            PtrTable exps, PtrTable dexps,
                                                            const int* __restrict__ expert,
                                                            const int* __restrict__ pos,
                                                            const int* __restrict__ assign,
                                                            const int* __restrict__ true_assign,
                                                            const int* __restrict__ load, float lambda_bal,
                                                            T* __restrict__ dgate, T* __restrict__ dfull, int B,
                                                            int k, int n, int D) {
  __shared__ float sdot[64];
  __shared__ int scorrect;
  const int b = blockIdx.x;
  if (b >= B) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) {
    int ok = 1;
    if (assign && true_assign)
      for (int j = 0; j < k; ++j) ok &= assign[b * k + j] == true_assign[b * k + j];
    scorrect = ok;
  }
  for (int j = wv; j < k; j += 4) {
    const int i = b * k + j;
    const int p = pos[i];
    const float w = gate ? ld1(gate, i) : 1.f;
    float dot = 0.f;
    if (p >= 0) {
      const T* ex = reinterpret_cast<const T*>(exps.p[expert[i]]) + (int64_t)p * D;
      T* dex = reinterpret_cast<T*>(dexps.p[expert[i]]);
      for (int c = lane; c < D; c += 64) {
        const float g = ld1(dout, (int64_t)b * D + c);
        if (dex) dex[(int64_t)p * D + c] = Cvt<T>::from_f(g * w);
        dot += g * ld1(ex, c);
      }
    }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) dot += __shfl_xor(dot, s);
    if (lane == 0) {
      if (j < 64) sdot[j] = dot;
      if (dgate) dgate[i] = Cvt<T>::from_f(dot);
    }
  }
  __syncthreads();
  if (!dfull) return;
  // row of the full-gate gradient: n entries, then made zero-mean
  __shared__ float srow[kMoeMaxExperts];
  for (int e = threadIdx.x; e < n; e += blockDim.x) {
    float v = lambda_bal * (float)load[e];
    if (scorrect)
      for (int j = 0; j < k && j < 64; ++j) {
        const int i = b * k + j;
        if (pos[i] >= 0 && expert[i] == e) v += sdot[j];
      }
    srow[e] = v;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    float s = 0.f;
    for (int e = threadIdx.x; e < n; e += 64) s += srow[e];
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) s += __shfl_xor(s, sh);
    if (threadIdx.x == 0) sdot[0] = s / n;  // sdot no longer needed
  }
  __syncthreads();
  const float mean = sdot[0];
  for (int e = threadIdx.x; e < n; e += blockDim.x) dfull[(int64_t)b * n + e] = Cvt<T>::from_f(srow[e] - mean);
}

PtrTable table(void* const* ptrs, int n) {
  PtrTable t;
  for (int i = 0; i < kMoeMaxExperts; ++i) t.p[i] = i < n ? ptrs[i] : nullptr;
  return t;
}

}  // namespace

#define FFK_MOE_DT(dt, ...)                               \
  do {                                                    \
    if (dt == DT_BF16) { using T = bf16_t; __VA_ARGS__; } \
    else { using T = float; __VA_ARGS__; }                \
  } while (0)

void topk_fwd(int dt, const void* x, void* vals, int* idx, int rows, int n, int k, hipStream_t st) {
  if (rows <= 0 || k <= 0) return;
  FFK_MOE_DT(dt, hipLaunchKernelGGL(topk_fwd_kernel<T>, dim3((rows + 3) / 4), dim3(256), 0, st, (const T*)x,
                                    (T*)vals, idx, rows, n, k));
}

void topk_bwd(int dt, const void* dvals, const int* idx, void* dx, int rows, int n, int k, hipStream_t st) {
  if (rows <= 0) return;
  FFK_MOE_DT(dt, hipLaunchKernelGGL(topk_bwd_kernel<T>, dim3((rows + 3) / 4), dim3(256), 0, st, (const T*)dvals,
                                    idx, (T*)dx, rows, n, k));
}

int64_t moe_route_ws_ints(int L, int n) {
  const int64_t nchunks = (L + 63) / 64;
  return 2 * nchunks * n;
}

void moe_route(const int* assign, int L, int n, int cap, int* expert, int* pos, int* load, int* ws, hipStream_t st) {
  if (L <= 0) return;
  const int nchunks = (L + 63) / 64;
  int* counts = ws;
  int* bases = ws + (int64_t)nchunks * n;
  hipLaunchKernelGGL(moe_count_kernel, dim3((nchunks + 3) / 4), dim3(256), 0, st, assign, L, n, counts);
  hipLaunchKernelGGL(moe_scan_kernel, dim3((n + 255) / 256), dim3(256), 0, st, counts, nchunks, n, bases, load);
  hipLaunchKernelGGL(moe_rank_kernel, dim3((nchunks + 3) / 4), dim3(256), 0, st, assign, L, n, cap, bases, expert,
                     pos);
}

void groupby_fwd(int dt, const void* data, const int* expert, const int* pos, void* const* outs, int n, int cap,
                 int L, int k, int D, hipStream_t st) {
  PtrTable t = table(outs, n);
  const int64_t elems = (int64_t)cap * D;
  FFK_MOE_DT(dt, {
    hipLaunchKernelGGL(moe_zero_kernel<T>, dim3((unsigned)std::min<int64_t>(256, (elems + 255) / 256), n), dim3(256),
                       0, st, t, n, elems);
    if (L > 0)
      hipLaunchKernelGGL(groupby_fwd_kernel<T>, dim3(L), dim3(256), 0, st, (const T*)data, expert, pos, t, L, k, D);
  });
}

void groupby_bwd(int dt, void* const* douts, int n, const int* expert, const int* pos, void* dx, int B, int k, int D,
                 hipStream_t st) {
  if (B <= 0) return;
  PtrTable t = table(douts, n);
  FFK_MOE_DT(dt, hipLaunchKernelGGL(groupby_bwd_kernel<T>, dim3(B), dim3(256), 0, st, t, expert, pos, (T*)dx, B, k,
                                    D));
}

void aggregate_fwd(int dt, const void* gate, void* const* exps, int n, const int* expert, const int* pos, void* out,
                   int B, int k, int D, hipStream_t st) {
  if (B <= 0) return;
  PtrTable t = table(exps, n);
  FFK_MOE_DT(dt, hipLaunchKernelGGL(aggregate_fwd_kernel<T>, dim3(B), dim3(256), 0, st, (const T*)gate, t, expert,
                                    pos, (T*)out, B, k, D));
}

void aggregate_bwd(int dt, const void* dout, const void* gate, void* const* exps, void* const* dexps, int n,
                   int cap, const int* expert, const int* pos, const int* assign, const int* true_assign,
                   const int* load, float lambda_bal, void* dgate, void* dfull, int B, int k, int D, hipStream_t st) {
  PtrTable te = table(exps, n), td = table(dexps, n);
  const int64_t elems = (int64_t)cap * D;
  FFK_MOE_DT(dt, {
    hipLaunchKernelGGL(moe_zero_kernel<T>, dim3((unsigned)std::min<int64_t>(256, (elems + 255) / 256), n), dim3(256),
                       0, st, td, n, elems);
    if (B > 0)
      hipLaunchKernelGGL(aggregate_bwd_kernel<T>, dim3(B), dim3(256), 0, st, (const T*)dout, (const T*)gate, te, td,
                         expert, pos, assign, true_assign, load, lambda_bal, (T*)dgate, (T*)dfull, B, k, n, D);
  });
}

}  // namespace ffk

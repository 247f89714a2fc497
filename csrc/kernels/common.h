// Shared device helpers for the flexflow_amd HIP kernel library (gfx950 / CDNA4 only).
//
// Conventions used by every kernel in csrc/kernels:
//   * wave = 64 lanes, block sizes are multiples of 64 (256 is the default);
//   * bf16 tensors travel as raw uint16_t and are converted with the native __bf16
//     type (hipcc lowers the f32->bf16 cast to v_cvt_pk_bf16_f32, NaN-preserving);
//   * memory-bound kernels move 16 B per lane (8 x bf16 / 4 x f32);
//   * MFMA fragment typedefs follow cdna_hip_programming.md §3.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <type_traits>

namespace ffk {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint16_t bf16_t;  // storage type

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

template <typename T> struct Cvt;
template <> struct Cvt<float> {
  __device__ __forceinline__ static float to_f(float v) { return v; }
  __device__ __forceinline__ static float from_f(float v) { return v; }
};
template <> struct Cvt<bf16_t> {
  __device__ __forceinline__ static float to_f(bf16_t v) { return bf2f(v); }
  __device__ __forceinline__ static bf16_t from_f(float v) { return f2bf(v); }
};

// 16-byte vector load/store of VEC elements of T (VEC*sizeof(T) == 16).
template <typename T> struct Vec16 {
  static constexpr int N = 16 / sizeof(T);
  T v[N];
};
template <typename T>
__device__ __forceinline__ void load16(const T* p, float* out) {
  constexpr int N = 16 / sizeof(T);
  uint4 raw = *reinterpret_cast<const uint4*>(p);
  const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = Cvt<T>::to_f(e[i]);
}
template <typename T>
__device__ __forceinline__ void store16(T* p, const float* in) {
  constexpr int N = 16 / sizeof(T);
  uint4 raw;
  T* e = reinterpret_cast<T*>(&raw);
#pragma unroll
  for (int i = 0; i < N; ++i) e[i] = Cvt<T>::from_f(in[i]);
  *reinterpret_cast<uint4*>(p) = raw;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64); `red` must hold NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (NT > 64) {
    __syncthreads();
    if (l == 0) red[w] = v;
    __syncthreads();
    v = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) v += red[i];
  }
  return v;
}
template <int NT>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (NT > 64) {
    __syncthreads();
    if (l == 0) red[w] = v;
    __syncthreads();
    v = -INFINITY;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) v = fmaxf(v, red[i]);
  }
  return v;
}

// Activation codes (match flexflow_amd.type.ActiMode numeric values).
// ACT_GRADMUL (kernel-internal): the 'pre-activation' operand already holds act'(z), stored by the
// producer's forward (bias_act_fwd with ACT_STORE_GRAD), so the backward multiplies by it.
enum Act : int { ACT_NONE = 10, ACT_RELU = 11, ACT_SIGMOID = 12, ACT_TANH = 13, ACT_GELU = 14, ACT_GRADMUL = 15 };
constexpr int ACT_STORE_GRAD = 0x100;  // bias_act_fwd flag: write act'(z) to zout instead of z

// erf with |error| < 1.5e-7 (Abramowitz & Stegun 7.1.26): one v_rcp, one v_exp and five FMAs
// instead of libm erff's branchy polynomial — the GELU epilogues evaluate it per output element.
// The reciprocal is the bare v_rcp_f32 (1 ulp): __frcp_rn / '1.f / x' lower to the IEEE division
// sequence (div_scale x2, rcp, div_fmas, div_fixup + refinement FMAs), which doubled the VALU cost
// of the GELU passes.
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
// e^x as the bare v_exp_f32 (2^(x log2 e)): __expf lowers to v_exp_f32 wrapped in a range reduction
// (v_rndne, v_cvt_i32, v_ldexp, three compares / selects: ~9 VALU instead of 2) that the activation
// functions below do not need — their arguments are <= 0 (GELU's e^(-x^2/2)) or feed a reciprocal
// that absorbs the overflow (sigmoid); results below 2^-126 flush to zero. Round 6: the GELU' pass
// of BERT-Large's FFN backward (bias_act_bwd) was VALU-bound on these sequences.
__device__ __forceinline__ float fast_expe(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
__device__ __forceinline__ float erf_poly_t(float t) {  // A&S 7.1.26 polynomial times t
  float y = __builtin_fmaf(1.061405429f, t, -1.453152027f);
  y = __builtin_fmaf(y, t, 1.421413741f);
  y = __builtin_fmaf(y, t, -0.284496736f);
  y = __builtin_fmaf(y, t, 0.254829592f);
  return y * t;
}
__device__ __forceinline__ float fast_erf(float x) {
  const float ax = fabsf(x);
  const float t = fast_rcp(__builtin_fmaf(0.3275911f, ax, 1.f));
  const float y = 1.f - erf_poly_t(t) * fast_expe(-ax * ax);
  return copysignf(y, x);
}

__device__ __forceinline__ float act_fwd(int act, float x) {
  switch (act) {
    case ACT_RELU: return fmaxf(x, 0.f);
    case ACT_SIGMOID: return fast_rcp(1.f + fast_expe(-x));
    case ACT_TANH: return tanhf(x);
    case ACT_GELU: return 0.5f * x * (1.f + fast_erf(x * 0.70710678118654752f));
    default: return x;
  }
}
// y = act(x) and g = act'(x) together (GELU: one erf / exp for both)
// derivative wrt pre-activation x
__device__ __forceinline__ float act_grad(int act, float x) {
  switch (act) {
    case ACT_RELU: return x > 0.f ? 1.f : 0.f;
    case ACT_SIGMOID: { float s = fast_rcp(1.f + fast_expe(-x)); return s * (1.f - s); }
    case ACT_TANH: { float t = tanhf(x); return 1.f - t * t; }
    case ACT_GRADMUL: return x;
    case ACT_GELU: {
      // Phi(x) + x phi(x); erf(x / sqrt 2) and phi share one exp(-x^2 / 2)
      const float au = fabsf(x) * 0.70710678118654752f;
      const float t = fast_rcp(__builtin_fmaf(0.3275911f, au, 1.f));
      const float e = fast_expe(-au * au);
      const float erf_abs = 1.f - erf_poly_t(t) * e;
      const float cdf = 0.5f + 0.5f * copysignf(erf_abs, x);
      return __builtin_fmaf(x * 0.3989422804014327f, e, cdf);
    }
    default: return 1.f;
  }
}
__device__ __forceinline__ void act_fwd_grad(int act, float x, float& y, float& g) {
  if (act == ACT_GELU) {
    const float au = fabsf(x) * 0.70710678118654752f;
    const float t = fast_rcp(__builtin_fmaf(0.3275911f, au, 1.f));
    const float e = fast_expe(-au * au);
    const float erf_abs = 1.f - erf_poly_t(t) * e;
    const float cdf = 0.5f + 0.5f * copysignf(erf_abs, x);
    y = x * cdf;
    g = __builtin_fmaf(x * 0.3989422804014327f, e, cdf);
    return;
  }
  y = act_fwd(act, x);
  g = act_grad(act, x);
}

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5 "XCD swizzle
// must be bijective"): blocks b, b+8, b+16... share an XCD, so give each XCD a contiguous chunk.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  constexpr int NX = 8;
  if (nwg <= NX) return bid;
  const int q = nwg / NX, r = nwg % NX, x = bid % NX;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / NX;
}

inline int ceil_div(int a, int b) { return (a + b - 1) / b; }
inline int64_t ceil_div64(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Grid size for grid-stride memory-bound kernels (Guideline 11): cap at 256 CU x 8 blocks.
inline int ew_grid(int64_t work_items, int block) {
  int64_t g = (work_items + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace ffk

#define FFK_CHECK(x)                                                              \
  do {                                                                            \
    hipError_t _e = (x);                                                          \
    if (_e != hipSuccess) {                                                       \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(_e), __FILE__, \
              __LINE__);                                                          \
      abort();                                                                    \
    }                                                                             \
  } while (0)

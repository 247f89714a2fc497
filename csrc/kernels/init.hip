// Parameter initialisers: uniform / normal / constant fill.
// Counter-based (splitmix64 of seed and GLOBAL element index): a shard initialised with its
// global offset gets exactly the values the unpartitioned tensor would have, so a TP/DP-sharded
// model starts bit-identical to the 1-GPU model.
// Replaces reference src/runtime/initializer_kernel.cu (curandGenerateUniform/Normal).
#include "common.h"
#include "ops.h"

namespace ffk {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float u01(uint64_t seed, uint64_t i, uint64_t stream) {
  const uint64_t z = mix64(seed * 0x9E3779B97F4A7C15ull + i * 2 + stream + 0x632BE59BD9B4E019ull);
  return ((float)(z >> 40) + 0.5f) * (1.0f / 16777216.0f);
}

template <typename T>
__global__ void uniform_kernel(T* out, int64_t n, float lo, float hi, uint64_t seed, int64_t offset) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = Cvt<T>::from_f(lo + (hi - lo) * u01(seed, offset + i, 0));
}
template <typename T>
__global__ void normal_kernel(T* out, int64_t n, float mean, float stdv, uint64_t seed, int64_t offset) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float a = u01(seed, offset + i, 0), b = u01(seed, offset + i, 1);
    const float r = sqrtf(-2.f * __logf(a));
    out[i] = Cvt<T>::from_f(mean + stdv * r * __cosf(6.283185307179586f * b));
  }
}
template <typename T>
__global__ void fill_kernel(T* out, int64_t n, float v) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = Cvt<T>::from_f(v);
}

void init_uniform(int dt, void* out, int64_t n, float lo, float hi, uint64_t seed, int64_t offset, hipStream_t st) {
  if (n == 0) return;
  if (dt == DT_BF16) hipLaunchKernelGGL(uniform_kernel<bf16_t>, dim3(ew_grid(n, 256)), dim3(256), 0, st, (bf16_t*)out, n, lo, hi, seed, offset);
  else hipLaunchKernelGGL(uniform_kernel<float>, dim3(ew_grid(n, 256)), dim3(256), 0, st, (float*)out, n, lo, hi, seed, offset);
}
void init_normal(int dt, void* out, int64_t n, float mean, float stdv, uint64_t seed, int64_t offset, hipStream_t st) {
  if (n == 0) return;
  if (dt == DT_BF16) hipLaunchKernelGGL(normal_kernel<bf16_t>, dim3(ew_grid(n, 256)), dim3(256), 0, st, (bf16_t*)out, n, mean, stdv, seed, offset);
  else hipLaunchKernelGGL(normal_kernel<float>, dim3(ew_grid(n, 256)), dim3(256), 0, st, (float*)out, n, mean, stdv, seed, offset);
}
void fill(int dt, void* out, int64_t n, float v, hipStream_t st) {
  if (n == 0) return;
  if (dt == DT_BF16) hipLaunchKernelGGL(fill_kernel<bf16_t>, dim3(ew_grid(n, 256)), dim3(256), 0, st, (bf16_t*)out, n, v);
  else hipLaunchKernelGGL(fill_kernel<float>, dim3(ew_grid(n, 256)), dim3(256), 0, st, (float*)out, n, v);
}

}  // namespace ffk

// Box copies for activation transfers (parallel/comm.py): the pack of every region a rank sends
// into one flat buffer, the unpack of a received flat buffer into the destination block, and the
// local block-to-block moves of a re-layout, each as ONE launch over a list of boxes, instead of one
// ATen slice copy per overlap region. Replaces the data movement of the reference's parallel-op
// kernels (src/parallel_ops/kernels/{partition,combine}_kernels.cu: per-region cudaMemcpy-style
// copies) and of concat_kernels.cu's per-input copies.
//
// A box is a rectangular region of up to kBoxDims dimensions with an element offset and strides on
// each side (the flat side has contiguous strides). The host coalesces dimensions contiguous on
// both sides and picks the widest vector (16 / 8 / 4 / 2 / 1 bytes) that divides every inner run,
// stride and offset, so a typical box is 1-3 dims of 16-B vectors. Descriptors live in a small
// device array the host builds once per transfer plan (no per-call H2D copy: graph-capturable).
// Grid: y = box, x = chunks of that box's vectors (grid-stride), 256 threads.
#include "common.h"
#include "ops.h"

namespace ffk {

namespace {

// one box: [src_off, dst_off, numel, ext[kBoxDims], sstr[kBoxDims], dstr[kBoxDims]] (int64, in
// units of the launch's vector), dims innermost last, leading unused dims with extent 1
constexpr int kBoxDims = 6;
constexpr int kBoxWords = 3 + 3 * kBoxDims;

template <typename V>
__global__ void __launch_bounds__(256) box_copy_kernel(const V* __restrict__ src, V* __restrict__ dst,
                                                       const int64_t* __restrict__ desc) {
  const int64_t* d = desc + (int64_t)blockIdx.y * kBoxWords;
  const int64_t n = d[2];
  const int64_t* ext = d + 3;
  const int64_t* ss = ext + kBoxDims;
  const int64_t* ds = ss + kBoxDims;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    int64_t rem = e, so = d[0], dof = d[1];
#pragma unroll
    for (int k = kBoxDims - 1; k >= 0; --k) {
      const int64_t x = ext[k];
      if (x == 1) continue;
      const int64_t q = rem / x, c = rem - q * x;
      so += c * ss[k];
      dof += c * ds[k];
      rem = q;
    }
    dst[dof] = src[so];
  }
}

template <typename T>
__global__ void __launch_bounds__(256) box_add_kernel(const T* __restrict__ src, T* __restrict__ dst,
                                                      const int64_t* __restrict__ desc) {
  const int64_t* d = desc + (int64_t)blockIdx.y * kBoxWords;
  const int64_t n = d[2];
  const int64_t* ext = d + 3;
  const int64_t* ss = ext + kBoxDims;
  const int64_t* ds = ss + kBoxDims;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    int64_t rem = e, so = d[0], dof = d[1];
#pragma unroll
    for (int k = kBoxDims - 1; k >= 0; --k) {
      const int64_t x = ext[k];
      if (x == 1) continue;
      const int64_t q = rem / x, c = rem - q * x;
      so += c * ss[k];
      dof += c * ds[k];
      rem = q;
    }
    dst[dof] = Cvt<T>::from_f(Cvt<T>::to_f(dst[dof]) + Cvt<T>::to_f(src[so]));
  }
}

}  // namespace

int box_words() { return kBoxWords; }
int box_dims() { return kBoxDims; }

// vec_bytes: 16 / 8 / 4 / 2 / 1 (copy) — the unit of every offset, extent and stride in desc;
// add: dt (DT_F32 / DT_BF16), desc in elements. max_n: the largest box (units) — sizes the grid.
void box_copy(const void* src, void* dst, const int64_t* desc, int nbox, int64_t max_n, int vec_bytes, int add,
              int dt, hipStream_t st) {
  if (nbox <= 0 || max_n <= 0) return;
  const int64_t blocks = std::min<int64_t>((max_n + 255) / 256, std::max<int64_t>(1, 8192 / nbox));
  dim3 grid((unsigned)std::max<int64_t>(blocks, 1), (unsigned)nbox);
  if (add) {
    if (dt == DT_F32)
      hipLaunchKernelGGL(box_add_kernel<float>, grid, dim3(256), 0, st, (const float*)src, (float*)dst, desc);
    else
      hipLaunchKernelGGL(box_add_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)src, (bf16_t*)dst, desc);
    return;
  }
  switch (vec_bytes) {
    case 16:
      hipLaunchKernelGGL(box_copy_kernel<uint4>, grid, dim3(256), 0, st, (const uint4*)src, (uint4*)dst, desc);
      break;
    case 8:
      hipLaunchKernelGGL(box_copy_kernel<uint2>, grid, dim3(256), 0, st, (const uint2*)src, (uint2*)dst, desc);
      break;
    case 4:
      hipLaunchKernelGGL(box_copy_kernel<uint32_t>, grid, dim3(256), 0, st, (const uint32_t*)src, (uint32_t*)dst,
                         desc);
      break;
    case 2:
      hipLaunchKernelGGL(box_copy_kernel<uint16_t>, grid, dim3(256), 0, st, (const uint16_t*)src, (uint16_t*)dst,
                         desc);
      break;
    default:
      hipLaunchKernelGGL(box_copy_kernel<uint8_t>, grid, dim3(256), 0, st, (const uint8_t*)src, (uint8_t*)dst, desc);
  }
}

}  // namespace ffk

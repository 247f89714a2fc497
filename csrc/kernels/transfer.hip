// Box copies for activation transfers (parallel/comm.py): the pack of every region a rank sends
// into one flat buffer, the unpack of a received flat buffer into the destination block, and the
// local block-to-block moves of a re-layout, each as ONE launch over a list of boxes, instead of one
// ATen slice copy per overlap region. Replaces the data movement of the reference's parallel-op
// kernels (src/parallel_ops/kernels/{partition,combine}_kernels.cu: per-region cudaMemcpy-style
// copies) and of concat_kernels.cu's per-input copies.
//
// A box is a rectangular region of up to kBoxDims dimensions with an element offset and strides on
// each side (the flat side has contiguous strides; a source stride may be negative: Reverse), read
// from one of up to kBoxSrcs source tensors (Concat's inputs in one launch). The host coalesces dimensions contiguous on
// both sides and picks the widest vector (16 / 8 / 4 / 2 / 1 bytes) that divides every inner run,
// stride and offset, so a typical box is 1-3 dims of 16-B vectors. Descriptors live in a small
// device array the host builds once per transfer plan (no per-call H2D copy: graph-capturable).
// Grid: y = box, x = chunks of that box's vectors (grid-stride), 256 threads.
#include "common.h"
#include "ops.h"

namespace ffk {

namespace {

// one box: [src index, src_off, dst_off, numel, ext[kBoxDims], sstr[kBoxDims], dstr[kBoxDims]]
// (int64, in units of the launch's vector), dims innermost last, leading unused dims with extent 1;
// the source is one of up to kBoxSrcs tensors (a concat's inputs), passed by value per launch
constexpr int kBoxDims = 6;
constexpr int kBoxWords = 4 + 3 * kBoxDims;

struct BoxSrcs {
  const void* p[kBoxSrcs];
};

// IT: int32_t when every offset a launch reaches and every box size fit (the host checks): the
// per-element index math is then 32-bit divisions (~10 VALU each instead of ~60 at 64 bits: the
// 64-bit form made a channel-last concat of 2-B elements compute-bound)
template <typename IT>
__device__ __forceinline__ void box_index(const int64_t* d, IT e, IT& so, IT& dof) {
  const int64_t* ext = d + 4;
  const int64_t* ss = ext + kBoxDims;
  const int64_t* ds = ss + kBoxDims;
  IT rem = e;
  so = (IT)d[1];
  dof = (IT)d[2];
#pragma unroll
  for (int k = kBoxDims - 1; k >= 0; --k) {
    const IT x = (IT)ext[k];
    if (x == 1) continue;
    const IT q = rem / x, c = rem - q * x;
    so += c * (IT)ss[k];
    dof += c * (IT)ds[k];
    rem = q;
  }
}

template <typename V, typename IT>
__global__ void __launch_bounds__(256) box_copy_kernel(BoxSrcs srcs, V* __restrict__ dst,
                                                       const int64_t* __restrict__ desc) {
  const int64_t* d = desc + (int64_t)blockIdx.y * kBoxWords;
  const V* __restrict__ src = reinterpret_cast<const V*>(srcs.p[d[0]]);
  const IT n = (IT)d[3];
  for (IT e = (IT)blockIdx.x * 256 + (IT)threadIdx.x; e < n; e += (IT)gridDim.x * 256) {
    IT so, dof;
    box_index<IT>(d, e, so, dof);
    dst[dof] = src[so];
  }
}

template <typename T>
__global__ void __launch_bounds__(256) box_add_kernel(BoxSrcs srcs, T* __restrict__ dst,
                                                      const int64_t* __restrict__ desc) {
  const int64_t* d = desc + (int64_t)blockIdx.y * kBoxWords;
  const T* __restrict__ src = reinterpret_cast<const T*>(srcs.p[d[0]]);
  const int64_t n = d[3];
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    int64_t so, dof;
    box_index<int64_t>(d, e, so, dof);
    dst[dof] = Cvt<T>::from_f(Cvt<T>::to_f(dst[dof]) + Cvt<T>::to_f(src[so]));
  }
}

}  // namespace

int box_words() { return kBoxWords; }
int box_dims() { return kBoxDims; }

// vec_bytes: 16 / 8 / 4 / 2 / 1 (copy) — the unit of every offset, extent and stride in desc;
// add: dt (DT_F32 / DT_BF16), desc in elements. max_n: the largest box (units) — sizes the grid.
void box_copy(const void* const* srcs, int nsrc, void* dst, const int64_t* desc, int nbox, int64_t max_n,
              int vec_bytes, int add, int dt, int idx32, hipStream_t st) {
  if (nbox <= 0 || max_n <= 0 || nsrc <= 0 || nsrc > kBoxSrcs) return;
  BoxSrcs s{};
  for (int i = 0; i < nsrc; ++i) s.p[i] = srcs[i];
  const int64_t blocks = std::min<int64_t>((max_n + 255) / 256, std::max<int64_t>(1, 8192 / nbox));
  dim3 grid((unsigned)std::max<int64_t>(blocks, 1), (unsigned)nbox);
  if (add) {
    if (dt == DT_F32) hipLaunchKernelGGL(box_add_kernel<float>, grid, dim3(256), 0, st, s, (float*)dst, desc);
    else hipLaunchKernelGGL(box_add_kernel<bf16_t>, grid, dim3(256), 0, st, s, (bf16_t*)dst, desc);
    return;
  }
  auto go = [&](auto vtag, auto itag) {
    using V = decltype(vtag);
    using IT = decltype(itag);
    hipLaunchKernelGGL((box_copy_kernel<V, IT>), grid, dim3(256), 0, st, s, (V*)dst, desc);
  };
  auto by_width = [&](auto itag) {
    switch (vec_bytes) {
      case 16: go(uint4{}, itag); break;
      case 8: go(uint2{}, itag); break;
      case 4: go(uint32_t{}, itag); break;
      case 2: go(uint16_t{}, itag); break;
      default: go(uint8_t{}, itag);
    }
  };
  if (idx32) by_width(int32_t{});
  else by_width(int64_t{});
}

// ------------------------------------------------------------------------------- concat
// Concat of dense inputs viewed as rows: x_i [outer][len_i] -> out [outer][row], row = sum len_i,
// input i at column off_i (units of V: 16 / 8 / 4 / 2 B). A contiguous tensor concatenated along
// dim a has outer = prod(shape[:a]); a channel-last [N, C, H, W] along C has outer = N*H*W and
// len_i = C_i — the NHWC channel concat of Inception's blocks. grid.y = input (its pointer, offset
// and length are uniform per workgroup), grid.x strides over that input's outer * len_i vectors:
// contiguous reads, writes in runs of len_i vectors, one 32-bit division per vector (the generic
// box kernel's 6-dim index math made this concat 0.4 ms/step slower than torch.cat, r5).
struct CatSrcs {
  const void* p[kBoxSrcs];
  int off[kBoxSrcs];
  int len[kBoxSrcs];
};

template <typename V>
__global__ void __launch_bounds__(256) concat_rows_kernel(CatSrcs s, V* __restrict__ out, int outer, int row) {
  const int i = blockIdx.y;
  const V* __restrict__ src = reinterpret_cast<const V*>(s.p[i]);
  const int len = s.len[i], off = s.off[i];
  const int n = outer * len;  // < 2^31 (host check)
  for (int e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) {
    const int o = e / len;
    out[(int64_t)o * row + off + (e - o * len)] = src[e];
  }
}

void concat_rows(const void* const* srcs, const int* lens, int nsrc, void* out, int outer, int vec_bytes,
                 hipStream_t st) {
  if (nsrc <= 0 || nsrc > kBoxSrcs || outer <= 0) return;
  CatSrcs s{};
  int row = 0, mx = 0;
  for (int i = 0; i < nsrc; ++i) {
    s.p[i] = srcs[i];
    s.off[i] = row;
    s.len[i] = lens[i];
    row += lens[i];
    mx = std::max(mx, lens[i]);
  }
  const int64_t blocks = std::min<int64_t>(((int64_t)outer * mx + 255) / 256, std::max<int64_t>(1, 8192 / nsrc));
  const dim3 grid((unsigned)std::max<int64_t>(blocks, 1), (unsigned)nsrc);
  switch (vec_bytes) {
    case 16: hipLaunchKernelGGL(concat_rows_kernel<uint4>, grid, dim3(256), 0, st, s, (uint4*)out, outer, row); break;
    case 8: hipLaunchKernelGGL(concat_rows_kernel<uint2>, grid, dim3(256), 0, st, s, (uint2*)out, outer, row); break;
    case 4: hipLaunchKernelGGL(concat_rows_kernel<uint32_t>, grid, dim3(256), 0, st, s, (uint32_t*)out, outer, row); break;
    default: hipLaunchKernelGGL(concat_rows_kernel<uint16_t>, grid, dim3(256), 0, st, s, (uint16_t*)out, outer, row);
  }
}

// ------------------------------------------------------------------------------- transpose
// dst [cols][rows] = src [rows][cols]^T for 2-byte elements, rows % 8 == 0 and cols % 8 == 0 (host
// check). The Linear layers keep a transposed bf16 copy of each weight, refreshed every training
// forward, so the input-gradient GEMM dx = dy . W reads W^T K-contiguous ("TN") instead of
// N-contiguous ("NN"): on MI355X the library's TN GEMM of BERT-Large's dgrad shapes is 14-25 %
// faster than its NN form (tuning/tunableop_gfx950.csv) and our ping-pong kernel's K-contiguous
// B path avoids the transposing LDS reads altogether. One 64 x 64 tile per workgroup through LDS:
// 16-B loads along source rows, 16-B stores along destination rows; the LDS row pitch of 72
// elements (144 B) keeps every 16-B chunk aligned and spreads the column reads over the banks.
// Grid: one workgroup per tile, or (max_blocks > 0) at most max_blocks workgroups striding over the
// tiles. (Refreshing on a side stream beside the forward GEMMs was measured slower than on the
// compute stream, with the full grid and with a 16-workgroup cap: kernels/__init__.py weight_t.)
// one 64 x 64 tile (r0, c0) of dst = src^T through the LDS image t (72-element row pitch)
__device__ __forceinline__ void transpose16_tile(const uint16_t* __restrict__ src, uint16_t* __restrict__ dst,
                                                 int rows, int cols, int r0, int c0, uint16_t* t) {
  constexpr int P = 72;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int id = threadIdx.x + 256 * j, r = id >> 3, ch = id & 7;
    uint4 v = {0u, 0u, 0u, 0u};
    if (r0 + r < rows && c0 + 8 * ch < cols)
      v = *reinterpret_cast<const uint4*>(src + (int64_t)(r0 + r) * cols + c0 + 8 * ch);
    *reinterpret_cast<uint4*>(t + r * P + 8 * ch) = v;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int id = threadIdx.x + 256 * j, oc = id >> 3, ch = id & 7;
    if (c0 + oc >= cols || r0 + 8 * ch >= rows) continue;
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      w[e] = (uint32_t)t[(8 * ch + 2 * e) * P + oc] | ((uint32_t)t[(8 * ch + 2 * e + 1) * P + oc] << 16);
    *reinterpret_cast<uint4*>(dst + (int64_t)(c0 + oc) * rows + r0 + 8 * ch) = uint4{w[0], w[1], w[2], w[3]};
  }
}

__global__ void __launch_bounds__(256) transpose16_kernel(const uint16_t* __restrict__ src,
                                                          uint16_t* __restrict__ dst, int rows, int cols) {
  __shared__ __attribute__((aligned(16))) uint16_t t[64 * 72];
  const int tc = (cols + 63) / 64;
  transpose16_tile(src, dst, rows, cols, (blockIdx.x / tc) * 64, (blockIdx.x % tc) * 64, t);
}

void transpose16(const void* src, void* dst, int rows, int cols, hipStream_t st) {
  if (rows <= 0 || cols <= 0) return;
  const int tiles = ((cols + 63) / 64) * ((rows + 63) / 64);
  hipLaunchKernelGGL(transpose16_kernel, dim3((unsigned)tiles), dim3(256), 0, st, (const uint16_t*)src, (uint16_t*)dst,
                     rows, cols);
}

// Every registered W^T of a model in ONE launch (the executor refreshes them at the start of each
// training forward): desc[i] = {src, dst, rows, cols, first tile}, tiles of matrix i numbered from
// its first tile; a workgroup finds its matrix by binary search over the n first-tile entries. The
// per-weight launches cost 5-6 us each at ~3 TB/s on BERT-Large's 4M-element weights (98 per step).
__global__ void __launch_bounds__(256) transpose16_batch_kernel(const int64_t* __restrict__ desc, int n) {
  __shared__ __attribute__((aligned(16))) uint16_t t[64 * 72];
  const int64_t tile = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {  // last matrix whose first tile <= tile
    const int mid = (lo + hi + 1) >> 1;
    if (desc[mid * 5 + 4] <= tile) lo = mid;
    else hi = mid - 1;
  }
  const int64_t* d = desc + lo * 5;
  const int rows = (int)d[2], cols = (int)d[3];
  const int tc = (cols + 63) / 64, k = (int)(tile - d[4]);
  transpose16_tile(reinterpret_cast<const uint16_t*>(d[0]), reinterpret_cast<uint16_t*>(d[1]), rows, cols,
                   (k / tc) * 64, (k % tc) * 64, t);
}

void transpose16_batch(const int64_t* desc, int n, int64_t tiles, hipStream_t st) {
  if (n <= 0 || tiles <= 0) return;
  hipLaunchKernelGGL(transpose16_batch_kernel, dim3((unsigned)tiles), dim3(256), 0, st, desc, n);
}

// ------------------------------------------------------------------------------- gather
// torch.gather along one dim of contiguous tensors whose other dims match (reference
// src/ops/gather.cc / kernels): out[o][j][i] = x[o][idx[o][j][i]][i]; the backward adds dy into an
// fp32 dx at the same positions (float atomics: indices may repeat, as in the reference's
// atomicAdd-based backward). Indices are clamped to the dim (an out-of-range index is a user
// error torch would raise on; here it must not become an out-of-bounds access).
template <typename T, typename I>
__global__ void __launch_bounds__(256) gather_fwd_kernel(const T* __restrict__ x, const I* __restrict__ idx,
                                                         T* __restrict__ out, int64_t n, int64_t dsz, int64_t inner,
                                                         int64_t xd) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int64_t o = e / (dsz * inner), i = e % inner;
    int64_t k = (int64_t)idx[e];
    k = k < 0 ? 0 : (k >= xd ? xd - 1 : k);
    out[e] = x[(o * xd + k) * inner + i];
  }
}

template <typename T, typename I>
__global__ void __launch_bounds__(256) gather_bwd_kernel(const T* __restrict__ dy, const I* __restrict__ idx,
                                                         float* __restrict__ dx, int64_t n, int64_t dsz, int64_t inner,
                                                         int64_t xd) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int64_t o = e / (dsz * inner), i = e % inner;
    int64_t k = (int64_t)idx[e];
    k = k < 0 ? 0 : (k >= xd ? xd - 1 : k);
    atomicAdd(dx + (o * xd + k) * inner + i, Cvt<T>::to_f(dy[e]));
  }
}

void gather_fwd(int dt, int idx64, const void* x, const void* idx, void* out, int64_t n, int64_t dsz, int64_t inner,
                int64_t xd, hipStream_t st) {
  if (n <= 0) return;
  const dim3 grid(ew_grid(n, 256));
  auto go = [&](auto tag) {
    using T = decltype(tag);
    if (idx64) hipLaunchKernelGGL((gather_fwd_kernel<T, int64_t>), grid, dim3(256), 0, st, (const T*)x,
                                  (const int64_t*)idx, (T*)out, n, dsz, inner, xd);
    else hipLaunchKernelGGL((gather_fwd_kernel<T, int32_t>), grid, dim3(256), 0, st, (const T*)x, (const int32_t*)idx,
                            (T*)out, n, dsz, inner, xd);
  };
  if (dt == DT_BF16) go(bf16_t{});
  else go(float{});
}

void gather_bwd(int dt, int idx64, const void* dy, const void* idx, float* dx, int64_t n, int64_t dsz, int64_t inner,
                int64_t xd, hipStream_t st) {
  if (n <= 0) return;
  const dim3 grid(ew_grid(n, 256));
  auto go = [&](auto tag) {
    using T = decltype(tag);
    if (idx64) hipLaunchKernelGGL((gather_bwd_kernel<T, int64_t>), grid, dim3(256), 0, st, (const T*)dy,
                                  (const int64_t*)idx, dx, n, dsz, inner, xd);
    else hipLaunchKernelGGL((gather_bwd_kernel<T, int32_t>), grid, dim3(256), 0, st, (const T*)dy,
                            (const int32_t*)idx, dx, n, dsz, inner, xd);
  };
  if (dt == DT_BF16) go(bf16_t{});
  else go(float{});
}

}  // namespace ffk

// Large-tile bf16 MFMA GEMM (256x128x64, 8 waves) with direct global->LDS DMA staging.
//
// Same math / layouts / epilogue contract as gemm.hip (A_K / B_K operand orientations, fused
// bias + activation + pre-activation store, beta accumulate, fp32 split-K partials), but built for
// the MI355X regime where the 128x128 register-staged kernel is L2-bandwidth bound
// (64 B/clk/CU of operand traffic at full MFMA rate vs ~47 here):
//   * tile 256(M) x 128(N) x 64(K), 512 threads = 8 waves as 4(M) x 2(N), 64x64 per wave
//     (4x4 mfma_f32_16x16x32_bf16 fragments, operands swapped so lanes own 4 output columns);
//     M = 8192-token BERT GEMMs with N = 1024 give exactly 256 tiles = one per CU;
//   * operands land in LDS by buffer_load ... lds (LDS-DMA, 16 B/lane, 1 KiB per wave
//     instruction): no staging VGPRs, hardware range check (num_records) zero-fills reads past
//     the end of the buffer so edge tiles never fault;
//   * conflict-free images written through the SOURCE address (rule 21: linear LDS destination,
//     inverse-swizzled global source, same XOR on the read): K-contiguous tiles as 128-B rows with
//     chunk ^ (row & 7) read by ds_read_b128; MN-contiguous tiles as 128-wide halves of 256-B
//     rows with the T10 image (b) XOR read by ds_read_b64_tr_b16;
//   * 3-stage LDS ring (3 x 48 KiB), counted `s_waitcnt vmcnt(6)` + raw s_barrier so the next
//     tile's DMA stays in flight across the barrier (cdna_hip_programming.md §5 "Pipelining
//     across barriers"; never __syncthreads in the loop, all LDS in one __shared__ array);
//   * XCD-aware bijective block remap + GROUP_M=8 ordering for L2 reuse; s_setprio around the
//     MFMA clusters (T5).
// Requires: 16-B aligned operand rows, K % 64 == 0 (a K tile never straddles rows), operands
// < 4 GiB. Anything else goes to gemm.hip.
#include "common.h"
#include "gemm.h"

namespace ffk {
namespace big {

constexpr int BM = 256, BN = 128, BK = 64, NT = 512;
constexpr int A_BYTES = BM * BK * 2;   // 32 KiB
constexpr int B_BYTES = BN * BK * 2;   // 16 KiB
constexpr int STAGE = A_BYTES + B_BYTES;
constexpr int NSTAGE = 3;

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ int swz_mn(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

// Issue the LDS-DMA loads of one operand tile. ROWS = extent along M (or N).
// K-contiguous: image [ROWS][64] with 128-B rows, piece = 8 rows.
// MN-contiguous: image [ROWS/128][64][128] (256-B rows), piece = 4 rows of one half.
template <bool KCONT, int ROWS>
__device__ __forceinline__ void dma_tile(__amdgpu_buffer_rsrc_t rsrc, char* lds, int64_t ld, int mn0, int k0,
                                         int wave, int lane) {
  constexpr int PIECES = ROWS * BK * 2 / 1024;
  constexpr int PER_WAVE = PIECES / 8;
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int piece = wave * PER_WAVE + i;
    int64_t elem;
    if (KCONT) {
      const int row = piece * 8 + (lane >> 3);
      const int pc = lane & 7;
      const int c = pc ^ (row & 7);
      elem = (int64_t)(mn0 + row) * ld + k0 + c * 8;
    } else {
      const int half = piece / 16;          // 16 pieces (64 rows x 256 B) per 128-wide half
      const int row = (piece % 16) * 4 + (lane >> 4);
      const int pc = lane & 15;
      const int c = pc ^ swz_mn(row);
      elem = (int64_t)(k0 + row) * ld + mn0 + half * 128 + c * 8;
    }
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_ptr_t)(lds + piece * 1024), 16, (int)(elem * 2), 0, 0, 0);
  }
}

template <bool KCONT>
__device__ __forceinline__ bf16x8 frag(const char* lds, int r0, int kk, int lane) {
  if (KCONT) {
    const int row = r0 + (lane & 15);
    const int c = kk * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(lds + row * 128 + ((c ^ (row & 7)) << 4));
  } else {
    const char* hl = lds + (r0 >> 7) * (BK * 256);
    const int rr = r0 & 127;
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int chunk = (rr >> 3) + (p >> 1);
    bf16x8 out;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int krow = 32 * kk + 8 * g + 4 * hf + q;
      const int off = krow * 256 + ((chunk ^ swz_mn(krow)) << 4) + 8 * (p & 1);
      typedef short v4s __attribute__((ext_vector_type(4)));
      v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(hl + off));
      bf16x4 b = __builtin_bit_cast(bf16x4, v);
      out[4 * hf + 0] = b[0];
      out[4 * hf + 1] = b[1];
      out[4 * hf + 2] = b[2];
      out[4 * hf + 3] = b[3];
    }
    return out;
  }
}

__device__ __forceinline__ void tile_coords(int bid, int tm, int tn, int& tile_m, int& tile_n) {
  const int nwg = tm * tn;
  bid = xcd_remap(bid, nwg);
  constexpr int GM = 8;
  const int per_group = GM * tn;
  const int group = bid / per_group;
  const int first_m = group * GM;
  const int gsize = min(tm - first_m, GM);
  const int in_g = bid % per_group;
  tile_m = first_m + in_g % gsize;
  tile_n = in_g / gsize;
}

template <bool A_K, bool B_K, int OUT_MODE>
__global__ void __launch_bounds__(NT, 1) gemm_big_kernel(GemmArgs p, int64_t a_bytes, int64_t b_bytes) {
  __shared__ __attribute__((aligned(16))) char smem[NSTAGE * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int tm = (p.M + BM - 1) / BM, tn = (p.N + BN - 1) / BN;
  int tile_m, tile_n;
  tile_coords(blockIdx.x, tm, tn, tile_m, tile_n);
  const int z = blockIdx.y;
  const int b = z / p.splitk, ks = z % p.splitk;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int kbeg = ks * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const int nk = (kend - kbeg + BK - 1) / BK;

  const bf16_t* Ab = p.A + (int64_t)b * p.sA;
  const bf16_t* Bb = p.B + (int64_t)b * p.sB;
  // range-checked descriptors over the rest of each operand buffer (reads past it return 0)
  const int64_t a_rem = a_bytes - (int64_t)b * p.sA * 2;
  const int64_t b_rem = b_bytes - (int64_t)b * p.sB * 2;
  __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)Ab, (short)0, (int)min(a_rem, (int64_t)0x7fffffff), 0x00020000);
  __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, (short)0, (int)min(b_rem, (int64_t)0x7fffffff), 0x00020000);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int t) {
    char* st = smem + (t % NSTAGE) * STAGE;
    const int k0 = kbeg + t * BK;
    dma_tile<A_K, BM>(ra, st, p.lda, m0, k0, wave, lane);
    dma_tile<B_K, BN>(rb, st + A_BYTES, p.ldb, n0, k0, wave, lane);
  };
  if (nk > 0) issue(0);
  if (nk > 1) issue(1);
  for (int t = 0; t < nk; ++t) {
    if (t + 1 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + 2 < nk) issue(t + 2);
    const char* cur = smem + (t % NSTAGE) * STAGE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag<B_K>(cur + A_BYTES, wn * 64 + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag<A_K>(cur, wm * 64 + i * 16, kk, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }

  const int mrow = m0 + wm * 64 + (lane & 15);
  const int ncol = n0 + wn * 64 + (lane >> 4) * 4;
  if (OUT_MODE == 2) {
    float* W = p.ws + (int64_t)z * p.M * p.N;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = mrow + i * 16;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = ncol + j * 16;
        float* dst = W + (int64_t)m * p.N + n;
        if (n + 3 < p.N && (p.N & 3) == 0) {
          *reinterpret_cast<float4*>(dst) = make_float4(acc[i][j][0] * p.alpha, acc[i][j][1] * p.alpha,
                                                        acc[i][j][2] * p.alpha, acc[i][j][3] * p.alpha);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) if (n + r < p.N) dst[r] = acc[i][j][r] * p.alpha;
        }
      }
    }
    return;
  }
  typedef typename std::conditional<OUT_MODE == 0, bf16_t, float>::type OutT;
  OutT* C = reinterpret_cast<OutT*>(p.C) + (int64_t)b * p.sC;
  bf16_t* Zp = p.Z ? reinterpret_cast<bf16_t*>(p.Z) + (int64_t)b * p.sC : nullptr;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = mrow + i * 16;
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = ncol + j * 16;
      if (n >= p.N) continue;
      float v[4];
      const bool full = p.vec_ok && (n + 3 < p.N);
      OutT* dst = C + (int64_t)m * p.ldc + n;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float x = acc[i][j][r] * p.alpha;
        if (p.beta != 0.f && n + r < p.N) x += p.beta * Cvt<OutT>::to_f(dst[r]);
        if (p.bias && n + r < p.N)
          x += p.bias_bf16 ? bf2f(((const bf16_t*)p.bias)[n + r]) : ((const float*)p.bias)[n + r];
        v[r] = x;
      }
      if (Zp) {
        bf16_t* zd = Zp + (int64_t)m * p.ldc + n;
        if (full) {
          ushort4 o; o.x = f2bf(v[0]); o.y = f2bf(v[1]); o.z = f2bf(v[2]); o.w = f2bf(v[3]);
          *reinterpret_cast<ushort4*>(zd) = o;
        } else {
          for (int r = 0; r < 4; ++r) if (n + r < p.N) zd[r] = f2bf(v[r]);
        }
      }
      if (p.act != ACT_NONE) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = act_fwd(p.act, v[r]);
      }
      if (full) {
        if (OUT_MODE == 0) {
          ushort4 o; o.x = f2bf(v[0]); o.y = f2bf(v[1]); o.z = f2bf(v[2]); o.w = f2bf(v[3]);
          *reinterpret_cast<ushort4*>(dst) = o;
        } else {
          *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) if (n + r < p.N) dst[r] = Cvt<OutT>::from_f(v[r]);
      }
    }
  }
}

template <int MODE>
static void launch(const GemmArgs& p, dim3 grid, hipStream_t s, int64_t ab, int64_t bb) {
  if (p.a_kcontig && p.b_kcontig) hipLaunchKernelGGL((gemm_big_kernel<true, true, MODE>), grid, dim3(NT), 0, s, p, ab, bb);
  else if (p.a_kcontig) hipLaunchKernelGGL((gemm_big_kernel<true, false, MODE>), grid, dim3(NT), 0, s, p, ab, bb);
  else if (p.b_kcontig) hipLaunchKernelGGL((gemm_big_kernel<false, true, MODE>), grid, dim3(NT), 0, s, p, ab, bb);
  else hipLaunchKernelGGL((gemm_big_kernel<false, false, MODE>), grid, dim3(NT), 0, s, p, ab, bb);
}

}  // namespace big

// Returns false if the shape/alignment is not eligible (caller uses the 128x128 kernel).
bool gemm_big_bf16(const GemmArgs& p0, int64_t a_bytes, int64_t b_bytes, hipStream_t stream) {
  using namespace big;
  GemmArgs p = p0;
  if (p.K % BK != 0 || a_bytes > 0x7fffffffLL || b_bytes > 0x7fffffffLL) return false;
  if (((uintptr_t)p.A & 15) || ((uintptr_t)p.B & 15) || p.lda % 8 || p.ldb % 8 || p.sA % 8 || p.sB % 8) return false;
  if (!p.a_kcontig && p.M % 8) return false;
  if (!p.b_kcontig && p.N % 8) return false;
  const int tm = (p.M + BM - 1) / BM, tn = (p.N + BN - 1) / BN;
  if ((int64_t)tm * tn * p.batch * p.splitk < 128) return false;  // too few tiles: 128x128 kernel fills better
  if (p.splitk > 1 && p.ws != nullptr) {
    p.kchunk = ((p.K + p.splitk - 1) / p.splitk + BK - 1) / BK * BK;
    dim3 grid(tm * tn, p.batch * p.splitk);
    launch<2>(p, grid, stream, a_bytes, b_bytes);
    return true;  // caller runs the reduction
  }
  p.splitk = 1;
  p.kchunk = p.K;
  dim3 grid(tm * tn, p.batch);
  if (p.out_f32) launch<1>(p, grid, stream, a_bytes, b_bytes);
  else launch<0>(p, grid, stream, a_bytes, b_bytes);
  return true;
}

}  // namespace ffk

// bf16 MFMA GEMM for gfx950 with fused epilogues.
//
//   C[b] = act( alpha * op(A[b]) . op(B[b])  + beta * C[b] + bias )      (fp32 accumulate)
//
// Operand layouts (template flags):
//   A_K = true : A is [M][K] row-major (K contiguous)      A_K = false : A is [K][M] (M contiguous)
//   B_K = true : B is [N][K] row-major (K contiguous)      B_K = false : B is [K][N] (N contiguous)
// so Linear forward (X.W^T) is <true,true>, dgrad (dY.W) is <true,false> and wgrad (dY^T.X) is
// <false,false>, all without materialising a transpose.
//
// Structure (cdna_hip_programming.md §5): 128x128x64 tile, 4 waves (2x2), each wave 64x64 via
// 4x4 mfma_f32_16x16x32_bf16 fragments; register-staged double-buffered LDS (global_load_dwordx4
// issued before the MFMAs of the current tile, ds_write after them, one barrier per K-tile).
// K-contiguous tiles are stored as 128-B rows with chunk ^= row&7 (conflict-free ds_read_b128);
// MN-contiguous tiles as 256-B rows with the dual-use XOR of T10 image (b), read with
// ds_read_b64_tr_b16 so the hardware does the transpose. Fragments are fed as MFMA(B, A) so the
// accumulator holds 4 consecutive output columns per lane -> 8/16-B epilogue stores.
// Block ids are remapped XCD-aware (T1, bijective) and grouped along M for L2 reuse.
// Split-K writes fp32 partial slabs that a second kernel reduces and finishes the epilogue.
//
// Replaces the reference's cuBLAS Linear/BatchMatmul kernels
// (reference: src/ops/kernels/linear_kernels.cu forward_kernel/backward_kernel,
//  src/ops/batch_matmul.cu).
#include "common.h"
#include "gemm.h"
#include "ops.h"

namespace ffk {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE_BYTES = BM * BK * 2;  // 16 KiB per operand tile

__device__ __forceinline__ int swz_mn(int row) {  // 256-B row image, T10 (b)
  return ((row & 3) << 2) | ((row >> 2) & 3);
}

// ALIGNED: rows of the contiguous dim start 16-B aligned and its extent is a multiple of 8, so a
// whole 8-element chunk is in or out of bounds and loads as one dwordx4. Otherwise (e.g. a 30522-
// wide vocab projection) each element is bounds-checked and loaded as a 16-bit value — only the
// operand that needs it pays, the MFMA/LDS pipeline is unchanged.
template <bool KCONT, int ROWS, bool ALIGNED = true>
struct Stager {
  // ROWS = 128 (the M or N extent of the tile)
  uint4 r[4];
  // g: operand base for this batch; ld: leading dim; mn0/k0 tile origin; mn_lim/k_lim bounds
  __device__ __forceinline__ void load(const bf16_t* __restrict__ g, int64_t ld, int mn0, int k0,
                                       int mn_lim, int k_lim, int tid) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int id = tid + i * NT;
      int mn, kk;
      if (KCONT) { mn = id >> 3; kk = (id & 7) * 8; }
      else { kk = id >> 4; mn = (id & 15) * 8; }
      const int gm = mn0 + mn, gk = k0 + kk;
      if (ALIGNED) {
        bool ok = KCONT ? (gm < mn_lim && gk < k_lim) : (gk < k_lim && gm < mn_lim);
        if (ok) {
          const bf16_t* p = KCONT ? g + (int64_t)gm * ld + gk : g + (int64_t)gk * ld + gm;
          r[i] = *reinterpret_cast<const uint4*>(p);
        } else {
          r[i] = make_uint4(0, 0, 0, 0);
        }
      } else {
        uint16_t e[8];
        if (KCONT) {
          const bool rok = gm < mn_lim;
          const bf16_t* p = g + (int64_t)gm * ld;
#pragma unroll
          for (int j = 0; j < 8; ++j) e[j] = (rok && gk + j < k_lim) ? p[gk + j] : (uint16_t)0;
        } else {
          const bool kok = gk < k_lim;
          const bf16_t* p = g + (int64_t)gk * ld;
#pragma unroll
          for (int j = 0; j < 8; ++j) e[j] = (kok && gm + j < mn_lim) ? p[gm + j] : (uint16_t)0;
        }
        r[i].x = e[0] | ((uint32_t)e[1] << 16);
        r[i].y = e[2] | ((uint32_t)e[3] << 16);
        r[i].z = e[4] | ((uint32_t)e[5] << 16);
        r[i].w = e[6] | ((uint32_t)e[7] << 16);
      }
    }
  }
  __device__ __forceinline__ void store(char* lds, int tid) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int id = tid + i * NT;
      int off;
      if (KCONT) {
        const int row = id >> 3, c = id & 7;
        off = row * 128 + ((c ^ (row & 7)) << 4);
      } else {
        const int row = id >> 4, c = id & 15;
        off = row * 256 + ((c ^ swz_mn(row)) << 4);
      }
      *reinterpret_cast<uint4*>(lds + off) = r[i];
    }
  }
};

// Read one 16x32 (rows x k) bf16 fragment for mfma_16x16x32: lane holds row r0+(l&15),
// k = 32*kk + 8*(l>>4) + j, j=0..7.
template <bool KCONT>
__device__ __forceinline__ bf16x8 read_frag(const char* lds, int r0, int kk, int lane) {
  if (KCONT) {
    const int row = r0 + (lane & 15);
    const int c = kk * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(lds + row * 128 + ((c ^ (row & 7)) << 4));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int chunk = (r0 >> 3) + (p >> 1);
    bf16x8 out;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int krow = 32 * kk + 8 * g + 4 * hf + q;
      const int off = krow * 256 + ((chunk ^ swz_mn(krow)) << 4) + 8 * (p & 1);
      typedef short v4s __attribute__((ext_vector_type(4)));
      v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) v4s*)(lds + off));
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

// OUT_MODE: 0 = bf16 output with full epilogue, 1 = fp32 output with full epilogue,
//           2 = fp32 split-K partial (alpha only, no beta/bias/act)
template <bool A_K, bool B_K, int OUT_MODE, bool A_AL = true, bool B_AL = true>
__global__ void __launch_bounds__(NT, 2) gemm_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tm = (p.M + BM - 1) / BM, tn = (p.N + BN - 1) / BN;
  int tile_m, tile_n;
  tile_coords(blockIdx.x, tm, tn, tile_m, tile_n);
  const int z = blockIdx.y;
  const int b = z / p.splitk, ks = z % p.splitk;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  const bf16_t* Ab = p.A + (int64_t)b * p.sA;
  const bf16_t* Bb = p.B + (int64_t)b * p.sB;
  const int kbeg = ks * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const int nk = (kend - kbeg + BK - 1) / BK;

  Stager<A_K, BM, A_AL> sa;
  Stager<B_K, BN, B_AL> sb;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    sa.load(Ab, p.lda, m0, kbeg, p.M, kend, tid);
    sb.load(Bb, p.ldb, n0, kbeg, p.N, kend, tid);
    sa.store(smem, tid);
    sb.store(smem + TILE_BYTES, tid);
    __syncthreads();
  }
  for (int t = 0; t < nk; ++t) {
    char* cur = smem + (t & 1) * 2 * TILE_BYTES;
    char* nxt = smem + ((t + 1) & 1) * 2 * TILE_BYTES;
    const bool more = (t + 1) < nk;
    if (more) {
      const int k1 = kbeg + (t + 1) * BK;
      sa.load(Ab, p.lda, m0, k1, p.M, kend, tid);
      sb.load(Bb, p.ldb, n0, k1, p.N, kend, tid);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag<A_K>(cur, wm * 64 + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = read_frag<B_K>(cur + TILE_BYTES, wn * 64 + j * 16, kk, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    if (more) {
      sa.store(nxt, tid);
      sb.store(nxt + TILE_BYTES, tid);
    }
    __syncthreads();
  }

  // Epilogue: lane holds C[m][n..n+3], m = m0+wm*64+i*16+(lane&15), n = n0+wn*64+j*16+(lane>>4)*4.
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
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] * p.alpha;
        float* dst = W + (int64_t)m * p.N + n;
        if (n + 3 < p.N && (p.N & 3) == 0) {
          *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) if (n + r < p.N) dst[r] = v[r];
        }
      }
    }
    return;
  }
  typedef typename std::conditional<OUT_MODE == 0, bf16_t, float>::type OutT;
  OutT* C = reinterpret_cast<OutT*>(p.C) + (int64_t)b * p.sC;
  bf16_t* Zp = p.Z ? reinterpret_cast<bf16_t*>(p.Z) + (int64_t)b * p.sC : nullptr;
  const bool vec_ok = p.vec_ok;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = mrow + i * 16;
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = ncol + j * 16;
      if (n >= p.N) continue;
      float v[4];
      const bool full = vec_ok && (n + 3 < p.N);
      OutT* dst = C + (int64_t)m * p.ldc + n;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float x = acc[i][j][r] * p.alpha;
        if (p.beta != 0.f && n + r < p.N) x += p.beta * Cvt<OutT>::to_f(dst[r]);
        if (p.bias && n + r < p.N) x += p.bias_bf16 ? bf2f(((const bf16_t*)p.bias)[n + r]) : ((const float*)p.bias)[n + r];
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

// Split-K reduction + epilogue: ws holds batch*splitk slabs of [M][N] fp32.
template <typename OutT>
__global__ void splitk_reduce_kernel(GemmArgs p) {
  const int64_t MN = (int64_t)p.M * p.N;
  const int64_t total = MN * p.batch;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int b = idx / MN;
    const int64_t e = idx % MN;
    const int m = e / p.N, n = e % p.N;
    float x = 0.f;
    const float* w = p.ws + (int64_t)b * p.splitk * MN + e;
    for (int s = 0; s < p.splitk; ++s) x += w[(int64_t)s * MN];
    OutT* C = reinterpret_cast<OutT*>(p.C) + (int64_t)b * p.sC + (int64_t)m * p.ldc + n;
    if (p.beta != 0.f) x += p.beta * Cvt<OutT>::to_f(*C);
    if (p.bias) x += p.bias_bf16 ? bf2f(((const bf16_t*)p.bias)[n]) : ((const float*)p.bias)[n];
    if (p.Z) reinterpret_cast<bf16_t*>(p.Z)[(int64_t)b * p.sC + (int64_t)m * p.ldc + n] = f2bf(x);
    *C = Cvt<OutT>::from_f(act_fwd(p.act, x));
  }
}

// Generic (unaligned / tiny) fallback: 16x16 threads, fp32 accumulate, any layout.
template <typename OutT>
__global__ void gemm_fallback_kernel(GemmArgs p, bool a_k, bool b_k) {
  const int b = blockIdx.z;
  const int m = blockIdx.y * 16 + threadIdx.y;
  const int n = blockIdx.x * 16 + threadIdx.x;
  if (m >= p.M || n >= p.N) return;
  const bf16_t* A = p.A + (int64_t)b * p.sA;
  const bf16_t* B = p.B + (int64_t)b * p.sB;
  float acc = 0.f;
  for (int k = 0; k < p.K; ++k) {
    float a = bf2f(a_k ? A[(int64_t)m * p.lda + k] : A[(int64_t)k * p.lda + m]);
    float bb = bf2f(b_k ? B[(int64_t)n * p.ldb + k] : B[(int64_t)k * p.ldb + n]);
    acc += a * bb;
  }
  OutT* C = reinterpret_cast<OutT*>(p.C) + (int64_t)b * p.sC + (int64_t)m * p.ldc + n;
  float x = acc * p.alpha;
  if (p.beta != 0.f) x += p.beta * Cvt<OutT>::to_f(*C);
  if (p.bias) x += p.bias_bf16 ? bf2f(((const bf16_t*)p.bias)[n]) : ((const float*)p.bias)[n];
  if (p.Z) reinterpret_cast<bf16_t*>(p.Z)[(int64_t)b * p.sC + (int64_t)m * p.ldc + n] = f2bf(x);
  *C = Cvt<OutT>::from_f(act_fwd(p.act, x));
}

template <bool AK, bool BK_, int MODE>
static void launch_tiled(const GemmArgs& p, dim3 grid, hipStream_t s, bool a_al, bool b_al) {
  if (a_al && b_al) hipLaunchKernelGGL((gemm_kernel<AK, BK_, MODE, true, true>), grid, dim3(NT), 0, s, p);
  else if (!a_al && b_al) hipLaunchKernelGGL((gemm_kernel<AK, BK_, MODE, false, true>), grid, dim3(NT), 0, s, p);
  else if (a_al && !b_al) hipLaunchKernelGGL((gemm_kernel<AK, BK_, MODE, true, false>), grid, dim3(NT), 0, s, p);
  else hipLaunchKernelGGL((gemm_kernel<AK, BK_, MODE, false, false>), grid, dim3(NT), 0, s, p);
}

template <int MODE>
static void dispatch_layout(const GemmArgs& p, dim3 grid, hipStream_t s, bool a_al, bool b_al) {
  if (p.a_kcontig && p.b_kcontig) launch_tiled<true, true, MODE>(p, grid, s, a_al, b_al);
  else if (p.a_kcontig && !p.b_kcontig) launch_tiled<true, false, MODE>(p, grid, s, a_al, b_al);
  else if (!p.a_kcontig && p.b_kcontig) launch_tiled<false, true, MODE>(p, grid, s, a_al, b_al);
  else launch_tiled<false, false, MODE>(p, grid, s, a_al, b_al);
}

static bool aligned16(const void* ptr) { return ((uintptr_t)ptr & 15) == 0; }

int64_t gemm_workspace_bytes(int M, int N, int K, int batch, int splitk) {
  if (splitk <= 1) return 0;
  return (int64_t)M * N * batch * splitk * 4;
}

int gemm_pick_splitk(int M, int N, int K, int batch, int impl) {
  // tile count of the kernel that will run
  int64_t tiles;
  if (impl == 6 || impl >= 60) return 1;  // persistent ping-pong kernel: every CU busy whatever the tile count
  if (impl == 2 && K % 32 == 0) {
    tiles = (int64_t)((M + 255) / 256) * ((N + gemm256_bn(M, N, batch, 1) - 1) / gemm256_bn(M, N, batch, 1)) * batch;
  } else if (impl >= 1 && K % 64 == 0) {
    tiles = (int64_t)((M + 255) / 256) * ((N + 127) / 128) * batch;
  } else {
    tiles = (int64_t)((M + BM - 1) / BM) * ((N + BN - 1) / BN) * batch;
  }
  if (tiles >= 256 || K < 1024) return 1;
  // minimise (waves of 256 CUs) / split, with a small charge per split for the fp32 slab reduce
  int best = 1;
  double best_cost = 1e30;
  for (int s = 1; s <= 16 && K / s >= 512; ++s) {
    const double cost = (double)((tiles * s + 255) / 256) / s + 0.03 * s;
    if (cost < best_cost - 1e-9) { best_cost = cost; best = s; }
  }
  return best;
}

static bool try_large(const GemmArgs& p, bool a_al, bool b_al, hipStream_t stream) {
  if (!(a_al && b_al && p.a_bytes > 0)) return false;
  if (p.impl >= 60 && p.impl < 70) {  // ablation of gemm_pp (timing only): 61 no loop DMA
    GemmArgs q = p;
    q.ablate = p.impl - 60;
    q.impl = 6;
    return gemm_pp_bf16(q, p.a_bytes, p.b_bytes, stream);
  }
  if (p.impl == 6 && gemm_pp_bf16(p, p.a_bytes, p.b_bytes, stream)) return true;
  if (p.impl >= 2 && gemm256_bf16(p, p.a_bytes, p.b_bytes, stream)) return true;
  if (p.impl >= 1 && gemm_big_bf16(p, p.a_bytes, p.b_bytes, stream)) return true;
  return false;
}

void gemm_bf16(GemmArgs p, hipStream_t stream) {
  if (p.M <= 0 || p.N <= 0 || p.batch <= 0) return;
  // 16-B aligned chunks of the contiguous dim for the vector staging path, per operand
  const bool a_al = aligned16(p.A) && (p.lda % 8 == 0) && (p.sA % 8 == 0) &&
                    (p.a_kcontig ? (p.K % 8 == 0) : (p.M % 8 == 0));
  const bool b_al = aligned16(p.B) && (p.ldb % 8 == 0) && (p.sB % 8 == 0) &&
                    (p.b_kcontig ? (p.K % 8 == 0) : (p.N % 8 == 0));
  const int osz = p.out_f32 ? 4 : 2;
  p.vec_ok = ((p.ldc % 4) == 0) && ((p.sC % 4) == 0) && (((uintptr_t)p.C) % (4 * osz) == 0) &&
             (p.Z == nullptr || ((uintptr_t)p.Z % 8) == 0);
  p.vec8_ok = (p.N % 8 == 0) && ((p.ldc % 8) == 0) && ((p.sC % 8) == 0) && (((uintptr_t)p.C) % 16 == 0) &&
              (p.Z == nullptr || ((uintptr_t)p.Z % 16) == 0) &&
              (p.bias == nullptr || ((uintptr_t)p.bias % 16) == 0);
  if (p.M * (int64_t)p.N * p.K < 64 * 64 * 64 && !(a_al && b_al)) {
    dim3 grid((p.N + 15) / 16, (p.M + 15) / 16, p.batch);
    if (p.out_f32) hipLaunchKernelGGL(gemm_fallback_kernel<float>, grid, dim3(16, 16), 0, stream, p, p.a_kcontig, p.b_kcontig);
    else hipLaunchKernelGGL(gemm_fallback_kernel<bf16_t>, grid, dim3(16, 16), 0, stream, p, p.a_kcontig, p.b_kcontig);
    return;
  }
  const int tm = (p.M + BM - 1) / BM, tn = (p.N + BN - 1) / BN;
  if (p.splitk > 1 && p.ws != nullptr) {
    p.kchunk = ((p.K + p.splitk - 1) / p.splitk + BK - 1) / BK * BK;
    dim3 grid(tm * tn, p.batch * p.splitk);
    if (!try_large(p, a_al, b_al, stream)) dispatch_layout<2>(p, grid, stream, a_al, b_al);
    if (p.skip_reduce) return;
    const int64_t total = (int64_t)p.M * p.N * p.batch;
    if (p.out_f32 && p.batch == 1 && p.ldc == p.N && !p.bias && !p.Z && p.act == ACT_NONE && total % 4 == 0 &&
        aligned16(p.C) && aligned16(p.ws)) {
      slab_sum(p.ws, reinterpret_cast<float*>(p.C), total, p.splitk, p.beta, stream);  // float4 slab reduce
      return;
    }
    if (p.out_f32) hipLaunchKernelGGL(splitk_reduce_kernel<float>, dim3(ew_grid(total, 256)), dim3(256), 0, stream, p);
    else hipLaunchKernelGGL(splitk_reduce_kernel<bf16_t>, dim3(ew_grid(total, 256)), dim3(256), 0, stream, p);
    return;
  }
  p.splitk = 1;
  p.kchunk = p.K;
  if (try_large(p, a_al, b_al, stream)) return;
  dim3 grid(tm * tn, p.batch);
  if (p.out_f32) dispatch_layout<1>(p, grid, stream, a_al, b_al);
  else dispatch_layout<0>(p, grid, stream, a_al, b_al);
}

}  // namespace ffk

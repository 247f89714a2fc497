// Persistent 256-row bf16 MFMA GEMM: one workgroup per CU walks its share of the output tiles and
// the LDS-DMA operand ring runs on across tile boundaries.
//
// Why: BERT-Large's forward and dgrad GEMMs are mostly K = 1024 (16384 x {1024, 3072, 4096, 30522}
// x 1024): only 32 K-tiles of 32 per output tile. In gemm256.hip every tile pays its own prologue
// (three K-tiles of DMA latency before the first MFMA) and its epilogue with the matrix pipe idle:
// ~1/4 of the tile's MFMA time at K = 1024. Here the DMAs of tile i+1's first K-tiles are issued
// during tile i's last K-steps (the ring index is a global step counter g = local tile * nk + k),
// so the next tile's operands are already landing while the accumulators of tile i are stored.
//
// Inner structure is gemm256.hip's (gemm256_tile.h): 256 x {256x32, 128x64} tiles, 8 waves in
// two ping-pong groups one barrier apart, 16 MFMAs per phase, counted vmcnt waits. The epilogue
// stores straight from the accumulators (the ring owns the LDS): each lane writes 4 consecutive
// columns (8 B bf16 / 16 B fp32) per fragment row; bias, beta * C, pre-activation store and
// activation are applied in registers. Tiles are dealt as tile = blockIdx.x + i * gridDim.x in the
// XCD-remapped, GROUP_M = 8 order, so the workgroups of one XCD walk neighbouring tiles together.
//
// Limits (the host launcher returns false otherwise): batch 1, no split-K, K % BK == 0, 16-B
// aligned operand rows, operands < 2 GiB.
#include "gemm256_tile.h"

namespace ffk {
namespace g256 {

// One K-tile of A (rows mm..) and B (rows / columns nn..) into a ring slot. The buffer resources
// are passed by value: captured by reference in a lambda they were spilled to scratch and every
// DMA went through a waterfall loop behind a vmcnt(0).
template <bool A_K, bool B_K, int BK, int A_BYTES, int A_PIECES, int PW>
__device__ __forceinline__ void stage(char* st, __amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb, int64_t lda,
                                      int64_t ldb, int mm, int nn, int k0, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int piece = wave * PW + i;
    if (piece < A_PIECES) dma_piece<A_K, BK>(ra, st, lda, mm, k0, piece, lane);
    else dma_piece<B_K, BK>(rb, st + A_BYTES, ldb, nn, k0, piece - A_PIECES, lane);
  }
}

template <bool A_K, bool B_K, int BN, int OUT_MODE>
__global__ void __launch_bounds__(NT, 1) gemm_persist_kernel(GemmArgs p, int64_t a_bytes, int64_t b_bytes) {
  constexpr int BK = Geo<BN>::BK, NBUF = Geo<BN>::NBUF, KK = BK / 32;
  constexpr int A_BYTES = BM * BK * 2;
  constexpr int B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int A_PIECES = A_BYTES / 1024, PIECES = STAGE / 1024;
  constexpr int PW = PIECES / 8;
  constexpr int WN = BN / 4;
  constexpr int NF = WN / 16;
  static_assert(PIECES % 8 == 0, "pieces must split evenly over 8 waves");
  __shared__ __attribute__((aligned(1024))) char smem[NBUF * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int tm = (p.M + BM - 1) / BM, tn = (p.N + BN - 1) / BN;
  const int T = tm * tn;
  const int nk = p.K / BK;
  const int G = gridDim.x;
  const int mine = (T - (int)blockIdx.x + G - 1) / G;  // tiles of this workgroup (grid <= T)
  const int total = mine * nk;                          // K-steps over all of them

  __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, (int)min(a_bytes, (int64_t)0x7fffffff), 0x00020000);
  __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, (int)min(b_bytes, (int64_t)0x7fffffff), 0x00020000);

  // general step -> (tile, k) mapping (prologue, and rings longer than a tile's K)
#define FF_PERSIST_ISSUE(gg)                                                                          \
  do {                                                                                                \
    const int lt_ = (gg) / nk, kt_ = (gg) - lt_ * nk;                                                 \
    int tm_, tn_;                                                                                     \
    tile_coords((int)blockIdx.x + lt_ * G, tm, tn, tm_, tn_);                                         \
    stage<A_K, B_K, BK, A_BYTES, A_PIECES, PW>(smem + ((gg) % NBUF) * STAGE, ra, rb, p.lda, p.ldb,    \
                                               tm_ * BM, tn_ * BN, kt_ * BK, wave, lane);             \
  } while (0)

  f32x4 acc[8][NF];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int pre = min(total, NBUF - 1);
  for (int g = 0; g < pre; ++g) FF_PERSIST_ISSUE(g);
  wait_tiles<PW, NBUF>(pre - 1);
  barrier();
  if (wr == 1) barrier();

  typedef typename std::conditional<OUT_MODE == 0, bf16_t, float>::type OutT;
  OutT* C = reinterpret_cast<OutT*>(p.C);
  bf16_t* Zp = reinterpret_cast<bf16_t*>(p.Z);

  // Coordinates of this workgroup's current and next tile; a refill DMA at step g + NBUF - 1 lands
  // in the next tile when it crosses the boundary (NBUF - 1 <= nk; shorter K takes the general path).
  int cur_m, cur_n, nxt_m = 0, nxt_n = 0;
  tile_coords((int)blockIdx.x, tm, tn, cur_m, cur_n);
  if (mine > 1) tile_coords((int)blockIdx.x + G, tm, tn, nxt_m, nxt_n);
  const bool short_k = nk < NBUF - 1;

  bf16x8 af[KK][4], bfr[KK][NF];
  int g = 0;
  for (int lt = 0; lt < mine; ++lt) {
    // the K loop holds no ordinary global loads (only LDS-DMA and LDS reads), so the compiler's
    // wait counting never drains the ring there; the epilogue's loads come after it
    for (int kt = 0; kt < nk; ++kt, ++g) {
      const char* cur = smem + (g % NBUF) * STAGE;
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
#pragma unroll
        for (int j = 0; j < NF; ++j) bfr[kk][j] = frag<B_K, BK>(cur + A_BYTES, wc * WN + j * 16, kk, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i) af[kk][i] = frag<A_K, BK>(cur, wr * 128 + i * 16, kk, lane);
      }
      lgkm0();
      barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NF; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[kk][j], af[kk][i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      barrier();
      // the refill may already belong to the next tile: the ring does not stop at tile boundaries
      if (g + NBUF - 1 < total) {
        if (short_k) {
          FF_PERSIST_ISSUE(g + NBUF - 1);
        } else {
          const int kn = kt + NBUF - 1;
          const bool nxt = kn >= nk;
          stage<A_K, B_K, BK, A_BYTES, A_PIECES, PW>(smem + ((g + NBUF - 1) % NBUF) * STAGE, ra, rb, p.lda, p.ldb,
                                                     (nxt ? nxt_m : cur_m) * BM, (nxt ? nxt_n : cur_n) * BN,
                                                     (nxt ? kn - nk : kn) * BK, wave, lane);
        }
      }
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i) af[kk][i] = frag<A_K, BK>(cur, wr * 128 + 64 + i * 16, kk, lane);
      wait_tiles<PW, NBUF>(min(total, g + NBUF) - (g + 2));
      lgkm0();
      barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NF; ++j)
            acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[kk][j], af[kk][i], acc[4 + i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      barrier();
    }

    // ---- tile lt is complete: store it while the next tile's first DMAs land
    const int tmi = cur_m, tni = cur_n;
    cur_m = nxt_m;
    cur_n = nxt_n;
    if (lt + 2 < mine) tile_coords((int)blockIdx.x + (lt + 2) * G, tm, tn, nxt_m, nxt_n);
    const int mrow = tmi * BM + wr * 128 + (lane & 15);
    const int ncol = tni * BN + wc * WN + (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = mrow + i * 16;
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        const int n = ncol + j * 16;
        f32x4 a = acc[i][j];
        acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (m >= p.M || n >= p.N) continue;
        float v[4];
        const bool full = p.vec_ok && (n + 3 < p.N);
        OutT* dst = C + (int64_t)m * p.ldc + n;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float x = a[r] * p.alpha;
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
  if (wr == 0) barrier();
#undef FF_PERSIST_ISSUE
}

template <int BN, int MODE>
static void launch(const GemmArgs& p, dim3 grid, hipStream_t s, int64_t ab, int64_t bb) {
  if (p.a_kcontig && p.b_kcontig) hipLaunchKernelGGL((gemm_persist_kernel<true, true, BN, MODE>), grid, dim3(NT), 0, s, p, ab, bb);
  else if (p.a_kcontig) hipLaunchKernelGGL((gemm_persist_kernel<true, false, BN, MODE>), grid, dim3(NT), 0, s, p, ab, bb);
  else if (p.b_kcontig) hipLaunchKernelGGL((gemm_persist_kernel<false, true, BN, MODE>), grid, dim3(NT), 0, s, p, ab, bb);
  else hipLaunchKernelGGL((gemm_persist_kernel<false, false, BN, MODE>), grid, dim3(NT), 0, s, p, ab, bb);
}

static int cu_count() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
      n = prop.multiProcessorCount;
    if (n <= 0) n = 256;
  }
  return n;
}

}  // namespace g256

bool gemm_persist_bf16(const GemmArgs& p, int64_t a_bytes, int64_t b_bytes, hipStream_t stream) {
  using namespace g256;
  if (p.batch != 1 || (p.splitk > 1 && p.ws != nullptr)) return false;
  const int bn = gemm256_bn(p.M, p.N, 1, 1);
  if (p.K % (bn == 256 ? 32 : 64) != 0 || p.K <= 0) return false;
  if (a_bytes > 0x7fffffffLL || b_bytes > 0x7fffffffLL || a_bytes <= 0 || b_bytes <= 0) return false;
  if (((uintptr_t)p.A & 15) || ((uintptr_t)p.B & 15) || p.lda % 8 || p.ldb % 8) return false;
  if (!p.a_kcontig && p.M % 8) return false;
  if (!p.b_kcontig && p.N % 8) return false;
  const int T = ((p.M + BM - 1) / BM) * ((p.N + bn - 1) / bn);
  dim3 grid(min(T, cu_count()));
  if (bn == 256) {
    if (p.out_f32) launch<256, 1>(p, grid, stream, a_bytes, b_bytes);
    else launch<256, 0>(p, grid, stream, a_bytes, b_bytes);
  } else {
    if (p.out_f32) launch<128, 1>(p, grid, stream, a_bytes, b_bytes);
    else launch<128, 0>(p, grid, stream, a_bytes, b_bytes);
  }
  return true;
}

}  // namespace ffk

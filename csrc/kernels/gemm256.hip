// 256 x {256x32, 128x64} bf16 MFMA GEMM, 8 waves in two ping-pong groups, 4/3-deep LDS-DMA ring.
//
// Why this structure (measured on the 256x128x64 kernel of gemm_big.hip with rocprofv3 --pmc,
// profiles/gemm_pmc_r1.txt): its waves spent ~32 % of their cycles parked at the per-K-tile
// barrier / vmcnt wait and only ~24 % issuing, while hipBLASLt's kernel parks ~16 %. Two waves
// share each SIMD and the single barrier per K-tile lines them up, so both read LDS at the same
// time and both issue MFMAs at the same time. Here:
//   * tile 256(M) x BN(N) x 32(K); waves = 2 (M) x 4 (N), 128 x BN/4 outputs per wave
//     (8 x BN/64 mfma_f32_16x16x32_bf16 fragments; operands swapped so a lane owns 4 consecutive
//     output columns -> 8-byte stores);
//   * each K-tile is two phases {LDS reads; barrier; 16 MFMAs; barrier}. Waves 4-7 run one
//     barrier behind waves 0-3 (one extra barrier at the start, balanced at the end), and waves w
//     and w+4 sit on the same SIMD (waves are dealt to SIMDs round-robin), so on every SIMD one
//     wave issues MFMAs while the other reads its next fragments — the ping-pong of
//     cdna_hip_programming.md "The 256^2 8-phase template"; s_setprio(1) around the MFMA bursts;
//   * LDS reads complete (lgkmcnt(0)) before each barrier, so a barrier proves every earlier read
//     of a ring slot is done: the DMA that refills slot (t+3)%4 (issued in tile t's second phase)
//     can never overwrite data a lagging wave still has to read;
//   * operands arrive by buffer_load ... lds (16 B / lane, 1 KiB per wave instruction, hardware
//     zero-fill past the end of the buffer); 4 slots of 32 KiB = 128 KiB in flight, tile t+1 is
//     waited for (counted vmcnt, never 0 in steady state) one phase before its first read;
//   * K-contiguous tiles are stored as 64-B rows with 16-B chunk ^ (((row >> 2) & 1) << 1): an
//     exhaustive search over chunk XORs of row bits for the four ds_read_b128 lane groups of the
//     16x16x32 operand pattern (16 rows x 4 chunks) gives this as conflict-free; MN-contiguous
//     tiles use 128-wide halves of 256-B rows with the T10 image (b) XOR, read by
//     ds_read_b64_tr_b16 (same image as gemm_big.hip);
//   * XCD-aware bijective block remap + GROUP_M = 8 tile order (per-XCD L2 reuse).
// Requires K % BK == 0 (split-K chunks are multiples of 64), 16-B aligned operand rows,
// operands < 2 GiB. Epilogue contract identical to gemm.hip (bias, activation, pre-activation
// store Z, alpha/beta, bf16 or fp32 C, fp32 split-K slabs).
#include "gemm256_tile.h"

namespace ffk {
namespace g256 {

template <bool A_K, bool B_K, int BN, int OUT_MODE>
__global__ void __launch_bounds__(NT, 1) gemm256_kernel(GemmArgs p, int64_t a_bytes, int64_t b_bytes) {
  constexpr int BK = Geo<BN>::BK, NBUF = Geo<BN>::NBUF, KK = BK / 32;
  constexpr int A_BYTES = BM * BK * 2;
  constexpr int B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int A_PIECES = A_BYTES / 1024, PIECES = STAGE / 1024;
  constexpr int PW = PIECES / 8;  // DMA instructions per wave per K-tile
  constexpr int WN = BN / 4;      // output columns per wave
  constexpr int NF = WN / 16;     // N fragments per wave
  static_assert(PIECES % 8 == 0, "pieces must split evenly over 8 waves");
  __shared__ __attribute__((aligned(1024))) char smem[NBUF * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int tm = (p.M + BM - 1) / BM, tn = (p.N + BN - 1) / BN;
  int tile_m, tile_n;
  tile_coords(blockIdx.x, tm, tn, tile_m, tile_n);
  const int z = blockIdx.y;
  const int b = z / p.splitk, ks = z % p.splitk;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int kbeg = ks * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const int nk = max(0, (kend - kbeg) / BK);

  const bf16_t* Ab = p.A + (int64_t)b * p.sA;
  const bf16_t* Bb = p.B + (int64_t)b * p.sB;
  const int64_t a_rem = a_bytes - (int64_t)b * p.sA * 2;
  const int64_t b_rem = b_bytes - (int64_t)b * p.sB * 2;
  __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)Ab, (short)0, (int)min(a_rem, (int64_t)0x7fffffff), 0x00020000);
  __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, (short)0, (int)min(b_rem, (int64_t)0x7fffffff), 0x00020000);

  f32x4 acc[8][NF];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int t) {
    char* st = smem + (t % NBUF) * STAGE;
    const int k0 = kbeg + t * BK;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int piece = wave * PW + i;
      if (piece < A_PIECES) dma_piece<A_K, BK>(ra, st, p.lda, m0, k0, piece, lane);
      else dma_piece<B_K, BK>(rb, st + A_BYTES, p.ldb, n0, k0, piece - A_PIECES, lane);
    }
  };

  // prologue: tiles 0..2 in flight, tile 0 landed everywhere before the first read
  const int pre = min(nk, NBUF - 1);
  for (int t = 0; t < pre; ++t) issue(t);
  wait_tiles<PW, NBUF>(pre - 1);
  barrier();
  if (wr == 1) barrier();  // ping-pong: the second wave group runs one barrier behind

  bf16x8 af[KK][4], bfr[KK][NF];
  for (int t = 0; t < nk; ++t) {
    const char* cur = smem + (t % NBUF) * STAGE;
    // ---- phase 0: rows 0..63 of this wave's 128
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
    // ---- phase 1: rows 64..127; refill slot (t+NBUF-1)%NBUF, make sure tile t+1 has landed
    if (t + NBUF - 1 < nk) issue(t + NBUF - 1);
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) af[kk][i] = frag<A_K, BK>(cur, wr * 128 + 64 + i * 16, kk, lane);
    wait_tiles<PW, NBUF>(min(nk, t + NBUF) - (t + 2));
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
  if (wr == 0) barrier();  // balance the barrier count of the two groups

  store_tile<WN, OUT_MODE>(p, acc, smem, wave, wr, wc, lane, m0, n0, b, z, tile_m);
}

template <int BN, int MODE>
static void launch(const GemmArgs& p, dim3 grid, hipStream_t s, int64_t ab, int64_t bb) {
  if (p.a_kcontig && p.b_kcontig) hipLaunchKernelGGL((gemm256_kernel<true, true, BN, MODE>), grid, dim3(NT), 0, s, p, ab, bb);
  else if (p.a_kcontig) hipLaunchKernelGGL((gemm256_kernel<true, false, BN, MODE>), grid, dim3(NT), 0, s, p, ab, bb);
  else if (p.b_kcontig) hipLaunchKernelGGL((gemm256_kernel<false, true, BN, MODE>), grid, dim3(NT), 0, s, p, ab, bb);
  else hipLaunchKernelGGL((gemm256_kernel<false, false, BN, MODE>), grid, dim3(NT), 0, s, p, ab, bb);
}

template <int BN>
static void launch_mode(const GemmArgs& p, dim3 grid, hipStream_t s, int64_t ab, int64_t bb, int mode) {
  if (mode == 2) launch<BN, 2>(p, grid, s, ab, bb);
  else if (mode == 1) launch<BN, 1>(p, grid, s, ab, bb);
  else launch<BN, 0>(p, grid, s, ab, bb);
}

}  // namespace g256

// Tile width for the 256-row kernel: time ~ (waves of 256 CUs) x (per-tile time), a 256x128 tile
// costing ~0.55 of a 256x256 one (half the MFMAs, a little more LDS traffic per flop).
int gemm256_bn(int M, int N, int batch, int splitk) {
  const int64_t t256 = (int64_t)((M + 255) / 256) * ((N + 255) / 256) * batch * splitk;
  const int64_t t128 = (int64_t)((M + 255) / 256) * ((N + 127) / 128) * batch * splitk;
  const double c256 = (double)((t256 + 255) / 256);
  const double c128 = 0.55 * (double)((t128 + 255) / 256);
  return c128 < c256 ? 128 : 256;
}

bool gemm256_bf16(const GemmArgs& p0, int64_t a_bytes, int64_t b_bytes, hipStream_t stream) {
  using namespace g256;
  GemmArgs p = p0;
  const int bn = gemm256_bn(p.M, p.N, p.batch, p.splitk > 1 && p.ws ? p.splitk : 1);
  if (p.K % (bn == 256 ? 32 : 64) != 0 || a_bytes > 0x7fffffffLL || b_bytes > 0x7fffffffLL || a_bytes <= 0 || b_bytes <= 0) return false;
  if (((uintptr_t)p.A & 15) || ((uintptr_t)p.B & 15) || p.lda % 8 || p.ldb % 8 || p.sA % 8 || p.sB % 8) return false;
  if (!p.a_kcontig && p.M % 8) return false;
  if (!p.b_kcontig && p.N % 8) return false;
  const bool split = p.splitk > 1 && p.ws != nullptr;
  if (!split) p.splitk = 1;
  p.kchunk = split ? ((p.K + p.splitk - 1) / p.splitk + 63) / 64 * 64 : p.K;
  const int tm = (p.M + BM - 1) / BM, tn = (p.N + bn - 1) / bn;
  dim3 grid(tm * tn, p.batch * p.splitk);
  const int mode = split ? 2 : (p.out_f32 ? 1 : 0);
  if (bn == 256) launch_mode<256>(p, grid, stream, a_bytes, b_bytes, mode);
  else launch_mode<128>(p, grid, stream, a_bytes, b_bytes, mode);
  return true;
}

bool gemm_dact_bf16(GemmArgs p, hipStream_t stream) {
  if (p.M <= 0 || p.N <= 0) return true;
  if (!p.zin || p.out_f32 || p.batch != 1 || p.beta != 0.f || p.bias || p.Z || p.act == ACT_NONE) return false;
  auto al16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  if (p.N % 8 || p.ldc % 8 || !al16(p.C) || !al16(p.zin) || (p.colpart && !al16(p.colpart))) return false;
  p.vec8_ok = true;
  p.vec_ok = true;
  p.dact = true;
  p.splitk = 1;
  p.ws = nullptr;
  // impl 6: the ping-pong kernel's DACT epilogue (NN dgrad layout; gemm_pp.hip), else the 256-row
  // kernel's
  if (p.impl == 6) return gemm_pp_bf16(p, p.a_bytes, p.b_bytes, stream);
  return gemm256_bf16(p, p.a_bytes, p.b_bytes, stream);
}

}  // namespace ffk

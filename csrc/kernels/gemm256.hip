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

  if (p.vec8_ok) {
    // Coalesced epilogue through LDS (the operand ring is free now: every wave has passed the
    // loop's last barrier). A wave writes 32 of its 128 output rows as fp32 into its own padded
    // [32][WN+4] LDS image (16-B writes, the +4-float pad makes the 8-lane write groups hit
    // distinct banks), then reads them back 8 consecutive columns per lane and applies
    // bias / beta*C / pre-activation store / activation with 16-B (bf16) or 32-B (fp32) accesses:
    // each row leaves as one contiguous 2*WN-byte segment instead of 16 scattered 8-byte pieces.
    // Only the wave's own rows are touched, and LDS executes a wave's instructions in order,
    // so no barrier is needed between the write and the read-back.
    constexpr int LDW = WN + 4;
    float* st = reinterpret_cast<float*>(smem) + wave * (32 * LDW);
    typedef typename std::conditional<OUT_MODE == 0, bf16_t, float>::type OutT2;
    OutT2* C = OUT_MODE == 2 ? nullptr : reinterpret_cast<OutT2*>(p.C) + (int64_t)b * p.sC;
    bf16_t* Zp = p.Z ? reinterpret_cast<bf16_t*>(p.Z) + (int64_t)b * p.sC : nullptr;
    float* W = OUT_MODE == 2 ? p.ws + (int64_t)z * p.M * p.N : nullptr;
    constexpr int CPR = WN / 8;  // 8-column chunks per row; a lane's chunk (lane % CPR) is fixed
    const bf16_t* Zin = reinterpret_cast<const bf16_t*>(p.zin);
    float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // column sums of this lane's chunk
    // dact: every pre-activation chunk this lane will need is requested up front (16 x 16 B in
    // flight per lane; the fragment registers of the main loop are dead by now), so the tile pays
    // one HBM latency instead of one per row group
    constexpr int ITS = 32 * CPR / 64;
    uint4 zpre[OUT_MODE == 0 ? 4 * ITS : 1];
    if (OUT_MODE == 0 && p.dact) {
#pragma unroll
      for (int qtr = 0; qtr < 4; ++qtr)
#pragma unroll
        for (int it = 0; it < ITS; ++it) {
          const int idx = it * 64 + lane;
          const int m = m0 + wr * 128 + qtr * 32 + idx / CPR;
          const int n = n0 + wc * WN + (idx % CPR) * 8;
          zpre[qtr * ITS + it] = (m < p.M && n < p.N)
                                     ? *reinterpret_cast<const uint4*>(Zin + (int64_t)m * p.ldc + n)
                                     : make_uint4(0, 0, 0, 0);
        }
    }
#pragma unroll
    for (int qtr = 0; qtr < 4; ++qtr) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) {
          const f32x4 v = acc[2 * qtr + i][j];
          *reinterpret_cast<float4*>(st + (i * 16 + (lane & 15)) * LDW + j * 16 + (lane >> 4) * 4) =
              make_float4(v[0] * p.alpha, v[1] * p.alpha, v[2] * p.alpha, v[3] * p.alpha);
        }
#pragma unroll
      for (int it = 0; it < 32 * CPR / 64; ++it) {
        const int idx = it * 64 + lane;
        const int r = idx / CPR, c8 = (idx % CPR) * 8;
        const int m = m0 + wr * 128 + qtr * 32 + r;
        const int n = n0 + wc * WN + c8;
        const float4 lo = *reinterpret_cast<const float4*>(st + r * LDW + c8);
        const float4 hi = *reinterpret_cast<const float4*>(st + r * LDW + c8 + 4);
        if (m >= p.M || n >= p.N) continue;
        float x[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        if (OUT_MODE == 2) {
          float4* d = reinterpret_cast<float4*>(W + (int64_t)m * p.N + n);
          d[0] = lo;
          d[1] = hi;
          continue;
        }
        OutT2* dst = C + (int64_t)m * p.ldc + n;
        if (OUT_MODE == 0 && p.dact) {
          // consumer dgrad * producer act'(pre-activation); the column sums feed the producer's
          // bias gradient (the separate bias_act_bwd pass re-read and re-wrote this whole tile)
          float zz[8];
          const uint4 zv = zpre[OUT_MODE == 0 ? qtr * ITS + it : 0];
          load16(reinterpret_cast<const bf16_t*>(&zv), zz);
          // round the GEMM result to bf16 first, as the unfused GEMM + bias_act_bwd pair does, so
          // the autotuner's choice between the two never changes the numerics beyond summation order
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            x[e] = bf2f(f2bf(x[e])) * act_grad(p.act, zz[e]);
            cs[e] += x[e];
          }
          store16(reinterpret_cast<bf16_t*>(dst), x);
          continue;
        }
        if (p.beta != 0.f) {
          float c[8];
          if (OUT_MODE == 0) load16(reinterpret_cast<const bf16_t*>(dst), c);
          else {
            const float4 c0 = reinterpret_cast<const float4*>(dst)[0], c1 = reinterpret_cast<const float4*>(dst)[1];
            c[0] = c0.x; c[1] = c0.y; c[2] = c0.z; c[3] = c0.w; c[4] = c1.x; c[5] = c1.y; c[6] = c1.z; c[7] = c1.w;
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] += p.beta * c[e];
        }
        if (p.bias) {
          float bb[8];
          if (p.bias_bf16) load16(reinterpret_cast<const bf16_t*>(p.bias) + n, bb);
          else {
            const float4 b0 = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p.bias) + n)[0];
            const float4 b1 = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p.bias) + n)[1];
            bb[0] = b0.x; bb[1] = b0.y; bb[2] = b0.z; bb[3] = b0.w; bb[4] = b1.x; bb[5] = b1.y; bb[6] = b1.z; bb[7] = b1.w;
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] += bb[e];
        }
        if (Zp) store16(Zp + (int64_t)m * p.ldc + n, x);
        if (p.act != ACT_NONE) {
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] = act_fwd(p.act, x[e]);
        }
        if (OUT_MODE == 0) store16(reinterpret_cast<bf16_t*>(dst), x);
        else {
          reinterpret_cast<float4*>(dst)[0] = make_float4(x[0], x[1], x[2], x[3]);
          reinterpret_cast<float4*>(dst)[1] = make_float4(x[4], x[5], x[6], x[7]);
        }
      }
    }
    if (OUT_MODE == 0 && p.dact && p.colpart) {
      // fold the 64 / CPR lanes that share a column chunk, then one lane per chunk stores the
      // wave's 128-row partial (row tile_m * 2 + wr of the [2 tm][N] slab; summed by col_reduce_add)
#pragma unroll
      for (int sh = CPR; sh < 64; sh <<= 1)
#pragma unroll
        for (int e = 0; e < 8; ++e) cs[e] += __shfl_xor(cs[e], sh);
      const int n = n0 + wc * WN + lane * 8;
      if (lane < CPR && n < p.N) {
        float4* d = reinterpret_cast<float4*>(p.colpart + (int64_t)(tile_m * 2 + wr) * p.N + n);
        d[0] = make_float4(cs[0], cs[1], cs[2], cs[3]);
        d[1] = make_float4(cs[4], cs[5], cs[6], cs[7]);
      }
    }
    return;
  }

  const int mrow = m0 + wr * 128 + (lane & 15);
  const int ncol = n0 + wc * WN + (lane >> 4) * 4;
  if (OUT_MODE == 2) {
    float* W = p.ws + (int64_t)z * p.M * p.N;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = mrow + i * 16;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < NF; ++j) {
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
  for (int i = 0; i < 8; ++i) {
    const int m = mrow + i * 16;
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < NF; ++j) {
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
  return gemm256_bf16(p, p.a_bytes, p.b_bytes, stream);
}

}  // namespace ffk

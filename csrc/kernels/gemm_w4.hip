// 256 x 256 x 64 bf16 MFMA GEMM with FOUR waves of 128 x 128 outputs each (one wave per SIMD,
// 256 AGPR accumulators per lane), a two-slot LDS-DMA ring and the K-tile split into two halves.
//
// Why this shape next to gemm256.hip (8 waves of 128 x 64, ping-pong pairs): a wave's LDS reads per
// K-step are (rows + columns) of its output block, so 128 x 128 blocks read 1/3 fewer LDS bytes per
// MFMA, and the per-phase barrier pairs of the ping-pong go away. One wave per SIMD has no partner
// to hide its LDS reads and DMA issue, so they are interleaved with its own MFMAs (groups of 4
// MFMAs pinned by sched_barrier). Why 64-deep K-tiles: with 32-deep ones a K-contiguous DMA piece
// covers 16 rows x 64 B, half of each 128-B line it touches, and a 256x256x32 build of this kernel
// ran 5-9 % slower on the BERT-Large forward shapes (profiles/gemm_bert_probe_r3_w4_v2.txt);
// ablating it (profiles/gemm_w4_ablation_r3.txt) priced the DMA issue at ~20 % of the main loop and
// the fragment reads at ~3-10 %. Spreading the DMA over both halves (A in three 32-KiB slots, B in
// two: 160 KiB) measured 1-4 % slower than this two-slot ring (profiles/gemm_bert_probe_r3_w4_v3.txt).
//
// Per K-tile t (slot t % 2), per wave:
//   half 0: 64 MFMAs on the kk = 0 fragments of tile t (registers, read during the previous
//           tile), reading tile t's kk = 1 fragments into the other register set;
//   lgkmcnt(0); wait for this wave's pieces of tile t+1; barrier (everyone has finished reading
//           tile t, and tile t+1 has landed everywhere);
//   half 1: 64 MFMAs on the kk = 1 fragments, staging tile t+2 into slot t % 2 (16 DMA pieces,
//           one per 4 MFMAs) and reading tile t+1's kk = 0 fragments.
// The MFMAs are inline asm on "+a" accumulators (hipcc's builtin picks the VGPR form with two
// fragment sets live and copies every result into the AGPR file); the hazards this hides from the
// compiler are padded explicitly (pin_acc + s_nop at both ends of the loop).
// Fragment images, swizzles, MFMA operand order and epilogue as gemm256_tile.h. Requires
// K % 128 == 0, 16-B aligned operand rows, operands < 2 GiB.
#include "gemm_w4_core.h"

namespace ffk {
namespace w4 {
using namespace g256;

template <bool A_K, bool B_K, int OUT_MODE>
__global__ void __launch_bounds__(NTH, 1) __attribute__((amdgpu_waves_per_eu(1, 1)))
gemm_w4_kernel(GemmArgs p, int64_t a_bytes, int64_t b_bytes) {
  constexpr int WN = 128, NF = 8;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
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

  const bool isA = wave < 2;
  const __amdgpu_buffer_rsrc_t rs = isA ? ra : rb;
  const int kstride = isA ? (A_K ? BK * 2 : BK * (int)p.lda * 2) : (B_K ? BK * 2 : BK * (int)p.ldb * 2);
  int boff[PW];
#pragma unroll
  for (int g = 0; g < PW; ++g) {
    const int pc = wave * PW + g;
    boff[g] = isA ? piece_off<A_K>(p.lda, m0, kbeg, pc, lane) : piece_off<B_K>(p.ldb, n0, kbeg, pc - A_PIECES, lane);
  }
  auto dma = [&](int slot, int t, int g) __attribute__((always_inline)) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(smem + slot * STAGE + (wave * PW + g) * 1024), 16, boff[g],
                                             t * kstride, 0, 0);
  };

  // prologue: tiles 0 and 1 in flight, tile 0 landed everywhere, its kk = 0 fragments in set 0
  for (int t = 0; t < min(nk, 2); ++t)
#pragma unroll
    for (int g = 0; g < PW; ++g) dma(t, t, g);
  if (nk > 1) vmcnt<16>();
  else vmcnt<0>();
  barrier();
  bf16x8 a0[8], b0[NF], a1[8], b1[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) b0[j] = frag64<B_K>(smem + A_BYTES, wc * WN + j * 16, 0, lane);
#pragma unroll
  for (int i = 0; i < 8; ++i) a0[i] = frag64<A_K>(smem, wr * 128 + i * 16, 0, lane);
  lgkm0();

  // 16 groups of 4 MFMAs on (ac, bc); group g < 8 also reads fragments g of (an, bn) from `src`
  // at sub-step kk; with `stage`, group g also issues DMA piece g of tile ts into slot `sslot`.
  auto half = [&](bf16x8(&ac)[8], bf16x8(&bc)[NF], bf16x8(&an)[8], bf16x8(&bn)[NF], const char* src, const char* srco,
                  int kk, bool stage, int sslot, int ts) __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      if (stage) dma(sslot, ts, g);
      if (g < 8) {
        bn[g] = frag64<B_K>((B_K ? src : srco) + A_BYTES, wc * WN + g * 16, kk, lane);
        an[g] = frag64<A_K>(A_K ? src : srco, wr * 128 + g * 16, kk, lane);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = g >> 1, j = (g & 1) * 4 + q;
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(bc[j]), "v"(ac[i]));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    lgkm0();
  };
  auto step = [&](auto slot_c, int t) __attribute__((always_inline)) {
    constexpr int S = decltype(slot_c)::value;  // t % 2
    const char* cur = smem + S * STAGE;
    const char* nxt = smem + (S ^ 1) * STAGE;
    // MN-contiguous fragments take two lane-dependent addresses each; with literal slot offsets
    // hipcc keeps an address set per slot live and spills. Opaque bases cost one v_add per read.
    int so = S * STAGE, sn = (S ^ 1) * STAGE;
    asm volatile("" : "+s"(so), "+s"(sn));
    half(a0, b0, a1, b1, cur, smem + so, 1, false, 0, 0);
    vmcnt<0>();  // tile t+1 (the only DMA in flight) has landed for this wave ...
    barrier();   // ... and for every wave; every wave has finished reading tile t
    half(a1, b1, a0, b0, nxt, smem + sn, 0, t + 2 < nk, S, t + 2);
  };
  // hazards the compiler cannot see around the asm MFMAs: the empty "+a" statements pin every
  // accumulator's zero-init before the nop (v_accvgpr_write -> MFMA C operand), and after the loop
  // every accumulator read behind the nop (MFMA D -> reader: 12 wait states for 8-pass XDL); hipcc
  // otherwise starts copying accumulators for the epilogue right behind the last MFMA.
  pin_acc(acc);
  asm volatile("s_nop 4");
  for (int t = 0; t < nk; t += 2) {  // nk even (K % 128 == 0, split-K chunks multiples of 128)
    step(std::integral_constant<int, 0>(), t);
    step(std::integral_constant<int, 1>(), t + 1);
  }
  asm volatile("s_nop 15\n\ts_nop 3");
  pin_acc(acc);
  barrier();  // every wave is done with the ring before it is reused as the epilogue stage
  store_tile<WN, OUT_MODE, false, false>(p, acc, smem, wave, wr, wc, lane, m0, n0, b, z, tile_m);
}

template <int MODE>
static void launch(const GemmArgs& p, dim3 grid, hipStream_t s, int64_t ab, int64_t bb) {
  if (p.a_kcontig && p.b_kcontig) hipLaunchKernelGGL((gemm_w4_kernel<true, true, MODE>), grid, dim3(NTH), 0, s, p, ab, bb);
  else if (p.a_kcontig) hipLaunchKernelGGL((gemm_w4_kernel<true, false, MODE>), grid, dim3(NTH), 0, s, p, ab, bb);
  else if (p.b_kcontig) hipLaunchKernelGGL((gemm_w4_kernel<false, true, MODE>), grid, dim3(NTH), 0, s, p, ab, bb);
  else hipLaunchKernelGGL((gemm_w4_kernel<false, false, MODE>), grid, dim3(NTH), 0, s, p, ab, bb);
}

}  // namespace w4

bool gemm_w4_bf16(const GemmArgs& p0, int64_t a_bytes, int64_t b_bytes, hipStream_t stream) {
  using namespace w4;
  GemmArgs p = p0;
  if (p.dact || !p.vec8_ok || p.K % 128 != 0 || a_bytes > 0x7fffffffLL || b_bytes > 0x7fffffffLL || a_bytes <= 0 ||
      b_bytes <= 0)
    return false;
  if (((uintptr_t)p.A & 15) || ((uintptr_t)p.B & 15) || p.lda % 8 || p.ldb % 8 || p.sA % 8 || p.sB % 8) return false;
  if (!p.a_kcontig && p.M % 8) return false;
  if (!p.b_kcontig && p.N % 8) return false;
  const bool split = p.splitk > 1 && p.ws != nullptr;
  if (!split) p.splitk = 1;
  p.kchunk = split ? ((p.K + p.splitk - 1) / p.splitk + 127) / 128 * 128 : p.K;
  const int tm = (p.M + BM - 1) / BM, tn = (p.N + BN - 1) / BN;
  dim3 grid(tm * tn, p.batch * p.splitk);
  const int mode = split ? 2 : (p.out_f32 ? 1 : 0);
  if (mode == 2) launch<2>(p, grid, stream, a_bytes, b_bytes);
  else if (mode == 1) launch<1>(p, grid, stream, a_bytes, b_bytes);
  else launch<0>(p, grid, stream, a_bytes, b_bytes);
  return true;
}

}  // namespace ffk

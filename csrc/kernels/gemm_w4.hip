// 256 x 256 x 32 bf16 MFMA GEMM with FOUR waves of 128 x 128 outputs each (one wave per SIMD,
// 256 accumulator registers per lane), a 4-slot LDS-DMA ring and ONE barrier per K-tile.
//
// Why this shape next to gemm256.hip (8 waves of 128 x 64, ping-pong pairs): a wave's LDS reads
// per K-tile are (rows + columns) of its output block, so 128 x 128 blocks read 1/3 fewer LDS
// bytes per MFMA than 128 x 64 ones, and the per-phase barrier pairs of the ping-pong go away.
// The vendor library's BERT-Large kernels have this geometry (MT256x256x64, wave tile 8 x 8 MFMA
// 16x16, 256 threads). One wave per SIMD has no partner to hide its LDS reads and DMA issue, so
// every K-tile interleaves them with its own MFMAs:
//   * tile t's fragments were read into one register set during tile t-1; tile t+1's are read
//     into the other set between tile t's 64 MFMAs (sched_group_barrier pins the interleave);
//   * the single barrier at the top of tile t proves (a) every wave has finished reading tile t
//     (its reads completed, lgkmcnt(0), before the barrier), so slot t % 4 can be refilled with
//     tile t+4 right after it, and (b) tile t+1 has landed for every wave (each wave waited
//     vmcnt for its own DMA pieces of t+1 before the barrier);
//   * every K-tile issues the same 8 DMA pieces per wave (pieces past the end of K are sent to an
//     out-of-range offset: hardware zero-fill into a dead slot), so the loop body is branch free
//     and the wait is always vmcnt(16) (tiles t+2 and t+3 stay in flight);
//   * XCD-aware bijective remap + GROUP_M = 8 tile order, as gemm256.hip.
// Same operand images, swizzles and epilogue as gemm256.hip (gemm256_tile.h). Requires K % 128 == 0
// (a multiple of 4 K-tiles per split-K chunk), 16-B aligned operand rows, operands < 2 GiB.
#include "gemm256_tile.h"

namespace ffk {
namespace w4 {
using namespace g256;

constexpr int BN = 256, BK = 32, NBUF = 4, NTH = 256;
constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
constexpr int A_PIECES = A_BYTES / 1024, PIECES = STAGE / 1024, PW = PIECES / 4;

// byte offset of this lane's 16 B of DMA piece pc of the K-tile starting at k0
template <bool KCONT>
__device__ __forceinline__ int piece_off(int64_t ld, int mn0, int k0, int pc, int lane) {
  constexpr int CPR = BK / 8;
  int64_t elem;
  if (KCONT) {
    const int row = pc * (64 / CPR) + lane / CPR;
    const int c = (lane % CPR) ^ swz_k<BK>(row);
    elem = (int64_t)(mn0 + row) * ld + k0 + c * 8;
  } else {
    const int half = pc / (BK / 4);
    const int krow = (pc % (BK / 4)) * 4 + (lane >> 4);
    const int c = (lane & 15) ^ swz_mn(krow);
    elem = (int64_t)(k0 + krow) * ld + mn0 + half * 128 + c * 8;
  }
  return (int)(elem * 2);
}

// Fragment read as frag<KCONT, BK>. The MN-contiguous (transposing) form is inline asm: hipcc puts
// an s_waitcnt vmcnt(0) in front of every ds_read_b64_tr_b16 builtin while LDS-DMA is in flight
// (it cannot tell that the read and the DMA touch different slots), which drains the whole ring
// once per fragment. The asm results are consumed only after the step's lgkmcnt(0).
template <bool KCONT>
__device__ __forceinline__ bf16x8 frag_w4(const char* tile, int r0, int lane) {
  if constexpr (KCONT) {
    return frag<true, BK>(tile, r0, 0, lane);
  } else {
    const char* hl = tile + (r0 >> 7) * (BK * 256);
    const int rr = r0 & 127;
    const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
    const int chunk = (rr >> 3) + (pp >> 1);
    const int k0 = 8 * g + q, k1 = 8 * g + 4 + q;
    const unsigned a0 = (unsigned)(uintptr_t)(hl + k0 * 256 + ((chunk ^ swz_mn(k0)) << 4) + 8 * (pp & 1));
    const unsigned a1 = (unsigned)(uintptr_t)(hl + k1 * 256 + ((chunk ^ swz_mn(k1)) << 4) + 8 * (pp & 1));
    typedef short v4s __attribute__((ext_vector_type(4)));
    v4s lo, hi;
    asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %3" : "=v"(lo), "=v"(hi) : "v"(a0), "v"(a1));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  }
}

template <bool A_K, bool B_K, int OUT_MODE>
__global__ void __launch_bounds__(NTH, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) gemm_w4_kernel(GemmArgs p, int64_t a_bytes, int64_t b_bytes) {
  constexpr int WN = 128, NF = 8;
  __shared__ __attribute__((aligned(1024))) char smem[NBUF * STAGE];

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

  // DMA pieces: waves 0-1 stage A, waves 2-3 stage B (wave-uniform), piece pc lands at slot + pc KiB.
  // A piece's source offset is its K-tile-0 offset plus t times the operand's K-tile stride;
  // pieces of tiles past the end of K go to an out-of-range offset (hardware zero-fill).
  const bool isA = wave < 2;
  const __amdgpu_buffer_rsrc_t rs = isA ? ra : rb;
  const int kstride = isA ? (A_K ? BK * 2 : BK * (int)p.lda * 2) : (B_K ? BK * 2 : BK * (int)p.ldb * 2);
  int boff[PW];
#pragma unroll
  for (int g = 0; g < PW; ++g) {
    const int pc = wave * PW + g;
    boff[g] = isA ? piece_off<A_K>(p.lda, m0, kbeg, pc, lane) : piece_off<B_K>(p.ldb, n0, kbeg, pc - A_PIECES, lane);
  }
  auto dma_off = [&](int t, int g) { return t < nk ? boff[g] + t * kstride : 0x7ffffff0; };
  auto dma = [&](int slot, int off, int g) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(smem + slot * STAGE + (wave * PW + g) * 1024), 16, off, 0, 0, 0);
  };
  auto read = [&](int slot, bf16x8(&af)[8], bf16x8(&bf)[NF]) {
    const char* cur = smem + slot * STAGE;
#pragma unroll
    for (int j = 0; j < NF; ++j) bf[j] = frag_w4<B_K>(cur + A_BYTES, wc * WN + j * 16, lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = frag_w4<A_K>(cur, wr * 128 + i * 16, lane);
  };

  // prologue: tiles 0..3 in flight, tile 0 landed everywhere, its fragments in set 0
#pragma unroll
  for (int t = 0; t < NBUF; ++t)
#pragma unroll
    for (int g = 0; g < PW; ++g) dma(t, dma_off(t, g), g);
  wait_vm<3 * PW>();
  barrier();
  bf16x8 a0[8], b0[NF], a1[8], b1[NF];
  read(0, a0, b0);
  lgkm0();

  // The MFMAs are inline asm with "+a" accumulators: with two fragment sets live (128 VGPRs),
  // hipcc otherwise picks the VGPR form of the builtin and copies all 256 accumulators into the
  // AGPR file after every MFMA, or spills them. The issue order is pinned group by group with
  // sched_barrier(0): 16 groups of 4 MFMAs, each carrying one LDS fragment read for tile t+1 and
  // (first 8 groups) one DMA piece for tile t+4. The loop is unrolled by the ring depth, so slot
  // offsets are immediates.
  auto step = [&](auto slot_c, int t, bf16x8(&ac)[8], bf16x8(&bc)[NF], bf16x8(&an)[8], bf16x8(&bn)[NF]) {
    constexpr int S = decltype(slot_c)::value;  // t % 4
    wait_vm<2 * PW>();  // this wave's pieces of tile t+1 have landed (t+2, t+3 stay in flight)
    barrier();          // ... and everyone's; every wave has finished reading tile t (slot S)
    const char* nx = smem + ((S + 1) % NBUF) * STAGE;
    // MN-contiguous fragments take two lane-dependent addresses each; with a literal slot offset
    // hipcc keeps a full address set per ring slot live (4 x 64 VGPRs) and spills. An opaque slot
    // base costs one v_add per read instead.
    int so = ((S + 1) % NBUF) * STAGE;
    asm volatile("" : "+s"(so));
    const char* nxo = smem + so;
    // The DMA offsets are computed up front and kept live to the end of the step: hipcc treats a
    // pending LDS-DMA as still reading its offset VGPR and puts an s_waitcnt vmcnt(0) (draining
    // the whole ring) in front of any later write of that register, e.g. a fragment read.
    int off[PW];
#pragma unroll
    for (int g = 0; g < PW; ++g) off[g] = dma_off(t + NBUF, g);
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      if (g < PW) dma(S, off[g], g);
      if (g < NF) bn[g] = frag_w4<B_K>((B_K ? nx : nxo) + A_BYTES, wc * WN + g * 16, lane);
      else an[g - NF] = frag_w4<A_K>(A_K ? nx : nxo, wr * 128 + (g - NF) * 16, lane);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = g >> 1, j = (g & 1) * 4 + q;
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(bc[j]), "v"(ac[i]));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    lgkm0();
#pragma unroll
    for (int g = 0; g < PW; ++g) asm volatile("" ::"v"(off[g]));
  };
  asm volatile("s_nop 4");  // v_accvgpr_write (zero-init) -> MFMA C operand
  for (int t = 0; t < nk; t += 4) {  // nk % 4 == 0 (K % 128 == 0, split-K chunks multiples of 128)
    step(std::integral_constant<int, 0>(), t, a0, b0, a1, b1);
    step(std::integral_constant<int, 1>(), t + 1, a1, b1, a0, b0);
    step(std::integral_constant<int, 2>(), t + 2, a0, b0, a1, b1);
    step(std::integral_constant<int, 3>(), t + 3, a1, b1, a0, b0);
  }
  asm volatile("s_nop 15\n\ts_nop 3");  // last MFMA's D -> first accumulator read of the epilogue
  // drain the (dummy) DMAs of the last tiles before the ring is reused as the epilogue stage
  wait_vm<0>();
  barrier();
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
  if (p.dact || !p.vec8_ok || p.K % 128 != 0 || a_bytes > 0x7fffffffLL || b_bytes > 0x7fffffffLL || a_bytes <= 0 || b_bytes <= 0) return false;
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

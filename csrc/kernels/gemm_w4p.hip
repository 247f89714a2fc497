// Persistent 4-wave 256 x 256 x 64 bf16 MFMA GEMM: one workgroup per CU walks its output tiles
// (tile = blockIdx.x, + gridDim.x, ...; XCD-grouped order of gemm256_tile.h tile_coords), and the
// next tile's first two K-tiles are requested by LDS-DMA BEFORE this tile's epilogue runs.
//
// Why: with one tile per workgroup (gemm_w4.hip) every CU reaches its epilogue at the same moment,
// so the whole chip stores its 128 KiB output tiles together (32 MiB at once: ~5 us of HBM write
// bandwidth) and then loads the next tiles' first K-tiles together — ~10 us per tile of prologue +
// epilogue in which no MFMA issues (BERT-Large K = 1024 GEMMs: 3-4 tiles per CU, a 25-30 % gap to
// hipBLASLt, whose kernels for these shapes are persistent stream-K launches of 256 workgroups).
// Here the DMA of tile i+1 is in flight while tile i's accumulators leave, and tile i's stores
// drain while tile i+1's main loop runs: the vmcnt waits of its first K-steps are counted so that
// they never wait for those stores (stores, loads and LDS-DMA retire in one in-order queue).
//
// The epilogue stages through a wave-private 8 KiB fp32 image outside the operand ring (16 rows x
// 128 columns per pass, 16-B chunks XOR-swizzled by row: conflict-free writes), so the ring can
// receive the next tile while it runs. Epilogues: alpha, bias (fp32 / bf16, loaded before the
// next tile's DMA is issued so the compiler's wait for it never covers the DMA), bf16 or fp32
// output. No activation / beta / split-K / pre-activation output (those run gemm_w4.hip).
// Main loop: gemm_w4.hip's (inline-asm MFMAs on AGPR accumulators, pinned issue order, two-slot
// ring, K-tile in halves around one barrier). Requires batch 1, K % 128 == 0, N % 8 == 0.
#include "gemm_w4_core.h"

namespace ffk {
namespace w4 {

constexpr int EPI_ROWS = 16;
constexpr int EPI_WAVE = EPI_ROWS * 128 * 4;  // bytes of one wave's fp32 staging image

template <bool A_K, bool B_K, bool F32OUT>
__global__ void __launch_bounds__(NTH, 1) __attribute__((amdgpu_waves_per_eu(1, 1)))
gemm_w4p_kernel(GemmArgs p, int64_t a_bytes, int64_t b_bytes) {
  constexpr int WN = 128, NF = 8;
  // stores per lane in one epilogue (16-B each): the count the first waits of a tile leave in flight
  constexpr int STORES = (F32OUT ? 2 : 1) * (128 / EPI_ROWS) * (EPI_ROWS * 128 / 8 / 64);
  constexpr int WAIT_K0 = (STORES + PW) > 63 ? 63 : (STORES + PW);
  constexpr int WAIT_K1 = (STORES + 2) > 63 ? 63 : (STORES + 2);  // + the tile's two bias loads
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE + 4 * EPI_WAVE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int tm = (p.M + BM - 1) / BM, tn = (p.N + BN - 1) / BN;
  const int total = tm * tn;
  const int nk = p.K / BK;
  int tile = blockIdx.x;
  if (tile >= total) return;

  __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, (int)min(a_bytes, (int64_t)0x7fffffff), 0x00020000);
  __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, (int)min(b_bytes, (int64_t)0x7fffffff), 0x00020000);
  const bool isA = wave < 2;
  const __amdgpu_buffer_rsrc_t rs = isA ? ra : rb;
  const int kstride = isA ? (A_K ? BK * 2 : BK * (int)p.lda * 2) : (B_K ? BK * 2 : BK * (int)p.ldb * 2);
  static_assert(PW == 16, "piece_lane_off assumes 16 pieces per wave");
  const int wl = wave & 1;
  const int gstride = isA ? piece_gstride<A_K>(p.lda) : piece_gstride<B_K>(p.ldb);
  int vb[4];
  auto set_tile = [&](int tmi, int tni) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      vb[q] = isA ? piece_lane_off<A_K>(p.lda, tmi * BM, 0, wl, q, lane)
                  : piece_lane_off<B_K>(p.ldb, tni * BN, 0, wl, q, lane);
  };
  auto dma = [&](int slot, int t, int g) __attribute__((always_inline)) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(smem + slot * STAGE + (wave * PW + g) * 1024), 16,
                                             vb[g & 3] + g * gstride, t * kstride, 0, 0);
  };

  int tile_m, tile_n;
  tile_coords(tile, tm, tn, tile_m, tile_n);
  set_tile(tile_m, tile_n);
#pragma unroll
  for (int g = 0; g < PW; ++g) dma(0, 0, g);
#pragma unroll
  for (int g = 0; g < PW; ++g) dma(1, 1, g);
  vmcnt<PW>();
  barrier();
  bf16x8 a0[8], b0[NF], a1[8], b1[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) b0[j] = frag64<B_K>(smem + A_BYTES, wc * WN + j * 16, 0, lane);
#pragma unroll
  for (int i = 0; i < 8; ++i) a0[i] = frag64<A_K>(smem, wr * 128 + i * 16, 0, lane);
  lgkm0();

  f32x4 acc[8][NF];
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
  auto step = [&](auto slot_c, int t, bool first) __attribute__((always_inline)) {
    constexpr int S = decltype(slot_c)::value;
    const char* cur = smem + S * STAGE;
    const char* nxt = smem + (S ^ 1) * STAGE;
    int so = S * STAGE, sn = (S ^ 1) * STAGE;
    asm volatile("" : "+s"(so), "+s"(sn));
    half(a0, b0, a1, b1, cur, smem + so, 1, false, 0, 0);
    // K-tile t+1 landed; on a tile's first step the previous epilogue's stores (issued after it)
    // may still be in flight
    if (first) vmcnt<WAIT_K1>();
    else vmcnt<0>();
    barrier();
    half(a1, b1, a0, b0, nxt, smem + sn, 0, t + 2 < nk, S, t + 2);
  };

  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  float* st = reinterpret_cast<float*>(smem + 2 * STAGE + wave * EPI_WAVE);
  typedef typename std::conditional<F32OUT, float, bf16_t>::type OutT;
  const int64_t c_bytes = (int64_t)p.M * p.ldc * (int64_t)sizeof(OutT);
  __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(p.C, (short)0, (int)min(c_bytes, (int64_t)0x7fffffff), 0x00020000);
  const int c8 = (lane & 15) * 8;  // this lane's 8-column chunk of the wave's 128 columns (fixed)
  // bias: two 16-B range-checked loads per tile whatever its type (a null bias has zero records and
  // reads zeros), so the counted waits see the same number of loads in every configuration
  const int bsz = p.bias ? (p.bias_bf16 ? 2 : 4) : 0;
  __amdgpu_buffer_rsrc_t rbias = __builtin_amdgcn_make_buffer_rsrc((void*)(p.bias ? p.bias : p.A), (short)0,
                                                                   p.N * bsz, 0x00020000);
  bool first_tile = true;
  for (;;) {
    // issued here (behind this tile's first K-tiles) and first used right after the main loop,
    // before the next tile's DMA: the wait hipcc puts in front of that use retires nothing else
    const int nb = tile_n * BN + wc * WN + c8;
    const u32x4 bia0 = __builtin_amdgcn_raw_buffer_load_b128(rbias, nb < p.N ? nb * bsz : 0x7ffffff0, 0, 0);
    const u32x4 bia1 = __builtin_amdgcn_raw_buffer_load_b128(rbias, nb < p.N ? nb * bsz + 16 : 0x7ffffff0, 0, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    pin_acc(acc);
    asm volatile("s_nop 4");
    for (int t = 0; t < nk; t += 2) {  // nk even
      step(std::integral_constant<int, 0>(), t, t == 0 && !first_tile);
      step(std::integral_constant<int, 1>(), t + 1, false);
    }
    asm volatile("s_nop 15\n\ts_nop 3");
    pin_acc(acc);
    barrier();  // every wave has finished reading the ring: the next tile may be staged into it

    const int m0 = tile_m * BM + wr * 128, n = tile_n * BN + wc * WN + c8;
    float bb[8];
    if (p.bias_bf16) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bb[2 * e] = __uint_as_float(bia0[e] << 16);
        bb[2 * e + 1] = __uint_as_float(bia0[e] & 0xffff0000u);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bb[e] = __uint_as_float(bia0[e]);
        bb[4 + e] = __uint_as_float(bia1[e]);
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) asm volatile("" : "+v"(bb[e]));  // materialised before the DMA below
    const int next = tile + (int)gridDim.x;
    const bool more = next < total;
    int ntm = 0, ntn = 0;
    if (more) {
      tile_coords(next, tm, tn, ntm, ntn);
      set_tile(ntm, ntn);
#pragma unroll
      for (int g = 0; g < PW; ++g) dma(0, 0, g);
#pragma unroll
      for (int g = 0; g < PW; ++g) dma(1, 1, g);
    }
    // epilogue: 8 passes of 16 rows; write a pass's accumulators into the wave's image, read it
    // back 8 consecutive columns per lane, one 16-B (bf16) / 2 x 16-B (fp32) store per row chunk
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      __builtin_amdgcn_sched_barrier(0);
      // re-define this pass's accumulators in the AGPR file right here: their AGPR -> VGPR copies
      // then follow this point (hipcc otherwise copied all 256 right after the loop and spilled,
      // and the spill reloads' vmcnt waits covered the next tile's DMA)
#pragma unroll
      for (int j = 0; j < NF; ++j) asm volatile("" : "+a"(acc[i][j]));
      const int r16 = lane & 15;
      // the staging image is written and read by inline asm: hipcc cannot tell it from the ring the
      // DMA above is filling and put an s_waitcnt vmcnt(0) in front of the first LDS write, which
      // made the epilogue wait for the next tile's K-tiles. A wave's LDS operations run in order,
      // so the read-back needs no wait behind the writes; the lgkmcnt(0) below covers the reads.
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        const f32x4 v = acc[i][j];
        const int ch = (j * 4 + (lane >> 4)) ^ (r16 & 7);
        const f32x4 w = {v[0] * p.alpha, v[1] * p.alpha, v[2] * p.alpha, v[3] * p.alpha};
        const unsigned a = (unsigned)(uintptr_t)(st + r16 * 128 + ch * 4);
        asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(w) : "memory");
      }
      f32x4 lov[4], hiv[4];
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int r = it * 4 + (lane >> 4);
        const int q0 = (2 * (lane & 15)) ^ (r & 7), q1 = (2 * (lane & 15) + 1) ^ (r & 7);
        const unsigned a0r = (unsigned)(uintptr_t)(st + r * 128 + q0 * 4);
        const unsigned a1r = (unsigned)(uintptr_t)(st + r * 128 + q1 * 4);
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3" : "=&v"(lov[it]), "=&v"(hiv[it]) : "v"(a0r), "v"(a1r) : "memory");
      }
      lgkm0();
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int r = it * 4 + (lane >> 4);
        const f32x4 lo = lov[it], hi = hiv[it];
        const int m = m0 + i * 16 + r;
        float x[8] = {lo[0] + bb[0], lo[1] + bb[1], lo[2] + bb[2], lo[3] + bb[3],
                      hi[0] + bb[4], hi[1] + bb[5], hi[2] + bb[6], hi[3] + bb[7]};
        // every lane issues its stores (the waits above count them): rows past M fall outside the
        // buffer's range and columns past N get an out-of-range offset, so the hardware drops them
        // ablate 1: every store dropped by the range check (issued, no memory traffic)
        const bool in = m < p.M && n < p.N && p.ablate == 0;
        const int off = in ? (int)(((int64_t)m * p.ldc + n) * (int64_t)sizeof(OutT)) : 0x7ffffff0;
        if constexpr (F32OUT) {
          u32x4 v0 = {__float_as_uint(x[0]), __float_as_uint(x[1]), __float_as_uint(x[2]), __float_as_uint(x[3])};
          u32x4 v1 = {__float_as_uint(x[4]), __float_as_uint(x[5]), __float_as_uint(x[6]), __float_as_uint(x[7])};
          __builtin_amdgcn_raw_buffer_store_b128(v0, rc, off, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b128(v1, rc, in ? off + 16 : off, 0, 0);
        } else {
          u32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = (uint32_t)f2bf(x[2 * e]) | ((uint32_t)f2bf(x[2 * e + 1]) << 16);
          __builtin_amdgcn_raw_buffer_store_b128(v, rc, off, 0, 0);
        }
      }
    }
    if (!more) break;
    tile = next;
    tile_m = ntm;
    tile_n = ntn;
    first_tile = false;
    vmcnt<WAIT_K0>();  // K-tile 0 of the next tile has landed for this wave (K-tile 1 and the stores may not) ...
    barrier();         // ... and for every wave
#pragma unroll
    for (int j = 0; j < NF; ++j) b0[j] = frag64<B_K>(smem + A_BYTES, wc * WN + j * 16, 0, lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) a0[i] = frag64<A_K>(smem, wr * 128 + i * 16, 0, lane);
    lgkm0();
  }
}

template <bool F32OUT>
static void launch_p(const GemmArgs& p, dim3 grid, hipStream_t s, int64_t ab, int64_t bb) {
  if (p.a_kcontig && p.b_kcontig) hipLaunchKernelGGL((gemm_w4p_kernel<true, true, F32OUT>), grid, dim3(NTH), 0, s, p, ab, bb);
  else if (p.a_kcontig) hipLaunchKernelGGL((gemm_w4p_kernel<true, false, F32OUT>), grid, dim3(NTH), 0, s, p, ab, bb);
  else if (p.b_kcontig) hipLaunchKernelGGL((gemm_w4p_kernel<false, true, F32OUT>), grid, dim3(NTH), 0, s, p, ab, bb);
  else hipLaunchKernelGGL((gemm_w4p_kernel<false, false, F32OUT>), grid, dim3(NTH), 0, s, p, ab, bb);
}

}  // namespace w4

static int g_cus = 0;

bool gemm_w4p_bf16(const GemmArgs& p, int64_t a_bytes, int64_t b_bytes, hipStream_t stream) {
  using namespace w4;
  if (p.dact || p.Z || p.act != ACT_NONE || p.beta != 0.f || p.batch != 1 || (p.splitk > 1 && p.ws) || !p.vec8_ok || p.K % 128 != 0 ||
      p.K <= 0 || a_bytes > 0x7fffffffLL || b_bytes > 0x7fffffffLL || a_bytes <= 0 || b_bytes <= 0)
    return false;
  if (((uintptr_t)p.A & 15) || ((uintptr_t)p.B & 15) || p.lda % 8 || p.ldb % 8) return false;
  if ((int64_t)p.M * p.ldc * (p.out_f32 ? 4 : 2) > 0x7fffff00LL) return false;  // buffer-store offsets
  if (!p.a_kcontig && p.M % 8) return false;
  if (!p.b_kcontig && p.N % 8) return false;
  if (p.bias && ((uintptr_t)p.bias & 15)) return false;
  if (g_cus == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_cus <= 0) g_cus = 256;
  }
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  dim3 grid(std::min(tiles, g_cus));
  if (p.out_f32) launch_p<true>(p, grid, stream, a_bytes, b_bytes);
  else launch_p<false>(p, grid, stream, a_bytes, b_bytes);
  return true;
}

}  // namespace ffk

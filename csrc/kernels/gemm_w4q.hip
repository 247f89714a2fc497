// Persistent 4-wave 256 x 256 bf16 MFMA GEMM with a 4-deep K ring (BK = 32): gemm_w4p.hip's tile
// walk and epilogue, with the operand ring cut into four 32-KiB slots instead of two 64-KiB ones.
//
// Why: gemm_w4p issues the LDS-DMA of K-tile t+2 in the middle of step t and waits for it in the
// middle of step t+1, one 2048-cycle step of MFMAs later (~0.85 us): under a whole-chip load an L2
// miss takes longer, and the waves sat on s_waitcnt 23-31 % of their cycles against hipBLASLt's
// 9 % (profiles/gemm_w4_vs_lib_pmc_r3.txt). Here K-tile t+4 is issued at the top of step t into the
// slot whose fragments were read during step t-1, and K-tile t+1 is waited for at the top of step
// t (its fragments are read during step t): every DMA has three 1024-cycle steps to land. The same
// 128 KiB ring + 32 KiB epilogue staging (160 KiB, one workgroup per CU).
//
// Step t (slot t % 4, compile-time through a 4x unrolled loop):
//   counted vmcnt: K-tile t+1 landed (t+2, t+3 and, on a tile's first steps, the previous tile's
//   epilogue stores may still be in flight) -> barrier -> 64 MFMAs on the fragments of K-tile t,
//   interleaved with the fragment reads of K-tile t+1 and the 8 DMA pieces of K-tile t+4 (slot t % 4).
// At the top of a tile's last step the ring is free: the next tile's bias and first four K-tiles
// are requested there, so they land under the last step and the epilogue.
// Requires batch 1, K % 128 == 0, N % 8 == 0 (same as gemm_w4p).
#include "gemm_w4_core.h"

namespace ffk {
namespace w4q {
using namespace g256;
using w4::vmcnt;

constexpr int BN = 256, BK = 32, NTH = 256, NSLOT = 4;
constexpr int A_BYTES = BM * BK * 2, STAGE = A_BYTES + BN * BK * 2;  // 16 + 16 KiB
constexpr int PW = STAGE / 1024 / 4;                                // DMA pieces per wave per K-tile (8)
constexpr int EPI_ROWS = 16;
constexpr int EPI_WAVE = EPI_ROWS * 128 * 4;

// Per-lane byte offset of piece g = 0..7 of wave-half wl (pieces wl * 8 + g of its operand) at
// K-tile 0, minus g * piece_gstride: K-contiguous pieces are 16 rows of 64 B (swizzle from lane
// bits only), MN-contiguous pieces 4 k-rows of one 128-wide half (swizzle sees g & 3 = q).
template <bool KCONT>
__device__ __forceinline__ int piece_lane_off(int64_t ld, int mn0, int wl, int q, int lane) {
  int64_t elem;
  if (KCONT) {
    const int row = wl * 128 + (lane >> 2);
    elem = (int64_t)(mn0 + row) * ld + (((lane & 3) ^ swz_k<BK>(row)) * 8);
  } else {
    const int swz = ((lane >> 4) << 2) | q;
    elem = (int64_t)(lane >> 4) * ld + mn0 + wl * 128 + ((lane & 15) ^ swz) * 8;
  }
  return (int)(elem * 2);
}
template <bool KCONT>
__device__ __forceinline__ int piece_gstride(int64_t ld) {
  return (int)((KCONT ? 16 : 4) * ld * 2);
}

// 16 x 32 fragment of a BK = 32 slot (gemm256_tile.h frag<KCONT, 32> layout); the MN-contiguous
// (transposing) read is inline asm for the reason given at w4::frag64
template <bool KCONT>
__device__ __forceinline__ bf16x8 fragq(const char* tile, int r0, int lane) {
  if constexpr (KCONT) {
    const int row = r0 + (lane & 15);
    const int c = lane >> 4;
    return *reinterpret_cast<const bf16x8*>(tile + row * (BK * 2) + ((c ^ swz_k<BK>(row)) << 4));
  } else {
    const char* hl = tile + (r0 >> 7) * (BK * 256);
    const int rr = r0 & 127;
    const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
    const int chunk = (rr >> 3) + (pp >> 1);
    const int k0 = 8 * g + q, k1 = k0 + 4;
    const unsigned a0 = (unsigned)(uintptr_t)(hl + k0 * 256 + ((chunk ^ swz_mn(k0)) << 4) + 8 * (pp & 1));
    const unsigned a1 = (unsigned)(uintptr_t)(hl + k1 * 256 + ((chunk ^ swz_mn(k1)) << 4) + 8 * (pp & 1));
    typedef short v4s __attribute__((ext_vector_type(4)));
    v4s lo, hi;
    asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %3" : "=&v"(lo), "=&v"(hi) : "v"(a0), "v"(a1));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  }
}

// s_waitcnt vmcnt with the allowance chosen at run time among compile-time immediates: n_after
// K-tiles (0..3) of this wave's DMAs may stay in flight, plus `stores` epilogue stores
template <int STORES>
__device__ __forceinline__ void wait_after(int n_after, bool stores) {
  constexpr int S = STORES;
  if (stores) {
    if (n_after >= 3) vmcnt<(3 * PW + S > 63 ? 63 : 3 * PW + S)>();
    else if (n_after == 2) vmcnt<(2 * PW + S > 63 ? 63 : 2 * PW + S)>();
    else if (n_after == 1) vmcnt<(PW + S > 63 ? 63 : PW + S)>();
    else vmcnt<(S > 63 ? 63 : S)>();
  } else {
    if (n_after >= 3) vmcnt<3 * PW>();
    else if (n_after == 2) vmcnt<2 * PW>();
    else if (n_after == 1) vmcnt<PW>();
    else vmcnt<0>();
  }
}

// ABL (timing-only builds, impl 50+ in the probes; outputs are NOT valid): bit 0 drops every
// store (range check), bit 1 issues no main-loop DMA (the MFMAs re-read the prologue's K-tiles),
// bit 2 also drops the per-step barrier — what is left is the MFMA + LDS-read stream alone;
// bit 3 keeps every DMA but re-reads K-tiles 0..3 (L2-resident: the issue cost without the latency);
// bit 5: global_load_lds instead of buffer_load ... lds (outputs valid; whole tiles only).
// CPOL: cache-policy bits of the operand DMAs (gfx950 CPol: sc0 = 1, nt = 2, sc1 = 16).
template <bool A_K, bool B_K, bool F32OUT, int ABL = 0, int CPOL = 0>
__global__ void __launch_bounds__(NTH, 1) __attribute__((amdgpu_waves_per_eu(1, 1)))
gemm_w4q_kernel(GemmArgs p, int64_t a_bytes, int64_t b_bytes) {
  constexpr int WN = 128, NF = 8;
  constexpr int STORES = (F32OUT ? 2 : 1) * (128 / EPI_ROWS) * (EPI_ROWS * 128 / 8 / 64);
  __shared__ __attribute__((aligned(1024))) char smem[NSLOT * STAGE + 4 * EPI_WAVE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int tm = (p.M + BM - 1) / BM, tn = (p.N + BN - 1) / BN;
  const int total = tm * tn;
  const int nk = p.K / BK;  // multiple of 4
  int tile = blockIdx.x;
  if (tile >= total) return;

  __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, (int)min(a_bytes, (int64_t)0x7fffffff), 0x00020000);
  __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, (int)min(b_bytes, (int64_t)0x7fffffff), 0x00020000);
  const bool isA = wave < 2;
  const __amdgpu_buffer_rsrc_t rs = isA ? ra : rb;
  const int kstride = isA ? (A_K ? BK * 2 : BK * (int)p.lda * 2) : (B_K ? BK * 2 : BK * (int)p.ldb * 2);
  const int wl = wave & 1;
  const int gstride = isA ? piece_gstride<A_K>(p.lda) : piece_gstride<B_K>(p.ldb);
  int vb[4];
  auto set_tile = [&](int tmi, int tni) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      vb[q] = isA ? piece_lane_off<A_K>(p.lda, tmi * BM, wl, q, lane) : piece_lane_off<B_K>(p.ldb, tni * BN, wl, q, lane);
  };
  // piece g of this wave's share of K-tile t into slot `slot`; dma() issues all 8 (prologue, seam)
  const char* gbase = (const char*)(isA ? p.A : p.B);
  auto dma1 = [&](int slot, int t, int g) __attribute__((always_inline)) {
    if constexpr (ABL & 32) {  // global_load_lds instead of the buffer form (timing ablation: no range check)
      typedef __attribute__((address_space(1))) void* gptr_t;
      __builtin_amdgcn_global_load_lds((gptr_t)(gbase + (int64_t)(vb[g & 3] + g * gstride) + (int64_t)t * kstride),
                                       (lds_ptr_t)(smem + slot * STAGE + (wave * PW + g) * 1024), 16, 0, 0);
    } else {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(smem + slot * STAGE + (wave * PW + g) * 1024), 16,
                                               vb[g & 3] + g * gstride, t * kstride, 0, CPOL);
    }
  };
  auto dma = [&](int slot, int t) __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < PW; ++g) dma1(slot, t, g);
  };

  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const int c8 = (lane & 15) * 8;
  const int bsz = p.bias ? (p.bias_bf16 ? 2 : 4) : 0;
  __amdgpu_buffer_rsrc_t rbias = __builtin_amdgcn_make_buffer_rsrc((void*)(p.bias ? p.bias : p.A), (short)0,
                                                                   p.N * bsz, 0x00020000);
  // bias of a tile: two range-checked 16-B loads issued BEFORE its K-tiles (so the counted waits
  // never see them); a null bias has zero records and reads zeros
  auto bias_load = [&](int tni, u32x4& b0, u32x4& b1) __attribute__((always_inline)) {
    const int nb = tni * BN + wc * WN + c8;
    b0 = __builtin_amdgcn_raw_buffer_load_b128(rbias, nb < p.N ? nb * bsz : 0x7ffffff0, 0, 0);
    b1 = __builtin_amdgcn_raw_buffer_load_b128(rbias, nb < p.N ? nb * bsz + 16 : 0x7ffffff0, 0, 0);
  };

  int tile_m, tile_n;
  tile_coords(tile, tm, tn, tile_m, tile_n);
  set_tile(tile_m, tile_n);
  u32x4 bia0, bia1;
  bias_load(tile_n, bia0, bia1);
#pragma unroll
  for (int s = 0; s < NSLOT; ++s) dma(s, s);
  vmcnt<3 * PW>();
  barrier();
  bf16x8 a0[8], b0[NF], a1[8], b1[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) b0[j] = fragq<B_K>(smem + A_BYTES, wc * WN + j * 16, lane);
#pragma unroll
  for (int i = 0; i < 8; ++i) a0[i] = fragq<A_K>(smem, wr * 128 + i * 16, lane);
  lgkm0();

  f32x4 acc[8][NF];
  float bb[8];
  bool first_tile = true;
  bool more = false;
  int ntm = 0, ntn = 0;

  // 64 MFMAs on (ac, bc) with the fragment reads of the slot at `src` into (an, bn) spread over them
  // K-contiguous reads take the slot base as a ds_read immediate (src); the transposing reads are
  // asm (no immediate), so their slot base is an opaque scalar (srco) added per read: otherwise
  // hipcc keeps one set of 16 lane addresses per slot and spills
  // The main-loop DMA pieces (dslot >= 0) go one per two MFMA groups: issued in a burst after the
  // barrier they held the wave's MFMA issue for ~25 % of the step (probe ablations: 'w4q_samek').
  auto mfmas = [&](bf16x8(&ac)[8], bf16x8(&bc)[NF], bf16x8(&an)[8], bf16x8(&bn)[NF], const char* src,
                   const char* srco, bool load, int dslot, int dt) __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      if (dslot >= 0 && (g & 1) == 0) dma1(dslot, dt, g >> 1);
      if (load && g < 8) {
        // (mixed layouts: both through the scalar base, which left hipcc the registers to not spill)
        constexpr bool IMM = A_K && B_K;
        bn[g] = fragq<B_K>((IMM ? src : srco) + A_BYTES, wc * WN + g * 16, lane);
        an[g] = fragq<A_K>(IMM ? src : srco, wr * 128 + g * 16, lane);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = g >> 1, j = (g & 1) * 4 + q;
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(bc[j]), "v"(ac[i]));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (load) lgkm0();
  };

  // step t on slot S = t % 4 (fragments of K-tile t in (ac, bc)). FULL: a step of a K-group that
  // is not the tile's last (K-tile t+4 exists: DMA it into slot S, and two K-tiles stay in flight
  // behind t+1). Otherwise the step is one of the last four: fewer in flight, no DMA, and the last
  // one (S == 3) has no fragments to read and starts the next tile's loads.
  auto step = [&](auto slot_c, auto full_c, int t, bf16x8(&ac)[8], bf16x8(&bc)[NF], bf16x8(&an)[8],
                  bf16x8(&bn)[NF]) __attribute__((always_inline)) {
    constexpr int S = decltype(slot_c)::value;
    constexpr bool FULL = decltype(full_c)::value;
    constexpr bool LAST = !FULL && S == 3;
    // K-tile t+1 landed: allowed in flight behind it are K-tiles t+2 .. min(t+3, nk-1) and, while
    // t+1 <= 3 on a tile after the first, the previous epilogue's stores
    constexpr int N_AFTER = FULL ? 2 : 2 - S;
    if constexpr (!LAST && !(ABL & 2)) wait_after<STORES>(N_AFTER, S < 3 && t < 3 && !first_tile);
    if constexpr (!(ABL & 4)) barrier();
    constexpr bool DMA = FULL && !(ABL & 2);
    if constexpr (LAST) {
      // the ring is free (every fragment read is done): the next tile's bias and K-tiles 0..3 go
      // out now, under this step's MFMAs and the epilogue. This tile's bias leaves its registers
      // first (its load retired long ago), so the compiler's wait for it covers nothing new.
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
      for (int e = 0; e < 8; ++e) asm volatile("" : "+v"(bb[e]));
      const int next = tile + (int)gridDim.x;
      more = next < total;
      if (more) {
        tile_coords(next, tm, tn, ntm, ntn);
        set_tile(ntm, ntn);
        bias_load(ntn, bia0, bia1);
#pragma unroll
        for (int s = 0; s < NSLOT; ++s) dma(s, s);
      }
    }
    int so = ((S + 1) & 3) * STAGE;
    asm volatile("" : "+s"(so));
    mfmas(ac, bc, an, bn, smem + ((S + 1) & 3) * STAGE, smem + so, !LAST, DMA ? S : -1, (ABL & 8) ? S : t + 4);
  };
  auto group = [&](auto full_c, int t) __attribute__((always_inline)) {
    step(std::integral_constant<int, 0>(), full_c, t, a0, b0, a1, b1);
    step(std::integral_constant<int, 1>(), full_c, t + 1, a1, b1, a0, b0);
    step(std::integral_constant<int, 2>(), full_c, t + 2, a0, b0, a1, b1);
    step(std::integral_constant<int, 3>(), full_c, t + 3, a1, b1, a0, b0);
  };

  float* st = reinterpret_cast<float*>(smem + NSLOT * STAGE + wave * EPI_WAVE);
  typedef typename std::conditional<F32OUT, float, bf16_t>::type OutT;
  const int64_t c_bytes = (int64_t)p.M * p.ldc * (int64_t)sizeof(OutT);
  __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(p.C, (short)0, (int)min(c_bytes, (int64_t)0x7fffffff), 0x00020000);
  for (;;) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    pin_acc(acc);
    asm volatile("s_nop 4");
    int t = 0;
    for (; t + 4 < nk; t += 4) group(std::true_type(), t);
    group(std::false_type(), t);
    asm volatile("s_nop 15\n\ts_nop 3");
    pin_acc(acc);

    const int m0 = tile_m * BM + wr * 128, n = tile_n * BN + wc * WN + c8;
    // epilogue (gemm_w4p.hip): 8 passes of 16 rows through the wave's fp32 staging image
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < NF; ++j) asm volatile("" : "+a"(acc[i][j]));
      const int r16 = lane & 15;
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
        const bool in = m < p.M && n < p.N && !(ABL & 1);
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
    tile += (int)gridDim.x;
    tile_m = ntm;
    tile_n = ntn;
    first_tile = false;
    // K-tile 0 of this tile landed (K-tiles 1..3 and the stores just issued may not have)
    vmcnt<(3 * PW + STORES > 63 ? 63 : 3 * PW + STORES)>();
    barrier();
#pragma unroll
    for (int j = 0; j < NF; ++j) b0[j] = fragq<B_K>(smem + A_BYTES, wc * WN + j * 16, lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) a0[i] = fragq<A_K>(smem, wr * 128 + i * 16, lane);
    lgkm0();
  }
}

template <bool F32OUT>
static void launch_q(const GemmArgs& p, dim3 grid, hipStream_t s, int64_t ab, int64_t bb) {
  if (p.a_kcontig && p.b_kcontig) hipLaunchKernelGGL((gemm_w4q_kernel<true, true, F32OUT>), grid, dim3(NTH), 0, s, p, ab, bb);
  else if (p.a_kcontig) hipLaunchKernelGGL((gemm_w4q_kernel<true, false, F32OUT>), grid, dim3(NTH), 0, s, p, ab, bb);
  else if (p.b_kcontig) hipLaunchKernelGGL((gemm_w4q_kernel<false, true, F32OUT>), grid, dim3(NTH), 0, s, p, ab, bb);
  else hipLaunchKernelGGL((gemm_w4q_kernel<false, false, F32OUT>), grid, dim3(NTH), 0, s, p, ab, bb);
}

}  // namespace w4q

static int g_cus_q = 0;

bool gemm_w4q_bf16(const GemmArgs& p, int64_t a_bytes, int64_t b_bytes, hipStream_t stream) {
  using namespace w4q;
  if (p.dact || p.Z || p.act != ACT_NONE || p.beta != 0.f || p.batch != 1 || (p.splitk > 1 && p.ws) || !p.vec8_ok || p.K % 128 != 0 ||
      p.K <= 0 || a_bytes > 0x7fffffffLL || b_bytes > 0x7fffffffLL || a_bytes <= 0 || b_bytes <= 0)
    return false;
  if (((uintptr_t)p.A & 15) || ((uintptr_t)p.B & 15) || p.lda % 8 || p.ldb % 8) return false;
  if ((int64_t)p.M * p.ldc * (p.out_f32 ? 4 : 2) > 0x7fffff00LL) return false;
  if (!p.a_kcontig && p.M % 8) return false;
  if (!p.b_kcontig && p.N % 8) return false;
  if (p.bias && ((uintptr_t)p.bias & 15)) return false;
  if (g_cus_q == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&g_cus_q, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_cus_q <= 0) g_cus_q = 256;
  }
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  dim3 grid(std::min(tiles, g_cus_q));
  if (p.ablate) {  // timing-only ablations: K-contiguous operands, bf16 output
    if (!p.a_kcontig || !p.b_kcontig || p.out_f32) return false;
    if (p.ablate == 1) hipLaunchKernelGGL((gemm_w4q_kernel<true, true, false, 1>), grid, dim3(NTH), 0, stream, p, a_bytes, b_bytes);
    else if (p.ablate == 3) hipLaunchKernelGGL((gemm_w4q_kernel<true, true, false, 3>), grid, dim3(NTH), 0, stream, p, a_bytes, b_bytes);
    else if (p.ablate == 7) hipLaunchKernelGGL((gemm_w4q_kernel<true, true, false, 7>), grid, dim3(NTH), 0, stream, p, a_bytes, b_bytes);
    else if (p.ablate == 9) hipLaunchKernelGGL((gemm_w4q_kernel<true, true, false, 9>), grid, dim3(NTH), 0, stream, p, a_bytes, b_bytes);
    else if (p.ablate == 32) {  // global_load_lds operands: whole tiles only (no range check)
      if (p.M % 256 || p.N % 256) return false;
      hipLaunchKernelGGL((gemm_w4q_kernel<true, true, false, 32>), grid, dim3(NTH), 0, stream, p, a_bytes, b_bytes);
    } else if (p.ablate == 21) hipLaunchKernelGGL((gemm_w4q_kernel<true, true, false, 0, 16>), grid, dim3(NTH), 0, stream, p, a_bytes, b_bytes);
    else if (p.ablate == 22) hipLaunchKernelGGL((gemm_w4q_kernel<true, true, false, 0, 2>), grid, dim3(NTH), 0, stream, p, a_bytes, b_bytes);
    else if (p.ablate == 23) hipLaunchKernelGGL((gemm_w4q_kernel<true, true, false, 0, 18>), grid, dim3(NTH), 0, stream, p, a_bytes, b_bytes);
    else if (p.ablate == 24) hipLaunchKernelGGL((gemm_w4q_kernel<true, true, false, 0, 1>), grid, dim3(NTH), 0, stream, p, a_bytes, b_bytes);
    else return false;
    return true;
  }
  if (p.out_f32) launch_q<true>(p, grid, stream, a_bytes, b_bytes);
  else launch_q<false>(p, grid, stream, a_bytes, b_bytes);
  return true;
}

}  // namespace ffk

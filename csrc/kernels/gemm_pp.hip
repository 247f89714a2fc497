// Persistent 8-wave ping-pong bf16 MFMA GEMM: 256 x 256 x 64 tiles, two waves per SIMD.
//
// Why (rounds 3-4, gemm_w4*.hip): with ONE wave per SIMD (4 waves of 128 x 128) every LDS-DMA
// issue and fragment read of the ring sits in the MFMA wave's own instruction stream; ablations
// priced the DMA issue at ~14 % of the main loop, which kept those kernels 8-14 % behind
// hipBLASLt. Here each SIMD holds two waves that own different halves of the tile's rows and
// alternate roles every ~1000 cycles:
//   * a COMPUTE phase: 64 back-to-back v_mfma_f32_16x16x32_bf16 on fragments already in registers
//     (128 x 64 outputs per wave, 128 accumulator VGPRs);
//   * a MEMORY phase: this group's share of the LDS-DMA for the next K-tiles, the 24 fragment
//     reads for its next compute phase and, at a tile boundary, the previous tile's epilogue.
// Group 0 (waves 0-3: tile rows 0-127) runs one phase ahead of group 1 (waves 4-7: rows
// 128-255); wave w and wave w+4 share a SIMD (cyclic dealing), so while one of them computes the
// other's memory work issues beside it — the MFMA pipe of every SIMD is fed from one wave while
// the other pays the issue cost. Phase p: group 0 reads / computes stage p/2, group 1 stage
// (p-1)/2; one s_barrier closes every phase (group 1 executes one extra barrier first).
//
// Every DMA offset is in the VGPR operand (the buffer range check does not cover soffset), so rows
// past the end of a K-contiguous operand read as zeros instead of past the allocation.
// Two-slot LDS ring (2 x 64 KiB). Stage u = (tile, K-tile) in this workgroup's tile walk; the
// K-tiles of consecutive tiles follow each other, so the ring never drains between tiles. Who
// stages what (each piece = one 1-KiB buffer_load ... lds; slot lifetimes in phases):
//   * A-rows-128..255 of u+1 (16) and the first half of every B quarter of u+1 (16): group 0 in its
//     memory phase 2u (their slot was last read by group 1 in phase 2u-1);
//   * A-rows-0..127 of u+2 (16) and the second half of every B quarter (16): group 1 in its memory
//     phase 2u+1 (A slot last read in 2u; a B quarter is read only by waves j and j+4, so wave j+4
//     refills it right behind its own reads). Eight pieces per wave per memory phase.
// Every piece has ~2 phases (~1 us) to land; each issuing wave retires its pieces with a counted
// vmcnt before the barrier that precedes their first read (never vmcnt(0) in steady state).
// The MFMAs are inline asm on VGPR accumulators, the first K-step of a tile uses a zero C operand
// (no accumulator clearing), and all LDS reads are inline asm (hipcc otherwise waits for the
// LDS-DMA in flight before each read).
//
// Epilogue: alpha, bias (fp32 / bf16), bf16 or fp32 output, through a wave-private LDS image into
// whole-row range-checked buffer stores (see epilogue()). Requires batch 1, beta 0, no activation, K % 64 == 0, 16-B aligned operand
// rows, operands and output < 2 GiB. Image formats / swizzles: gemm_pp_core.h, gemm256_tile.h.
#include "gemm_pp_core.h"

namespace ffk {
namespace pp {
using namespace ppcore;

constexpr int NTHR = 512;
constexpr int NFB = 4;     // 16-column B fragments per wave (64 columns)

typedef short v4s __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// No AGPRs anywhere in this kernel: when a function uses AGPRs, LLVM splits the 256-register budget
// of two waves per SIMD 128 / 128 between VGPRs and AGPRs, and 128 accumulators + 96 fragment
// registers + addressing do not fit the halves (hipcc spilled 100-300 registers). In VGPR form the
// MFMAs read and write the one 256-register pool, and the epilogue needs no AGPR -> VGPR copies.
template <int OFF>
__device__ __forceinline__ bf16x8 ds128(unsigned a) {
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "n"(OFF));
  return r;
}
template <bool ZERO>
__device__ __forceinline__ void mfma(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  if constexpr (ZERO) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=v"(acc) : "v"(b), "v"(a));
  else asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(b), "v"(a));
}
template <int OFF>
__device__ __forceinline__ v4s dstr(unsigned a) {
  v4s r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "n"(OFF));
  return r;
}
__device__ __forceinline__ bf16x8 join(v4s lo, v4s hi) {
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// counted wait with a run-time count (the counts differ at tile boundaries and at the end)
template <int EPI>
__device__ __forceinline__ void vmcnt_rt(int n) {
  switch (n) {
    case 8: vmcnt<8>(); break;
    case EPI: vmcnt<EPI>(); break;
    case EPI + 8: vmcnt<EPI + 8>(); break;
    default: vmcnt<0>(); break;
  }
}

// The lane id, opaque to the optimiser: every lane-dependent address is re-derived from it where it
// is used (a few VALU per phase) instead of being hoisted into long-lived registers, which this
// kernel does not have (224 of its 256 VGPRs are accumulators and fragments).
__device__ __forceinline__ int opaque_lane() {
  int l = (int)(threadIdx.x & 63);
  asm volatile("" : "+v"(l));
  return l;
}

// VMEM ops of one epilogue: 2 bias loads (one wasted for a bf16 bias keeps the count fixed) + 16 row
// stores (bf16) or 32 (fp32).
// ACT (bf16 output only): activation in the epilogue, the pre-activation (z + bias) stored to Z in
// the same pass (16 more stores; issued out of range when Z is null so the count stays fixed)
// DACT (bf16 output only; round 6): the dgrad of a Linear fused with its producer's activation
// backward — C = (alpha A.B) * act'(zin), zin read in C's layout (16 more loads, two per row pass,
// each pass's pair requested one pass ahead so that no wait covers the previous pass's stores),
// plus the per-128-row fp32 column sums of that product for the producer's bias gradient (2 more
// stores). (Round 5's first attempt loaded every zin row up front and summed columns per element
// pass: ~150 VGPRs spilled; here the sums are 8 registers folded across lanes once per tile.)
// HB = false (no bias): no bias loads, and no 8 bias registers live across the 8 row passes — with
// them the bf16-output epilogue spilled ~12 VGPRs to scratch inside the main loop, and each reload's
// s_waitcnt vmcnt(0) also waited for the LDS-DMA pieces in flight (round 6).
template <bool F32OUT, bool ACT = false, bool DACT = false, bool HB = true>
constexpr int epi_ops() { return DACT ? 16 + 14 + 2 : (F32OUT ? 32 : 16) + (HB ? 2 : 0) + (ACT ? 16 : 0); }

// ACTK: 0, or the activation (ACT_RELU / ACT_GELU) as a compile-time constant: one code path per
// instantiation (a run-time switch over every activation cost ~10 more VGPR spills). DK: 0, or
// ACT_GRADMUL for the DACT epilogue (zin already holds act'(z), stored by the producer's forward).
// (Evaluating GELU' from z here was tried: ~14 VALU per element in the memory phase, 96 B/lane of
// spills, and wrong results on 1/3 of the elements on gfx950 — not built.)
template <bool A_K, bool B_K, bool F32OUT, bool SPLIT, int ACTK = 0, int DK = 0, bool HB = true>
__global__ void __attribute__((amdgpu_flat_work_group_size(NTHR, NTHR), amdgpu_waves_per_eu(2, 2)))
gemm_pp_kernel(GemmArgs p, int64_t a_bytes, int64_t b_bytes) {
  constexpr bool DACT = DK != 0;
  // DACT: + 32 B per lane of running column sums (8 waves x 2 KiB, 160 KiB in all)
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE + 4 * 4096 + (DACT ? 8 * 2048 : 0)];
  constexpr bool ACT = ACTK != 0;
  constexpr int EPI = epi_ops<F32OUT, ACT, DACT, HB>();
  static_assert(!ACT || (!F32OUT && !SPLIT), "activation epilogue: bf16 output, no split-K");
  static_assert(!DACT || (!F32OUT && !SPLIT && !ACT), "dgrad-activation epilogue: bf16 output, no split-K");

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wj = wave & 3;  // grp: rows grp*128.. of the tile; wj: columns wj*64..
  const int tm = (p.M + BM - 1) / BM, tn = (p.N + BN - 1) / BN;
  // work units: output tiles x split-K slices (unit = tile * S + slice; slices write fp32 slabs
  // ws[slice][M][N] that slab_sum folds; S = 1: the tile's output straight into C)
  // slice s of a tile covers K-tiles [s nkt / S, (s + 1) nkt / S) (any S <= nkt: S is chosen so
  // that the units fill the CUs, e.g. 48 tiles x 5 slices)
  // (a template parameter: the run-time form cost the unsplit kernel ~20 SGPRs, spilled to VGPR
  // lanes and read back in every memory phase)
  const int S = SPLIT ? p.splitk : 1;
  const int total = tm * tn * S;
  const int nkt = p.K / BK;
  const int first = blockIdx.x;
  if (first >= total || nkt < S) return;
  const int ntiles = (total - 1 - first) / (int)gridDim.x + 1;
  auto unit_nk = [&](int unit) __attribute__((always_inline)) {
    if (S == 1) return nkt;
    const int sl = unit % S;
    return (sl + 1) * nkt / S - sl * nkt / S;
  };
  int U = 0;  // stages of this workgroup
  for (int tl = 0; tl < ntiles; ++tl) U += unit_nk(first + tl * (int)gridDim.x);

  __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, (int)min(a_bytes, (int64_t)0x7fffffff), 0x00020000);
  __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, (int)min(b_bytes, (int64_t)0x7fffffff), 0x00020000);

  // ---- LDS-DMA: per-lane (tile independent) source offsets; the tile / K-tile part is scalar and
  // added to them per issue.
  // VGPRs are scarce (128 AGPR accumulators + 96 fragment registers of the 256): a K-contiguous
  // operand needs one offset register (piece_lane_off does not depend on the piece there), an
  // MN-contiguous one two (q enters as an XOR of the 16-B chunk: off(q) = base + (x ^ 16 q)).
  const int gsA = piece_gstride<A_K>(p.lda), gsB = piece_gstride<true>(p.ldb);
  const int awl = grp ^ 1;  // A half this wave stages: group 0 stages rows 128.., group 1 rows 0..
  // per-lane DMA source offset = base + chunk: for an MN-contiguous operand the piece's q = g & 3
  // enters as an XOR of the chunk part only (bits 4-5 of the base need not be zero)
  auto voff = [&](bool is_a, int& base, int& chunk) __attribute__((always_inline)) {
    const int l = opaque_lane();
    const bool kc = A_K;
    const int64_t ld = p.lda;
    const int wl = awl;
    if (kc) {
      base = piece_lane_off<true>(ld, 0, 0, wl, 0, l);
      chunk = 0;
    } else {
      base = (int)(((l >> 4) * (int)ld + wl * 128) * 2);
      chunk = ((l & 15) ^ (((l >> 4) & 3) << 2)) * 16;
    }
  };
  auto unit_coords = [&](int unit, int& tmi, int& tni, int& sl) __attribute__((always_inline)) {
    const int t = S > 1 ? unit / S : unit;
    sl = S > 1 ? unit - t * S : 0;
    tile_coords(t, tm, tn, tmi, tni);
  };
  // Each wave stages an increasing sequence of stages (group 0: 0, 1, 2, ...; group 1 the A rows
  // 0..127 of 0, 1, 2, ...), so the scalar source bases are kept in a cursor that adds one K-step
  // per stage and re-derives the tile coordinates only when it crosses into the next tile.
  const int ka = A_K ? BK * 2 : BK * (int)p.lda * 2, kb = B_K ? BK * 2 : BK * (int)p.ldb * 2;
  int c_kt = 0, c_tl = 0, c_sa = 0, c_sb = 0, c_nk = 0;
  auto cursor_tile = [&]() __attribute__((always_inline)) {
    int tmi, tni, sl;
    unit_coords(first + c_tl * (int)gridDim.x, tmi, tni, sl);
    const int m0 = tmi * BM, n0 = tni * BN, k0 = (sl * nkt / S) * BK;
    c_nk = unit_nk(first + c_tl * (int)gridDim.x);
    c_sa = __builtin_amdgcn_readfirstlane(A_K ? (int)(((int64_t)m0 * p.lda + k0) * 2) : (int)(((int64_t)k0 * p.lda + m0) * 2));
    c_sb = __builtin_amdgcn_readfirstlane(B_K ? (int)(((int64_t)n0 * p.ldb + k0) * 2) : (int)(((int64_t)k0 * p.ldb + n0) * 2));
  };
  auto cursor_next = [&]() __attribute__((always_inline)) {
    if (++c_kt == c_nk) {
      c_kt = 0;
      if (++c_tl < ntiles) cursor_tile();
    } else {
      c_sa += ka;
      c_sb += kb;
    }
  };
  cursor_tile();
  // A pieces of half `awl`, g = 4 wj + t (4 per wave)
  auto dma_a = [&](int u) __attribute__((always_inline)) {
    const int sa = c_sa;
    char* dst = smem + (u & 1) * STAGE + awl * 16 * 1024;
    int vb, vc;
    voff(true, vb, vc);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int g = wj * 4 + t;
      const int vo = (A_K ? vb : vb + (vc ^ (16 * t))) + (sa + g * gsA);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)(dst + g * 1024), 16, vo, 0, 0, 0);
    }
  };
  // B pieces of this wave's 64-column quarter (8 per stage: group 0 issues 0..3 of stage u + 1,
  // group 1 pieces 4..7 of stage u + 2). Only wave j and wave j + 4 read quarter j, so a group-1
  // wave may refill it as soon as its own reads of the stage are done. K-contiguous: piece t =
  // rows 64 j + 8 t .. + 7 (128-B rows). MN-contiguous: the quarter is its own [64 k][64 n] image
  // (128-B k-rows, 16-B chunk c stored at c ^ s(k), s(k) = (k & 2) | ((k >> 1) & 4)); piece t =
  // k-rows 8 t .. 8 t + 7.
  auto dma_b = [&](int u, int t0) __attribute__((always_inline)) {
    const int sb = c_sb;
    const int l = opaque_lane();
    char* dst = smem + (u & 1) * STAGE + A_BYTES + wj * (B_K ? 8 * 1024 : 8192);
    if constexpr (B_K) {
      const int vb = piece_lane_off<true>(p.ldb, 0, 0, 0, 0, l) + sb + wj * 64 * (int)p.ldb * 2;
#pragma unroll
      for (int t = t0; t < t0 + 4; ++t)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr_t)(dst + t * 1024), 16, vb + t * gsB, 0, 0, 0);
    } else {
      const int vb = (l >> 3) * (int)p.ldb * 2 + sb + wj * 128;
      const int x = ((l & 7) ^ ((l >> 3) & 2)) * 16;
#pragma unroll
      for (int t = t0; t < t0 + 4; ++t)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr_t)(dst + t * 1024), 16,
                                                 vb + (x ^ (64 * (t & 1))) + t * 8 * (int)p.ldb * 2, 0, 0, 0);
    }
  };

  // ---- fragment reads: per-lane LDS addresses, derived per phase (slot 1 adds STAGE)
  const unsigned sbase = (unsigned)(uintptr_t)smem;
  // K-contiguous images: 128-B rows, chunk ^ (row & 7); fragment i of a 16-row block at +2048 i,
  // and the kk = 1 chunk is the kk = 0 one with bit 2 flipped (address ^ 64).
  // MN-contiguous images (128-wide halves of 256-B k-rows, chunk ^ swz_mn(krow)), read by
  // ds_read_b64_tr_b16: lane (g, q, pp) reads k-row 8g + q (+4 for the second read) at chunk
  // (rr >> 3) + (pp >> 1); with rr = 16 i (+ 64 for odd B waves) the XOR'd chunk is
  // (2 i [+ 8]) ^ (swz ^ (pp >> 1)), so a read costs one v_xor + v_add off per-lane constants
  bf16x8 af[2][8], bfr[2][NFB];
  auto read_frags = [&](int slot) __attribute__((always_inline)) {
    const unsigned so = slot ? (unsigned)STAGE : 0u;
    const int lane = opaque_lane();
    const int l16 = lane & 15, lg = lane >> 4;
    const unsigned aK = sbase + (grp * 128 + l16) * 128 + ((lg ^ (lane & 7)) << 4);
    const unsigned bK = sbase + A_BYTES + (wj * 64 + l16) * 128 + ((lg ^ (lane & 7)) << 4);
    const int q4 = l16 >> 2, pp = l16 & 3;
    const int kr = 8 * lg + q4;
    const unsigned aM = sbase + grp * (BK * 256) + kr * 256 + 8 * (pp & 1);
    const unsigned T0 = (unsigned)((swz_mn(kr) ^ (pp >> 1)) << 4);
    const unsigned T1 = (unsigned)((swz_mn(kr + 4) ^ (pp >> 1)) << 4);
    // B quarter image (see dma_b): k-row kr at kr * 128, chunk 2 jj + (pp >> 1) stored at
    // ^ s(kr), s(kr) = (q4 & 2) | ((lg & 1) << 2) for kr = 8 lg + q4 (also for kr + 4, kr + 32):
    // address = bQ + ((32 jj) ^ TQ), the k + 4 and kk = 1 reads at +512 / +4096
    const unsigned bQ = sbase + A_BYTES + wj * 8192 + kr * 128 + 16 * (pp >> 1) + 8 * (pp & 1);
    const unsigned TQ = (unsigned)(((q4 & 2) | ((lg & 1) << 2)) << 4);
    if constexpr (B_K) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const unsigned a = (bK + so) ^ (kk * 64);
        bfr[kk][0] = ds128<0>(a);
        bfr[kk][1] = ds128<2048>(a);
        bfr[kk][2] = ds128<4096>(a);
        bfr[kk][3] = ds128<6144>(a);
      }
    } else {
#pragma unroll
      for (int jj = 0; jj < NFB; ++jj) {
        const unsigned a0 = bQ + so + ((32u * jj) ^ TQ);
        bfr[0][jj] = join(dstr<0>(a0), dstr<512>(a0));
        bfr[1][jj] = join(dstr<4096>(a0), dstr<4096 + 512>(a0));
      }
    }
    if constexpr (A_K) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const unsigned a = (aK + so) ^ (kk * 64);
        af[kk][0] = ds128<0>(a);
        af[kk][1] = ds128<2048>(a);
        af[kk][2] = ds128<4096>(a);
        af[kk][3] = ds128<6144>(a);
        af[kk][4] = ds128<8192>(a);
        af[kk][5] = ds128<10240>(a);
        af[kk][6] = ds128<12288>(a);
        af[kk][7] = ds128<14336>(a);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const unsigned c = 32 * i;
        const unsigned a0 = aM + so + (c ^ T0), a1 = aM + so + (c ^ T1);
        af[0][i] = join(dstr<0>(a0), dstr<1024>(a1));
        af[1][i] = join(dstr<8192>(a0), dstr<8192 + 1024>(a1));
      }
    }
  };

  f32x4 acc[8][NFB];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int jj = 0; jj < NFB; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](auto zero_c) __attribute__((always_inline)) {
    constexpr bool Z = decltype(zero_c)::value;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int jj = 0; jj < NFB; ++jj) mfma<Z>(acc[i][jj], bfr[0][jj], af[0][i]);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int jj = 0; jj < NFB; ++jj) mfma<false>(acc[i][jj], bfr[1][jj], af[1][i]);
    __builtin_amdgcn_s_setprio(0);
  };

  // ---- epilogue
  typedef typename std::conditional<F32OUT, float, bf16_t>::type OutT;
  const int64_t c_bytes = (int64_t)p.M * p.ldc * (int64_t)sizeof(OutT);
  __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(p.C, (short)0, (int)min(c_bytes, (int64_t)0x7fffffff), 0x00020000);
  // split-K: one range-checked descriptor over all slabs ([S][M][N] fp32, ldc = N)
  const int64_t ws_bytes = (int64_t)S * p.M * p.N * 4;
  if constexpr (SPLIT) rc = __builtin_amdgcn_make_buffer_rsrc(p.ws, (short)0, (int)min(ws_bytes, (int64_t)0x7fffffff), 0x00020000);
  const int64_t ldo = SPLIT ? p.N : p.ldc;
  const int bsz = p.bias ? (p.bias_bf16 ? 2 : 4) : 0;
  __amdgpu_buffer_rsrc_t rbias = __builtin_amdgcn_make_buffer_rsrc((void*)(p.bias ? p.bias : p.A), (short)0, p.N * bsz, 0x00020000);
  const float alpha = p.alpha;
  // ACT: the pre-activation store (same layout as C); a null Z gets an empty range (stores dropped)
  __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc((void*)(ACT && p.Z ? p.Z : p.C), (short)0,
                                                                ACT && p.Z ? (int)min(c_bytes, (int64_t)0x7fffffff) : 0,
                                                                0x00020000);
  // DACT: zin (bf16, C's layout) and the column-sum partials [2 * ceil(M / 256)][N] (a null colpart
  // gets an empty range: its stores are dropped)
  const int64_t zin_bytes = (int64_t)p.M * p.ldc * 2;
  const int64_t cp_bytes = DACT && p.colpart ? (int64_t)2 * ((p.M + BM - 1) / BM) * p.N * 4 : 0;
  __amdgpu_buffer_rsrc_t rzin = __builtin_amdgcn_make_buffer_rsrc((void*)(DACT ? p.zin : p.C), (short)0,
                                                                  DACT ? (int)min(zin_bytes, (int64_t)0x7fffffff) : 0,
                                                                  0x00020000);
  __amdgpu_buffer_rsrc_t rcp = __builtin_amdgcn_make_buffer_rsrc((void*)(DACT && p.colpart ? (void*)p.colpart : p.C),
                                                                 (short)0, (int)min(cp_bytes, (int64_t)0x7fffffff),
                                                                 0x00020000);
  // Epilogue through a wave-private fp32 staging image (16 rows x 64 columns, 4 KiB, outside the
  // ring): the accumulator layout puts 4 consecutive columns of one row in a lane, so direct 8-B
  // stores leave a wave as 16 scattered 32-B row pieces per instruction, store-issue bound at
  // ~7 B/clk/CU (MI355X_MICROARCH.md, epilogue store tail). Here each 16-row block is written to
  // the image (16-B chunk c of row r at c ^ r: conflict-free), read back as 8 consecutive columns
  // per lane and stored as whole 128-B (bf16) / 256-B (fp32) row segments, with bias and alpha.
  // A wave's LDS operations execute in order, so the read-back needs no wait behind the writes.
  auto epilogue = [&](int tl) __attribute__((always_inline)) {
    int tmi, tni, sl;
    unit_coords(first + tl * (int)gridDim.x, tmi, tni, sl);
    const int lane = opaque_lane();
    const int cc = lane & 7;
    const unsigned st = sbase + 2 * STAGE + wj * 4096;
    const int m0 = tmi * BM + grp * 128;
    const int n = tni * BN + wj * 64 + 8 * cc;  // this lane's 8 read-back columns
    const bool nin = n < p.N;
    float bb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if constexpr (DACT || !HB) {
      // no bias (dgrad): no bias registers live across the passes
    } else if (p.bias_bf16) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rbias, nin ? n * 2 : -16, 0, 0);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bb[2 * e] = __uint_as_float(v[e] << 16);
        bb[2 * e + 1] = __uint_as_float(v[e] & 0xffff0000u);
      }
    } else {
      const u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(rbias, nin ? n * 4 : -16, 0, 0);
      const u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(rbias, nin ? n * 4 + 16 : -16, 0, 0);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bb[e] = __uint_as_float(v0[e]);
        bb[4 + e] = __uint_as_float(v1[e]);
      }
    }
    // DACT: zin rows of pass i (rows m0 + 16 i + rr8 + 8 h, columns n..n+7), requested one pass
    // ahead (after pass i - 1 consumed its pair, before its stores: the wait for them covers no
    // store); cs: this lane's column sums over its rows. Waiting for zin pair 0 also retires every
    // DMA piece older than the epilogue, so the memory phase's counted wait stays correct whatever
    // the epilogue's VMEM count.
    auto zin_off = [&](int i, int h) __attribute__((always_inline)) {
      const int m = m0 + 16 * i + (opaque_lane() >> 3) + 8 * h;
      return (m < p.M && nin) ? (int)(((int64_t)m * p.ldc + n) * 2) : -16;
    };
    u32x4 zq[2];
    // the lane's running column sums live in its own 32 B of LDS between passes (in registers,
    // next to the 128 accumulators, they spilled ~16 VGPRs to scratch): read, add, write per pass;
    // a wave's LDS operations execute in order
    const unsigned csa = sbase + 2 * STAGE + 4 * 4096 + wave * 2048 + (lane << 5);
    if constexpr (DACT) {
      const f32x4 zz = {0.f, 0.f, 0.f, 0.f};
      asm volatile("ds_write_b128 %0, %1\n\tds_write_b128 %0, %1 offset:16" ::"v"(csa), "v"(zz) : "memory");
      zq[0] = __builtin_amdgcn_raw_buffer_load_b128(rzin, zin_off(0, 0), 0, 0);
      zq[1] = __builtin_amdgcn_raw_buffer_load_b128(rzin, zin_off(0, 1), 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      __builtin_amdgcn_sched_barrier(0);
      // addresses re-derived per pass (kept across the 8 passes they cost registers the
      // allocator does not have next to the 128 accumulators)
      const int ln = opaque_lane();
      const int w16 = ln & 15, wg = ln >> 4, rc8 = ln & 7, rr8 = ln >> 3;
#pragma unroll
      for (int jj = 0; jj < NFB; ++jj) {
        const unsigned a = st + w16 * 256 + (((4 * jj + wg) ^ w16) << 4);
        asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(acc[i][jj]) : "memory");
      }
      f32x4 lo[2], hi[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int rr = rr8 + 8 * h;
        const unsigned a0 = st + rr * 256 + (((2 * rc8) ^ rr) << 4);
        const unsigned a1 = st + rr * 256 + (((2 * rc8 + 1) ^ rr) << 4);
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3" : "=&v"(lo[h]), "=&v"(hi[h]) : "v"(a0), "v"(a1) : "memory");
      }
      lgkm0();
      __builtin_amdgcn_sched_barrier(0);
      u32x4 ov[2];  // DACT: this pass's two output rows, stored after the next zin pair is requested
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int m = m0 + 16 * i + rr8 + 8 * h;
        const bool in = m < p.M && nin;
        const int off = in ? (int)(((int64_t)sl * p.M * p.N + (int64_t)m * ldo + n) * (int64_t)sizeof(OutT)) : -16;
        float x[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          x[e] = __builtin_fmaf(lo[h][e], alpha, bb[e]);
          x[4 + e] = __builtin_fmaf(hi[h][e], alpha, bb[4 + e]);
        }
        if constexpr (F32OUT) {
          const u32x4 o0 = {__float_as_uint(x[0]), __float_as_uint(x[1]), __float_as_uint(x[2]), __float_as_uint(x[3])};
          const u32x4 o1 = {__float_as_uint(x[4]), __float_as_uint(x[5]), __float_as_uint(x[6]), __float_as_uint(x[7])};
          __builtin_amdgcn_raw_buffer_store_b128(o0, rc, off, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b128(o1, rc, in ? off + 16 : off, 0, 0);
        } else {
          if constexpr (DACT) {
            const u32x4 zv = zq[h];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float z0 = __uint_as_float(zv[e] << 16), z1 = __uint_as_float(zv[e] & 0xffff0000u);
              // the GEMM result rounded to bf16 first, as the unfused GEMM + bias_act_bwd pair
              // does: the autotuner's pick changes the numerics by summation order only
              x[2 * e] = bf2f(f2bf(x[2 * e])) * act_grad(DK, z0);
              x[2 * e + 1] = bf2f(f2bf(x[2 * e + 1])) * act_grad(DK, z1);
            }
            {  // running column sums += this row (in LDS; see csa)
              f32x4 c0, c1;
              asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)"
                           : "=&v"(c0), "=&v"(c1) : "v"(csa) : "memory");
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                c0[e] += x[e];
                c1[e] += x[4 + e];
              }
              asm volatile("ds_write_b128 %0, %1\n\tds_write_b128 %0, %2 offset:16" ::"v"(csa), "v"(c0), "v"(c1) : "memory");
            }
          }
          if constexpr (ACT) {
            u32x4 zo;
#pragma unroll
            for (int e = 0; e < 4; ++e) zo[e] = (uint32_t)f2bf(x[2 * e]) | ((uint32_t)f2bf(x[2 * e + 1]) << 16);
            __builtin_amdgcn_raw_buffer_store_b128(zo, rz, off, 0, 0);
#pragma unroll
            for (int e = 0; e < 8; ++e) x[e] = act_fwd(ACTK, x[e]);
          }
          u32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = (uint32_t)f2bf(x[2 * e]) | ((uint32_t)f2bf(x[2 * e + 1]) << 16);
          if constexpr (DACT) ov[h] = o;
          else __builtin_amdgcn_raw_buffer_store_b128(o, rc, off, 0, 0);
        }
      }
      if constexpr (DACT) {
        if (i < 7) {  // the next pass's zin pair, then this pass's stores
          zq[0] = __builtin_amdgcn_raw_buffer_load_b128(rzin, zin_off(i + 1, 0), 0, 0);
          zq[1] = __builtin_amdgcn_raw_buffer_load_b128(rzin, zin_off(i + 1, 1), 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int m = m0 + 16 * i + rr8 + 8 * h;
          const int off = (m < p.M && nin) ? (int)(((int64_t)m * ldo + n) * 2) : -16;
          __builtin_amdgcn_raw_buffer_store_b128(ov[h], rc, off, 0, 0);
        }
      }
    }
    if constexpr (DACT) {
      // fold the 8 row lanes of each column group (lane bits 3-5), then lanes 0-7 store this wave's
      // 64 column sums of its 128 rows: colpart row 2 * tile_m + group
      float cs[8];
      {
        f32x4 c0, c1;
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(c0), "=&v"(c1) : "v"(csa) : "memory");
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          cs[e] = c0[e];
          cs[4 + e] = c1[e];
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        cs[e] += __shfl_xor(cs[e], 8);
        cs[e] += __shfl_xor(cs[e], 16);
        cs[e] += __shfl_xor(cs[e], 32);
      }
      const bool st0 = nin && (opaque_lane() >> 3) == 0;
      const int co = st0 ? (int)(((int64_t)(2 * tmi + grp) * p.N + n) * 4) : -16;
      const u32x4 c0 = {__float_as_uint(cs[0]), __float_as_uint(cs[1]), __float_as_uint(cs[2]), __float_as_uint(cs[3])};
      const u32x4 c1 = {__float_as_uint(cs[4]), __float_as_uint(cs[5]), __float_as_uint(cs[6]), __float_as_uint(cs[7])};
      __builtin_amdgcn_raw_buffer_store_b128(c0, rcp, co, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(c1, rcp, st0 ? co + 16 : co, 0, 0);
    }
  };

  // ---- prologue: stage 0 (all of it) and A rows 0..127 of stage 1 land before the first phase
  if (grp == 0) {
    dma_b(0, 0);
    dma_a(0);
    cursor_next();
  } else {
    dma_a(0);
    dma_b(0, 4);
    cursor_next();
    if (U > 1) {
      dma_a(1);
      dma_b(1, 4);
      cursor_next();
    }
  }
  vmcnt<0>();
  barrier();
  if (grp == 1) barrier();  // group 1 runs one phase behind

  // memory phase of stage u (epi: the previous tile's epilogue first)
  auto mem_phase = [&](int u, bool epi, int tl_prev) __attribute__((always_inline)) {
    if (epi) epilogue(tl_prev);
    int after;  // VMEM ops issued after the piece this wave retires at the end of the phase
    if (grp == 0) {
      const bool iss = u + 1 < U && !(p.ablate & 1);
      if (iss) {
        dma_b(u + 1, 0);  // first: the compute phase's vmcnt(4) retires these and leaves the A rows
        dma_a(u + 1);
        cursor_next();
      }
      after = (epi ? EPI : 0) + (iss ? 8 : 0);  // retires A rows 128.. of stage u
    } else {
      const bool iss = u + 2 < U && !(p.ablate & 1);
      if (iss) dma_a(u + 2);
      after = (epi ? EPI : 0) + (iss ? 8 : 0);  // retires A rows 0..127 / B 4..7 of stage u + 1
    }
    read_frags(u & 1);
    lgkm0();
    if (grp == 1 && u + 2 < U && !(p.ablate & 1)) {
      // this wave's B quarter of slot u & 1 is free only now: its partner (wave j) read it in the
      // previous phase, and this wave's own reads just completed
      dma_b(u + 2, 4);
      cursor_next();
    }
    vmcnt_rt<EPI>(after);
    barrier();
  };
  auto compute_phase = [&](int u, auto zero_c) __attribute__((always_inline)) {
    compute(zero_c);
    if (grp == 0 && u + 1 < U && !(p.ablate & 1)) vmcnt<4>();  // B of stage u + 1 (its A rows 128.. may still fly)
    barrier();
  };

  int u = 0;
  mem_phase(0, false, 0);
  for (int tl = 0; tl < ntiles; ++tl) {
    compute_phase(u, std::true_type());
    const int nk = unit_nk(first + tl * (int)gridDim.x);
    for (int kt = 1; kt < nk; ++kt) {
      mem_phase(u + 1, false, 0);
      ++u;
      compute_phase(u, std::false_type());
    }
    ++u;
    // MFMA -> accumulator read distance before the epilogue (inline asm: hipcc pads nothing)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3");
    if (tl + 1 < ntiles) {
      mem_phase(u, true, tl);
    } else {
      epilogue(tl);
      if (grp == 0) barrier();  // balance the barrier count of the two groups
    }
  }
}

template <bool F32OUT, bool SPLIT, int ACTK, bool HB>
static void launch_hb(const GemmArgs& p, dim3 grid, hipStream_t s, int64_t ab, int64_t bb) {
  if (p.a_kcontig && p.b_kcontig) hipLaunchKernelGGL((gemm_pp_kernel<true, true, F32OUT, SPLIT, ACTK, 0, HB>), grid, dim3(NTHR), 0, s, p, ab, bb);
  else if (p.a_kcontig) hipLaunchKernelGGL((gemm_pp_kernel<true, false, F32OUT, SPLIT, ACTK, 0, HB>), grid, dim3(NTHR), 0, s, p, ab, bb);
  else if (p.b_kcontig) hipLaunchKernelGGL((gemm_pp_kernel<false, true, F32OUT, SPLIT, ACTK, 0, HB>), grid, dim3(NTHR), 0, s, p, ab, bb);
  else hipLaunchKernelGGL((gemm_pp_kernel<false, false, F32OUT, SPLIT, ACTK, 0, HB>), grid, dim3(NTHR), 0, s, p, ab, bb);
}
template <bool F32OUT, bool SPLIT, int ACTK = 0>
static void launch(const GemmArgs& p, dim3 grid, hipStream_t s, int64_t ab, int64_t bb) {
  if (SPLIT || !p.bias) launch_hb<F32OUT, SPLIT, ACTK, false>(p, grid, s, ab, bb);  // split-K never has a bias
  else launch_hb<F32OUT, SPLIT, ACTK, true>(p, grid, s, ab, bb);
}

// the DACT epilogue is built for the dgrad layout only: A = dY [M][K] K-contiguous, B = W [K][N]
// N-contiguous (the weight of the consumer Linear as stored)
template <int DK>
static void launch_dact(const GemmArgs& p, dim3 grid, hipStream_t s, int64_t ab, int64_t bb) {
  hipLaunchKernelGGL((gemm_pp_kernel<true, false, false, false, 0, DK>), grid, dim3(NTHR), 0, s, p, ab, bb);
}

}  // namespace pp

static int g_pp_cus = 0;

bool gemm_pp_bf16(const GemmArgs& p, int64_t a_bytes, int64_t b_bytes, hipStream_t stream) {
  using namespace pp;
  // activation epilogue (bias + act, optional pre-activation store): bf16 output, no split-K
  const bool act = !p.dact && (p.Z || p.act != ACT_NONE);
  if (p.dact) {  // dgrad-activation epilogue (gemm_dact_bf16 sets it): NN layout, bf16 out, no bias
    if (!p.zin || p.out_f32 || p.bias || p.Z || p.beta != 0.f || p.batch != 1 || (p.splitk > 1 && p.ws) ||
        !p.a_kcontig || p.b_kcontig || p.act != ACT_GRADMUL ||
        ((uintptr_t)p.zin & 15) || (p.colpart && ((uintptr_t)p.colpart & 15)) ||
        (int64_t)p.M * p.ldc * 2 > 0x7fffff00LL || (int64_t)2 * ((p.M + BM - 1) / BM) * p.N * 4 > 0x7fffff00LL)
      return false;
  }
  if (act && (p.out_f32 || (p.act != ACT_NONE && p.act != ACT_RELU && p.act != ACT_GELU) || (p.splitk > 1 && p.ws) ||
              ((uintptr_t)p.Z & 15)))
    return false;
  const bool split = p.splitk > 1 && p.ws;
  if (split && (!p.out_f32 || p.bias || p.alpha != 1.f || p.K / BK < p.splitk ||
                (int64_t)p.splitk * p.M * p.N * 4 > 0x7fffff00LL))
    return false;
  if ((p.beta != 0.f && !split) || p.batch != 1 || p.K % BK != 0 ||
      p.K <= 0 || a_bytes > 0x7fffffffLL || b_bytes > 0x7fffffffLL || a_bytes <= 0 || b_bytes <= 0)
    return false;
  if (((uintptr_t)p.A & 15) || ((uintptr_t)p.B & 15) || p.lda % 8 || p.ldb % 8) return false;
  if ((int64_t)p.M * p.ldc * (p.out_f32 ? 4 : 2) > 0x7fffff00LL) return false;  // buffer-store offsets
  if (!p.a_kcontig && p.M % 8) return false;
  if (!p.b_kcontig && p.N % 8) return false;
  if (p.N % 8 || p.ldc % 8 || ((uintptr_t)p.C & 15)) return false;  // whole 8-column row stores
  if (p.bias && ((uintptr_t)p.bias & 15)) return false;
  if (g_pp_cus == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&g_pp_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_pp_cus <= 0) g_pp_cus = 256;
  }
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN) * (split ? p.splitk : 1);
  dim3 grid(std::min(tiles, g_pp_cus));
  if (p.dact) {
    launch_dact<ACT_GRADMUL>(p, grid, stream, a_bytes, b_bytes);
  } else if (split) launch<true, true>(p, grid, stream, a_bytes, b_bytes);  // split-K: fp32 slabs only
  else if (p.out_f32) launch<true, false>(p, grid, stream, a_bytes, b_bytes);
  else if (act && p.act == ACT_GELU) launch<false, false, ACT_GELU>(p, grid, stream, a_bytes, b_bytes);
  else if (act && p.act == ACT_RELU) launch<false, false, ACT_RELU>(p, grid, stream, a_bytes, b_bytes);
  else if (act) launch<false, false, ACT_NONE>(p, grid, stream, a_bytes, b_bytes);  // Z store, no activation
  else launch<false, false>(p, grid, stream, a_bytes, b_bytes);
  return true;
}

}  // namespace ffk

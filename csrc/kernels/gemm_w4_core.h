// Shared pieces of the 4-wave 256 x 256 x 64 MFMA GEMMs: gemm_w4.hip (one tile per workgroup,
// split-K, every epilogue) and gemm_w4p.hip (persistent). Geometry, DMA piece offsets, the
// transposing fragment read and the counted vmcnt helper; see gemm_w4.hip for the design.
#pragma once
#include "gemm256_tile.h"

namespace ffk {
namespace w4 {
using namespace g256;

constexpr int BN = 256, BK = 64, NTH = 256;
constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
constexpr int A_PIECES = A_BYTES / 1024, PIECES = STAGE / 1024, PW = PIECES / 4;

// counted wait on this wave's vector-memory queue (loads, stores, LDS-DMA; in issue order)
template <int N>
__device__ __forceinline__ void vmcnt() {
  static_assert(N >= 0 && N <= 63, "vmcnt is a 6-bit count");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <bool KCONT>
__device__ __forceinline__ int piece_off(int64_t ld, int mn0, int k0, int pc, int lane) {
  int64_t elem;
  if (KCONT) {  // 8 rows x 128 B
    const int row = pc * 8 + (lane >> 3);
    const int c = (lane & 7) ^ swz_k<BK>(row);
    elem = (int64_t)(mn0 + row) * ld + k0 + c * 8;
  } else {  // 4 k-rows of one 128-wide half (256 B each)
    const int half = pc / (BK / 4);
    const int krow = (pc % (BK / 4)) * 4 + (lane >> 4);
    const int c = (lane & 15) ^ swz_mn(krow);
    elem = (int64_t)(k0 + krow) * ld + mn0 + half * 128 + c * 8;
  }
  return (int)(elem * 2);
}

// piece_off(ld, mn0, k0, wl * 16 + g, lane) == piece_lane_off(ld, mn0, k0, wl, g & 3, lane) +
// g * piece_gstride(ld): the per-lane part of a wave's 16 pieces depends on g only through the
// MN-contiguous swizzle's g & 3 (K-contiguous: not at all), so a wave keeps 1 or 4 VGPRs of DMA
// offsets instead of 16 (the persistent kernel spilled them, and the spill reloads put counted
// vmcnt waits in front of every DMA issue). The g-dependent part is added per issue (one VALU add
// with a scalar operand) and stays in the VGPR offset, which the buffer range check covers.
template <bool KCONT>
__device__ __forceinline__ int piece_lane_off(int64_t ld, int mn0, int k0, int wl, int q, int lane) {
  int64_t elem;
  if (KCONT) {
    elem = (int64_t)(mn0 + wl * 128 + (lane >> 3)) * ld + k0 + (((lane & 7) ^ (lane >> 3)) * 8);
  } else {
    const int swz = (((lane >> 4) & 3) << 2) | q;
    elem = (int64_t)(k0 + (lane >> 4)) * ld + mn0 + wl * 128 + ((lane & 15) ^ swz) * 8;
  }
  return (int)(elem * 2);
}
template <bool KCONT>
__device__ __forceinline__ int piece_gstride(int64_t ld) {
  return (int)((KCONT ? 8 : 4) * ld * 2);
}

// frag<KCONT, 64>(tile, r0, kk). The MN-contiguous (transposing) form is inline asm: hipcc puts an
// s_waitcnt vmcnt(0) in front of every ds_read_b64_tr_b16 builtin while LDS-DMA is in flight (it
// cannot tell that the read and the DMA touch different slots), which drains the ring once per
// fragment. The asm results are consumed only after the half's lgkmcnt(0).
template <bool KCONT>
__device__ __forceinline__ bf16x8 frag64(const char* tile, int r0, int kk, int lane) {
  if constexpr (KCONT) {
    return frag<true, BK>(tile, r0, kk, lane);
  } else {
    const char* hl = tile + (r0 >> 7) * (BK * 256);
    const int rr = r0 & 127;
    const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
    const int chunk = (rr >> 3) + (pp >> 1);
    const int k0 = 32 * kk + 8 * g + q, k1 = k0 + 4;
    const unsigned a0 = (unsigned)(uintptr_t)(hl + k0 * 256 + ((chunk ^ swz_mn(k0)) << 4) + 8 * (pp & 1));
    const unsigned a1 = (unsigned)(uintptr_t)(hl + k1 * 256 + ((chunk ^ swz_mn(k1)) << 4) + 8 * (pp & 1));
    typedef short v4s __attribute__((ext_vector_type(4)));
    v4s lo, hi;
    asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %3" : "=&v"(lo), "=&v"(hi) : "v"(a0), "v"(a1));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  }
}

}  // namespace w4
}  // namespace ffk

// Tile geometry, LDS-DMA piece offsets and the counted vmcnt helper of the persistent ping-pong
// GEMM (gemm_pp.hip). (Rounds 3-4 shared them with the 4-wave kernels gemm_w4{,p,q}.hip, removed
// in round 5: the ping-pong kernel matched or beat them at every zoo call site they won.)
#pragma once
#include "gemm256_tile.h"

namespace ffk {
namespace ppcore {
using namespace g256;

constexpr int BN = 256, BK = 64;
constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;

// counted wait on this wave's vector-memory queue (loads, stores, LDS-DMA; in issue order)
template <int N>
__device__ __forceinline__ void vmcnt() {
  static_assert(N >= 0 && N <= 63, "vmcnt is a 6-bit count");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Byte offset of lane `lane`'s 16-B piece g of a wave's 128-row slab = piece_lane_off(..., g & 3,
// lane) + g * piece_gstride(ld): K-contiguous pieces are 8 rows x 128 B (chunk c of row r at
// c ^ (r & 7)), MN-contiguous pieces 4 k-rows of a 128-wide half (16-B chunk c of k-row k at
// c ^ swz_mn(k)). The per-lane part depends on g only through the MN swizzle's g & 3, so a wave
// keeps 1 or 4 VGPRs of DMA offsets instead of 16 (spilling them put counted vmcnt waits in front
// of every DMA issue). The g-dependent part is added per issue (one VALU add with a scalar operand)
// and stays in the VGPR offset, which the buffer range check covers.
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

}  // namespace ppcore
}  // namespace ffk

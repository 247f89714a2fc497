// Shared tile machinery of the 256-row MFMA GEMMs (gemm256.hip: one output tile per workgroup;
// kept separate so that variants can be built as their own translation units, guide rule 19).
#pragma once
#include "common.h"
#include "gemm.h"

namespace ffk {
namespace g256 {

constexpr int BM = 256, NT = 512;

// K-tile geometry per output-tile width: BN = 256 -> BK = 32 with a 4-slot ring (4 x 32 KiB);
// BN = 128 -> BK = 64 with a 3-slot ring (3 x 48 KiB), so that each phase still issues 16 MFMAs
// per wave (8 would be too short to cover the other group's LDS reads).
template <int BN> struct Geo;
template <> struct Geo<256> { static constexpr int BK = 32, NBUF = 4; };
template <> struct Geo<128> { static constexpr int BK = 64, NBUF = 3; };

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// 16-B chunk swizzle of a K-contiguous row of BK bf16 (64-B rows: 4 chunks, 128-B rows: 8 chunks)
template <int BK>
__device__ __forceinline__ int swz_k(int row) {
  if constexpr (BK == 32) return ((row >> 2) & 1) << 1;
  else return row & 7;
}
__device__ __forceinline__ int swz_mn(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

// One 1-KiB DMA piece of an operand tile. K-contiguous: 1024 / (2 BK) rows of 2 BK bytes.
// MN-contiguous: 4 k-rows of one 128-wide half (256 B each).
template <bool KCONT, int BK>
__device__ __forceinline__ void dma_piece(__amdgpu_buffer_rsrc_t rsrc, char* lds_tile, int64_t ld, int mn0, int k0,
                                          int piece, int lane) {
  constexpr int CPR = BK / 8;  // 16-B chunks per K-contiguous row
  int64_t elem;
  if (KCONT) {
    const int row = piece * (64 / CPR) + lane / CPR;
    const int c = (lane % CPR) ^ swz_k<BK>(row);
    elem = (int64_t)(mn0 + row) * ld + k0 + c * 8;
  } else {
    const int half = piece / (BK / 4);
    const int krow = (piece % (BK / 4)) * 4 + (lane >> 4);
    const int c = (lane & 15) ^ swz_mn(krow);
    elem = (int64_t)(k0 + krow) * ld + mn0 + half * 128 + c * 8;
  }
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_ptr_t)(lds_tile + piece * 1024), 16, (int)(elem * 2), 0, 0, 0);
}

// 16 (rows along M or N) x 32 (k, sub-step kk of the K-tile) fragment for mfma_f32_16x16x32_bf16.
template <bool KCONT, int BK>
__device__ __forceinline__ bf16x8 frag(const char* tile, int r0, int kk, int lane) {
  if (KCONT) {
    const int row = r0 + (lane & 15);
    const int c = kk * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(tile + row * (BK * 2) + ((c ^ swz_k<BK>(row)) << 4));
  } else {
    const char* hl = tile + (r0 >> 7) * (BK * 256);
    const int rr = r0 & 127;
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int chunk = (rr >> 3) + (p >> 1);
    bf16x8 out;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int krow = 32 * kk + 8 * g + 4 * hf + q;
      const int off = krow * 256 + ((chunk ^ swz_mn(krow)) << 4) + 8 * (p & 1);
      typedef short v4s __attribute__((ext_vector_type(4)));
      v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(hl + off));
      bf16x4 b = __builtin_bit_cast(bf16x4, v);
      out[4 * hf + 0] = b[0];
      out[4 * hf + 1] = b[1];
      out[4 * hf + 2] = b[2];
      out[4 * hf + 3] = b[3];
    }
    return out;
  }
}

__device__ __forceinline__ void tile_coords(int bid, int tm, int tn, int& tile_m, int& tile_n) {
  const int nwg = tm * tn;
  bid = xcd_remap(bid, nwg);
  constexpr int GM = 8;
  const int per_group = GM * tn;
  const int group = bid / per_group;
  const int first_m = group * GM;
  const int gsize = min(tm - first_m, GM);
  const int in_g = bid % per_group;
  tile_m = first_m + in_g % gsize;
  tile_n = in_g / gsize;
}

__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N == 0 || N == 4 || N == 6 || N == 8 || N == 12, "add the vmcnt immediate");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
}

// Wait until at most `tiles_after` tiles' worth of this wave's DMAs are outstanding.
template <int PW, int NBUF>
__device__ __forceinline__ void wait_tiles(int tiles_after) {
  if constexpr (NBUF >= 4) {
    if (tiles_after >= 2) { wait_vm<2 * PW>(); return; }
  }
  if (tiles_after >= 1) wait_vm<PW>();
  else wait_vm<0>();
}

__device__ __forceinline__ void lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

}  // namespace g256
}  // namespace ffk

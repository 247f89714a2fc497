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
  static_assert(N == 0 || N == 4 || N == 6 || N == 8 || N == 12 || N == 16 || N == 24, "add the vmcnt immediate");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
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

// Orders every accumulator against neighbouring asm statements (see the 4-wave kernels).
template <int NF>
__device__ __forceinline__ void pin_acc(f32x4 (&acc)[8][NF]) {
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) asm volatile("" : "+a"(acc[i][j]));
}

// Epilogue of a 256-row tile whose waves each own 128 rows x WN columns (acc[i][j]: rows
// wr*128 + 16 i + (lane & 15), columns wc*WN + 16 j + 4 (lane >> 4) + r; the MFMA operands are
// swapped so that a lane holds 4 consecutive columns), gemm256.hip (8 waves, WN = BN/4). The LDS
// operand ring must be free when it is called.
template <int WN, int OUT_MODE, bool DACT = true, bool SCATTER = true>
__device__ __forceinline__ void store_tile(const GemmArgs& p, f32x4 (&acc)[8][WN / 16], char* smem, int wave, int wr,
                                           int wc, int lane, int m0, int n0, int b, int z, int tile_m) {
  constexpr int NF = WN / 16;
  if (!SCATTER || p.vec8_ok) {
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
    uint4 zpre[OUT_MODE == 0 && DACT ? 4 * ITS : 1];
    if (OUT_MODE == 0 && DACT && p.dact) {
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
      // one quarter's accumulators at a time: without the fence hipcc hoists every accumulator
      // read (256 AGPR -> VGPR copies in the 4-wave kernel) to the top and spills
      __builtin_amdgcn_sched_barrier(0);
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
        if (OUT_MODE == 0 && DACT && p.dact) {
          // consumer dgrad * producer act'(pre-activation); the column sums feed the producer's
          // bias gradient (the separate bias_act_bwd pass re-read and re-wrote this whole tile)
          float zz[8];
          const uint4 zv = zpre[OUT_MODE == 0 && DACT ? qtr * ITS + it : 0];
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
    if (OUT_MODE == 0 && DACT && p.dact && p.colpart) {
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

  if constexpr (SCATTER) {
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
}

}  // namespace g256
}  // namespace ffk

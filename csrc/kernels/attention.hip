// Flash attention (forward + backward), bf16 in/out, fp32 accumulate, gfx950 MFMA 32x32x16.
//
// Forward (per workgroup: 4 waves x 32 query rows, K/V tiles of 64 keys double-buffered in LDS):
//   S^T = K . Q^T with swapped operands so each lane owns ONE query row (lane&31) and 32 of the
//   tile's 64 keys -> online softmax is lane-local plus one xor-32 exchange (T12 idea);
//   the fp32 S^T accumulator is converted to bf16 and used directly as the B operand of
//   O^T += V^T . P^T (cdna_hip_programming.md §3 'An accumulator tile as the next MFMA's operand');
//   V^T fragments come from ds_read_b64_tr_b16 on the row-major V tile (T10).
//   LDS images use an XOR swizzle found by exhaustive search to be conflict-free for both the
//   ds_read_b128 K reads and the transposed V reads (128-B rows), or T10 image (b) for 256-B rows.
// Backward (per workgroup: 4 waves x 32 keys; loop over 64-query tiles):
//   S, dP are computed with the KEY on the lane so P and dS feed dV^T and dK^T as B operands with
//   no data movement; dS^T goes through LDS once for dQ = dS . K, whose per-key-block partials are
//   written with plain fp32 stores (no atomics, deterministic) and summed by a finishing kernel.
// Strided Q/K/V/O views are supported so that the fused QKV projection output [B,S,3,H,D] and the
// [B,S,H,D] output feed/leave the kernel without permute copies.
//
// Reference counterpart: src/ops/attention.cu (cuDNN multi-head attention, fwd+bwd); the
// reference HIP build disables it entirely (src/ops/attention.cpp:33-43 '#if 0').
#include "common.h"
#include "ops.h"
#include "attention.h"

namespace ffk {

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

template <int D>
__device__ __forceinline__ int aswz(int row) {
  if (D == 64) return (((row >> 1) & 1) << 2) | ((row >> 3) & 1) | (((row >> 4) & 1) << 1);
  else return ((row & 3) << 2) | ((row >> 2) & 3);
}
// byte offset of element (row, col) of a [rows][D] bf16 tile image
template <int D>
__device__ __forceinline__ int aoff(int row, int col) {
  const int ch = col >> 3;
  return row * (D * 2) + ((ch ^ aswz<D>(row)) << 4) + ((col & 7) << 1);
}

// 2^x as the bare v_exp_f32. exp2f() lowers to v_exp_f32 wrapped in a denormal range fix-up
// (v_cmp + 2 v_cndmask + v_add + v_ldexp: six VALU ops per score element instead of one); softmax
// probabilities below 2^-126 are irrelevant (they flush to 0, exp2(-inf) stays 0).
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

typedef short v4s __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x4 tr_read(const char* lds, int off) {
  v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(lds + off));
  return __builtin_bit_cast(bf16x4, v);
}

// Stage a [ROWS][D] bf16 tile (rows r0.., clamp at rlim) from global (row stride ss) into regs.
template <int D, int ROWS, int NTH>
struct TileStage {
  static constexpr int CH = ROWS * D / 8 / NTH;  // 16-B chunks per thread
  uint4 r[CH];
  __device__ __forceinline__ void load(const bf16_t* g, int64_t ss, int r0, int rlim, int tid) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int id = tid + i * NTH;
      const int row = id / (D / 8), c = id % (D / 8);
      if (r0 + row < rlim) r[i] = *reinterpret_cast<const uint4*>(g + (int64_t)(r0 + row) * ss + c * 8);
      else r[i] = make_uint4(0, 0, 0, 0);
    }
  }
  __device__ __forceinline__ void store(char* lds, int tid) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int id = tid + i * NTH;
      const int row = id / (D / 8), c = id % (D / 8);
      *reinterpret_cast<uint4*>(lds + aoff<D>(row, c * 8)) = r[i];
    }
  }
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// Same [64][D] tile image as TileStage::store, written by the LDS-DMA path (buffer_load ... lds):
// no staging registers, so the forward needs 32 fewer VGPRs (4 workgroups per CU instead of 3 at
// D = 64). Each wave instruction fills one 1-KiB piece, lane l landing at piece + 16 l; the XOR
// swizzle is applied on the global side (lane l of slot s fetches chunk (s % CPR) ^ aswz(row)).
// Rows past the sequence end read as zero (buffer range check), like TileStage's clamp.
template <int D, int NWAVES>
__device__ __forceinline__ void dma_tile(__amdgpu_buffer_rsrc_t rs, char* lds_tile, int64_t ss, int r0, int wave,
                                         int lane) {
  constexpr int PIECES = 64 * D * 2 / 1024, CPR = D / 8;
#pragma unroll
  for (int i = 0; i < PIECES / NWAVES; ++i) {
    const int piece = i * NWAVES + wave;
    const int slot = piece * 64 + lane;
    const int row = slot / CPR;
    const int ch = (slot % CPR) ^ aswz<D>(row);
    const int off = (int)(((int64_t)(r0 + row) * ss + ch * 8) * 2);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(lds_tile + piece * 1024), 16, off, 0, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 cat8(bf16x4 lo, bf16x4 hi) {
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

__device__ __forceinline__ bf16x8 pack8(const f32x16& a, int base) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (__bf16)a[base + j];
  return o;
}

// ------------------------------------------------------------------------------------ forward
// MASK = false (no ragged key tile, not causal) compiles the mask test out. 1-D grid through
// xcd_remap: the query blocks of one (batch, head) share an XCD and its L2 copy of K / V. The O
// tile leaves through LDS as whole rows (16 B per lane). Together -5 % at B32 H16 S512 D64
// (scripts/lab/attn_fwd_lab.hip, profiles/attn_fwd_lab_r2.txt).
template <int D, bool MASK, bool DMA>
__global__ void __launch_bounds__(256, DMA ? 4 : 2) attn_fwd_kernel(AttnArgs a) {
  constexpr int KV = 64;
  constexpr int TB = KV * D * 2;  // bytes of one K or V tile
  __shared__ __attribute__((aligned(16))) char smem[4 * TB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int nqb = (a.Sq + 127) / 128;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = lid / nqb, b = bh / a.H, hh = bh % a.H;
  const int qblk0 = (lid % nqb) * 128;
  const int q0 = qblk0 + wave * 32;
  const int qrow = q0 + (lane & 31);
  const bf16_t* Q = a.q + (int64_t)b * a.q_sb + (int64_t)hh * a.q_sh;
  const bf16_t* K = a.k + (int64_t)b * a.k_sb + (int64_t)hh * a.k_sh;
  const bf16_t* V = a.v + (int64_t)b * a.v_sb + (int64_t)hh * a.v_sh;

  bf16x8 qf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    if (qrow < a.Sq) qf[s] = *reinterpret_cast<const bf16x8*>(Q + (int64_t)qrow * a.q_ss + 16 * s + 8 * h);
    else qf[s] = bf16x8{};
  }
  f32x16 oacc[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) oacc[i] = f32x16{};
  float m = -INFINITY, lsum = 0.f;
  const float sl2 = a.scale * LOG2E;

  // This lane's fragment byte offsets inside a K / V tile image, computed once: the 32-row key
  // half (kt), the V tile and the double-buffer slot are additive (ds_read immediates; the swizzle
  // does not see row bit 5), only the swizzled chunk bits need a register each. Recomputing them
  // per tile was ~100 of the loop's ~300 VALU instructions.
  const int G = lane >> 4, qi = (lane & 15) >> 2, pi = lane & 3;
  int ko[D / 16], vo[D / 32][2][2];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    ko[s] = aoff<D>(lane & 31, 16 * s + 8 * h);
    asm volatile("" : "+v"(ko[s]));  // keep in a register (no per-tile rematerialisation)
  }
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int hi = 0; hi < 2; ++hi) {
        vo[dt][s2][hi] = aoff<D>(16 * s2 + 4 * h + qi + 8 * hi, dt * 32 + 16 * (G & 1) + 4 * pi);
        asm volatile("" : "+v"(vo[dt][s2][hi]));
      }

  int nkv = (a.Sk + KV - 1) / KV;
  if (a.causal) nkv = min(nkv, (min(qblk0 + 128, a.Sq) + KV - 1) / KV);

  TileStage<D, KV, 256> sk, sv;
  const int kb = (int)min((int64_t)0x7fffffff, ((int64_t)(a.Sk - 1) * a.k_ss + D) * 2);
  const int vb = (int)min((int64_t)0x7fffffff, ((int64_t)(a.Sk - 1) * a.v_ss + D) * 2);
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc((void*)K, (short)0, kb, 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void*)V, (short)0, vb, 0x00020000);
  if (nkv > 0) {
    if (DMA) {
      dma_tile<D, 4>(rk, smem, a.k_ss, 0, wave, lane);
      dma_tile<D, 4>(rv, smem + TB, a.v_ss, 0, wave, lane);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      sk.load(K, a.k_ss, 0, a.Sk, tid);
      sv.load(V, a.v_ss, 0, a.Sk, tid);
      sk.store(smem, tid);
      sv.store(smem + TB, tid);
    }
    __syncthreads();
  }
  // one K/V tile; the double-buffer slot PAR is a compile-time constant (the loop below is unrolled
  // by two) so that the slot base is an immediate of every ds_read, not a per-address add
  auto tile = [&](auto par, int t) {
    constexpr int PAR = decltype(par)::value;
    const char* kl = smem + PAR * 2 * TB;
    const char* vl = kl + TB;
    char* nk = smem + (PAR ^ 1) * 2 * TB;
    const bool more = t + 1 < nkv;
    if (more) {
      if (DMA) {
        dma_tile<D, 4>(rk, nk, a.k_ss, (t + 1) * KV, wave, lane);
        dma_tile<D, 4>(rv, nk + TB, a.v_ss, (t + 1) * KV, wave, lane);
      } else {
        sk.load(K, a.k_ss, (t + 1) * KV, a.Sk, tid);
        sv.load(V, a.v_ss, (t + 1) * KV, a.Sk, tid);
      }
    }
    // S^T[key][q] for keys 32kt..32kt+31 of this tile
    f32x16 sacc[2] = {f32x16{}, f32x16{}};
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kl + ko[s] + kt * 32 * 2 * D);
        sacc[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], sacc[kt], 0, 0, 0);
      }
    }
    // mask (only on tiles that cross the sequence end or the causal diagonal: a wave-uniform
    // test), online softmax on the raw scores (lane-local + xor-32 partner), scale folded into
    // one FMA per element: p = exp2(s * sl2 - m * sl2)
    const int kbase = t * KV;
    const bool need_mask = MASK && ((kbase + KV > a.Sk) || (a.causal && kbase + KV - 1 > q0));
    if (need_mask) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kbase + 32 * kt + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (key >= a.Sk || (a.causal && key > qrow)) sacc[kt][r] = -INFINITY;
        }
      }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sacc[kt][r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * sl2;
    // deferred max (cdna_hip_programming.md T13): the running max moves (and O / l are rescaled)
    // only when some row's tile max exceeds it by more than a.rescale_thr (log2 units); otherwise P is
    // taken against the old max and stays <= 2^rescale_thr. Decided before this tile's P exists, so
    // nothing is ever at two scales.
    if (!__all(mx <= m + a.rescale_thr)) {
      const float mnew = fmaxf(m, mx);
      const float alpha = fast_exp2(m - (mnew == -INFINITY ? 0.f : mnew));
      lsum *= alpha;
#pragma unroll
      for (int i = 0; i < D / 32; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[i][r] *= alpha;
      m = mnew;
    }
    const float msafe = m == -INFINITY ? 0.f : m;
    float rs0 = 0.f, rs1 = 0.f;  // two chains: half the dependent-add latency
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = fast_exp2(__builtin_fmaf(sacc[kt][r], sl2, -msafe));
        sacc[kt][r] = p;
        if (r & 1) rs1 += p;
        else rs0 += p;
      }
    }
    float rs = rs0 + rs1;
    rs += __shfl_xor(rs, 32, 64);
    lsum += rs;
    // O^T[d][q] += V^T[d][key] . P^T[key][q]
    bf16x8 pf[2][2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) { pf[kt][0] = pack8(sacc[kt], 0); pf[kt][1] = pack8(sacc[kt], 8); }
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16x4 lo = tr_read(vl, vo[dt][s2][0] + kt * 32 * 2 * D);
          const bf16x4 hi = tr_read(vl, vo[dt][s2][1] + kt * 32 * 2 * D);
          oacc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cat8(lo, hi), pf[kt][s2], oacc[dt], 0, 0, 0);
        }
      }
    }
    if (more) {
      if (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else {
        sk.store(nk, tid);
        sv.store(nk + TB, tid);
      }
    }
    __syncthreads();
  };
  for (int t = 0; t < nkv; t += 2) {
    tile(std::integral_constant<int, 0>{}, t);
    if (t + 1 < nkv) tile(std::integral_constant<int, 1>{}, t + 1);
  }
  // epilogue: O^T accumulators (lane = query row, d = 32dt + 8g + 4h + 0..3) -> [128 q][D] LDS
  // image (16-B chunks XOR-swizzled by row & 7) -> whole-row 16-B stores
  __syncthreads();  // the last tile's V reads are done: the K/V buffers are free
  {
    const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
    const int row = wave * 32 + (lane & 31);
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 4 * dt + g;
        *reinterpret_cast<uint2*>(smem + row * (D * 2) + ((c ^ (row & 7)) << 4) + 8 * h) =
            make_uint2((unsigned)f2bf(oacc[dt][4 * g] * inv) | ((unsigned)f2bf(oacc[dt][4 * g + 1] * inv) << 16),
                       (unsigned)f2bf(oacc[dt][4 * g + 2] * inv) | ((unsigned)f2bf(oacc[dt][4 * g + 3] * inv) << 16));
      }
    if (h == 0 && a.lse && qrow < a.Sq) a.lse[(int64_t)bh * a.Sq + qrow] = lsum > 0.f ? (m * LN2 + __logf(lsum)) : INFINITY;
  }
  __syncthreads();
  {
    constexpr int CPR = D / 8;
    bf16_t* Ob = a.o + (int64_t)b * a.o_sb + (int64_t)hh * a.o_sh;
#pragma unroll
    for (int i = 0; i < 128 * CPR / 256; ++i) {
      const int id = tid + i * 256, r = id / CPR, c = id % CPR;
      if (qblk0 + r < a.Sq)
        *reinterpret_cast<uint4*>(Ob + (int64_t)(qblk0 + r) * a.o_ss + 8 * c) =
            *reinterpret_cast<const uint4*>(smem + r * (D * 2) + ((c ^ (r & 7)) << 4));
    }
  }
}

// ------------------------------------------------------------------ forward, 64 rows per wave
// attn_fwd_kernel with two 32-row query blocks per wave (256 rows per 4-wave workgroup, two
// workgroups per CU at <= 256 registers): every K fragment, V fragment and DMA piece serves two
// row blocks. Why: summing a wave-tile's issue cycles (16 MFMAs hold the SIMD's issue for 128
// cycles, ~176 VALU instructions ~720, 4 LDS-DMA pieces ~250-400, 24 LDS reads ~150) gives ~1400
// per 512 cycles of MFMA work. Measured (profiles/attn_fwd_variants_r4.txt): +2..6 % for S >= 512
// (708 -> 725-740 TF/s at B32 H16 S512, 794 -> 840 at S4096), -1..7 % at S = 256; taking the row
// sums on the matrix core (ones x P^T) as well did not help. Bitwise equal to the 4-wave kernel.
// D = 64; the default for Sq >= 512 (variant 3).
template <bool MASK>
__global__ void __launch_bounds__(256, 2) attn_fwd2_kernel(AttnArgs a) {
  constexpr int D = 64, KV = 64, QB = 2, ROWS = 4 * 32 * QB;
  constexpr int TB = KV * D * 2;
  __shared__ __attribute__((aligned(16))) char smem[ROWS * D * 2 > 4 * TB ? ROWS * D * 2 : 4 * TB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int nqb = (a.Sq + ROWS - 1) / ROWS;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = lid / nqb, b = bh / a.H, hh = bh % a.H;
  const int qblk0 = (lid % nqb) * ROWS;
  const int q0 = qblk0 + wave * 32 * QB;  // rows q0 + 32 qb + (lane & 31)
  const bf16_t* Q = a.q + (int64_t)b * a.q_sb + (int64_t)hh * a.q_sh;
  const bf16_t* K = a.k + (int64_t)b * a.k_sb + (int64_t)hh * a.k_sh;
  const bf16_t* V = a.v + (int64_t)b * a.v_sb + (int64_t)hh * a.v_sh;

  bf16x8 qf[QB][D / 16];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    const int qrow = q0 + 32 * qb + (lane & 31);
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      if (qrow < a.Sq) qf[qb][s] = *reinterpret_cast<const bf16x8*>(Q + (int64_t)qrow * a.q_ss + 16 * s + 8 * h);
      else qf[qb][s] = bf16x8{};
    }
  }
  f32x16 oacc[QB][D / 32];
  float m[QB], lsum[QB];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
#pragma unroll
    for (int i = 0; i < D / 32; ++i) oacc[qb][i] = f32x16{};
    m[qb] = -INFINITY;
    lsum[qb] = 0.f;
  }
  const float sl2 = a.scale * LOG2E;

  const int G = lane >> 4, qi = (lane & 15) >> 2, pi = lane & 3;
  int ko[D / 16], vo[D / 32][2][2];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    ko[s] = aoff<D>(lane & 31, 16 * s + 8 * h);
    asm volatile("" : "+v"(ko[s]));
  }
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int hi = 0; hi < 2; ++hi) {
        vo[dt][s2][hi] = aoff<D>(16 * s2 + 4 * h + qi + 8 * hi, dt * 32 + 16 * (G & 1) + 4 * pi);
        asm volatile("" : "+v"(vo[dt][s2][hi]));
      }

  int nkv = (a.Sk + KV - 1) / KV;
  if (a.causal) nkv = min(nkv, (min(qblk0 + ROWS, a.Sq) + KV - 1) / KV);
  const int kb = (int)min((int64_t)0x7fffffff, ((int64_t)(a.Sk - 1) * a.k_ss + D) * 2);
  const int vb = (int)min((int64_t)0x7fffffff, ((int64_t)(a.Sk - 1) * a.v_ss + D) * 2);
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc((void*)K, (short)0, kb, 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void*)V, (short)0, vb, 0x00020000);
  if (nkv > 0) {
    dma_tile<D, 4>(rk, smem, a.k_ss, 0, wave, lane);
    dma_tile<D, 4>(rv, smem + TB, a.v_ss, 0, wave, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  auto tile = [&](auto par, int t) {
    constexpr int PAR = decltype(par)::value;
    const char* kl = smem + PAR * 2 * TB;
    const char* vl = kl + TB;
    char* nk = smem + (PAR ^ 1) * 2 * TB;
    const bool more = t + 1 < nkv;
    if (more) {
      dma_tile<D, 4>(rk, nk, a.k_ss, (t + 1) * KV, wave, lane);
      dma_tile<D, 4>(rv, nk + TB, a.v_ss, (t + 1) * KV, wave, lane);
    }
    f32x16 sacc[QB][2];
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) sacc[qb][0] = sacc[qb][1] = f32x16{};
#pragma unroll
    for (int s = 0; s < D / 16; ++s)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kl + ko[s] + kt * 32 * 2 * D);
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
          sacc[qb][kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[qb][s], sacc[qb][kt], 0, 0, 0);
      }
    const int kbase = t * KV;
    bf16x8 pf[QB][2][2];
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
      const int qrow = q0 + 32 * qb + (lane & 31);
      const bool need_mask = MASK && ((kbase + KV > a.Sk) || (a.causal && kbase + KV - 1 > q0 + 32 * qb));
      if (need_mask) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = kbase + 32 * kt + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (key >= a.Sk || (a.causal && key > qrow)) sacc[qb][kt][r] = -INFINITY;
          }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sacc[qb][kt][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * sl2;
      if (!__all(mx <= m[qb] + a.rescale_thr)) {
        const float mnew = fmaxf(m[qb], mx);
        const float alpha = fast_exp2(m[qb] - (mnew == -INFINITY ? 0.f : mnew));
        lsum[qb] *= alpha;
#pragma unroll
        for (int i = 0; i < D / 32; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) oacc[qb][i][r] *= alpha;
        m[qb] = mnew;
      }
      const float msafe = m[qb] == -INFINITY ? 0.f : m[qb];
      float rs0 = 0.f, rs1 = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fast_exp2(__builtin_fmaf(sacc[qb][kt][r], sl2, -msafe));
          sacc[qb][kt][r] = p;
          if (r & 1) rs1 += p;
          else rs0 += p;
        }
      float rs = rs0 + rs1;
      rs += __shfl_xor(rs, 32, 64);
      lsum[qb] += rs;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) { pf[qb][kt][0] = pack8(sacc[qb][kt], 0); pf[qb][kt][1] = pack8(sacc[qb][kt], 8); }
    }
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16x4 lo = tr_read(vl, vo[dt][s2][0] + kt * 32 * 2 * D);
          const bf16x4 hi = tr_read(vl, vo[dt][s2][1] + kt * 32 * 2 * D);
          const bf16x8 vf = cat8(lo, hi);
#pragma unroll
          for (int qb = 0; qb < QB; ++qb)
            oacc[qb][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[qb][kt][s2], oacc[qb][dt], 0, 0, 0);
        }
    if (more) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  for (int t = 0; t < nkv; t += 2) {
    tile(std::integral_constant<int, 0>{}, t);
    if (t + 1 < nkv) tile(std::integral_constant<int, 1>{}, t + 1);
  }
  __syncthreads();
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    const float inv = lsum[qb] > 0.f ? 1.f / lsum[qb] : 0.f;
    const int row = wave * 32 * QB + 32 * qb + (lane & 31);
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 4 * dt + g;
        *reinterpret_cast<uint2*>(smem + row * (D * 2) + ((c ^ (row & 7)) << 4) + 8 * h) =
            make_uint2((unsigned)f2bf(oacc[qb][dt][4 * g] * inv) | ((unsigned)f2bf(oacc[qb][dt][4 * g + 1] * inv) << 16),
                       (unsigned)f2bf(oacc[qb][dt][4 * g + 2] * inv) | ((unsigned)f2bf(oacc[qb][dt][4 * g + 3] * inv) << 16));
      }
    const int qrow = q0 + 32 * qb + (lane & 31);
    if (h == 0 && a.lse && qrow < a.Sq)
      a.lse[(int64_t)bh * a.Sq + qrow] = lsum[qb] > 0.f ? (m[qb] * LN2 + __logf(lsum[qb])) : INFINITY;
  }
  __syncthreads();
  {
    constexpr int CPR = D / 8;
    bf16_t* Ob = a.o + (int64_t)b * a.o_sb + (int64_t)hh * a.o_sh;
#pragma unroll
    for (int i = 0; i < ROWS * CPR / 256; ++i) {
      const int id = tid + i * 256, r = id / CPR, c = id % CPR;
      if (qblk0 + r < a.Sq)
        *reinterpret_cast<uint4*>(Ob + (int64_t)(qblk0 + r) * a.o_ss + 8 * c) =
            *reinterpret_cast<const uint4*>(smem + r * (D * 2) + ((c ^ (r & 7)) << 4));
    }
  }
}

// ------------------------------------------------------------------------------------ backward
// delta[bh][q] = sum_d dO[q][d] * O[q][d]
template <int D>
__global__ void attn_bwd_pre_kernel(AttnArgs a) {
  // delta[row] = sum_d O[row][d] * dO[row][d]: D/8 lanes per row, one 16-B load of each per lane
  constexpr int LPR = D / 8;
  const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t row = gt / LPR;
  const int part = (int)(gt % LPR);
  const int64_t total = (int64_t)a.B * a.H * a.Sq;
  float s = 0.f;
  if (row < total) {
    const int bh = (int)(row / a.Sq), q = (int)(row % a.Sq), b = bh / a.H, hh = bh % a.H;
    const bf16_t* O = a.o + (int64_t)b * a.o_sb + (int64_t)hh * a.o_sh + (int64_t)q * a.o_ss + part * 8;
    const bf16_t* dO = a.dout + (int64_t)b * a.do_sb + (int64_t)hh * a.do_sh + (int64_t)q * a.do_ss + part * 8;
    float o[8], d[8];
    load16(O, o);
    load16(dO, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += o[j] * d[j];
  }
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (row < total && part == 0) {
    a.delta[row] = s;
    a.lse2[row] = a.lse[row] * LOG2E;  // the DMA backward reads lse in log2 units
  }
}

// dS^T image [key][64 queries] (128-B rows): byte offset of (key row, query q), q % 4 == 0. The
// 8-B unit index is XORed with f(row) = row[2:0] | (row[1]^row[3])<<3 — found by exhaustive search
// over linear XOR maps to be conflict-free both for the 8-B writes (16 consecutive key rows per
// lane group, banks mod 32) and for the ds_read_b64_tr_b16 reads of the dQ stage (banks mod 64);
// the unswizzled image cost ~57 % extra LDS cycles (SQ_LDS_BANK_CONFLICT, profiles/attn_pmc_r1.txt).
// Workgroup barrier that orders LDS only: __syncthreads() also waits vmcnt(0), which here would
// stall every q-tile on the dQ partial stores (and on the next tile's prefetch) for a full
// memory round trip.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ int dst_off(int row, int q) {
  const int f = (row & 7) | ((((row >> 1) ^ (row >> 3)) & 1) << 3);
  return row * 128 + (((q >> 2) ^ f) << 3) + (q & 3) * 2;
}

__device__ __forceinline__ unsigned pack_bf2(float x, float y) {
  return (unsigned)f2bf(x) | ((unsigned)f2bf(y) << 16);
}

// NW waves x 32 keys per workgroup (NW = 8 at D = 64: 256 keys; 4 at D = 128), loop over 64-query
// tiles. Shaped by measurements (scripts/lab/attn_bwd_lab.hip, profiles/attn_bwd_lab_r2.txt):
//  * MASK = false (no ragged blocks, not causal) drops every bounds / mask test; with MASK the
//    key / causal mask runs only on 32x32 blocks that cross the sequence end or the diagonal (a
//    per-element select on every block cost the kernel ~30 %).
//  * Prologue: the K and V blocks go row-coalesced into LDS (K stays there for dQ; V is staged in
//    the tile buffers) and the per-lane K^T / V^T fragments are read from LDS — not per-lane
//    gathers at the 6 KB row stride of a fused QKV projection.
//  * Epilogue: dK / dV are staged through LDS and stored as whole 128/256-B rows, 16 B per lane
//    (the per-lane 8-B stores scattered over 32 rows were store-issue bound: ~8 % of the kernel).
//  * dQ tiles are computed transposed (dQ^T = K^T . dS^T: lane = query, 4 consecutive d per
//    register quad), so partials move as 16-B vectors.
//  * CHAIN: one launch per key block; launch p adds its dQ contribution to the fp32 running sum
//    left by launch p - 1 (cache-resident, read back by the same lanes that will rewrite it) and the
//    last contributing block writes the bf16 dQ — no per-key-block slabs and no finishing pass
//    (228 -> 163 us at B32 H16 S512 D64). It needs B*H workgroups per launch to fill the chip, so
//    small batch x heads use one launch with per-key-block slabs + attn_dq_finish_kernel.
//  * 1-D grid through xcd_remap: the key blocks of one (batch, head) share an XCD (and its L2 copy
//    of Q / dO).
//  * DMA: the next Q / dO tile and its lse2 / delta rows go global -> LDS by buffer_load ... lds
//    (no staging registers, no ds_write of the tile); vmcnt also counts stores, so the dQ tile's
//    global stores are issued after the end-of-tile barrier, behind the wait for the DMA.
template <int D, int NW, bool MASK, bool CHAIN, bool DMA = false>
__global__ void __launch_bounds__(64 * NW, 8 / NW) attn_bwd_kernel(AttnArgs a, int nkb, int pass) {
  constexpr int NT = 64 * NW;
  constexpr int QT = 64;       // queries per loop step
  constexpr int KB = 32 * NW;  // keys per workgroup
  constexpr int QB = QT * D * 2;
  // LDS: 2 x {Q tile, dO tile, lse, delta} (double-buffered: tile t+1 is fetched into registers
  // while tile t is computed), K block image, dS^T image [KB][QT]
  constexpr int TILE = 2 * QB + 2 * QT * 4;
  static_assert(2 * TILE >= KB * D * 2, "tile buffers stage the V block and the dV image");
  // dQ stage: NTILE (d x query) 32x32 tiles per q-tile; with more waves than tiles, KSPLIT waves
  // share a tile's key range and the upper parts hand their fp32 partial to part 0 through LDS
  constexpr int NTILE = 2 * (D / 32);
  constexpr int KSPLIT = NW > NTILE ? NW / NTILE : 1;
  constexpr int DQX = KSPLIT > 1 ? NTILE * (KSPLIT - 1) * 32 * 32 * 4 : 0;
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE + KB * D * 2 + KB * QT * 2 + DQX];
  char* k_l = smem + 2 * TILE;
  char* ds_l = k_l + KB * D * 2;
  float* dqx_l = reinterpret_cast<float*>(ds_l + KB * QT * 2);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int groups = CHAIN ? 1 : nkb;  // workgroups per (batch, head) in this launch
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = lid / groups, b = bh / a.H, hh = bh % a.H;
  const int kblk = CHAIN ? pass : lid % groups;
  const int kb0 = kblk * KB;
  const int key = kb0 + wave * 32 + (lane & 31);
  const bf16_t* Q = a.q + (int64_t)b * a.q_sb + (int64_t)hh * a.q_sh;
  const bf16_t* K = a.k + (int64_t)b * a.k_sb + (int64_t)hh * a.k_sh;
  const bf16_t* V = a.v + (int64_t)b * a.v_sb + (int64_t)hh * a.v_sh;
  const bf16_t* dO = a.dout + (int64_t)b * a.do_sb + (int64_t)hh * a.do_sh;
  const float* LSE = a.lse + (int64_t)bh * a.Sq;
  const float* DL = a.delta + (int64_t)bh * a.Sq;
  const float sl2 = a.scale * LOG2E;
  static_assert(!DMA || NW >= 2 * (D / 32), "DMA defers one dQ tile per wave past the barrier");
  // DMA: buffer resources over this (batch, head)'s Q / dO rows and lse2 / delta entries
  const int qbytes = (int)min((int64_t)0x7fffffff, ((int64_t)(a.Sq - 1) * a.q_ss + D) * 2);
  const int dbytes = (int)min((int64_t)0x7fffffff, ((int64_t)(a.Sq - 1) * a.do_ss + D) * 2);
  const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc((void*)Q, (short)0, qbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rdo = __builtin_amdgcn_make_buffer_rsrc((void*)dO, (short)0, dbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rl =
      __builtin_amdgcn_make_buffer_rsrc((void*)(a.lse2 + (int64_t)bh * a.Sq), (short)0, a.Sq * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rdl = __builtin_amdgcn_make_buffer_rsrc((void*)DL, (short)0, a.Sq * 4, 0x00020000);
  // chain: slab 0 carries the running dQ sum; otherwise one fp32 slab per key block
  const bool chain = CHAIN || nkb == 1;
  float* dq_part = a.dq_acc + (int64_t)(chain ? 0 : kblk) * a.B * a.H * a.Sq * D + (int64_t)bh * a.Sq * D;
  bf16_t* dQb = a.dq + (int64_t)b * a.dq_sb + (int64_t)hh * a.dq_sh;

  // K block -> LDS (kept for dQ), V block -> tile buffers; K^T / V^T fragments (B operands, key on
  // the lane) from the LDS images
  bf16x8 kf[D / 16], vf[D / 16];
  {
    TileStage<D, KB, NT> sk, sv;
    sk.load(K, a.k_ss, kb0, MASK ? a.Sk : 1 << 30, tid);
    sv.load(V, a.v_ss, kb0, MASK ? a.Sk : 1 << 30, tid);
    sk.store(k_l, tid);
    sv.store(smem, tid);
  }
  __syncthreads();
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    const int row = wave * 32 + (lane & 31);
    kf[s] = *reinterpret_cast<const bf16x8*>(k_l + aoff<D>(row, 16 * s + 8 * h));
    vf[s] = *reinterpret_cast<const bf16x8*>(smem + aoff<D>(row, 16 * s + 8 * h));
  }
  f32x16 dk[D / 32], dv[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) { dk[i] = f32x16{}; dv[i] = f32x16{}; }
  const int qt_begin = (MASK && a.causal) ? kb0 / QT : 0;
  const int nqt = (a.Sq + QT - 1) / QT;
  const int G = lane >> 4, qi = (lane & 15) >> 2, pi = lane & 3;

  TileStage<D, QT, NT> sq, sd;
  float lse_r = INFINITY, dl_r = 0.f;
  auto fetch = [&](int t) {  // global -> registers
    const int qbase = t * QT;
    sq.load(Q, a.q_ss, qbase, MASK ? a.Sq : 1 << 30, tid);
    sd.load(dO, a.do_ss, qbase, MASK ? a.Sq : 1 << 30, tid);
    if (tid < QT) {
      const int q = qbase + tid;
      lse_r = (!MASK || q < a.Sq) ? LSE[q] * LOG2E : INFINITY;
      dl_r = (!MASK || q < a.Sq) ? DL[q] : 0.f;
    }
  };
  auto stash = [&](int t) {  // registers -> LDS buffer t & 1
    char* tb = smem + (t & 1) * TILE;
    sq.store(tb, tid);
    sd.store(tb + QB, tid);
    if (tid < QT) {
      reinterpret_cast<float*>(tb + 2 * QB)[tid] = lse_r;
      reinterpret_cast<float*>(tb + 2 * QB)[QT + tid] = dl_r;
    }
  };
  // DMA: tile t's Q / dO image (the TileStage layout) and lse2 / delta rows into buffer t & 1;
  // rows past Sq read as zero (range check), which makes their P x dO and dS x Q terms zero
  auto dma_rows = [&](int t) {
    char* tb = smem + (t & 1) * TILE;
    dma_tile<D, NW>(rq, tb, a.q_ss, t * QT, wave, lane);
    dma_tile<D, NW>(rdo, tb + QB, a.do_ss, t * QT, wave, lane);
    if (wave == NW - 1) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rl, (lds_ptr_t)(tb + 2 * QB), 4, (t * QT + lane) * 4, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rdl, (lds_ptr_t)(tb + 2 * QB + QT * 4), 4, (t * QT + lane) * 4, 0, 0, 0);
    }
  };
  if constexpr (DMA) {
    __syncthreads();  // every wave has its V fragments: the tile buffers can be overwritten
    if (qt_begin < nqt) {
      dma_rows(qt_begin);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  } else {
    if (qt_begin < nqt) fetch(qt_begin);
    __syncthreads();  // every wave has its V fragments: the tile buffers can be overwritten
    if (qt_begin < nqt) stash(qt_begin);
    __syncthreads();
  }

  for (int t = qt_begin; t < nqt; ++t) {
    const int qbase = t * QT;
    char* tb = smem + (t & 1) * TILE;
    const char* q_l = tb;
    const char* do_l = tb + QB;
    const float* lse_l = reinterpret_cast<const float*>(tb + 2 * QB);
    const float* dl_l = lse_l + QT;
    const bool more = t + 1 < nqt;
    if (more) {  // in flight during this tile's MFMAs
      if constexpr (DMA) dma_rows(t + 1);  // buffer (t+1)&1: its readers finished before tile t-1's mid barrier
      else fetch(t + 1);
    }
    // chain, key block > 0: the previous launch's dQ running sum for this wave's dQ tile, requested
    // now so its HBM round trip runs under the tile's MFMAs (read at its use below, the load sat on
    // the workgroup's critical path once per query tile)
    float4 prev[4];
    if constexpr (NW >= 2 * (D / 32)) {
      const int tile = wave % (2 * (D / 32));
      const int q = qbase + 32 * (tile / (D / 32)) + (lane & 31);
      if (chain && kblk > 0 && wave < 2 * (D / 32) && (!MASK || q < a.Sq)) {
        const float* prow = dq_part + (int64_t)q * D + 32 * (tile % (D / 32)) + 4 * h;
#pragma unroll
        for (int g = 0; g < 4; ++g) prev[g] = *reinterpret_cast<const float4*>(prow + 8 * g);
      }
    }
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      // S[q][key] and dP[q][key] for 32 queries x this wave's 32 keys
      f32x16 sacc = f32x16{}, pacc = f32x16{};
#pragma unroll
      for (int s = 0; s < D / 16; ++s) {
        const int row = 32 * qt + (lane & 31);
        const bf16x8 qa = *reinterpret_cast<const bf16x8*>(q_l + aoff<D>(row, 16 * s + 8 * h));
        const bf16x8 da = *reinterpret_cast<const bf16x8*>(do_l + aoff<D>(row, 16 * s + 8 * h));
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kf[s], sacc, 0, 0, 0);
        pacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, vf[s], pacc, 0, 0, 0);
      }
      // P = exp2(S*sl2 - lse2), dS = P * (dP - delta); accumulator rows 4g..4g+3 are 4 consecutive
      // queries, so their lse / delta come in as one 16-B LDS read each
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const float4 L4 = *reinterpret_cast<const float4*>(lse_l + 32 * qt + 8 * g4 + 4 * h);
        const float lv[4] = {L4.x, L4.y, L4.z, L4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) sacc[4 * g4 + j] = fast_exp2(sacc[4 * g4 + j] * sl2 - lv[j]);
      }
      if (MASK) {
        const bool need = (kb0 + wave * 32 + 31 >= a.Sk) || (a.causal && kb0 + wave * 32 + 31 > qbase + 32 * qt);
        if (need) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int q = qbase + 32 * qt + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (key >= a.Sk || (a.causal && key > q)) sacc[r] = 0.f;
          }
        }
      }
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const float4 D4 = *reinterpret_cast<const float4*>(dl_l + 32 * qt + 8 * g4 + 4 * h);
        const float dv4[4] = {D4.x, D4.y, D4.z, D4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) pacc[4 * g4 + j] = sacc[4 * g4 + j] * (pacc[4 * g4 + j] - dv4[j]);
      }
      const bf16x8 pb0 = pack8(sacc, 0), pb1 = pack8(sacc, 8);
      const bf16x8 sb0 = pack8(pacc, 0), sb1 = pack8(pacc, 8);
      // dV^T[d][key] += dO^T[d][q] . P[q][key];  dK^T[d][key] += Q^T[d][q] . dS[q][key]
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) {
        const int col = dt * 32 + 16 * (G & 1) + 4 * pi;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int r0 = 32 * qt + 16 * s2 + 4 * h + qi;
          const bf16x8 ao = cat8(tr_read(do_l, aoff<D>(r0, col)), tr_read(do_l, aoff<D>(r0 + 8, col)));
          const bf16x8 aq = cat8(tr_read(q_l, aoff<D>(r0, col)), tr_read(q_l, aoff<D>(r0 + 8, col)));
          dv[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ao, s2 ? pb1 : pb0, dv[dt], 0, 0, 0);
          dk[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aq, s2 ? sb1 : sb0, dk[dt], 0, 0, 0);
        }
      }
      // dS^T image [key][q] (key = wave*32 + lane&31): the packed dS quads, 4 queries per 8-B write
      {
        const int krow = wave * 32 + (lane & 31);
        const bf16x4 parts[4] = {sb0.lo, sb0.hi, sb1.lo, sb1.hi};
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<bf16x4*>(ds_l + dst_off(krow, 32 * qt + 8 * g + 4 * h)) = parts[g];
      }
    }
    lds_barrier();
    // the dQ tile's running-sum / final store (deferred past the end-of-tile barrier under DMA)
    auto put_dq = [&](f32x16& acc, int tile, int part) {
      const int qt = tile / (D / 32), dt = tile % (D / 32);
      const int q = qbase + 32 * qt + (lane & 31);
      if (part == 0 && (!MASK || q < a.Sq)) {
        float* prow = dq_part + (int64_t)q * D + 32 * dt + 4 * h;
        if (chain && kblk > 0) {
          // the previous launch's running sum (written by this lane of the same wave position);
          // a causal block's query tiles all had key block kblk - 1 contributing too
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            float4 pv;
            if constexpr (NW >= 2 * (D / 32)) pv = prev[g];  // prefetched at the top of the tile
            else pv = *reinterpret_cast<const float4*>(prow + 8 * g);
            acc[4 * g] += pv.x; acc[4 * g + 1] += pv.y; acc[4 * g + 2] += pv.z; acc[4 * g + 3] += pv.w;
          }
        }
        // last key block contributing to this query tile: the last one, or (causal) the diagonal's
        int last = nkb - 1;
        if (MASK && a.causal) last = min(last, (qbase + QT - 1) / KB);
        if (chain && kblk == last) {
          bf16_t* drow = dQb + (int64_t)q * a.dq_ss + 32 * dt + 4 * h;
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<uint2*>(drow + 8 * g) = make_uint2(pack_bf2(acc[4 * g] * a.scale, acc[4 * g + 1] * a.scale),
                                                                 pack_bf2(acc[4 * g + 2] * a.scale, acc[4 * g + 3] * a.scale));
        } else {
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<float4*>(prow + 8 * g) = make_float4(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]);
        }
      }
    };
    auto add_parts = [&](f32x16& acc, int tile) {
#pragma unroll
      for (int p2 = 1; p2 < KSPLIT; ++p2) {
        const float* o = dqx_l + ((p2 - 1) * NTILE + tile) * 1024;
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {
          const float4 v = *reinterpret_cast<const float4*>(o + (r4 * 64 + lane) * 4);
          acc[4 * r4] += v.x; acc[4 * r4 + 1] += v.y; acc[4 * r4 + 2] += v.z; acc[4 * r4 + 3] += v.w;
        }
      }
    };
    f32x16 dq_keep;
    int dq_tile = -1, dq_kpart = 0;
    // dQ^T tile (d x query) = K^T . dS^T over this block's keys: wave -> (qt, dt) tiles (and, with
    // KSPLIT > 1, a 1/KSPLIT slice of the keys); lane = query, rows = d (r&3) + 8(r>>2) + 4h
    for (int tile = wave % NTILE; tile < NTILE; tile += (NW < NTILE ? NW : NTILE)) {
      const int qt = tile / (D / 32), dt = tile % (D / 32);
      const int part = KSPLIT > 1 ? wave / NTILE : 0;
      constexpr int KS_PER = KB / 16 / KSPLIT;
      f32x16 acc = f32x16{};
      // fully unrolled the 16-step form (4 waves: one wave per tile) spilled 14 VGPRs
#pragma unroll(KS_PER > 8 ? 4 : KS_PER)
      for (int ks = part * KS_PER; ks < (part + 1) * KS_PER; ++ks) {
        const int kr = 16 * ks + 8 * h + qi;
        const int cq = 32 * qt + 16 * (G & 1) + 4 * pi;
        const bf16x8 af = cat8(tr_read(ds_l, dst_off(kr, cq)), tr_read(ds_l, dst_off(kr + 4, cq)));
        const int cd = 32 * dt + 16 * (G & 1) + 4 * pi;
        const bf16x8 bk = cat8(tr_read(k_l, aoff<D>(kr, cd)), tr_read(k_l, aoff<D>(kr + 4, cd)));
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bk, af, acc, 0, 0, 0);
      }
      if constexpr (KSPLIT > 1) {
        // parts 1.. park their partial in LDS (lane-major: conflict-free 16-B rows), part 0 adds
        // (under DMA after the end-of-tile barrier, which then orders the exchange: one barrier less)
        float* slot = dqx_l + ((part - 1) * NTILE + tile) * 1024;
        if (part > 0) {
#pragma unroll
          for (int r4 = 0; r4 < 4; ++r4)
            *reinterpret_cast<float4*>(slot + (r4 * 64 + lane) * 4) =
                make_float4(acc[4 * r4], acc[4 * r4 + 1], acc[4 * r4 + 2], acc[4 * r4 + 3]);
        }
        if constexpr (!DMA) {
          lds_barrier();
          if (part == 0) add_parts(acc, tile);
        }
      }
      if constexpr (DMA) {
        dq_keep = acc;
        dq_tile = tile;
        dq_kpart = part;
      } else {
        put_dq(acc, tile, part);
      }
    }
    if constexpr (DMA) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile t+1 landed (and older dQ stores done)
      lds_barrier();
      if (dq_tile >= 0) {
        if constexpr (KSPLIT > 1) {
          if (dq_kpart == 0) add_parts(dq_keep, dq_tile);
        }
        put_dq(dq_keep, dq_tile, dq_kpart);
      }
    } else {
      if (more) stash(t + 1);  // other buffer: its last readers finished before this tile's first sync
      lds_barrier();           // tile t+1 visible; dS^T reads of tile t done before it is rewritten
    }
  }
  // slabs, causal: query tiles before qt_begin get nothing from this key block; zero its rows
  if (MASK && a.causal && !chain) {
    for (int64_t i = tid; i < (int64_t)min(qt_begin * QT, a.Sq) * D; i += NT) dq_part[i] = 0.f;
  }
  // dK (K block image) and dV (tile buffers) through LDS, 16-B chunks XOR-swizzled by row & 7;
  // the loop's last barrier retired every read of both regions
  if (qt_begin >= nqt) __syncthreads();
  {
    char* dv_l = smem;
    const int row = wave * 32 + (lane & 31);
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 4 * dt + g;
        const int off = row * (D * 2) + ((c ^ (row & 7)) << 4) + 8 * h;
        *reinterpret_cast<uint2*>(k_l + off) = make_uint2(pack_bf2(dk[dt][4 * g] * a.scale, dk[dt][4 * g + 1] * a.scale),
                                                          pack_bf2(dk[dt][4 * g + 2] * a.scale, dk[dt][4 * g + 3] * a.scale));
        *reinterpret_cast<uint2*>(dv_l + off) = make_uint2(pack_bf2(dv[dt][4 * g], dv[dt][4 * g + 1]),
                                                           pack_bf2(dv[dt][4 * g + 2], dv[dt][4 * g + 3]));
      }
    }
    lds_barrier();
    bf16_t* dKb = a.dk + (int64_t)b * a.dk_sb + (int64_t)hh * a.dk_sh;
    bf16_t* dVb = a.dv + (int64_t)b * a.dv_sb + (int64_t)hh * a.dv_sh;
    constexpr int CPR = D / 8;  // 16-B chunks per row
#pragma unroll
    for (int i = 0; i < KB * CPR / NT; ++i) {
      const int id = tid + i * NT, r = id / CPR, c = id % CPR;
      const int off = r * (D * 2) + ((c ^ (r & 7)) << 4);
      if (!MASK || kb0 + r < a.Sk) {
        *reinterpret_cast<uint4*>(dKb + (int64_t)(kb0 + r) * a.dk_ss + 8 * c) = *reinterpret_cast<const uint4*>(k_l + off);
        *reinterpret_cast<uint4*>(dVb + (int64_t)(kb0 + r) * a.dv_ss + 8 * c) = *reinterpret_cast<const uint4*>(dv_l + off);
      }
    }
  }
}

// Backward, one barrier per query tile (the default backward, variant 10; D = 64, 8 waves x 32 keys, LDS-DMA tiles):
// attn_bwd_kernel software-pipelined over the query tiles. Iteration t computes S / dP / dV / dK
// of tile t (its dS^T into one of two LDS images) and the dQ of tile t-1 from the other image, so
// the one end-of-iteration barrier orders the tile buffers, both dS^T images and the DMA of tile
// t+1 at once (attn_bwd_kernel: three barriers per tile, two with DMA), and a wave's dQ MFMAs do
// not depend on its S / dP work of the same iteration. dQ^T runs on 16x16x32 MFMAs: 16 (d x query)
// tiles of 16 x 16, two per wave sharing the K^T operand, each over all KB keys, so no wave hands
// a partial sum to another (no exchange buffer: the second dS^T image takes its LDS).
template <bool MASK, bool CHAIN, bool SB = false>
__global__ void __launch_bounds__(512, 1) attn_bwd1b_kernel(AttnArgs a, int nkb, int pass) {
  constexpr int D = 64, NW = 8, NT = 64 * NW, QT = 64, KB = 32 * NW, QB = QT * D * 2;
  constexpr int TILE = 2 * QB + 2 * QT * 4;  // Q tile, dO tile, lse2, delta
  constexpr int DS = KB * QT * 2;            // one dS^T image [KB][QT]
  static_assert(2 * TILE >= KB * D * 2, "tile buffers stage the V block and the dV image");
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE + KB * D * 2 + 2 * DS];
  char* k_l = smem + 2 * TILE;
  char* ds0 = k_l + KB * D * 2;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5;
  const bool late = a.stagger && __builtin_amdgcn_readfirstlane(wave) >= NW / 2;
  const int groups = CHAIN ? 1 : nkb;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = lid / groups, b = bh / a.H, hh = bh % a.H;
  const int kblk = CHAIN ? pass : lid % groups;
  const int kb0 = kblk * KB;
  const int key = kb0 + wave * 32 + (lane & 31);
  const bf16_t* Q = a.q + (int64_t)b * a.q_sb + (int64_t)hh * a.q_sh;
  const bf16_t* K = a.k + (int64_t)b * a.k_sb + (int64_t)hh * a.k_sh;
  const bf16_t* V = a.v + (int64_t)b * a.v_sb + (int64_t)hh * a.v_sh;
  const bf16_t* dO = a.dout + (int64_t)b * a.do_sb + (int64_t)hh * a.do_sh;
  const float* DL = a.delta + (int64_t)bh * a.Sq;
  const float sl2 = a.scale * LOG2E;
  const int qbytes = (int)min((int64_t)0x7fffffff, ((int64_t)(a.Sq - 1) * a.q_ss + D) * 2);
  const int dbytes = (int)min((int64_t)0x7fffffff, ((int64_t)(a.Sq - 1) * a.do_ss + D) * 2);
  const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc((void*)Q, (short)0, qbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rdo = __builtin_amdgcn_make_buffer_rsrc((void*)dO, (short)0, dbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rl =
      __builtin_amdgcn_make_buffer_rsrc((void*)(a.lse2 + (int64_t)bh * a.Sq), (short)0, a.Sq * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rdl = __builtin_amdgcn_make_buffer_rsrc((void*)DL, (short)0, a.Sq * 4, 0x00020000);
  const bool chain = CHAIN || nkb == 1;
  float* dq_part = a.dq_acc + (int64_t)(chain ? 0 : kblk) * a.B * a.H * a.Sq * D + (int64_t)bh * a.Sq * D;
  bf16_t* dQb = a.dq + (int64_t)b * a.dq_sb + (int64_t)hh * a.dq_sh;

  bf16x8 kf[D / 16], vf[D / 16];
  {
    TileStage<D, KB, NT> sk, sv;
    sk.load(K, a.k_ss, kb0, MASK ? a.Sk : 1 << 30, tid);
    sv.load(V, a.v_ss, kb0, MASK ? a.Sk : 1 << 30, tid);
    sk.store(k_l, tid);
    sv.store(smem, tid);
  }
  __syncthreads();
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    const int row = wave * 32 + (lane & 31);
    kf[s] = *reinterpret_cast<const bf16x8*>(k_l + aoff<D>(row, 16 * s + 8 * h));
    vf[s] = *reinterpret_cast<const bf16x8*>(smem + aoff<D>(row, 16 * s + 8 * h));
  }
  f32x16 dk[D / 32], dv[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) { dk[i] = f32x16{}; dv[i] = f32x16{}; }

  const int qt_begin = (MASK && a.causal) ? kb0 / QT : 0;
  const int nqt = (a.Sq + QT - 1) / QT;
  const int G = lane >> 4, qi = (lane & 15) >> 2, pi = lane & 3, l16 = lane & 15;
  auto dma_rows = [&](int t) {
    char* tb = smem + (t & 1) * TILE;
    dma_tile<D, NW>(rq, tb, a.q_ss, t * QT, wave, lane);
    dma_tile<D, NW>(rdo, tb + QB, a.do_ss, t * QT, wave, lane);
    if (wave == NW - 1) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rl, (lds_ptr_t)(tb + 2 * QB), 4, (t * QT + lane) * 4, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rdl, (lds_ptr_t)(tb + 2 * QB + QT * 4), 4, (t * QT + lane) * 4, 0, 0, 0);
    }
  };
  __syncthreads();  // every wave has its V fragments: the tile buffers can be overwritten
  if (qt_begin < nqt) {
    dma_rows(qt_begin);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();

  // dQ^T mapping: rows d0 .. d0+15, query columns q0 + {0..15, 16..31} of the tile
  const int dq_d0 = 16 * (wave & 3), dq_q0 = 32 * (wave >> 2);
  f32x4 dqa[2];
  float4 prevq[2];
  // one iteration: S / dP / dV / dK of tile t (s_tile), dQ of tile t-1 (dq_tile); the first and
  // last iterations are peeled so that the steady-state body is one basic block in which the
  // scheduler can interleave the two independent halves
  auto prefetch = [&](int t) {  // the previous launch's running sum of tile t-1's dQ
    const int pq = (t - 1) * QT;
    if (chain && kblk > 0) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int q = pq + dq_q0 + 16 * j + l16;
        if (!MASK || q < a.Sq) prevq[j] = *reinterpret_cast<const float4*>(dq_part + (int64_t)q * D + dq_d0 + 4 * G);
      }
        }
  };
  // hook(stage): stage 2 qt after the S / dP MFMAs, 2 qt + 1 after the dV / dK MFMAs of half qt
  auto s_tile = [&](int t, auto hook) {
    const int qbase = t * QT;
    const char* tb = smem + (t & 1) * TILE;
    const char* q_l = tb;
    const char* do_l = tb + QB;
    const float* lse_l = reinterpret_cast<const float*>(tb + 2 * QB);
    const float* dl_l = lse_l + QT;
    char* ds_l = ds0 + (t & 1) * DS;
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      f32x16 sacc = f32x16{}, pacc = f32x16{};
#pragma unroll
      for (int s = 0; s < D / 16; ++s) {
        const int row = 32 * qt + (lane & 31);
        const bf16x8 qa = *reinterpret_cast<const bf16x8*>(q_l + aoff<D>(row, 16 * s + 8 * h));
        const bf16x8 da = *reinterpret_cast<const bf16x8*>(do_l + aoff<D>(row, 16 * s + 8 * h));
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kf[s], sacc, 0, 0, 0);
        pacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, vf[s], pacc, 0, 0, 0);
      }
      // stagger (a.stagger): waves w and w + 4 share a SIMD and would otherwise reach the
      // softmax VALU together; waves 4-7 run the dQ chunk after it instead, so one wave of each
      // pair issues MFMAs while its partner runs the exp / dS arithmetic (MI355X_MICROARCH.md,
      // 'Two waves per SIMD', item 9)
      if (!late) hook(2 * qt);
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const float4 L4 = *reinterpret_cast<const float4*>(lse_l + 32 * qt + 8 * g4 + 4 * h);
        const float lv[4] = {L4.x, L4.y, L4.z, L4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) sacc[4 * g4 + j] = fast_exp2(sacc[4 * g4 + j] * sl2 - lv[j]);
      }
      if (MASK) {
        const bool need = (kb0 + wave * 32 + 31 >= a.Sk) || (a.causal && kb0 + wave * 32 + 31 > qbase + 32 * qt);
        if (need) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int q = qbase + 32 * qt + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (key >= a.Sk || (a.causal && key > q)) sacc[r] = 0.f;
          }
        }
      }
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const float4 D4 = *reinterpret_cast<const float4*>(dl_l + 32 * qt + 8 * g4 + 4 * h);
        const float dv4[4] = {D4.x, D4.y, D4.z, D4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) pacc[4 * g4 + j] = sacc[4 * g4 + j] * (pacc[4 * g4 + j] - dv4[j]);
      }
      const bf16x8 pb0 = pack8(sacc, 0), pb1 = pack8(sacc, 8);
      const bf16x8 sb0 = pack8(pacc, 0), sb1 = pack8(pacc, 8);
      if (late) hook(2 * qt);
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) {
        const int col = dt * 32 + 16 * (G & 1) + 4 * pi;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int r0 = 32 * qt + 16 * s2 + 4 * h + qi;
          const bf16x8 ao = cat8(tr_read(do_l, aoff<D>(r0, col)), tr_read(do_l, aoff<D>(r0 + 8, col)));
          const bf16x8 aq = cat8(tr_read(q_l, aoff<D>(r0, col)), tr_read(q_l, aoff<D>(r0 + 8, col)));
          dv[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ao, s2 ? pb1 : pb0, dv[dt], 0, 0, 0);
          dk[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aq, s2 ? sb1 : sb0, dk[dt], 0, 0, 0);
        }
      }
      hook(2 * qt + 1);
      const int krow = wave * 32 + (lane & 31);
      const bf16x4 parts[4] = {sb0.lo, sb0.hi, sb1.lo, sb1.hi};
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<bf16x4*>(ds_l + dst_off(krow, 32 * qt + 8 * g + 4 * h)) = parts[g];
    }
  };
  // dQ^T (16 d x 16 queries, two tiles) = K^T . dS^T of tile t-1 over key slices [32 k0, 32 k1)
  auto dq_chunk = [&](int t, int k0, int k1) {
    const char* dsl = ds0 + ((t - 1) & 1) * DS;
    if (k0 == 0) dqa[0] = dqa[1] = f32x4{};
#pragma unroll
    for (int ks = k0; ks < k1; ++ks) {
      const int kr = 32 * ks + 8 * G + qi;
      const bf16x8 ka = cat8(tr_read(k_l, aoff<D>(kr, dq_d0 + 4 * pi)), tr_read(k_l, aoff<D>(kr + 4, dq_d0 + 4 * pi)));
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int cq = dq_q0 + 16 * j + 4 * pi;
        const bf16x8 sbq = cat8(tr_read(dsl, dst_off(kr, cq)), tr_read(dsl, dst_off(kr + 4, cq)));
        dqa[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, sbq, dqa[j], 0, 0, 0);
      }
    }
  };
  auto dq_tile = [&](int t) { dq_chunk(t, 0, KB / 32); };
  // dbp (fused QKV-bias gradient, non-causal chain): column sums of the final dQ (last pass) and of
  // this block's dK / dV, as partials [B*H][2][D] (dQ, per query half of the waves) and
  // [nkb][B*H][D] (dK, dV) that attn_bias_fold adds into the bias gradient
  const bool bsum = a.dbp != nullptr;
  float dqs[4] = {0.f, 0.f, 0.f, 0.f};
  auto dq_store = [&](int t) {  // after the barrier: vmcnt counts stores, the next wait is a tile away
    const int pq = (t - 1) * QT;
    int last = nkb - 1;
    if (MASK && a.causal) last = min(last, (pq + QT - 1) / KB);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int q = pq + dq_q0 + 16 * j + l16;
      if (!MASK || q < a.Sq) {
        f32x4 acc = dqa[j];
        if (chain && kblk > 0) {
          acc[0] += prevq[j].x; acc[1] += prevq[j].y; acc[2] += prevq[j].z; acc[3] += prevq[j].w;
        }
        if (chain && kblk == last) {
          const unsigned w0 = pack_bf2(acc[0] * a.scale, acc[1] * a.scale), w1 = pack_bf2(acc[2] * a.scale, acc[3] * a.scale);
          *reinterpret_cast<uint2*>(dQb + (int64_t)q * a.dq_ss + dq_d0 + 4 * G) = make_uint2(w0, w1);
          if (bsum) {  // the bias gradient sums the stored (bf16) dQ, as the unfused column sum would
            dqs[0] += __uint_as_float(w0 << 16); dqs[1] += __uint_as_float(w0 & 0xffff0000u);
            dqs[2] += __uint_as_float(w1 << 16); dqs[3] += __uint_as_float(w1 & 0xffff0000u);
          }
        } else {
          *reinterpret_cast<float4*>(dq_part + (int64_t)q * D + dq_d0 + 4 * G) = make_float4(acc[0], acc[1], acc[2], acc[3]);
        }
      }
    }
  };
  auto finish = [&]() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile t+1 landed; older dQ stores done
    lds_barrier();
  };
  if (qt_begin < nqt) {
    if (qt_begin + 1 < nqt) dma_rows(qt_begin + 1);
    s_tile(qt_begin, [](int) {});
    finish();
    for (int t = qt_begin + 1; t < nqt; ++t) {
      if (t + 1 < nqt) dma_rows(t + 1);  // buffer (t+1)&1: read during iteration t-1, before its barrier
      prefetch(t);
      // tile t-1's dQ in four key-slice chunks between the S / dP and dV / dK stages of tile t
      s_tile(t, [&](int st) {
        if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
        dq_chunk(t, 2 * st, 2 * st + 2);
        if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
      });
      finish();
      dq_store(t);
    }
    prefetch(nqt);
    dq_tile(nqt);
    finish();
    dq_store(nqt);
  }
  if (MASK && a.causal && !chain) {
    for (int64_t i = tid; i < (int64_t)min(qt_begin * QT, a.Sq) * D; i += NT) dq_part[i] = 0.f;
  }
  if (bsum && kblk == nkb - 1) {  // dQ column sums: over the 16 query lanes of each d quad
#pragma unroll
    for (int off = 1; off < 16; off <<= 1)
#pragma unroll
      for (int i = 0; i < 4; ++i) dqs[i] += __shfl_xor(dqs[i], off, 64);
    if (l16 == 0)
      *reinterpret_cast<float4*>(a.dbp + ((int64_t)bh * 2 + (wave >> 2)) * D + dq_d0 + 4 * G) =
          make_float4(dqs[0], dqs[1], dqs[2], dqs[3]);
  }
  if (qt_begin >= nqt) __syncthreads();
  {
    char* dv_l = smem;
    const int row = wave * 32 + (lane & 31);
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 4 * dt + g;
        const int off = row * (D * 2) + ((c ^ (row & 7)) << 4) + 8 * h;
        *reinterpret_cast<uint2*>(k_l + off) = make_uint2(pack_bf2(dk[dt][4 * g] * a.scale, dk[dt][4 * g + 1] * a.scale),
                                                          pack_bf2(dk[dt][4 * g + 2] * a.scale, dk[dt][4 * g + 3] * a.scale));
        *reinterpret_cast<uint2*>(dv_l + off) = make_uint2(pack_bf2(dv[dt][4 * g], dv[dt][4 * g + 1]),
                                                           pack_bf2(dv[dt][4 * g + 2], dv[dt][4 * g + 3]));
      }
    }
    lds_barrier();
    bf16_t* dKb = a.dk + (int64_t)b * a.dk_sb + (int64_t)hh * a.dk_sh;
    bf16_t* dVb = a.dv + (int64_t)b * a.dv_sb + (int64_t)hh * a.dv_sh;
    constexpr int CPR = D / 8;
    static_assert(NT % CPR == 0, "a thread's chunk column is fixed");
    float sk[8] = {}, sv[8] = {};
#pragma unroll
    for (int i = 0; i < KB * CPR / NT; ++i) {
      const int id = tid + i * NT, r = id / CPR, c = id % CPR;
      const int off = r * (D * 2) + ((c ^ (r & 7)) << 4);
      if (!MASK || kb0 + r < a.Sk) {
        const uint4 kv4 = *reinterpret_cast<const uint4*>(k_l + off);
        const uint4 vv4 = *reinterpret_cast<const uint4*>(dv_l + off);
        *reinterpret_cast<uint4*>(dKb + (int64_t)(kb0 + r) * a.dk_ss + 8 * c) = kv4;
        *reinterpret_cast<uint4*>(dVb + (int64_t)(kb0 + r) * a.dv_ss + 8 * c) = vv4;
        if (bsum) {
          const unsigned kw[4] = {kv4.x, kv4.y, kv4.z, kv4.w}, vw[4] = {vv4.x, vv4.y, vv4.z, vv4.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            sk[2 * e] += __uint_as_float(kw[e] << 16); sk[2 * e + 1] += __uint_as_float(kw[e] & 0xffff0000u);
            sv[2 * e] += __uint_as_float(vw[e] << 16); sv[2 * e + 1] += __uint_as_float(vw[e] & 0xffff0000u);
          }
        }
      }
    }
    if (bsum) {  // dK / dV column sums: lanes l, l^8, l^16, l^32 share the chunk, then the 8 waves via LDS
#pragma unroll
      for (int off = 8; off < 64; off <<= 1)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          sk[e] += __shfl_xor(sk[e], off, 64);
          sv[e] += __shfl_xor(sv[e], off, 64);
        }
      float* red = reinterpret_cast<float*>(ds0);  // the dS^T images are dead here
      if (lane < CPR) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          red[(wave * CPR + lane) * 8 + e] = sk[e];
          red[NW * CPR * 8 + (wave * CPR + lane) * 8 + e] = sv[e];
        }
      }
      __syncthreads();
      if (tid < 2 * D) {
        const int which = tid / D, d = tid % D;  // d = 8 * chunk + e
        float acc = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) acc += red[which * NW * CPR * 8 + (w * CPR + d / 8) * 8 + d % 8];
        float* part = a.dbp + (int64_t)a.B * a.H * 2 * D + (int64_t)which * nkb * a.B * a.H * D;
        part[((int64_t)kblk * a.B * a.H + bh) * D + d] = acc;
      }
    }
  }
}

// db[which][h][d] += the partials of attn_bwd1b_kernel: dQ over (batch, query half), dK / dV over
// (key block, batch) — the fused QKV projection's bias gradient in its [3][H][D] layout. One
// workgroup per (which, head): 1024 / D groups of D threads each sum a few of the partial rows
// (coalesced D-float rows, independent loads), then fold through LDS (one thread per output
// looping over all rows was latency-bound: 21 us per call; 4 groups per head still 9 us).
__global__ void __launch_bounds__(1024) attn_bias_fold_kernel(const float* __restrict__ part, float* __restrict__ db,
                                                              int B, int H, int D, int nkb) {
  __shared__ float red[1024];
  const int which = blockIdx.x / H, h = blockIdx.x % H;
  const int d = threadIdx.x % D, grp = threadIdx.x / D, ngrp = blockDim.x / D;
  float s = 0.f;
  if (grp < ngrp) {
    if (which == 0) {  // rows (b, x): part[((b*H + h)*2 + x)*D + d]
      for (int r = grp; r < 2 * B; r += ngrp) s += part[((int64_t)((r >> 1) * H + h) * 2 + (r & 1)) * D + d];
    } else {  // rows (kb, b): p[((kb*B + b)*H + h)*D + d]
      const float* p = part + (int64_t)B * H * 2 * D + (int64_t)(which - 1) * nkb * B * H * D;
      for (int r = grp; r < nkb * B; r += ngrp) s += p[((int64_t)r * H + h) * D + d];
    }
  }
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x < D) {
    float t = 0.f;
    for (int g = 0; g < ngrp; ++g) t += red[g * D + threadIdx.x];
    db[((int64_t)which * H + h) * D + threadIdx.x] += t;
  }
}

// dq[q][d] = scale * sum_kb dq_part[kb][bh][q][d]
template <int D>
__global__ void attn_dq_finish_kernel(AttnArgs a, int nkb) {
  const int64_t per = (int64_t)a.B * a.H * a.Sq * D;
  const int64_t nv = per / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    float4 s = reinterpret_cast<const float4*>(a.dq_acc)[i];
    for (int kb = 1; kb < nkb; ++kb) {
      const float4 t = reinterpret_cast<const float4*>(a.dq_acc + kb * per)[i];
      s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
    }
    const int64_t e = i * 4;
    const int d = e % D;
    const int64_t q = (e / D) % a.Sq;
    const int64_t bh = e / ((int64_t)D * a.Sq);
    const int b = bh / a.H, hh = bh % a.H;
    bf16_t* dst = a.dq + (int64_t)b * a.dq_sb + (int64_t)hh * a.dq_sh + q * a.dq_ss + d;
    ushort4 o;
    o.x = f2bf(s.x * a.scale); o.y = f2bf(s.y * a.scale); o.z = f2bf(s.z * a.scale); o.w = f2bf(s.w * a.scale);
    *reinterpret_cast<ushort4*>(dst) = o;
  }
}

// Backward variant: 10 (default) = attn_bwd1b_kernel (one barrier per query tile, fenced dQ
// chunks, LDS-DMA tiles) chained per key block when B*H workgroups fill the chip (>= 256), else
// attn_bwd_kernel with LDS-DMA Q / dO tiles (one launch with per-key-block dQ slabs + finishing
// pass); 2 = attn_bwd_kernel without DMA (also what every variant falls back to without 16-B
// aligned Q / dO rows; D = 128 always takes it with 4 waves). B32 H16 S512 D64: 2 / 10 = 161 / 151 us
// (profiles/attn_bwd_r5.txt). Round 6 removed the structures measured slower (4-wave slabs and
// 4-wave chained, the one-wave-per-SIMD key-group kernel, the unfenced and the slab forms of
// attn_bwd1b_kernel); rounds 1-5 measurements: docs/PERFORMANCE.md. Settable for A/B runs in one
// process (attn_set_bwd_variant); default from FF_ATTN_BWD; other values mean 10.
static int g_bwd_variant = -1;
int attn_bwd_variant() {
  if (g_bwd_variant < 0) {
    const char* e = getenv("FF_ATTN_BWD");
    g_bwd_variant = (e && atoi(e) == 2) ? 2 : 10;
  }
  return g_bwd_variant;
}
void attn_set_bwd_variant(int v) { g_bwd_variant = v == 2 ? 2 : 10; }

// keys per backward workgroup
static int bwd_keys(int D) { return D == 64 ? 256 : 128; }

int64_t attn_bwd_slab_floats(int B, int H, int Sq, int Sk, int D) {
  const int nkb = (Sk + bwd_keys(D) - 1) / bwd_keys(D);
  return (int64_t)nkb * B * H * Sq * D;
}

int64_t attn_bwd_workspace_floats(int B, int H, int Sq, int Sk, int D) {
  const int nkb = (Sk + bwd_keys(D) - 1) / bwd_keys(D);
  // slabs, delta, lse2, bias-gradient partials (attn_bwd1b_kernel)
  return (int64_t)nkb * B * H * Sq * D + 2 * (int64_t)B * H * Sq + (int64_t)B * H * D * (2 + 2 * nkb);
}

// Forward structure: 3 (default) = 64 rows per wave (attn_fwd2_kernel; D = 64 and Sq >= 512, else
// 1), 1 = 4 waves with LDS-DMA K/V staging, 0 = 4 waves through registers (also the fallback
// without 16-B aligned K / V rows, and D = 128). All three run the same per-row arithmetic (bitwise
// equal outputs). Removed in round 6 as measured slower: the persistent 64-rows-per-wave kernel
// and the 8-wave ping-pong (profiles/attn_fwd_variants_r4.txt, attn_fwd_pingpong_r4.txt).
// attn_set_fwd_variant; default from FF_ATTN_FWD; other values mean 3.
static int g_fwd_variant = -1;
int attn_fwd_variant() {
  if (g_fwd_variant < 0) {
    const char* e = getenv("FF_ATTN_FWD");
    const int v = e ? atoi(e) : 3;
    g_fwd_variant = (v == 0 || v == 1) ? v : 3;
  }
  return g_fwd_variant;
}
void attn_set_fwd_variant(int v) { g_fwd_variant = (v == 0 || v == 1) ? v : 3; }

// Deferred-max threshold of the forward (log2 units; 0 = rescale whenever a row max grows, the
// textbook online softmax). Default 8 (P <= 256 in bf16 between rescales), FF_ATTN_RESCALE_THR.
static float g_rescale_thr = -1.f;
float attn_rescale_thr() {
  if (g_rescale_thr < 0.f) {
    const char* e = getenv("FF_ATTN_RESCALE_THR");
    g_rescale_thr = e ? fmaxf(0.f, (float)atof(e)) : 8.f;
  }
  return g_rescale_thr;
}
void attn_set_rescale_thr(float t) { g_rescale_thr = fmaxf(0.f, t); }

// attn_bwd1b_kernel wave stagger (AttnArgs.stagger): FF_ATTN_STAGGER, attn_set_stagger (A/B)
static int g_stagger = -1;
int attn_stagger() {
  if (g_stagger < 0) {
    const char* e = getenv("FF_ATTN_STAGGER");
    g_stagger = e ? (atoi(e) != 0) : 0;
  }
  return g_stagger;
}
void attn_set_stagger(int v) { g_stagger = v != 0; }

void attn_fwd(AttnArgs a, hipStream_t st) {
  const dim3 grid((unsigned)((a.Sq + 127) / 128 * a.B * a.H));
  const bool mask = a.causal || a.Sk % 64 != 0;
  a.rescale_thr = attn_rescale_thr();
  // the DMA path needs 16-B aligned K / V rows and buffer offsets below 2 GiB
  const bool dma_ok = ((uintptr_t)a.k & 15) == 0 && ((uintptr_t)a.v & 15) == 0 && a.k_ss % 8 == 0 &&
                      a.v_ss % 8 == 0 && (int64_t)(a.Sk + 64) * a.k_ss * 2 < 0x7fffffffLL &&
                      (int64_t)(a.Sk + 64) * a.v_ss * 2 < 0x7fffffffLL;
  const bool dma = attn_fwd_variant() >= 1 && dma_ok;
  // 64 query rows per wave (attn_fwd2_kernel): 2-6 % faster from S = 512 up, slower at S = 256
  // (half the workgroups), profiles/attn_fwd_variants_r4.txt
  if (attn_fwd_variant() == 3 && dma_ok && a.D == 64 && a.Sq >= 512) {
    const dim3 g3((unsigned)((a.Sq + 255) / 256 * a.B * a.H));
    if (mask) hipLaunchKernelGGL((attn_fwd2_kernel<true>), g3, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((attn_fwd2_kernel<false>), g3, dim3(256), 0, st, a);
    return;
  }
  if (a.D == 64) {
    if (dma) {
      if (mask) hipLaunchKernelGGL((attn_fwd_kernel<64, true, true>), grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((attn_fwd_kernel<64, false, true>), grid, dim3(256), 0, st, a);
    } else {
      if (mask) hipLaunchKernelGGL((attn_fwd_kernel<64, true, false>), grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((attn_fwd_kernel<64, false, false>), grid, dim3(256), 0, st, a);
    }
  } else if (a.D == 128) {
    if (mask) hipLaunchKernelGGL((attn_fwd_kernel<128, true, false>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((attn_fwd_kernel<128, false, false>), grid, dim3(256), 0, st, a);
  }
}

template <int D, int NW, bool DMA = false>
static void launch_bwd_main(AttnArgs a, int nkb, bool chain, hipStream_t st) {
  const bool mask = a.causal || a.Sk % (32 * NW) != 0 || a.Sq % 64 != 0;
  const int bh = a.B * a.H;
  if (chain) {
    for (int p = 0; p < nkb; ++p) {
      if (mask) hipLaunchKernelGGL((attn_bwd_kernel<D, NW, true, true, DMA>), dim3(bh), dim3(64 * NW), 0, st, a, nkb, p);
      else hipLaunchKernelGGL((attn_bwd_kernel<D, NW, false, true, DMA>), dim3(bh), dim3(64 * NW), 0, st, a, nkb, p);
    }
  } else {
    if (mask) hipLaunchKernelGGL((attn_bwd_kernel<D, NW, true, false, DMA>), dim3(bh * nkb), dim3(64 * NW), 0, st, a, nkb, 0);
    else hipLaunchKernelGGL((attn_bwd_kernel<D, NW, false, false, DMA>), dim3(bh * nkb), dim3(64 * NW), 0, st, a, nkb, 0);
  }
}

bool attn_bwd(AttnArgs a, hipStream_t st) {
  bool bias_done = false;
  a.stagger = attn_stagger();
  const int v = attn_bwd_variant();
  const int nkb = (a.Sk + bwd_keys(a.D) - 1) / bwd_keys(a.D);
  const int64_t rows = (int64_t)a.B * a.H * a.Sq;
  const dim3 gpre((unsigned)((rows * (a.D / 8) + 255) / 256));
  const int64_t per = (int64_t)a.B * a.H * a.Sq * a.D;
  const dim3 gfin(ew_grid(per / 4, 256));
  // chained launches (one per key block, the fp32 dQ sum carried between them) once B*H
  // workgroups fill the chip; every attn_bwd_kernel launch with a single key block writes the
  // final dQ itself, so only the slab form with several key blocks needs the finishing pass
  const bool chain = a.B * a.H >= 256;
  const bool finish = !chain && nkb > 1;
  // the DMA paths need 16-B aligned Q / dO rows and buffer offsets below 2 GiB
  const bool dma_ok = v == 10 && ((uintptr_t)a.q & 15) == 0 && ((uintptr_t)a.dout & 15) == 0 && a.q_ss % 8 == 0 &&
                      a.do_ss % 8 == 0 && (int64_t)(a.Sq + 64) * a.q_ss * 2 < 0x7fffffffLL &&
                      (int64_t)(a.Sq + 64) * a.do_ss * 2 < 0x7fffffffLL;
  if (a.D == 64) {
    hipLaunchKernelGGL(attn_bwd_pre_kernel<64>, gpre, dim3(256), 0, st, a);
    if (chain && dma_ok) {
      const bool m = a.causal || a.Sk % 256 != 0 || a.Sq % 64 != 0;
      const int bh = a.B * a.H;
      // fused bias-gradient sums: non-causal (every query tile's last key block is the last launch)
      if (a.causal) a.dbp = nullptr;
      bias_done = a.dbp != nullptr;
      for (int p = 0; p < nkb; ++p) {
        if (m) hipLaunchKernelGGL((attn_bwd1b_kernel<true, true>), dim3(bh), dim3(512), 0, st, a, nkb, p);
        else hipLaunchKernelGGL((attn_bwd1b_kernel<false, true, true>), dim3(bh), dim3(512), 0, st, a, nkb, p);
      }
    } else if (dma_ok) {
      launch_bwd_main<64, 8, true>(a, nkb, chain, st);
    } else {
      launch_bwd_main<64, 8>(a, nkb, chain, st);
    }
    if (finish) hipLaunchKernelGGL(attn_dq_finish_kernel<64>, gfin, dim3(256), 0, st, a, nkb);
  } else if (a.D == 128) {
    hipLaunchKernelGGL(attn_bwd_pre_kernel<128>, gpre, dim3(256), 0, st, a);
    launch_bwd_main<128, 4>(a, nkb, chain, st);
    if (finish) hipLaunchKernelGGL(attn_dq_finish_kernel<128>, gfin, dim3(256), 0, st, a, nkb);
  }
  if (bias_done)
    hipLaunchKernelGGL(attn_bias_fold_kernel, dim3((unsigned)(3 * a.H)), dim3(1024), 0, st, a.dbp, a.dbias, a.B, a.H,
                       a.D, nkb);
  return bias_done;
}

}  // namespace ffk

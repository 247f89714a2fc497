// Attention-backward lab: prices the parts of the main backward kernel by switching them off one
// at a time (knob bits), and hosts candidate restructurings next to the production kernel.
// Standalone executable (no torch): production attn_fwd / attn_bwd (csrc/kernels/attention.hip)
// provide O, lse, delta and the reference dQ/dK/dV; every lab variant is timed with hip events in
// interleaved rounds and diffed against the reference.
//   build: scripts/lab/build_lab.sh   run: scripts/lab/attn_bwd_lab [B H S]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "attention.h"
#include "common.h"

namespace lab {
using namespace ffk;

constexpr float LOG2E = 1.4426950408889634f;

template <int D>
__device__ __forceinline__ int aswz(int row) {
  if (D == 64) return (((row >> 1) & 1) << 2) | ((row >> 3) & 1) | (((row >> 4) & 1) << 1);
  else return ((row & 3) << 2) | ((row >> 2) & 3);
}
template <int D>
__device__ __forceinline__ int aoff(int row, int col) {
  const int ch = col >> 3;
  return row * (D * 2) + ((ch ^ aswz<D>(row)) << 4) + ((col & 7) << 1);
}
typedef short v4s __attribute__((ext_vector_type(4)));
__device__ __forceinline__ bf16x4 tr_read(const char* lds, int off) {
  v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(lds + off));
  return __builtin_bit_cast(bf16x4, v);
}
__device__ __forceinline__ bf16x8 cat8(bf16x4 lo, bf16x4 hi) {
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
template <int D, int ROWS, int NTH>
struct TileStage {
  static constexpr int CH = ROWS * D / 8 / NTH;
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
__device__ __forceinline__ bf16x8 pack8(const f32x16& a, int base) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (__bf16)a[base + j];
  return o;
}
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ int dst_off(int row, int q) {
  const int f = (row & 7) | ((((row >> 1) ^ (row >> 3)) & 1) << 3);
  return row * 128 + (((q >> 2) ^ f) << 3) + (q & 3) * 2;
}

enum : int { K_NO_DQ = 1, K_NO_DQ_STORE = 2, K_NO_EXP = 4, K_NO_PREFETCH = 8, K_NO_DKDV = 16, K_NO_DS_WRITE = 32,
             // candidate changes
             K_DQT = 64,     // dQ^T = K^T . dS^T (swapped operands): lane = query, 4 float4 stores per tile
             K_SBW = 128,    // dS^T image written from the packed bf16 dS (no second conversion)
             K_PRIO = 256,   // s_setprio 1 for the second half of the waves
             K_DQ4 = 512,
             K_NO_EPI = 1024,     // dK/dV stores skipped (epilogue price)
             K_WIDE_EPI = 2048,   // dK/dV as 16-B stores after a permlane32 swap of the h halves
             K_ONE_TILE = 4096,   // one query tile per workgroup (fixed per-workgroup cost)
             K_LDS_EPI = 8192,    // dK/dV staged through LDS, stored as whole 128-B rows (16 B/lane)
             K_LDS_PRO = 16384,   // K and V blocks loaded row-coalesced into LDS, fragments read from LDS
             K_XCD = 32768 };     // 1-D grid through xcd_remap: the key blocks of one (b, h) share an XCD

__device__ __forceinline__ unsigned pk2(float x, float y) {
  return (unsigned)f2bf(x) | ((unsigned)f2bf(y) << 16);
}
// acc: lane = key row (lane & 31), d = 32 dt + 8 g + 4 h + (0..3); 16-B stores of 8 consecutive d
__device__ __forceinline__ void store_wide(bf16_t* row, const f32x16& acc, float sc, int dt, int h) {
  unsigned dw[4][2];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    dw[g][0] = pk2(acc[4 * g] * sc, acc[4 * g + 1] * sc);
    dw[g][1] = pk2(acc[4 * g + 2] * sc, acc[4 * g + 3] * sc);
  }
#pragma unroll
  for (int gp = 0; gp < 2; ++gp) {
    const auto r0 = __builtin_amdgcn_permlane32_swap(dw[2 * gp][0], dw[2 * gp + 1][0], false, false);
    const auto r1 = __builtin_amdgcn_permlane32_swap(dw[2 * gp][1], dw[2 * gp + 1][1], false, false);
    *reinterpret_cast<uint4*>(row + 32 * dt + 8 * (2 * gp + h)) = make_uint4(r0[0], r1[0], r0[1], r1[1]);
  }
}  // dQ stage on waves 0..NTILE-1 only, full key range each, no LDS hand-off

// Copy of production attn_bwd_kernel<64, 8> (non-causal) with knob bits.
template <int D, int NW, int KN>
__global__ void __launch_bounds__(64 * NW, 8 / NW) bwd_knob(AttnArgs a) {
  constexpr int NT = 64 * NW, QT = 64, KB = 32 * NW, QB = QT * D * 2;
  constexpr int TILE = 2 * QB + 2 * QT * 4;
  constexpr int NTILE = 2 * (D / 32);
  constexpr int KSPLIT = NW > NTILE ? NW / NTILE : 1;
  constexpr int DQX = KSPLIT > 1 ? NTILE * (KSPLIT - 1) * 32 * 32 * 4 : 0;
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE + KB * D * 2 + KB * QT * 2 + DQX];
  char* k_l = smem + 2 * TILE;
  char* ds_l = k_l + KB * D * 2;
  float* dqx_l = reinterpret_cast<float*>(ds_l + KB * QT * 2);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int nkb = a.Sk / KB;
  const int lid = (KN & K_XCD) ? xcd_remap(blockIdx.x, nkb * a.B * a.H) : 0;
  const int bh = (KN & K_XCD) ? lid / nkb : blockIdx.y, b = bh / a.H, hh = bh % a.H;
  const int kblk = (KN & K_XCD) ? lid % nkb : blockIdx.x;
  const int kb0 = kblk * KB;
  const int key = kb0 + wave * 32 + (lane & 31);
  const bf16_t* Q = a.q + (int64_t)b * a.q_sb + (int64_t)hh * a.q_sh;
  const bf16_t* K = a.k + (int64_t)b * a.k_sb + (int64_t)hh * a.k_sh;
  const bf16_t* V = a.v + (int64_t)b * a.v_sb + (int64_t)hh * a.v_sh;
  const bf16_t* dO = a.dout + (int64_t)b * a.do_sb + (int64_t)hh * a.do_sh;
  const float* LSE = a.lse + (int64_t)bh * a.Sq;
  const float* DL = a.delta + (int64_t)bh * a.Sq;
  const float sl2 = a.scale * LOG2E;
  if ((KN & K_PRIO) && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  bf16x8 kf[D / 16], vf[D / 16];
  if (KN & K_LDS_PRO) {
    {
      TileStage<D, KB, NT> st, sv;
      st.load(K, a.k_ss, kb0, a.Sk, tid);
      sv.load(V, a.v_ss, kb0, a.Sk, tid);
      st.store(k_l, tid);
      sv.store(ds_l, tid);
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      const int row = wave * 32 + (lane & 31);
      kf[s] = *reinterpret_cast<const bf16x8*>(k_l + aoff<D>(row, 16 * s + 8 * h));
      vf[s] = *reinterpret_cast<const bf16x8*>(ds_l + aoff<D>(row, 16 * s + 8 * h));
    }
  } else {
    {
      TileStage<D, KB, NT> st;
      st.load(K, a.k_ss, kb0, a.Sk, tid);
      st.store(k_l, tid);
    }
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      kf[s] = *reinterpret_cast<const bf16x8*>(K + (int64_t)key * a.k_ss + 16 * s + 8 * h);
      vf[s] = *reinterpret_cast<const bf16x8*>(V + (int64_t)key * a.v_ss + 16 * s + 8 * h);
    }
  }
  f32x16 dk[D / 32], dv[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) { dk[i] = f32x16{}; dv[i] = f32x16{}; }
  const int nqt = (KN & K_ONE_TILE) ? 1 : (a.Sq + QT - 1) / QT;
  const int G = lane >> 4, qi = (lane & 15) >> 2, pi = lane & 3;
  float* dq_part = a.dq_acc + (int64_t)kblk * a.B * a.H * a.Sq * D + (int64_t)bh * a.Sq * D;
  TileStage<D, QT, NT> sq, sd;
  float lse_r = INFINITY, dl_r = 0.f;
  auto fetch = [&](int t) {
    const int qbase = t * QT;
    sq.load(Q, a.q_ss, qbase, a.Sq, tid);
    sd.load(dO, a.do_ss, qbase, a.Sq, tid);
    if (tid < QT) {
      lse_r = LSE[qbase + tid] * LOG2E;
      dl_r = DL[qbase + tid];
    }
  };
  auto stash = [&](int t) {
    char* tb = smem + (t & 1) * TILE;
    sq.store(tb, tid);
    sd.store(tb + QB, tid);
    if (tid < QT) {
      reinterpret_cast<float*>(tb + 2 * QB)[tid] = lse_r;
      reinterpret_cast<float*>(tb + 2 * QB)[QT + tid] = dl_r;
    }
  };
  fetch(0);
  stash(0);
  if (KN & K_NO_PREFETCH) stash(1);
  __syncthreads();
  for (int t = 0; t < nqt; ++t) {
    const int qbase = t * QT;
    char* tb = smem + (t & 1) * TILE;
    const char* q_l = tb;
    const char* do_l = tb + QB;
    const float* lse_l = reinterpret_cast<const float*>(tb + 2 * QB);
    const float* dl_l = lse_l + QT;
    const bool more = t + 1 < nqt;
    if (!(KN & K_NO_PREFETCH) && more) fetch(t + 1);
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
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int q0l = 32 * qt + 8 * g4 + 4 * h;
        const float4 L4 = *reinterpret_cast<const float4*>(lse_l + q0l);
        const float4 D4 = *reinterpret_cast<const float4*>(dl_l + q0l);
        const float lv[4] = {L4.x, L4.y, L4.z, L4.w}, dv4[4] = {D4.x, D4.y, D4.z, D4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 4 * g4 + j;
          float p = (KN & K_NO_EXP) ? sacc[r] * sl2 - lv[j] : exp2f(sacc[r] * sl2 - lv[j]);
          sacc[r] = p;
          pacc[r] = p * (pacc[r] - dv4[j]);
        }
      }
      const bf16x8 pb0 = pack8(sacc, 0), pb1 = pack8(sacc, 8);
      const bf16x8 sb0 = pack8(pacc, 0), sb1 = pack8(pacc, 8);
      if (!(KN & K_NO_DKDV)) {
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
      } else {
        // keep P / dS live
        dv[0][0] += (float)pb0[0] + (float)pb1[1];
        dk[0][0] += (float)sb0[0] + (float)sb1[1];
      }
      if ((KN & K_SBW) && !(KN & K_NO_DS_WRITE)) {
        const int krow = wave * 32 + (lane & 31);
        typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));
        const bf16x4v parts[4] = {sb0.lo, sb0.hi, sb1.lo, sb1.hi};
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<bf16x4v*>(ds_l + dst_off(krow, 32 * qt + 8 * g + 4 * h)) = parts[g];
      } else if (!(KN & K_NO_DS_WRITE)) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int ql = 32 * qt + 8 * g + 4 * h;
          const int krow = wave * 32 + (lane & 31);
          ushort4 o;
          o.x = f2bf(pacc[4 * g + 0]); o.y = f2bf(pacc[4 * g + 1]);
          o.z = f2bf(pacc[4 * g + 2]); o.w = f2bf(pacc[4 * g + 3]);
          *reinterpret_cast<ushort4*>(ds_l + dst_off(krow, ql)) = o;
        }
      } else {
        dk[1][0] += pacc[0] + pacc[15];
      }
    }
    lds_barrier();
    if (!(KN & K_NO_DQ)) {
      constexpr bool DQ4 = (KN & K_DQ4) != 0;
      constexpr int KSP = DQ4 ? 1 : KSPLIT;
      for (int tile = wave % NTILE; tile < NTILE && (!DQ4 || wave < NTILE); tile += (NW < NTILE ? NW : NTILE)) {
        const int qt = tile / (D / 32), dt = tile % (D / 32);
        const int part = KSP > 1 ? wave / NTILE : 0;
        constexpr int KS_PER = KB / 16 / KSP;
        f32x16 acc = f32x16{};
#pragma unroll
        for (int ks = part * KS_PER; ks < (part + 1) * KS_PER; ++ks) {
          const int cq = 32 * qt + 16 * (G & 1) + 4 * pi;
          const int kr = 16 * ks + 8 * h + qi;
          const bf16x8 af = cat8(tr_read(ds_l, dst_off(kr, cq)), tr_read(ds_l, dst_off(kr + 4, cq)));
          const int cd = 32 * dt + 16 * (G & 1) + 4 * pi;
          const bf16x8 bk = cat8(tr_read(k_l, aoff<D>(kr, cd)), tr_read(k_l, aoff<D>(kr + 4, cd)));
          if (KN & K_DQT) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bk, af, acc, 0, 0, 0);
          else acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bk, acc, 0, 0, 0);
        }
        if constexpr (KSP > 1) {
          float* slot = dqx_l + ((part - 1) * NTILE + tile) * 1024;
          if (part > 0) {
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4)
              *reinterpret_cast<float4*>(slot + (r4 * 64 + lane) * 4) =
                  make_float4(acc[4 * r4], acc[4 * r4 + 1], acc[4 * r4 + 2], acc[4 * r4 + 3]);
          }
          lds_barrier();
          if (part == 0) {
#pragma unroll
            for (int p2 = 1; p2 < KSP; ++p2) {
              const float* o = dqx_l + ((p2 - 1) * NTILE + tile) * 1024;
#pragma unroll
              for (int r4 = 0; r4 < 4; ++r4) {
                const float4 v = *reinterpret_cast<const float4*>(o + (r4 * 64 + lane) * 4);
                acc[4 * r4] += v.x; acc[4 * r4 + 1] += v.y; acc[4 * r4 + 2] += v.z; acc[4 * r4 + 3] += v.w;
              }
            }
          }
        }
        if (part == 0) {
          const bool st = !(KN & K_NO_DQ_STORE) || a.causal == 12345;
          if (st && (KN & K_DQT)) {
            // acc: lane = query (lane & 31), rows = d (r&3) + 8(r>>2) + 4h -> 4 consecutive d per float4
            const int q = qbase + 32 * qt + (lane & 31);
#pragma unroll
            for (int g = 0; g < 4; ++g)
              *reinterpret_cast<float4*>(dq_part + (int64_t)q * D + 32 * dt + 8 * g + 4 * h) =
                  make_float4(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]);
          } else if (st) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int q = qbase + 32 * qt + (r & 3) + 8 * (r >> 2) + 4 * h;
              const int d = 32 * dt + (lane & 31);
              dq_part[(int64_t)q * D + d] = acc[r];
            }
          }
        }
      }
    }
    if (!(KN & K_NO_PREFETCH) && more) stash(t + 1);
    lds_barrier();
  }
  if (KN & K_LDS_EPI) {
    // [KB][D] bf16 images of dK (K block region) and dV (dS^T region), 16-B chunks XOR-swizzled
    // by row & 7; the loop's last barrier has retired every read of both regions
    char* dk_l = k_l;
    char* dv_l = ds_l;
    const int row = wave * 32 + (lane & 31);
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 4 * dt + g;
        const int off = row * (D * 2) + ((c ^ (row & 7)) << 4) + 8 * h;
        *reinterpret_cast<uint2*>(dk_l + off) = make_uint2(pk2(dk[dt][4 * g] * a.scale, dk[dt][4 * g + 1] * a.scale),
                                                           pk2(dk[dt][4 * g + 2] * a.scale, dk[dt][4 * g + 3] * a.scale));
        *reinterpret_cast<uint2*>(dv_l + off) = make_uint2(pk2(dv[dt][4 * g], dv[dt][4 * g + 1]),
                                                           pk2(dv[dt][4 * g + 2], dv[dt][4 * g + 3]));
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
      if (!(KN & K_NO_EPI) || a.causal == 12345) {
        *reinterpret_cast<uint4*>(dKb + (int64_t)(kb0 + r) * a.dk_ss + 8 * c) = *reinterpret_cast<const uint4*>(dk_l + off);
        *reinterpret_cast<uint4*>(dVb + (int64_t)(kb0 + r) * a.dv_ss + 8 * c) = *reinterpret_cast<const uint4*>(dv_l + off);
      }
    }
  } else if (!(KN & K_NO_EPI) || a.causal == 12345) {
    bf16_t* dK = a.dk + (int64_t)b * a.dk_sb + (int64_t)hh * a.dk_sh + (int64_t)key * a.dk_ss;
    bf16_t* dV = a.dv + (int64_t)b * a.dv_sb + (int64_t)hh * a.dv_sh + (int64_t)key * a.dv_ss;
    if (KN & K_WIDE_EPI) {
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) {
        store_wide(dK, dk[dt], a.scale, dt, h);
        store_wide(dV, dv[dt], 1.f, dt, h);
      }
    } else {
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * h;
        ushort4 o;
        o.x = f2bf(dk[dt][4 * g + 0] * a.scale); o.y = f2bf(dk[dt][4 * g + 1] * a.scale);
        o.z = f2bf(dk[dt][4 * g + 2] * a.scale); o.w = f2bf(dk[dt][4 * g + 3] * a.scale);
        *reinterpret_cast<ushort4*>(dK + d) = o;
        o.x = f2bf(dv[dt][4 * g + 0]); o.y = f2bf(dv[dt][4 * g + 1]);
        o.z = f2bf(dv[dt][4 * g + 2]); o.w = f2bf(dv[dt][4 * g + 3]);
        *reinterpret_cast<ushort4*>(dV + d) = o;
      }
    }
    }
  }
}

template <int D>
__global__ void dq_finish(AttnArgs a, int nkb) {
  const int64_t per = (int64_t)a.B * a.H * a.Sq * D;
  const int64_t nv = per / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
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

}  // namespace lab

#include "attn_bwd_seq.inc"
struct Variant { const char* name; void (*launch)(ffk::AttnArgs, hipStream_t); bool check; };
#include "attn_bwd_lab_variants.inc"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static float bf2f_h(uint16_t v) { uint32_t u = (uint32_t)v << 16; float f; memcpy(&f, &u, 4); return f; }
static uint16_t f2bf_h(float f) { uint32_t u; memcpy(&u, &f, 4); u += 0x7fff + ((u >> 16) & 1); return (uint16_t)(u >> 16); }


int main(int argc, char** argv) {
  int B = argc > 1 ? atoi(argv[1]) : 32, H = argc > 2 ? atoi(argv[2]) : 16, S = argc > 3 ? atoi(argv[3]) : 512;
  const int D = 64;
  const int64_t nqkv = (int64_t)B * S * 3 * H * D, no = (int64_t)B * S * H * D;
  std::vector<uint16_t> hq(nqkv), hdo(no);
  std::mt19937 rng(1);
  std::normal_distribution<float> nd(0.f, 1.f);
  for (auto& x : hq) x = f2bf_h(nd(rng));
  for (auto& x : hdo) x = f2bf_h(nd(rng));
  uint16_t *qkv, *o, *dout, *dqkv_ref, *dqkv;
  float *lse, *ws;
  CK(hipMalloc(&qkv, nqkv * 2)); CK(hipMalloc(&dqkv_ref, nqkv * 2)); CK(hipMalloc(&dqkv, nqkv * 2));
  CK(hipMalloc(&o, no * 2)); CK(hipMalloc(&dout, no * 2));
  CK(hipMalloc(&lse, (int64_t)B * H * S * 4));
  const int64_t wsf = ffk::attn_bwd_workspace_floats(B, H, S, S, D) + 8 * (int64_t)B * H * S * D;
  CK(hipMalloc(&ws, wsf * 4));
  CK(hipMemcpy(qkv, hq.data(), nqkv * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dout, hdo.data(), no * 2, hipMemcpyHostToDevice));
  ffk::AttnArgs a;
  const int64_t sb = (int64_t)S * 3 * H * D, sh = D, ss = 3 * H * D;
  const int64_t ob = (int64_t)S * H * D, oh = D, os = H * D;
  a.q = qkv; a.k = qkv + H * D; a.v = qkv + 2 * H * D;
  a.q_sb = a.k_sb = a.v_sb = sb; a.q_sh = a.k_sh = a.v_sh = sh; a.q_ss = a.k_ss = a.v_ss = ss;
  a.o = o; a.o_sb = ob; a.o_sh = oh; a.o_ss = os;
  a.dout = dout; a.do_sb = ob; a.do_sh = oh; a.do_ss = os;
  a.lse = lse; a.B = B; a.H = H; a.Sq = a.Sk = S; a.D = D; a.scale = 1.f / sqrtf((float)D); a.causal = 0;
  a.dq_sb = a.dk_sb = a.dv_sb = sb; a.dq_sh = a.dk_sh = a.dv_sh = sh; a.dq_ss = a.dk_ss = a.dv_ss = ss;
  a.delta = ws + 8 * (int64_t)B * H * S * D;
  a.dq_acc = ws;
  ffk::attn_fwd(a, 0);
  ffk::AttnArgs r = a;
  r.dq = dqkv_ref; r.dk = dqkv_ref + H * D; r.dv = dqkv_ref + 2 * H * D;
  ffk::attn_bwd(r, 0);  // also leaves delta in ws
  CK(hipDeviceSynchronize());
  std::vector<uint16_t> ref(nqkv), got(nqkv);
  CK(hipMemcpy(ref.data(), dqkv_ref, nqkv * 2, hipMemcpyDeviceToHost));
  a.dq = dqkv; a.dk = dqkv + H * D; a.dv = dqkv + 2 * H * D;

  const auto& vars = lab_variants();
  const double flops = 10.0 * B * H * (double)S * S * D;
  std::vector<std::vector<float>> times(vars.size());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int reps = 20;
  for (int round = 0; round < 3; ++round) {
    for (size_t i = 0; i < vars.size(); ++i) {
      vars[i].launch(a, 0);
      CK(hipEventRecord(e0, 0));
      for (int k = 0; k < reps; ++k) vars[i].launch(a, 0);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      times[i].push_back(ms / reps);
    }
  }
  printf("B=%d H=%d S=%d D=%d  (main kernel + dq finish where the variant has one)\n", B, H, S, D);
  for (size_t i = 0; i < vars.size(); ++i) {
    float best = 1e9;
    for (float t : times[i]) best = std::min(best, t);
    double err = -1;
    if (vars[i].check) {
      CK(hipMemset(dqkv, 0, nqkv * 2));
      vars[i].launch(a, 0);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(got.data(), dqkv, nqkv * 2, hipMemcpyDeviceToHost));
      err = 0;
      for (int64_t j = 0; j < nqkv; ++j) err = std::max(err, (double)fabsf(bf2f_h(got[j]) - bf2f_h(ref[j])));
    }
    printf("%-34s %8.1f us  %6.1f TF/s  maxdiff %.4g   rounds", vars[i].name, best * 1e3, flops / best / 1e9, err);
    for (float t : times[i]) printf(" %.1f", t * 1e3);
    printf("\n");
  }
  return 0;
}

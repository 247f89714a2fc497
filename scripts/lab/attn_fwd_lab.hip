// Attention-forward lab: the production forward kernel with switches (F_* bits) that turn one
// part off at a time or swap in a candidate, timed against production and diffed.
//   build: scripts/lab/build_lab.sh   run: scripts/lab/attn_fwd_lab [B H S]
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
constexpr float LN2 = 0.6931471805599453f;
enum : int { F_NO_EXP = 1, F_NO_PV = 2, F_NO_RESCALE = 4, F_ONE_TILE = 8, F_NO_EPI = 16, F_LDS_EPI = 32,
             F_NO_MASKTEST = 64, F_XCD = 256, F_TREE = 512 };
// max / sum of the 32 scores of a lane as balanced trees (the serial chains were 32 dependent
// ops), and the xor-32 partner exchange with v_permlane32_swap instead of ds_bpermute
__device__ __forceinline__ float tree_max(const f32x16& a, const f32x16& b) {
  float t[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) t[i] = fmaxf(a[i], b[i]);
#pragma unroll
  for (int w = 8; w > 0; w >>= 1)
#pragma unroll
    for (int i = 0; i < w; ++i) t[i] = fmaxf(t[i], t[i + w]);
  return t[0];
}
__device__ __forceinline__ float tree_sum(const f32x16& a, const f32x16& b) {
  float t[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) t[i] = a[i] + b[i];
#pragma unroll
  for (int w = 8; w > 0; w >>= 1)
#pragma unroll
    for (int i = 0; i < w; ++i) t[i] = t[i] + t[i + w];
  return t[0];
}
__device__ __forceinline__ float swap32(float x) {  // value of lane l ^ 32
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}
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
__device__ __forceinline__ unsigned pk2(float x, float y) { return (unsigned)f2bf(x) | ((unsigned)f2bf(y) << 16); }

template <int D, int KN>
__global__ void __launch_bounds__(256, 2) fwd_knob(AttnArgs a) {
  constexpr int KV = 64;
  constexpr int TB = KV * D * 2;  // bytes of one K or V tile
  __shared__ __attribute__((aligned(16))) char smem[4 * TB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int nqb = (a.Sq + 127) / 128;
  const int lid = (KN & F_XCD) ? xcd_remap(blockIdx.x, gridDim.x) : 0;
  const int bh = (KN & F_XCD) ? lid / nqb : blockIdx.y, b = bh / a.H, hh = bh % a.H;
  const int qblk0 = ((KN & F_XCD) ? lid % nqb : blockIdx.x) * 128;
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

  int nkv = (KN & F_ONE_TILE) ? 1 : (a.Sk + KV - 1) / KV;
  if (a.causal) nkv = min(nkv, (min(qblk0 + 128, a.Sq) + KV - 1) / KV);

  TileStage<D, KV, 256> sk, sv;
  if (nkv > 0) {
    sk.load(K, a.k_ss, 0, a.Sk, tid);
    sv.load(V, a.v_ss, 0, a.Sk, tid);
    sk.store(smem, tid);
    sv.store(smem + TB, tid);
    __syncthreads();
  }
  for (int t = 0; t < nkv; ++t) {
    const char* kl = smem + (t & 1) * 2 * TB;
    const char* vl = kl + TB;
    char* nk = smem + ((t + 1) & 1) * 2 * TB;
    const bool more = t + 1 < nkv;
    if (more) {
      sk.load(K, a.k_ss, (t + 1) * KV, a.Sk, tid);
      sv.load(V, a.v_ss, (t + 1) * KV, a.Sk, tid);
    }
    // S^T[key][q] for keys 32kt..32kt+31 of this tile
    f32x16 sacc[2] = {f32x16{}, f32x16{}};
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const int row = 32 * kt + (lane & 31);
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kl + aoff<D>(row, 16 * s + 8 * h));
        sacc[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], sacc[kt], 0, 0, 0);
      }
    }
    // mask (only on tiles that cross the sequence end or the causal diagonal: a wave-uniform
    // test), online softmax on the raw scores (lane-local + xor-32 partner), scale folded into
    // one FMA per element: p = exp2(s * sl2 - m * sl2)
    const int kbase = t * KV;
    const bool need_mask = !(KN & F_NO_MASKTEST) && ((kbase + KV > a.Sk) || (a.causal && kbase + KV - 1 > q0));
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
    if (KN & F_TREE) {
      mx = tree_max(sacc[0], sacc[1]);
      mx = fmaxf(mx, swap32(mx)) * sl2;
    } else {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sacc[kt][r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * sl2;
    }
    const float mnew = fmaxf(m, mx);
    const float msafe = mnew == -INFINITY ? 0.f : mnew;
    const float alpha = exp2f(m - msafe);
    float rs = 0.f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = (KN & F_NO_EXP) ? __builtin_fmaf(sacc[kt][r], sl2, -msafe) : exp2f(__builtin_fmaf(sacc[kt][r], sl2, -msafe));
        sacc[kt][r] = p;
        if (!(KN & F_TREE)) rs += p;
      }
    }
    if (KN & F_TREE) rs = tree_sum(sacc[0], sacc[1]) + 0.f, rs += swap32(rs);
    else rs += __shfl_xor(rs, 32, 64);
    lsum = lsum * alpha + rs;
    m = mnew;
    if (!(KN & F_NO_RESCALE)) {
#pragma unroll
    for (int i = 0; i < D / 32; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) oacc[i][r] *= alpha;
    }
    // O^T[d][q] += V^T[d][key] . P^T[key][q]
    bf16x8 pf[2][2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) { pf[kt][0] = pack8(sacc[kt], 0); pf[kt][1] = pack8(sacc[kt], 8); }
    const int G = lane >> 4, qi = (lane & 15) >> 2, pi = lane & 3;
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) {
      const int col = dt * 32 + 16 * (G & 1) + 4 * pi;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int r0 = 32 * kt + 16 * s2 + 4 * h + qi;
          const bf16x4 lo = tr_read(vl, aoff<D>(r0, col));
          const bf16x4 hi = tr_read(vl, aoff<D>(r0 + 8, col));
          bf16x8 vf;
          vf[0] = lo[0]; vf[1] = lo[1]; vf[2] = lo[2]; vf[3] = lo[3];
          vf[4] = hi[0]; vf[5] = hi[1]; vf[6] = hi[2]; vf[7] = hi[3];
          if (!(KN & F_NO_PV)) oacc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[kt][s2], oacc[dt], 0, 0, 0);
          else oacc[dt][0] += (float)vf[0] + (float)pf[kt][s2][1];
        }
      }
    }
    if (more) {
      sk.store(nk, tid);
      sv.store(nk + TB, tid);
    }
    __syncthreads();
  }
  // epilogue
  if ((KN & F_LDS_EPI)) {
    // O^T acc: lane = query row, d = 32dt + 8g + 4h + (0..3); stage [128 q][D] rows in LDS
    __syncthreads();
    const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
    char* ol = smem;
    const int row = wave * 32 + (lane & 31);
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 4 * dt + g;
        const int off = row * (D * 2) + ((c ^ (row & 7)) << 4) + 8 * h;
        *reinterpret_cast<uint2*>(ol + off) = make_uint2(pk2(oacc[dt][4 * g] * inv, oacc[dt][4 * g + 1] * inv),
                                                         pk2(oacc[dt][4 * g + 2] * inv, oacc[dt][4 * g + 3] * inv));
      }
    if (h == 0 && a.lse && qrow < a.Sq) a.lse[(int64_t)bh * a.Sq + qrow] = lsum > 0.f ? (m * LN2 + __logf(lsum)) : INFINITY;
    __syncthreads();
    constexpr int CPR = D / 8;
    bf16_t* Ob = a.o + (int64_t)b * a.o_sb + (int64_t)hh * a.o_sh;
#pragma unroll
    for (int i = 0; i < 128 * CPR / 256; ++i) {
      const int id = tid + i * 256, r = id / CPR, c = id % CPR;
      if (qblk0 + r < a.Sq && (!(KN & F_NO_EPI) || a.causal == 12345))
        *reinterpret_cast<uint4*>(Ob + (int64_t)(qblk0 + r) * a.o_ss + 8 * c) =
            *reinterpret_cast<const uint4*>(ol + r * (D * 2) + ((c ^ (r & 7)) << 4));
    }
  } else if (qrow < a.Sq && (!(KN & F_NO_EPI) || a.causal == 12345)) {
    const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
    bf16_t* O = a.o + (int64_t)b * a.o_sb + (int64_t)hh * a.o_sh + (int64_t)qrow * a.o_ss;
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * h;
        ushort4 o;
        o.x = f2bf(oacc[dt][4 * g + 0] * inv);
        o.y = f2bf(oacc[dt][4 * g + 1] * inv);
        o.z = f2bf(oacc[dt][4 * g + 2] * inv);
        o.w = f2bf(oacc[dt][4 * g + 3] * inv);
        *reinterpret_cast<ushort4*>(O + d) = o;
      }
    }
    if (h == 0 && a.lse) a.lse[(int64_t)bh * a.Sq + qrow] = lsum > 0.f ? (m * LN2 + __logf(lsum)) : INFINITY;
  }
}


template <int KN>
void launch(ffk::AttnArgs a, hipStream_t st) {
  const int nqb = (a.Sq + 127) / 128;
  if (KN & F_XCD) hipLaunchKernelGGL((fwd_knob<64, KN>), dim3(nqb * a.B * a.H), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((fwd_knob<64, KN>), dim3(nqb, a.B * a.H), dim3(256), 0, st, a);
}
void launch_prod(ffk::AttnArgs a, hipStream_t st) { ffk::attn_fwd(a, st); }
}  // namespace lab

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
static float bf2f_h(uint16_t v) { uint32_t u = (uint32_t)v << 16; float f; memcpy(&f, &u, 4); return f; }
static uint16_t f2bf_h(float f) { uint32_t u; memcpy(&u, &f, 4); u += 0x7fff + ((u >> 16) & 1); return (uint16_t)(u >> 16); }
struct Variant { const char* name; void (*launch)(ffk::AttnArgs, hipStream_t); bool check; };

int main(int argc, char** argv) {
  using namespace lab;
  int B = argc > 1 ? atoi(argv[1]) : 32, H = argc > 2 ? atoi(argv[2]) : 16, S = argc > 3 ? atoi(argv[3]) : 512;
  const int D = 64;
  const int64_t nqkv = (int64_t)B * S * 3 * H * D, no = (int64_t)B * S * H * D;
  std::vector<uint16_t> hq(nqkv);
  std::mt19937 rng(1);
  std::normal_distribution<float> nd(0.f, 1.f);
  for (auto& x : hq) x = f2bf_h(nd(rng));
  uint16_t *qkv, *o, *o_ref;
  float *lse, *lse_ref;
  CK(hipMalloc(&qkv, nqkv * 2)); CK(hipMalloc(&o, no * 2)); CK(hipMalloc(&o_ref, no * 2));
  CK(hipMalloc(&lse, (int64_t)B * H * S * 4)); CK(hipMalloc(&lse_ref, (int64_t)B * H * S * 4));
  CK(hipMemcpy(qkv, hq.data(), nqkv * 2, hipMemcpyHostToDevice));
  ffk::AttnArgs a;
  const int64_t sb = (int64_t)S * 3 * H * D, sh = D, ss = 3 * H * D;
  a.q = qkv; a.k = qkv + H * D; a.v = qkv + 2 * H * D;
  a.q_sb = a.k_sb = a.v_sb = sb; a.q_sh = a.k_sh = a.v_sh = sh; a.q_ss = a.k_ss = a.v_ss = ss;
  a.o_sb = (int64_t)S * H * D; a.o_sh = D; a.o_ss = H * D;
  a.B = B; a.H = H; a.Sq = a.Sk = S; a.D = D; a.scale = 1.f / sqrtf((float)D); a.causal = 0;
  ffk::AttnArgs r = a;
  r.o = o_ref; r.lse = lse_ref;
  ffk::attn_fwd(r, 0);
  CK(hipDeviceSynchronize());
  std::vector<uint16_t> ref(no), got(no);
  CK(hipMemcpy(ref.data(), o_ref, no * 2, hipMemcpyDeviceToHost));
  a.o = o; a.lse = lse;
  static const std::vector<Variant> vars = {
      {"production", launch_prod, true},
      {"knob: none", launch<0>, true},
      {"knob: no exp", launch<F_NO_EXP>, false},
      {"knob: no PV MFMA", launch<F_NO_PV>, false},
      {"knob: no rescale", launch<F_NO_RESCALE>, false},
      {"knob: no O stores", launch<F_NO_EPI>, false},
      {"knob: one KV tile", launch<F_ONE_TILE>, false},
      {"knob: one KV tile, no O stores", launch<F_ONE_TILE | F_NO_EPI>, false},
      {"knob: no mask test", launch<F_NO_MASKTEST>, true},
      {"cand: LDS epilogue", launch<F_LDS_EPI>, true},
      {"cand: XCD grouping", launch<F_XCD>, true},
      {"cand: XCD + LDS epilogue", launch<F_XCD | F_LDS_EPI>, true},
      {"cand: XCD + LDS epi + no mask test", launch<F_XCD | F_LDS_EPI | F_NO_MASKTEST>, true},
      {"cand: tree reductions + permlane32", launch<F_TREE>, true},
      {"cand: all above + tree", launch<F_XCD | F_LDS_EPI | F_NO_MASKTEST | F_TREE>, true},
  };
  const double flops = 4.0 * B * H * (double)S * S * D;
  std::vector<std::vector<float>> times(vars.size());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int round = 0; round < 3; ++round)
    for (size_t i = 0; i < vars.size(); ++i) {
      vars[i].launch(a, 0);
      CK(hipEventRecord(e0, 0));
      for (int k = 0; k < 20; ++k) vars[i].launch(a, 0);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      times[i].push_back(ms / 20);
    }
  printf("attention forward B=%d H=%d S=%d D=%d\n", B, H, S, D);
  for (size_t i = 0; i < vars.size(); ++i) {
    float best = 1e9;
    for (float t : times[i]) best = std::min(best, t);
    double err = -1;
    if (vars[i].check) {
      CK(hipMemset(o, 0, no * 2));
      vars[i].launch(a, 0);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(got.data(), o, no * 2, hipMemcpyDeviceToHost));
      err = 0;
      for (int64_t j = 0; j < no; ++j) err = std::max(err, (double)fabsf(bf2f_h(got[j]) - bf2f_h(ref[j])));
    }
    printf("%-36s %8.1f us  %6.1f TF/s  maxdiff %.4g\n", vars[i].name, best * 1e3, flops / best / 1e9, err);
  }
  return 0;
}

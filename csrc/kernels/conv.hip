// 2-D convolution (NCHW or channel-last tensors, bf16, fp32 accumulate) as implicit GEMMs on MFMA 32x32x16.
//
// Reference: src/ops/conv_2d.cu (cuDNN forward / backward-data / backward-filter with algorithm
// search). MI355X design:
//   * Activations are channel-last ([N][H][W][G][Cp]) so that every MFMA operand fragment — 8
//     consecutive reduction elements — is ONE 16-B load of 8 channels at one pixel. The framework
//     keeps CNN activations channel-last end to end (kernels.CHANNELS_LAST), so such an operand
//     with Cg % 8 == 0 is read in place; NCHW operands (and channel counts that are not a multiple
//     of 8, e.g. an RGB input) are re-laid out per call into channel-padded copies (Cp = Cg
//     rounded up to 8). The weights are packed the same way ([G][rows][KH][KW][Cp], zero tail to
//     the K tile).
//   * forward and backward-data are the same kernel (conv_igemm_kernel): rows = output channels
//     (forward) / input channels (backward-data), columns = output pixels of the call, reduction
//     = (kh, kw, 8-channel chunk). The gather of a chunk is a bounds test on the shifted pixel
//     (forward: ih = oh*s - p + kh; backward-data: oh = (ih + p - kh) / s when divisible). Tiles
//     128 x 128 x 32 through double-buffered, XOR-swizzled LDS images (conflict-free b128 reads),
//     4 waves x (2 x 2) MFMA tiles, bias + ReLU fused into the store: NCHW straight from the
//     accumulators, channel-last through an LDS [pixel][channel] image so that each pixel's
//     channels leave as whole 16-B chunks.
//   * backward-filter (conv_wgrad_kernel): rows = output channels, columns = the flattened
//     (kh, kw, input channel) axis, reduction = output pixels, split over workgroups. Both
//     operands arrive as [pixel][channel] images and are read transposed with ds_read_b64_tr_b16 —
//     the attention dV^T = dO^T . P operand path; the splits' fp32 tiles go to slabs that one
//     reduce pass adds into the weight gradient (no atomics).
#include <stdexcept>

#include "common.h"
#include "ops.h"

namespace ffk {

namespace {

typedef short v4s __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x4 trr(const char* lds, int off) {
  v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(lds + off));
  return __builtin_bit_cast(bf16x4, v);
}
__device__ __forceinline__ bf16x8 cat(bf16x4 lo, bf16x4 hi) {
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
// [rows][32] bf16 image (64-B rows): 16-B chunk c of row r, XOR-swizzled by (r >> 2) & 3 so that
// 16 consecutive rows read at one chunk column hit 16 distinct bank groups
__device__ __forceinline__ int off32(int r, int c) { return r * 64 + ((c ^ ((r >> 2) & 3)) << 4); }
}  // namespace

// ------------------------------------------------------------------------------- re-layouts
// x [N][G*Cg][HW] -> xt [N][HW][G][Cp] (channels zero-padded to Cp per group)
// A workgroup transposes a 64-pixel x 64-channel tile of one (image, group) through LDS: loads are
// one channel row of 64 consecutive pixels per wave instruction, stores are whole 16-B
// 8-channel chunks, consecutive lanes on consecutive chunks / pixels (the pixel-per-thread
// version with 64-bit index math and pixel-strided 16-B stores ran at ~1 TB/s)
constexpr int NHWC_ROW = 72;  // LDS row (one pixel): 64 channels + 8 pad, 144 B (16-B aligned)
__global__ void __launch_bounds__(256) conv_nhwc_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ xt, int N,
                                                        int G, int Cg, int HW, int Cp) {
  __shared__ __attribute__((aligned(16))) uint16_t tile[64 * NHWC_ROW];
  const int hw0 = blockIdx.x * 64, ct = blockIdx.y;
  const int ng = blockIdx.z, n = ng / G, g = ng - n * G;
  const int c0 = ct * 64;
  const int t = threadIdx.x, px = t & 63;
  const bf16_t* src = x + ((int64_t)n * G + g) * Cg * HW;
#pragma unroll 4
  for (int r = t >> 6; r < 64; r += 4) {
    const int c = c0 + r, hw = hw0 + px;
    tile[px * NHWC_ROW + r] = (c < Cg && hw < HW) ? src[(int64_t)c * HW + hw] : (uint16_t)0;
  }
  __syncthreads();
  const int nch = min(8, (Cp - c0) / 8);  // 8-channel chunks of this tile inside Cp
  for (int k = t; k < 64 * 8; k += 256) {
    const int pi = k >> 3, ch = k & 7, hw = hw0 + pi;
    if (ch < nch && hw < HW)
      *reinterpret_cast<uint4*>(xt + (((int64_t)n * HW + hw) * G + g) * Cp + c0 + ch * 8) =
          *reinterpret_cast<const uint4*>(tile + pi * NHWC_ROW + ch * 8);
  }
}

static void launch_nhwc(const bf16_t* x, bf16_t* xt, int N, int G, int Cg, int HW, int Cp, hipStream_t st) {
  const dim3 grid((unsigned)((HW + 63) / 64), (unsigned)((Cp + 63) / 64), (unsigned)(N * G));
  hipLaunchKernelGGL(conv_nhwc_kernel, grid, dim3(256), 0, st, x, xt, N, G, Cg, HW, Cp);
}

// w [G*Kg][Cg][KH][KW] -> wp [G][Kg][KH][KW][Cp] + zero tail to Kp per row (forward operand), or
// (transpose = 1) wp [G][Cg][KH][KW][Kgp] + tail (backward-data operand: rows = input channels)
// wp2 (optional): the transposed image too (Kp2 per row), in the same launch — the forward packs the
// backward-data operand of its step along with its own (conv2d_fwd's wpack_bwd)
__global__ void __launch_bounds__(256) conv_pack_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ wp, int G,
                                                        int Kg, int Cg, int KH, int KW, int Kp, int transpose,
                                                        bf16_t* __restrict__ wp2 = nullptr, int Kp2 = 0) {
  // 32-bit index math (weights are far below 2^31 elements; the host checks): the 64-bit divisions
  // of the first version made a 37k-element pack take ~8 us
  const unsigned total1 = wp ? (unsigned)G * (transpose ? Cg : Kg) * Kp : 0u;
  const unsigned total = total1 + (wp2 ? (unsigned)G * Cg * Kp2 : 0u);
  const unsigned stride = gridDim.x * blockDim.x;
  for (unsigned i0 = blockIdx.x * blockDim.x + threadIdx.x; i0 < total; i0 += stride) {
    const bool second = i0 >= total1;
    const int tr = second ? 1 : transpose;
    const unsigned K_ = second ? (unsigned)Kp2 : (unsigned)Kp;
    const unsigned i = second ? i0 - total1 : i0;
    const unsigned rows = tr ? Cg : Kg;  // GEMM rows per group
    const int red = tr ? Kg : Cg;        // reduction channels
    const unsigned redp = (red + 7) / 8 * 8;
    const unsigned gr = i / K_, k = i - gr * K_;
    const unsigned g = gr / rows, row = gr - g * rows;
    const unsigned t = k / redp, c = k - t * redp;
    const unsigned kh = t / KW, kw = t - kh * KW;
    uint16_t v = 0;
    if ((int)kh < KH && (int)c < red) {
      const unsigned co = tr ? c : row, ci = tr ? row : c;
      v = w[((((size_t)g * Kg + co) * Cg + ci) * KH + kh) * KW + kw];
    }
    (second ? wp2 : wp)[i] = v;
  }
}

// ------------------------------------------------------------------------------- fwd / bwd-data
struct IGemmArgs {
  const bf16_t* A;   // packed weights [G][M][Kp]
  const bf16_t* B;   // channel-last source [N][Hs][Ws][G][Cs]
  bf16_t* out;       // NCHW [N][G*M][Ho][Wo], or (out_nhwc) channel-last [N][Ho][Wo][G][M]
  const bf16_t* bias;
  int N, G, M, Kp;   // rows per group, padded reduction length (multiple of 32)
  int Hs, Ws, Cs;    // source geometry (Cs = padded channels per group)
  int Ho, Wo;        // output geometry (columns = N * Ho * Wo)
  int KH, KW, sh, sw, ph, pw;
  int relu;
  int out_nhwc;      // channel-last output (M % 8 == 0)
  int accum;         // add into the existing output (a gradient summed over several consumers)
  int nph;           // backward-data by stride phase (sh * sw sub-GEMMs, grid z = G * nph); 0 / 1: off
  // backward-data of a convolution whose input came from a bias + ReLU convolution (its only
  // consumer): the epilogue writes that producer's pre-activation gradient dx * (y > 0) (dmask = its
  // channel-last output y) and adds the per-channel sums of it into row (phase * gridDim.x +
  // blockIdx.x) of dpart ([rows][G * M] fp32, zeroed by the host), folded into the producer's bias
  // gradient afterwards (Executor._plan_dact_fusion; the producer skips its own mask + sum pass)
  const bf16_t* dmask = nullptr;
  float* dpart = nullptr;
};

// Column -> output pixel of the implicit GEMMs: the identity, or (stride-phase backward-data) the
// pixel (n, py + sh jy, px + sw jx) of phase column (n, jy, jx)
struct IdPix {
  __device__ __forceinline__ int64_t operator()(int64_t p) const { return p; }
};
struct PhasePix {
  int Hq, Wq, py, px, sh, sw, H, W;
  __device__ __forceinline__ int64_t operator()(int64_t p) const {
    const int64_t HW = (int64_t)Hq * Wq;
    const int64_t n = p / HW;
    const int r = (int)(p - n * HW), jy = r / Wq, jx = r - jy * Wq;
    return (n * H + py + sh * jy) * W + px + sw * jx;
  }
};

// Epilogue of the implicit GEMMs: acc[i][j] row = channel (r&3) + 8(r>>2) + 4h of the wave's
// (BM/2)-row block, column = pixel lane & 31 of its (BN/2)-pixel block; bias, ReLU, accumulate.
// smem: >= BN * (2 BM + 16) bytes, free (every wave past its last read of the K loop's images).
template <int BM, int BN, class PixMap = IdPix>
__device__ __forceinline__ void igemm_epilogue(const IGemmArgs& a, f32x16 (&acc)[BM / 64][BN / 64], char* smem,
                                               int m0, int64_t p0, int64_t P, int g, PixMap pix = PixMap{}) {
  constexpr int MI = BM / 64, NB = BN / 64, RS = BM * 2 + 16;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  if (a.out_nhwc) {
    const int64_t ldo = (int64_t)a.G * a.M;
    constexpr int ITERS = BN * (BM / 8) / 256;
    static_assert(ITERS * 256 == BN * (BM / 8), "whole store passes");
    // the producer's outputs for every chunk this thread stores, all requested up front (one
    // dependent global load per pass exposed its latency 8 times per tile)
    uint4 ym[ITERS];
    if (a.dmask) {
#pragma unroll
      for (int it = 0; it < ITERS; ++it) {
        const int k = tid + 256 * it, px = k / (BM / 8), c = k % (BM / 8);
        const int64_t p = p0 + px;
        const int m = m0 + c * 8;
        ym[it] = (p < P && m < a.M) ? *reinterpret_cast<const uint4*>(a.dmask + pix(p) * ldo + (int64_t)g * a.M + m)
                                    : make_uint4(0, 0, 0, 0);
      }
    }
    // stage the tile as [pixel][channel] in LDS (the K loop's buffers are free after its last
    // barrier), then store whole 16-B channel chunks: a pixel's BM channels are one contiguous run
    // of the channel-last output, consecutive lanes on consecutive chunks. The lane's bias values
    // (4 consecutive channels per (i, q); M % 8 == 0 here) are loaded once, 8 B at a time.
    float bv[MI][4][4];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = m0 + (BM / 2) * wm + 32 * i + 8 * q + 4 * h;
        uint2 raw = make_uint2(0, 0);
        if (a.bias && m < a.M) raw = *reinterpret_cast<const uint2*>(a.bias + g * a.M + m);
        bv[i][q][0] = bf2f((bf16_t)(raw.x & 0xffff));
        bv[i][q][1] = bf2f((bf16_t)(raw.x >> 16));
        bv[i][q][2] = bf2f((bf16_t)(raw.y & 0xffff));
        bv[i][q][3] = bf2f((bf16_t)(raw.y >> 16));
      }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int px = (BN / 2) * wn + 32 * j + (lane & 31);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int ml = (BM / 2) * wm + 32 * i + 8 * q + 4 * h;
          uint16_t e[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            float v = acc[i][j][4 * q + k] + bv[i][q][k];
            if (a.relu) v = fmaxf(v, 0.f);
            e[k] = f2bf(v);
          }
          uint2 pk;
          pk.x = (uint32_t)e[0] | ((uint32_t)e[1] << 16);
          pk.y = (uint32_t)e[2] | ((uint32_t)e[3] << 16);
          *reinterpret_cast<uint2*>(smem + px * RS + ml * 2) = pk;
        }
      }
    }
    __syncthreads();
    // dact: this thread's 8 channels (chunk c = tid % (BM / 8): 256 is a multiple of BM / 8, so c
    // is fixed across the loop) summed over the pixels it stores
    float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
      const int k = tid + 256 * it;
      const int px = k / (BM / 8), c = k % (BM / 8);
      const int64_t p = p0 + px;
      const int m = m0 + c * 8;
      if (p < P && m < a.M) {
        const int64_t eoff = pix(p) * ldo + (int64_t)g * a.M + m;
        uint4* dst = reinterpret_cast<uint4*>(a.out + eoff);
        uint4 v = *reinterpret_cast<const uint4*>(smem + px * RS + c * 16);
        if (a.dmask) {  // the producer's ReLU: keep the gradient where its output was positive
          const uint4 yv = ym[it];
          const uint32_t* yw = reinterpret_cast<const uint32_t*>(&yv);
          uint32_t* vw = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const bool lo_on = bf2f((bf16_t)(yw[q] & 0xffff)) > 0.f, hi_on = bf2f((bf16_t)(yw[q] >> 16)) > 0.f;
            vw[q] = (lo_on ? (vw[q] & 0xffffu) : 0u) | (hi_on ? (vw[q] & 0xffff0000u) : 0u);
            csum[2 * q] += bf2f((bf16_t)(vw[q] & 0xffff));
            csum[2 * q + 1] += bf2f((bf16_t)(vw[q] >> 16));
          }
        }
        if (a.accum) {  // fp32 sum of the staged value and the existing gradient, one rounding
          const uint4 o = *dst;
          const uint32_t* ow = reinterpret_cast<const uint32_t*>(&o);
          uint32_t* vw = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float lo = bf2f((bf16_t)(vw[k] & 0xffff)) + bf2f((bf16_t)(ow[k] & 0xffff));
            const float hi = bf2f((bf16_t)(vw[k] >> 16)) + bf2f((bf16_t)(ow[k] >> 16));
            vw[k] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
          }
        }
        *dst = v;
      }
    }
    if (a.dpart) {
      // fold the 256 / (BM / 8) threads that share a chunk through LDS, then one thread per
      // channel adds the workgroup's partial into its slab row
      constexpr int CPT = BM / 8, TPC = 256 / CPT;
      __syncthreads();  // every thread is done reading the staged tile
      float* red = reinterpret_cast<float*>(smem);  // [TPC][BM]
      const int c = tid % CPT, t = tid / CPT;
#pragma unroll
      for (int e = 0; e < 8; ++e) red[t * BM + c * 8 + e] = csum[e];
      __syncthreads();
      if (tid < BM) {
        float sum = 0.f;
        for (int q = 0; q < TPC; ++q) sum += red[q * BM + tid];
        const int m = m0 + tid;
        constexpr bool kPhase = std::is_same<PixMap, PhasePix>::value;
        const int row = (kPhase ? (int)(blockIdx.z % a.nph) * (int)gridDim.x : 0) + (int)blockIdx.x;
        if (m < a.M) a.dpart[(int64_t)row * ldo + (int64_t)g * a.M + m] = sum;
      }
    }
    return;
  }
  const int64_t HoWo = (int64_t)a.Ho * a.Wo;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int64_t p = p0 + (BN / 2) * wn + 32 * j + (lane & 31);
    if (p >= P) continue;
    const int64_t rp = pix(p), n = rp / HoWo, pp = rp - n * HoWo;
    bf16_t* ob = a.out + (n * a.G + g) * (int64_t)a.M * HoWo + pp;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + (BM / 2) * wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m >= a.M) continue;
        float v = acc[i][j][r];
        if (a.bias) v += bf2f(a.bias[g * a.M + m]);
        if (a.relu) v = fmaxf(v, 0.f);
        if (a.accum) v += bf2f(ob[(int64_t)m * HoWo]);
        ob[(int64_t)m * HoWo] = f2bf(v);
      }
    }
  }
}

template <bool BWD, int BM, int BN>
__global__ void __launch_bounds__(256) conv_igemm_kernel(IGemmArgs a) {
  // MI / NB: MFMA row / column tiles per wave (BM / 2 rows x BN / 2 pixels per wave)
  constexpr int BK = 32, MI = BM / 64, NB = BN / 64;
  constexpr int TA = BM * BK * 2, TB = BN * BK * 2;
  constexpr int RS = BM * 2 + 16;  // channel-last epilogue: [pixel][BM channels] rows, 16-B pad
  constexpr int SMEM = 2 * (TA + TB) > BN * RS ? 2 * (TA + TB) : BN * RS;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  const int g = blockIdx.z;
  const int m0 = blockIdx.y * BM;
  const int64_t P = (int64_t)a.N * a.Ho * a.Wo;
  const int64_t p0 = (int64_t)blockIdx.x * BN;
  const int C8 = a.Cs / 8;
  const bf16_t* Ag = a.A + (int64_t)g * a.M * a.Kp;
  // this thread's staging slots: rows r and r + 64 of both tiles, 16-B chunk c
  const int sr = tid >> 2, sc = tid & 3;
  const bf16_t* arow[MI];
  bool aok[MI];
  int64_t pbase[NB];
  int prow[NB], pcol[NB];
  bool pok[NB];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int m = m0 + sr + 64 * i;
    aok[i] = m < a.M;
    arow[i] = Ag + (int64_t)(aok[i] ? m : 0) * a.Kp + sc * 8;
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int64_t p = p0 + sr + 64 * i;
    pok[i] = p < P;
    const int64_t pp = pok[i] ? p : 0;
    const int64_t n = pp / ((int64_t)a.Ho * a.Wo);
    const int rem = (int)(pp - n * a.Ho * a.Wo);
    prow[i] = rem / a.Wo;
    pcol[i] = rem - prow[i] * a.Wo;
    pbase[i] = n * a.Hs * a.Ws;
  }
  // reduction chunk of this thread at K-step 0: chunk index sc -> (kh, kw, c8)
  int c8 = sc % C8, kw = (sc / C8) % a.KW, kh = sc / C8 / a.KW;
  uint4 ra[MI], rb[NB];
  auto load = [&](int ks) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
      ra[i] = aok[i] ? *reinterpret_cast<const uint4*>(arow[i] + ks * BK) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      bool ok = pok[i] && kh < a.KH;
      int sy, sx;
      if (!BWD) {
        sy = prow[i] * a.sh - a.ph + kh;
        sx = pcol[i] * a.sw - a.pw + kw;
      } else {  // source (output-gradient) pixel whose window at (kh, kw) covers this input pixel
        const int ny = prow[i] + a.ph - kh, nx = pcol[i] + a.pw - kw;
        ok = ok && ny >= 0 && nx >= 0 && ny % a.sh == 0 && nx % a.sw == 0;
        sy = ny / a.sh;
        sx = nx / a.sw;
      }
      ok = ok && sy >= 0 && sy < a.Hs && sx >= 0 && sx < a.Ws;
      rb[i] = ok ? *reinterpret_cast<const uint4*>(a.B + ((pbase[i] + (int64_t)sy * a.Ws + sx) * a.G + g) * a.Cs +
                                                    c8 * 8)
                 : make_uint4(0, 0, 0, 0);
    }
    // advance this thread's chunk by BK / 8 = 4 chunks
    c8 += 4;
    while (c8 >= C8) {
      c8 -= C8;
      if (++kw == a.KW) { kw = 0; ++kh; }
    }
  };
  auto stash = [&](int buf) {
    char* la = smem + buf * (TA + TB);
    char* lb = la + TA;
#pragma unroll
    for (int i = 0; i < MI; ++i) *reinterpret_cast<uint4*>(la + off32(sr + 64 * i, sc)) = ra[i];
#pragma unroll
    for (int i = 0; i < NB; ++i) *reinterpret_cast<uint4*>(lb + off32(sr + 64 * i, sc)) = rb[i];
  };
  f32x16 acc[MI][NB];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x16{};
  const int nks = a.Kp / BK;
  load(0);
  stash(0);
  __syncthreads();
  for (int ks = 0; ks < nks; ++ks) {
    const int buf = ks & 1;
    const char* la = smem + buf * (TA + TB);
    const char* lb = la + TA;
    if (ks + 1 < nks) load(ks + 1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[MI], bfr[NB];
#pragma unroll
      for (int i = 0; i < MI; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(la + off32((BM / 2) * wm + 32 * i + (lane & 31), 2 * kk + h));
#pragma unroll
      for (int j = 0; j < NB; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(lb + off32((BN / 2) * wn + 32 * j + (lane & 31), 2 * kk + h));
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (ks + 1 < nks) stash(buf ^ 1);
    __syncthreads();
  }
  igemm_epilogue<BM, BN>(a, acc, smem, m0, p0, P, g);
}

// ------------------------------------------------------------------------------- fwd / bwd-data (LDS-DMA)
// The same implicit GEMM with K steps of 64 (one barrier per 64-deep step: at 32 the barrier and the
// fragment-read restart dominated) and operand tiles written straight into LDS by buffer_load ...
// lds (no staging registers). Each wave instruction fills one 1-KiB piece = 8 rows of 128 B, lane
// l landing at row l / 8, slot l % 8; the XOR swizzle (chunk c of row r at slot c ^ (r & 7)) is
// applied on the global side, so lane l always fetches chunk (l & 7) ^ (l >> 3) of its rows and
// keeps ONE (kh, kw, c8) reduction cursor. Padding taps, rows past M and pixels past P read an
// offset beyond the buffer's range, which returns zeros. Two LDS buffers: the DMA for step k + 1
// is issued right after the barrier that retires step k and runs under step k's MFMAs.
typedef __attribute__((address_space(3))) void* lds_ptr_t;
__device__ __forceinline__ int off64(int r, int c) { return r * 128 + ((c ^ (r & 7)) << 4); }

// PH (backward-data, stride > 1): one sub-GEMM per stride phase (py, px) = (ih % sh, iw % sw).
// The input pixels of a phase receive only the taps kh = kh0 + sh th, kw = kw0 + sw tw (kh0 =
// (py + ph) % sh), and their output-gradient source is (jy + oy0 - th, jx + ox0 - tw): a dense
// GEMM over ~1 / (sh sw) of the taps. Without phases every input pixel walks all KH x KW taps and
// 3 of 4 (stride 2) read zeros: the MFMA work of the stride-2 convolutions' backward-data was 4x.
template <bool BWD, int BM, int BN, bool PH = false>
__global__ void __launch_bounds__(256) conv_igemm_dma_kernel(IGemmArgs a) {
  constexpr int BK = 64, MI = BM / 64, NB = BN / 64;
  constexpr int TA = BM * BK * 2, TB = BN * BK * 2;
  constexpr int WA = TA / 1024 / 4, WB = TB / 1024 / 4;  // 1-KiB pieces per wave per step
  constexpr int RS = BM * 2 + 16;
  constexpr int SMEM = 2 * (TA + TB) > BN * RS ? 2 * (TA + TB) : BN * RS;
  constexpr int BAD = 0x7ffffff0;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  int g = blockIdx.z;
  const int m0 = blockIdx.y * BM;
  int64_t P = (int64_t)a.N * a.Ho * a.Wo;
  const int64_t p0 = (int64_t)blockIdx.x * BN;
  const int C8 = a.Cs / 8;
  // stride phase (PH): column geometry Hq x Wq, tap subset KHq x KWq from (kh0, kw0)
  PhasePix pm{a.Ho, a.Wo, 0, 0, 1, 1, a.Ho, a.Wo};
  int KHq = a.KH, KWq = a.KW, kh0 = 0, kw0 = 0, oy0 = 0, ox0 = 0;
  if (PH) {
    const int nph = a.sh * a.sw, phz = (int)blockIdx.z % nph;
    g = (int)blockIdx.z / nph;
    pm.py = phz / a.sw;
    pm.px = phz % a.sw;
    pm.sh = a.sh;
    pm.sw = a.sw;
    pm.Hq = (a.Ho - pm.py + a.sh - 1) / a.sh;
    pm.Wq = (a.Wo - pm.px + a.sw - 1) / a.sw;
    kh0 = (pm.py + a.ph) % a.sh;
    kw0 = (pm.px + a.pw) % a.sw;
    KHq = (a.KH - kh0 + a.sh - 1) / a.sh;
    KWq = (a.KW - kw0 + a.sw - 1) / a.sw;
    oy0 = (pm.py + a.ph - kh0) / a.sh;
    ox0 = (pm.px + a.pw - kw0) / a.sw;
    P = (int64_t)a.N * pm.Hq * pm.Wq;
    if (p0 >= P) return;  // whole workgroup: this phase has fewer columns than the grid's widest
  }
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.A + (int64_t)g * a.M * a.Kp), (short)0, a.M * a.Kp * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.B, (short)0, (int)((int64_t)a.N * a.Hs * a.Ws * a.G * a.Cs * 2), 0x00020000);
  const int ch = (lane & 7) ^ (lane >> 3);  // this lane's 16-B chunk of every 128-B row it loads
  int aoff[WA];
#pragma unroll
  for (int i = 0; i < WA; ++i) {
    const int m = m0 + (i * 4 + wave) * 8 + (lane >> 3);
    aoff[i] = m < a.M ? (m * a.Kp + (PH ? 0 : ch * 8)) * 2 : BAD;
  }
  int pbase[WB], prow[WB], pcol[WB];
  bool pok[WB];
  const int Hc = PH ? pm.Hq : a.Ho, Wc = PH ? pm.Wq : a.Wo;  // column image geometry
#pragma unroll
  for (int i = 0; i < WB; ++i) {
    const int64_t p = p0 + (i * 4 + wave) * 8 + (lane >> 3);
    pok[i] = p < P;
    const int64_t pp = pok[i] ? p : 0;
    const int n = (int)(pp / ((int64_t)Hc * Wc));
    const int rem = (int)(pp - (int64_t)n * Hc * Wc);
    prow[i] = rem / Wc;
    pcol[i] = rem - prow[i] * Wc;
    pbase[i] = n * a.Hs * a.Ws;
  }
  // reduction cursor of this lane's chunk: K index ks * 8 + ch -> (kh, kw, c8); with PH, (th, tw,
  // c8) over the phase's taps (kh, kw below hold th, tw)
  const int KWc = PH ? (KWq > 0 ? KWq : 1) : a.KW, KHc = PH ? KHq : a.KH;
  const bool unit_stride = a.sh == 1 && a.sw == 1;  // backward-data without the stride divisions
  // fast addressing (forward, stride phases, stride-1 backward-data): the source pixel is
  // (yb + SG kh, xb + SG kw), so a piece's byte offset is its pixel base plus a per-lane tap term
  // computed once per step — the operand issue is the kernel's VALU bottleneck
  constexpr int SG = BWD ? -1 : 1;
  const bool fast = PH || !BWD || unit_stride;
  const int GC2 = a.G * a.Cs * 2;
  int yb[WB], xb[WB], pixb[WB];
#pragma unroll
  for (int i = 0; i < WB; ++i) {
    yb[i] = PH ? prow[i] + oy0 : (!BWD ? prow[i] * a.sh - a.ph : prow[i] + a.ph);
    xb[i] = PH ? pcol[i] + ox0 : (!BWD ? pcol[i] * a.sw - a.pw : pcol[i] + a.pw);
    pixb[i] = (pbase[i] + yb[i] * a.Ws + xb[i]) * GC2 + g * a.Cs * 2;
  }
  int c8 = ch % C8, kw = (ch / C8) % KWc, kh = ch / C8 / KWc;
  auto issue = [&](int buf, int ks) {
    char* la = smem + buf * (TA + TB);
    char* lb = la + TA;
    int acol = ks * (BK * 2);
    if (PH) acol = kh < KHc ? (((kh0 + a.sh * kh) * a.KW + kw0 + a.sw * kw) * a.Cs + c8 * 8) * 2 : BAD;
#pragma unroll
    for (int i = 0; i < WA; ++i) {
      const int off = (aoff[i] == BAD || acol == BAD) ? BAD : aoff[i] + acol;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)(la + (i * 4 + wave) * 1024), 16, off, 0, 0, 0);
    }
    if (fast) {
      const int tap = (SG * kh * a.Ws + SG * kw) * GC2 + c8 * 16;
#pragma unroll
      for (int i = 0; i < WB; ++i) {
        const bool ok = pok[i] && kh < KHc && (unsigned)(yb[i] + SG * kh) < (unsigned)a.Hs &&
                        (unsigned)(xb[i] + SG * kw) < (unsigned)a.Ws;
        const int off = ok ? pixb[i] + tap : BAD;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr_t)(lb + (i * 4 + wave) * 1024), 16, off, 0, 0, 0);
      }
    } else {
#pragma unroll
    for (int i = 0; i < WB; ++i) {
      bool ok = pok[i] && kh < KHc;
      int sy, sx;
      if (PH) {
        sy = prow[i] + oy0 - kh;
        sx = pcol[i] + ox0 - kw;
      } else if (!BWD) {
        sy = prow[i] * a.sh - a.ph + kh;
        sx = pcol[i] * a.sw - a.pw + kw;
      } else if (unit_stride) {  // backward-data, stride 1: the source pixel is the shifted one
        sy = prow[i] + a.ph - kh;
        sx = pcol[i] + a.pw - kw;
      } else {  // source (output-gradient) pixel whose window at (kh, kw) covers this input pixel
        const int ny = prow[i] + a.ph - kh, nx = pcol[i] + a.pw - kw;
        ok = ok && ny >= 0 && nx >= 0 && ny % a.sh == 0 && nx % a.sw == 0;
        sy = ny / a.sh;
        sx = nx / a.sw;
      }
      ok = ok && sy >= 0 && sy < a.Hs && sx >= 0 && sx < a.Ws;
      const int off = ok ? (((pbase[i] + sy * a.Ws + sx) * a.G + g) * a.Cs + c8 * 8) * 2 : BAD;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr_t)(lb + (i * 4 + wave) * 1024), 16, off, 0, 0, 0);
    }
    }
    c8 += 8;  // next step: 8 chunks on
    while (c8 >= C8) {
      c8 -= C8;
      if (++kw == KWc) { kw = 0; ++kh; }
    }
  };
  f32x16 acc[MI][NB];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x16{};
  const int nks = PH ? (KHq * KWq * C8 + 7) / 8 : a.Kp / BK;  // a phase without taps: zeros
  if (nks > 0) issue(0, 0);
  for (int ks = 0; ks < nks; ++ks) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // step ks visible to all waves; every wave is done reading the other buffer
    if (ks + 1 < nks) issue((ks + 1) & 1, ks + 1);
    const char* la = smem + (ks & 1) * (TA + TB);
    const char* lb = la + TA;
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      bf16x8 af[MI], bfr[NB];
#pragma unroll
      for (int i = 0; i < MI; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(la + off64((BM / 2) * wm + 32 * i + (lane & 31), 2 * kk + h));
#pragma unroll
      for (int j = 0; j < NB; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(lb + off64((BN / 2) * wn + 32 * j + (lane & 31), 2 * kk + h));
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();  // the epilogue reuses the images
  if (PH) igemm_epilogue<BM, BN>(a, acc, smem, m0, p0, P, g, pm);
  else igemm_epilogue<BM, BN>(a, acc, smem, m0, p0, P, g);
}

// ------------------------------------------------------------------------------- bwd-filter
// dW as an implicit GEMM: rows = output channels (TM per workgroup), columns = the flattened
// (kh, kw, input channel) reduction axis of the forward (128 per workgroup, so 1x1 and k x k
// convolutions both fill whole tiles), reduction = output pixels in steps of 64, split over S
// workgroups per tile. Both operands are [pixel][channel] images (dy rows; x rows gathered at the
// pixel shifted by each column's (kh, kw)) read transposed from LDS with ds_read_b64_tr_b16. Each
// split writes its fp32 tile to a slab and wgrad_reduce_kernel adds the S slabs into dW (no
// atomics), re-indexing (kh, kw, c) columns to the [K][C][KH][KW] weight layout.
struct WGradArgs {
  const bf16_t* dy;   // [N][OH][OW][G][Kgs]
  const bf16_t* x;    // [N][H][W][G][Cp]
  float* ws;          // [G][S][Kg][NC] fp32 partial tiles
  int N, G, Kg, Kgs, Cp, H, W, OH, OW, KH, KW, sh, sw, ph, pw;
  int NC;             // KH * KW * Cp columns
  int S;              // pixel splits per tile
};

// [rows][TC] bf16 image (TC = 64 or 128 channels per row): the attention kernels' swizzles,
// conflict-free for 16-B row writes and ds_read_b64_tr_b16 column reads
template <int TC>
__device__ __forceinline__ int offc(int row, int col) {
  const int sw = TC == 64 ? ((((row >> 1) & 1) << 2) | ((row >> 3) & 1) | (((row >> 4) & 1) << 1))
                          : (((row & 3) << 2) | ((row >> 2) & 3));
  return row * (TC * 2) + ((((col >> 3) ^ sw)) << 4) + ((col & 7) << 1);
}

// TM output channels x 128 columns per workgroup; 4 waves in 2 x 2, each (TM/2) x 64 as
// (TM/64) x 2 MFMA tiles of 32 x 32
template <int TM>
__global__ void __launch_bounds__(256, 2) conv_wgrad_kernel(WGradArgs a) {  // 2 waves / SIMD: <= 256 registers
  constexpr int TN = 128, BP = 64;
  constexpr int TIA = BP * TM * 2, TIB = BP * TN * 2;
  constexpr int CA = TM / 8, CB = TN / 8;                   // 16-B chunks per pixel row
  constexpr int LA = BP * CA / 256, LB = BP * CB / 256;     // chunks per thread per step
  constexpr int MTM = TM / 64, MTN = TN / 64;
  __shared__ __attribute__((aligned(16))) char smem[2 * (TIA + TIB)];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  const int co0 = blockIdx.x * TM, n0 = blockIdx.y * TN;
  const int g = blockIdx.z / a.S, split = blockIdx.z % a.S;
  const int64_t P = (int64_t)a.N * a.OH * a.OW;
  const int64_t nsteps = (P + BP - 1) / BP;
  const int64_t s0 = nsteps * split / a.S, s1 = nsteps * (split + 1) / a.S;
  // A (dy) slots: rows tid / CA + (256 / CA) i, chunk tid % CA (fixed)
  const int ach = tid % CA;
  const bool aok = co0 + ach * 8 < a.Kgs;
  const bf16_t* abase = a.dy + (int64_t)g * a.Kgs + co0 + ach * 8;
  const int64_t astride = (int64_t)a.G * a.Kgs;
  // B (x) slots: rows tid / CB + 16 i, column chunk tid % CB (fixed): its (kh, kw, c)
  const int bch = tid % CB;
  const int col = n0 + bch * 8;
  const bool bok = col < a.NC;
  const int kpos = bok ? col / a.Cp : 0, bc = col - kpos * a.Cp;
  const int kh = kpos / a.KW, kw = kpos - kh * a.KW;
  const bf16_t* bbase = a.x + (int64_t)g * a.Cp + bc;
  int bn[LB], boh[LB], bow[LB];
  const int dq = BP / a.OW, dr = BP - dq * a.OW;
#pragma unroll
  for (int i = 0; i < LB; ++i) {
    const int64_t p = s0 * BP + tid / CB + (256 / CB) * i;
    bn[i] = (int)(p / ((int64_t)a.OH * a.OW));
    const int rem = (int)(p - (int64_t)bn[i] * a.OH * a.OW);
    boh[i] = rem / a.OW;
    bow[i] = rem - boh[i] * a.OW;
  }
  uint4 ra[LA], rb[LB];
  int64_t st_cur = s0;
  auto load = [&]() {
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int64_t p = st_cur * BP + tid / CA + (256 / CA) * i;
      ra[i] = (aok && p < P) ? *reinterpret_cast<const uint4*>(abase + p * astride) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      uint4 v = make_uint4(0, 0, 0, 0);
      const int ih = boh[i] * a.sh - a.ph + kh, iw = bow[i] * a.sw - a.pw + kw;
      if (bok && bn[i] < a.N && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W)
        v = *reinterpret_cast<const uint4*>(bbase + ((((int64_t)bn[i] * a.H + ih) * a.W + iw) * a.G) * a.Cp);
      rb[i] = v;
      // next step: 64 pixels on
      bow[i] += dr;
      boh[i] += dq;
      if (bow[i] >= a.OW) { bow[i] -= a.OW; ++boh[i]; }
      if (boh[i] >= a.OH) { bn[i] += boh[i] / a.OH; boh[i] %= a.OH; }
    }
    ++st_cur;
  };
  auto stash = [&](int buf) {
    char* la = smem + buf * (TIA + TIB);
    char* lb = la + TIA;
#pragma unroll
    for (int i = 0; i < LA; ++i)
      *reinterpret_cast<uint4*>(la + offc<TM>(tid / CA + (256 / CA) * i, ach * 8)) = ra[i];
#pragma unroll
    for (int i = 0; i < LB; ++i)
      *reinterpret_cast<uint4*>(lb + offc<TN>(tid / CB + (256 / CB) * i, bch * 8)) = rb[i];
  };
  f32x16 acc[MTM][MTN];
#pragma unroll
  for (int i = 0; i < MTM; ++i)
#pragma unroll
    for (int j = 0; j < MTN; ++j) acc[i][j] = f32x16{};
  const int G4 = lane >> 4, qi = (lane & 15) >> 2, pi = lane & 3;
  if (s0 < s1) {
    load();
    stash(0);
  }
  __syncthreads();
  for (int64_t st = s0; st < s1; ++st) {
    const int buf = (int)((st - s0) & 1);
    const char* la = smem + buf * (TIA + TIB);
    const char* lb = la + TIA;
    const bool more = st + 1 < s1;
    if (more) load();
#pragma unroll
    for (int ks = 0; ks < BP / 16; ++ks) {
      const int r0 = 16 * ks + 4 * h + qi;
      bf16x8 fa[MTM], fb[MTN];
#pragma unroll
      for (int i = 0; i < MTM; ++i) {
        const int c = (TM / 2) * wm + 32 * i + 16 * (G4 & 1) + 4 * pi;
        fa[i] = cat(trr(la, offc<TM>(r0, c)), trr(la, offc<TM>(r0 + 8, c)));
      }
#pragma unroll
      for (int j = 0; j < MTN; ++j) {
        const int c = (TN / 2) * wn + 32 * j + 16 * (G4 & 1) + 4 * pi;
        fb[j] = cat(trr(lb, offc<TN>(r0, c)), trr(lb, offc<TN>(r0 + 8, c)));
      }
#pragma unroll
      for (int i = 0; i < MTM; ++i)
#pragma unroll
        for (int j = 0; j < MTN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (more) stash(buf ^ 1);
    __syncthreads();
  }
  // acc[i][j]: row = output channel, column = lane & 31; every split writes its whole slab tile
  // (zeros for an empty split) so that the reduce reads defined values
  float* slab = a.ws + ((int64_t)(g * a.S + split) * a.Kg) * a.NC;
#pragma unroll
  for (int j = 0; j < MTN; ++j) {
    const int cc = n0 + (TN / 2) * wn + 32 * j + (lane & 31);
    if (cc >= a.NC) continue;
#pragma unroll
    for (int i = 0; i < MTM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + (TM / 2) * wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (co < a.Kg) slab[(int64_t)co * a.NC + cc] = acc[i][j][r];
      }
    }
  }
}

// The same backward-filter GEMM with both [64 pixel][channel] images written by LDS-DMA. A piece
// is 1 KiB of whole image rows (TC = 128: 4 rows of 256 B; 64: 8 rows of 128 B); lane l lands at
// row l / (TC / 8), slot l % (TC / 8) and fetches the chunk slot ^ swizzle(row) of offc<TC>, so a
// lane's column chunk is fixed per piece for the whole kernel: the x gather keeps one (kh, kw, c)
// per piece and only advances the pixels. Out-of-range pixels / channels / padding taps read
// beyond the buffer range (zeros).
template <int TC>
__device__ __forceinline__ int offc_swz(int row) {
  return TC == 64 ? ((((row >> 1) & 1) << 2) | ((row >> 3) & 1) | (((row >> 4) & 1) << 1))
                  : (((row & 3) << 2) | ((row >> 2) & 3));
}

// BP pixels per stage, NS stages in the ring (NS - 1 in flight under the MFMAs of the current one)
template <int TM, int BP = 64, int NS = 2>
__global__ void __launch_bounds__(256, 2) conv_wgrad_dma_kernel(WGradArgs a) {
  constexpr int TN = 128;
  constexpr int TIA = BP * TM * 2, TIB = BP * TN * 2;
  constexpr int WA = TIA / 1024 / 4, WB = TIB / 1024 / 4;  // pieces per wave per step
  constexpr int RA = 1024 / (TM * 2), RB = 1024 / (TN * 2);  // image rows per piece
  constexpr int MTM = TM / 64, MTN = TN / 64;
  constexpr int BAD = 0x7ffffff0;
  __shared__ __attribute__((aligned(16))) char smem[NS * (TIA + TIB)];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  const int co0 = blockIdx.x * TM, n0 = blockIdx.y * TN;
  const int g = blockIdx.z / a.S, split = blockIdx.z % a.S;
  const int64_t P = (int64_t)a.N * a.OH * a.OW;
  const int64_t nsteps = (P + BP - 1) / BP;
  const int64_t s0 = nsteps * split / a.S, s1 = nsteps * (split + 1) / a.S;
  const __amdgpu_buffer_rsrc_t rdy =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.dy, (short)0, (int)(P * a.G * a.Kgs * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.x, (short)0, (int)((int64_t)a.N * a.H * a.W * a.G * a.Cp * 2), 0x00020000);
  // A (dy) pieces: fixed channel chunk per piece, pixel = step * 64 + row
  int arow[WA], acol[WA];
#pragma unroll
  for (int i = 0; i < WA; ++i) {
    const int row = (i * 4 + wave) * RA + lane / (TM / 8);
    const int c = (lane % (TM / 8)) ^ offc_swz<TM>(row);
    arow[i] = row;
    acol[i] = co0 + c * 8 < a.Kgs ? (g * a.Kgs + co0 + c * 8) : -1;
  }
  // B (x) pieces: fixed column chunk (kh, kw, c) per piece, tracked pixel (n, oh, ow)
  int bkh[WB], bkw[WB], bcol[WB], bn[WB], boh[WB], bow[WB];
  const int dq = BP / a.OW, dr = BP - dq * a.OW;
#pragma unroll
  for (int i = 0; i < WB; ++i) {
    const int row = (i * 4 + wave) * RB + lane / (TN / 8);
    const int c = (lane % (TN / 8)) ^ offc_swz<TN>(row);
    const int col = n0 + c * 8;
    const int kpos = col / a.Cp, cc = col - kpos * a.Cp;
    bkh[i] = col < a.NC ? kpos / a.KW : 1 << 20;  // past the image: always a padding tap
    bkw[i] = kpos % a.KW;
    bcol[i] = g * a.Cp + cc;
    const int64_t p = s0 * BP + row;
    bn[i] = (int)(p / ((int64_t)a.OH * a.OW));
    const int rem = (int)(p - (int64_t)bn[i] * a.OH * a.OW);
    boh[i] = rem / a.OW;
    bow[i] = rem - boh[i] * a.OW;
  }
  // 32-bit cursors (both buffers are under 2 GiB on this path): the per-step address work is the
  // kernel's issue bottleneck at small Kg (profiles/conv_wgrad_pmc_r4.txt)
  const int ldy2 = a.G * a.Kgs * 2, lx2 = a.G * a.Cp * 2, P32 = (int)P;
  // x pieces: the output pixel's input origin (ihb, iwb) = (oh sh, ow sw) and its byte offset pixb
  // advance incrementally; the piece's fixed tap (kh - ph, kw - pw) and channel are one constant
  const int stepB = (dr * a.sw + dq * a.sh * a.W) * lx2, wrapW = (a.sh * a.W - a.OW * a.sw) * lx2,
            wrapH = (a.H * a.W - a.OH * a.sh * a.W) * lx2;
  int ihb[WB], iwb[WB], pixb[WB], tapb[WB];
#pragma unroll
  for (int i = 0; i < WB; ++i) {
    ihb[i] = boh[i] * a.sh;
    iwb[i] = bow[i] * a.sw;
    pixb[i] = ((bn[i] * a.H + ihb[i]) * a.W + iwb[i]) * lx2;
    bkh[i] -= a.ph;  // from here on: the tap's offset from the window origin
    bkw[i] -= a.pw;
    tapb[i] = (bkh[i] * a.W + bkw[i]) * lx2 + bcol[i] * 2;
  }
  int pa[WA], aoffs[WA];
#pragma unroll
  for (int i = 0; i < WA; ++i) {
    pa[i] = (int)(s0 * BP) + arow[i];
    aoffs[i] = pa[i] * ldy2 + acol[i] * 2;
  }
  auto issue = [&](int buf, int64_t st) {
    char* la = smem + buf * (TIA + TIB);
    char* lb = la + TIA;
#pragma unroll
    for (int i = 0; i < WA; ++i) {
      const int off = (acol[i] >= 0 && pa[i] < P32) ? aoffs[i] : BAD;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rdy, (lds_ptr_t)(la + (i * 4 + wave) * 1024), 16, off, 0, 0, 0);
      pa[i] += BP;
      aoffs[i] += BP * ldy2;
    }
#pragma unroll
    for (int i = 0; i < WB; ++i) {
      const bool ok = bn[i] < a.N && (unsigned)(ihb[i] + bkh[i]) < (unsigned)a.H &&
                      (unsigned)(iwb[i] + bkw[i]) < (unsigned)a.W;
      const int off = ok ? pixb[i] + tapb[i] : BAD;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr_t)(lb + (i * 4 + wave) * 1024), 16, off, 0, 0, 0);
      bow[i] += dr;  // next step: BP pixels on
      boh[i] += dq;
      iwb[i] += dr * a.sw;
      ihb[i] += dq * a.sh;
      pixb[i] += stepB;
      if (bow[i] >= a.OW) {
        bow[i] -= a.OW;
        ++boh[i];
        iwb[i] -= a.OW * a.sw;
        ihb[i] += a.sh;
        pixb[i] += wrapW;
      }
      if (boh[i] >= a.OH) {  // next image(s): usually one, no integer division
        const int k = boh[i] < 2 * a.OH ? 1 : boh[i] / a.OH;
        boh[i] -= k * a.OH;
        ihb[i] -= k * a.OH * a.sh;
        bn[i] += k;
        pixb[i] += k * wrapH;
      }
    }
  };
  f32x16 acc[MTM][MTN];
#pragma unroll
  for (int i = 0; i < MTM; ++i)
#pragma unroll
    for (int j = 0; j < MTN; ++j) acc[i][j] = f32x16{};
  const int G4 = lane >> 4, qi = (lane & 15) >> 2, pi = lane & 3;
#pragma unroll
  for (int q = 0; q < NS - 1; ++q)
    if (s0 + q < s1) issue(q, s0 + q);
  for (int64_t st = s0; st < s1; ++st) {
    // stage st landed (the NS - 2 stages issued after it may stay in flight)
    if (NS > 2 && st + NS - 2 < s1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * (WA + WB)) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // stage st visible to all waves; every wave is done reading stage st - 1's buffer
    if (st + NS - 1 < s1) issue((int)((st + NS - 1 - s0) % NS), st + NS - 1);
    const char* la = smem + (int)((st - s0) % NS) * (TIA + TIB);
    const char* lb = la + TIA;
#pragma unroll
    for (int ks = 0; ks < BP / 16; ++ks) {
      const int r0 = 16 * ks + 4 * h + qi;
      bf16x8 fa[MTM], fb[MTN];
#pragma unroll
      for (int i = 0; i < MTM; ++i) {
        const int c = (TM / 2) * wm + 32 * i + 16 * (G4 & 1) + 4 * pi;
        fa[i] = cat(trr(la, offc<TM>(r0, c)), trr(la, offc<TM>(r0 + 8, c)));
      }
#pragma unroll
      for (int j = 0; j < MTN; ++j) {
        const int c = (TN / 2) * wn + 32 * j + 16 * (G4 & 1) + 4 * pi;
        fb[j] = cat(trr(lb, offc<TN>(r0, c)), trr(lb, offc<TN>(r0 + 8, c)));
      }
#pragma unroll
      for (int i = 0; i < MTM; ++i)
#pragma unroll
        for (int j = 0; j < MTN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  }
  float* slab = a.ws + ((int64_t)(g * a.S + split) * a.Kg) * a.NC;
#pragma unroll
  for (int j = 0; j < MTN; ++j) {
    const int cc = n0 + (TN / 2) * wn + 32 * j + (lane & 31);
    if (cc >= a.NC) continue;
#pragma unroll
    for (int i = 0; i < MTM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + (TM / 2) * wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (co < a.Kg) slab[(int64_t)co * a.NC + cc] = acc[i][j][r];
      }
    }
  }
}

// dW[g*Kg + m][c][kh][kw] += sum over the S slabs of column (kh*KW + kw)*Cp + c (c < Cg). A
// workgroup owns 16 consecutive slab elements and folds their S partials in 16 strided groups (a
// thread per element looping over S serially was latency-bound: ~0.5 us per 4 loads, S ~ 300)
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ ws, float* __restrict__ dw, int G,
                                                           int S, int Kg, int NC, int Cg, int Cp, int KK) {
  __shared__ float sh[16][17];
  const int64_t total = (int64_t)G * Kg * NC, slab = (int64_t)Kg * NC;
  const int el = threadIdx.x & 15, sg = threadIdx.x >> 4;
  const int64_t i = (int64_t)blockIdx.x * 16 + el;
  float v = 0.f;
  int g = 0;
  int64_t rem = 0;
  if (i < total) {
    g = (int)(i / slab);
    rem = i - (int64_t)g * slab;
    const float* p = ws + (int64_t)g * S * slab + rem;
    int s = sg;
    for (; s + 48 < S; s += 64) v += (p[s * slab] + p[(s + 16) * slab]) + (p[(s + 32) * slab] + p[(s + 48) * slab]);
    for (; s < S; s += 16) v += p[s * slab];
  }
  sh[sg][el] = v;
  __syncthreads();
  if (sg != 0 || i >= total) return;
  for (int k = 1; k < 16; ++k) v += sh[k][el];
  const int m = (int)(rem / NC), colx = (int)(rem - (int64_t)m * NC);
  const int kp = colx / Cp, c = colx - kp * Cp;
  if (c < Cg) dw[((int64_t)(g * Kg + m) * Cg + c) * KK + kp] += v;
}

// The same fold for few splits (S <= 32): a thread per 4 consecutive slab elements (one 16-B load
// per split, fixed order), grid-stride. wgrad_reduce_kernel's 16 row-groups x 16 elements per
// workgroup left 12 of 16 groups idle at S = 4 and launched 147k workgroups for a 512 x 4608
// gradient: 73 us, 1.5x the backward-filter GEMM it reduces (profiles/conv_wgrad_pmc_r4.txt).
__global__ void __launch_bounds__(256) wgrad_reduce4_kernel(const float* __restrict__ ws, float* __restrict__ dw, int G,
                                                            int S, int Kg, int NC, int Cg, int Cp, int KK) {
  const int64_t slab = (int64_t)Kg * NC, total4 = (int64_t)G * slab / 4;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total4; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = q * 4;
    const int g = (int)(i / slab);
    const int64_t rem = i - (int64_t)g * slab;
    const float* p = ws + (int64_t)g * S * slab + rem;
    float4 v = *reinterpret_cast<const float4*>(p);
    for (int s = 1; s < S; ++s) {
      const float4 t = *reinterpret_cast<const float4*>(p + s * slab);
      v.x += t.x;
      v.y += t.y;
      v.z += t.z;
      v.w += t.w;
    }
    // NC and Cp are multiples of 8: the 4 columns share one row and one (kh, kw)
    const int m = (int)(rem / NC), colx = (int)(rem - (int64_t)m * NC);
    const int kp = colx / Cp, c = colx - kp * Cp;
    float* d = dw + ((int64_t)(g * Kg + m) * Cg + c) * KK + kp;
    if (KK == 1 && c + 3 < Cg && ((uintptr_t)d & 15) == 0) {
      float4 o = *reinterpret_cast<float4*>(d);
      o.x += v.x;
      o.y += v.y;
      o.z += v.z;
      o.w += v.w;
      *reinterpret_cast<float4*>(d) = o;
    } else {
      const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (c + k < Cg) d[k * KK] += vv[k];
    }
  }
}

// Few splits and a k x k filter: a workgroup per gradient row m. The S slab rows (column order
// (kh, kw, c)) are summed with coalesced 16-B loads into an LDS row (padded by one float per tap,
// so the transposing reads below are conflict-free), then the dW row ([c][kh][kw] order) is
// updated with coalesced read-modify-writes. wgrad_reduce4_kernel's dW updates were 4-B stores at
// a KH*KW stride.
constexpr int WRED_ROW_FLOATS = 16384;  // 64 KiB of LDS
__global__ void __launch_bounds__(256) wgrad_reduce_row_kernel(const float* __restrict__ ws, float* __restrict__ dw, int G,
                                                               int S, int Kg, int NC, int Cg, int Cp, int KK) {
  __shared__ float row[WRED_ROW_FLOATS];
  const int g = blockIdx.x / Kg, m = blockIdx.x - g * Kg;
  const int64_t slab = (int64_t)Kg * NC;
  const float* base = ws + (int64_t)g * S * slab + (int64_t)m * NC;
  for (int j = threadIdx.x * 4; j < NC; j += 1024) {
    float4 v = *reinterpret_cast<const float4*>(base + j);
    for (int s = 1; s < S; ++s) {
      const float4 t = *reinterpret_cast<const float4*>(base + s * slab + j);
      v.x += t.x;
      v.y += t.y;
      v.z += t.z;
      v.w += t.w;
    }
    const int kp = j / Cp, c = j - kp * Cp;  // Cp % 8 == 0: one tap per 4 columns
    float* r = row + kp * (Cp + 1) + c;
    r[0] = v.x;
    r[1] = v.y;
    r[2] = v.z;
    r[3] = v.w;
  }
  __syncthreads();
  float* d = dw + (int64_t)(g * Kg + m) * Cg * KK;
  for (int e = threadIdx.x; e < Cg * KK; e += 256) {
    const int c = e / KK, kp = e - c * KK;
    d[e] += row[kp * (Cp + 1) + c];
  }
}

// ------------------------------------------------------------------------------- host
static int round8(int v) { return (v + 7) / 8 * 8; }
static int kpad(int KH, int KW, int redp) { return (KH * KW * redp + 63) / 64 * 64; }  // whole 64-deep K steps

// 128-row tiles, or 64 when the GEMM has at most 64 rows (narrow layers: half the MFMA work of a
// 128-row tile would be padding); 128 pixels per tile while that gives at least two workgroups per
// CU, else 64 (twice the workgroups for the same work: the K loop is latency-bound at one
// workgroup per CU)
// The LDS-DMA kernel needs both operands addressable by 31-bit byte offsets (buffer range); the
// register-staged kernel takes the rest.
template <bool BWD, int BM>
static void launch_igemm_bm(const IGemmArgs& a, int64_t P, int M, int G, hipStream_t st) {
  const int64_t t128 = ((P + 127) / 128) * ((M + BM - 1) / BM) * G;
  const bool dma = (int64_t)a.N * a.Hs * a.Ws * a.G * a.Cs * 2 < 0x7fff0000LL && (int64_t)a.M * a.Kp * 2 < 0x7fff0000LL;
  if (BWD && dma && a.nph > 1) {  // stride phases: grid over the widest phase (py = px = 0)
    const int64_t Pq = (int64_t)a.N * ((a.Ho + a.sh - 1) / a.sh) * ((a.Wo + a.sw - 1) / a.sw);
    const unsigned gz = (unsigned)(G * a.nph), gy = (unsigned)((M + BM - 1) / BM);
    if (t128 >= 512) hipLaunchKernelGGL((conv_igemm_dma_kernel<true, BM, 128, true>), dim3((unsigned)((Pq + 127) / 128), gy, gz), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((conv_igemm_dma_kernel<true, BM, 64, true>), dim3((unsigned)((Pq + 63) / 64), gy, gz), dim3(256), 0, st, a);
    return;
  }
  const dim3 g128((unsigned)((P + 127) / 128), (M + BM - 1) / BM, G), g64((unsigned)((P + 63) / 64), (M + BM - 1) / BM, G);
  if (t128 >= 512) {
    if (dma) hipLaunchKernelGGL((conv_igemm_dma_kernel<BWD, BM, 128>), g128, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((conv_igemm_kernel<BWD, BM, 128>), g128, dim3(256), 0, st, a);
  } else {
    if (dma) hipLaunchKernelGGL((conv_igemm_dma_kernel<BWD, BM, 64>), g64, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((conv_igemm_kernel<BWD, BM, 64>), g64, dim3(256), 0, st, a);
  }
}
template <bool BWD>
static void launch_igemm(const IGemmArgs& a, int64_t P, int M, int G, hipStream_t st) {
  if (M <= 64) launch_igemm_bm<BWD, 64>(a, P, M, G, st);
  else launch_igemm_bm<BWD, 128>(a, P, M, G, st);
}

// backward-filter tiling: 64-row tiles for narrow outputs, else 128. Pixel splits: about as many
// workgroups as fit the CUs at once (3 per CU at 64 rows, 2 at 128: LDS), each over at least 4
// steps of 64 pixels; slabs capped at 64 MB
static int wgrad_tm(int Kg) { return Kg <= 64 ? 64 : 128; }
// FF_CONV_WGRAD_SLOTS scales the workgroup target (percent, default 100): fewer splits write and
// re-read fewer fp32 slabs, more splits fill the CUs
static int wgrad_slot_pct() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("FF_CONV_WGRAD_SLOTS");
    v = e ? std::max(1, atoi(e)) : 100;
  }
  return v;
}
static int wgrad_splits(int64_t P, int G, int Kg, int NC) {
  const int TM = wgrad_tm(Kg);
  const int64_t tiles = (int64_t)G * ((Kg + TM - 1) / TM) * ((NC + 127) / 128);
  const int64_t nsteps = (P + 63) / 64, slots = (TM == 64 ? 768 : 512) * (int64_t)wgrad_slot_pct() / 100;
  int64_t S = std::min<int64_t>(nsteps / 4, (slots + tiles - 1) / tiles);
  S = std::min<int64_t>(S, (int64_t)(16 << 20) / std::max<int64_t>(1, (int64_t)G * Kg * NC));
  return (int)std::max<int64_t>(1, S);
}

static int64_t align8(int64_t v) { return (v + 7) / 8 * 8; }

// backward-filter ring: 0 = two 64-pixel stages, 1 = four 32-pixel stages (FF_CONV_WGRAD_PIPE)
static int conv_wgrad_pipe() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("FF_CONV_WGRAD_PIPE");
    v = e ? atoi(e) : 0;
  }
  return v;
}

// stride-phase backward-data (conv_igemm_dma_kernel<.., PH>): FF_CONV_DGRAD_PHASES=0 turns it off
static bool conv_dgrad_phases() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("FF_CONV_DGRAD_PHASES");
    v = e ? atoi(e) != 0 : 1;
  }
  return v != 0;
}

int64_t conv_ws_elems(int N, int C, int H, int W, int K, int OH, int OW, int KH, int KW, int G) {
  // bf16 elements: channel-last input + channel-last output gradient + packed weights (fwd / bwd)
  // + the backward-filter fp32 slabs (2 bf16 elements each)
  const int Cg = C / G, Kg = K / G, Cp = round8(Cg), Kgp = round8(Kg);
  const int64_t xt = align8((int64_t)N * H * W * G * Cp), yt = align8((int64_t)N * OH * OW * G * Kgp);
  const int64_t wf = (int64_t)G * Kg * kpad(KH, KW, Cp), wb = (int64_t)G * Cg * kpad(KH, KW, Kgp);
  const int NC = KH * KW * Cp;
  const int64_t slabs = (int64_t)wgrad_splits((int64_t)N * OH * OW, G, Kg, NC) * G * Kg * NC;
  return xt + yt + align8(std::max(wf, wb)) + 2 * slabs + 64;
}

int64_t conv_wpack_elems(int C, int K, int KH, int KW, int G) {
  return (int64_t)G * (C / G) * kpad(KH, KW, round8(K / G));
}

void conv2d_fwd(const void* x, const void* w, const void* bias, void* y, void* ws, const int* geom, int relu,
                int x_nhwc, int y_nhwc, hipStream_t st, void* wpack_bwd) {
  const int N = geom[0], C = geom[1], H = geom[2], W = geom[3], K = geom[4], OH = geom[5], OW = geom[6];
  const int KH = geom[7], KW = geom[8], sh = geom[9], sw = geom[10], ph = geom[11], pw = geom[12], G = geom[13];
  const int Cg = C / G, Kg = K / G, Cp = round8(Cg);
  bf16_t* xt = (bf16_t*)ws;
  bf16_t* wp = xt + align8((int64_t)N * H * W * G * Cp) + align8((int64_t)N * OH * OW * G * round8(Kg));
  const int Kp = kpad(KH, KW, Cp);
  // a channel-last input (Cg % 8 == 0, so Cp == Cg) is the implicit GEMM's B operand as it is
  const bf16_t* src = (const bf16_t*)x;
  if (!x_nhwc) {
    launch_nhwc((const bf16_t*)x, xt, N, G, Cg, H * W, Cp, st);
    src = xt;
  }
  // a 1 x 1 filter over 64k input channels per group IS the packed operand ([G][Kg][Cg], rows of
  // Kp == Cg): no pack pass (36 of ResNet-50's 53 forward convolutions)
  const bf16_t* A = wp;
  const bool no_pack = KH == 1 && KW == 1 && Cg % 64 == 0 && Kp == Cg;
  if (no_pack) A = (const bf16_t*)w;
  const int Kpb = kpad(KH, KW, round8(Kg));
  const int64_t packed = (no_pack ? 0 : (int64_t)G * Kg * Kp) + (wpack_bwd ? (int64_t)G * Cg * Kpb : 0);
  if (packed >= (1ll << 31)) throw std::runtime_error("conv2d: packed weights of 2^31 or more elements");
  if (packed > 0)
    hipLaunchKernelGGL(conv_pack_kernel, dim3(ew_grid(packed, 256)), dim3(256), 0, st, (const bf16_t*)w,
                       no_pack ? nullptr : wp, G, Kg, Cg, KH, KW, Kp, 0, (bf16_t*)wpack_bwd, Kpb);
  IGemmArgs a{A, src, (bf16_t*)y, (const bf16_t*)bias, N, G, Kg, Kp, H, W, Cp, OH, OW, KH, KW, sh, sw, ph, pw, relu,
              y_nhwc, 0};
  launch_igemm<false>(a, (int64_t)N * OH * OW, Kg, G, st);
}

// rows of the dact partial slab conv2d_bwd writes (an upper bound over its tilings)
int64_t conv_dact_rows(const int* geom) {
  const int N = geom[0], H = geom[2], W = geom[3], sh = geom[9], sw = geom[10];
  const int nph = conv_dgrad_phases() ? sh * sw : 1;
  if (nph > 1) return (int64_t)nph * (((int64_t)N * ((H + sh - 1) / sh) * ((W + sw - 1) / sw) + 63) / 64);
  return ((int64_t)N * H * W + 63) / 64;
}

void conv2d_bwd(const void* x, const void* w, const void* dy, void* dx, float* dw, void* ws, const int* geom,
                int need_dx, int x_nhwc, int dy_nhwc, int accum_dx, hipStream_t st, const void* wpack,
                const void* dmask, float* dpart) {
  const int N = geom[0], C = geom[1], H = geom[2], W = geom[3], K = geom[4], OH = geom[5], OW = geom[6];
  const int KH = geom[7], KW = geom[8], sh = geom[9], sw = geom[10], ph = geom[11], pw = geom[12], G = geom[13];
  const int Cg = C / G, Kg = K / G, Cp = round8(Cg), Kgp = round8(Kg);
  bf16_t* xt = (bf16_t*)ws;
  bf16_t* yt = xt + align8((int64_t)N * H * W * G * Cp);
  bf16_t* wp = yt + align8((int64_t)N * OH * OW * G * Kgp);
  float* slabs = (float*)(wp + align8(std::max((int64_t)G * Kg * kpad(KH, KW, Cp), (int64_t)G * Cg * kpad(KH, KW, Kgp))));
  const bf16_t* ysrc = (const bf16_t*)dy;
  if (!dy_nhwc) {
    launch_nhwc((const bf16_t*)dy, yt, N, G, Kg, OH * OW, Kgp, st);
    ysrc = yt;
  }
  if (need_dx) {
    const int Kp = kpad(KH, KW, Kgp);
    // the operand packed by this step's forward (wpack), or packed here
    if ((int64_t)G * Cg * Kp >= (1ll << 31)) throw std::runtime_error("conv2d: packed weights of 2^31 or more elements");
    if (!wpack)
      hipLaunchKernelGGL(conv_pack_kernel, dim3(ew_grid((int64_t)G * Cg * Kp, 256)), dim3(256), 0, st,
                         (const bf16_t*)w, wp, G, Kg, Cg, KH, KW, Kp, 1, nullptr, 0);
    IGemmArgs a{wpack ? (const bf16_t*)wpack : wp, ysrc, (bf16_t*)dx, nullptr, N, G, Cg, Kp, OH, OW, Kgp, H, W, KH, KW, sh, sw, ph, pw, 0, x_nhwc,
                accum_dx, conv_dgrad_phases() ? sh * sw : 1};
    if (dmask && x_nhwc && !accum_dx && Cg % 8 == 0) {
      a.dmask = (const bf16_t*)dmask;
      a.dpart = dpart;
      if (dpart) hipMemsetAsync(dpart, 0, conv_dact_rows(geom) * (int64_t)C * sizeof(float), st);
    }
    launch_igemm<true>(a, (int64_t)N * H * W, Cg, G, st);
  }
  if (dw) {
    // the forward's channel-last input copy is rebuilt here (the workspace is per call) unless
    // the input is channel-last already
    const bf16_t* xsrc = (const bf16_t*)x;
    if (!x_nhwc) {
      launch_nhwc((const bf16_t*)x, xt, N, G, Cg, H * W, Cp, st);
      xsrc = xt;
    }
    const int NC = KH * KW * Cp, TM = wgrad_tm(Kg);
    const int64_t P = (int64_t)N * OH * OW;
    const int S = wgrad_splits(P, G, Kg, NC);
    WGradArgs b{ysrc, xsrc, slabs, N, G, Kg, Kgp, Cp, H, W, OH, OW, KH, KW, sh, sw, ph, pw, NC, S};
    const dim3 grid((Kg + TM - 1) / TM, (NC + 127) / 128, G * S);
    const bool dma = P * G * Kgp * 2 < 0x7fff0000LL && (int64_t)N * H * W * G * Cp * 2 < 0x7fff0000LL;
    if (dma && conv_wgrad_pipe() == 1) {  // 32-pixel stages, 4 deep
      if (TM == 128) hipLaunchKernelGGL((conv_wgrad_dma_kernel<128, 32, 4>), grid, dim3(256), 0, st, b);
      else hipLaunchKernelGGL((conv_wgrad_dma_kernel<64, 32, 4>), grid, dim3(256), 0, st, b);
    } else if (dma) {
      if (TM == 128) hipLaunchKernelGGL(conv_wgrad_dma_kernel<128>, grid, dim3(256), 0, st, b);
      else hipLaunchKernelGGL(conv_wgrad_dma_kernel<64>, grid, dim3(256), 0, st, b);
    } else {
      if (TM == 128) hipLaunchKernelGGL(conv_wgrad_kernel<128>, grid, dim3(256), 0, st, b);
      else hipLaunchKernelGGL(conv_wgrad_kernel<64>, grid, dim3(256), 0, st, b);
    }
    if (S <= 32 && KH * KW > 1 && KH * KW * (Cp + 1) <= WRED_ROW_FLOATS)
      hipLaunchKernelGGL(wgrad_reduce_row_kernel, dim3((unsigned)(G * Kg)), dim3(256), 0, st, slabs, dw, G, S, Kg, NC, Cg,
                         Cp, KH * KW);
    else if (S <= 32)
      hipLaunchKernelGGL(wgrad_reduce4_kernel, dim3(ew_grid((int64_t)G * Kg * NC / 4, 256)), dim3(256), 0, st, slabs, dw,
                         G, S, Kg, NC, Cg, Cp, KH * KW);
    else
      hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)(((int64_t)G * Kg * NC + 15) / 16)), dim3(256), 0, st, slabs,
                         dw, G, S, Kg, NC, Cg, Cp, KH * KW);
  }
}

}  // namespace ffk

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
//   * backward-filter (conv_wgrad_kernel): rows = output channels, columns = input channels of
//     one (kh, kw), reduction = output pixels, split over workgroups. Both operands arrive as
//     [pixel][channel] images (the channel-last copies) and are read transposed with
//     ds_read_b64_tr_b16 — the attention dV^T = dO^T . P operand path — and each workgroup adds its
//     fp32 32x32 tiles into the fp32 weight gradient with float atomics.
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
__global__ void __launch_bounds__(256) conv_pack_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ wp, int G,
                                                        int Kg, int Cg, int KH, int KW, int Kp, int transpose) {
  const int rows = transpose ? Cg : Kg;         // GEMM rows per group
  const int red = transpose ? Kg : Cg;          // reduction channels
  const int redp = (red + 7) / 8 * 8;
  const int64_t total = (int64_t)G * rows * Kp;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int k = (int)(i % Kp);
    const int64_t gr = i / Kp;
    const int row = (int)(gr % rows), g = (int)(gr / rows);
    const int c = k % redp, t = k / redp, kw = t % KW, kh = t / KW;
    uint16_t v = 0;
    if (kh < KH && c < red) {
      const int co = transpose ? c : row, ci = transpose ? row : c;
      v = w[(((int64_t)(g * Kg + co) * Cg + ci) * KH + kh) * KW + kw];
    }
    wp[i] = v;
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
};

template <bool BWD, int BN>
__global__ void __launch_bounds__(256) conv_igemm_kernel(IGemmArgs a) {
  constexpr int BM = 128, BK = 32, NB = BN / 64;  // NB: pixel rows per thread / MFMA columns per wave
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
  const bf16_t* arow[2];
  bool aok[2];
  int64_t pbase[NB];
  int prow[NB], pcol[NB];
  bool pok[NB];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
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
  uint4 ra[2], rb[NB];
  auto load = [&](int ks) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
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
    for (int i = 0; i < 2; ++i) *reinterpret_cast<uint4*>(la + off32(sr + 64 * i, sc)) = ra[i];
#pragma unroll
    for (int i = 0; i < NB; ++i) *reinterpret_cast<uint4*>(lb + off32(sr + 64 * i, sc)) = rb[i];
  };
  f32x16 acc[2][NB];
#pragma unroll
  for (int i = 0; i < 2; ++i)
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
      bf16x8 af[2], bfr[NB];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(la + off32(64 * wm + 32 * i + (lane & 31), 2 * kk + h));
#pragma unroll
      for (int j = 0; j < NB; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(lb + off32((BN / 2) * wn + 32 * j + (lane & 31), 2 * kk + h));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (ks + 1 < nks) stash(buf ^ 1);
    __syncthreads();
  }
  // epilogue: acc[i][j] row = channel (r&3) + 8(r>>2) + 4h, column = pixel lane & 31
  if (a.out_nhwc) {
    // stage the tile as [pixel][channel] in LDS (the K loop's buffers are free after its last
    // barrier), then store whole 16-B channel chunks: a pixel's BM channels are one contiguous run
    // of the channel-last output, consecutive lanes on consecutive chunks
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int px = (BN / 2) * wn + 32 * j + (lane & 31);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int ml = 64 * wm + 32 * i + 8 * q + 4 * h;
          uint16_t e[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int m = m0 + ml + k;
            float v = acc[i][j][4 * q + k];
            if (a.bias && m < a.M) v += bf2f(a.bias[g * a.M + m]);
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
    const int64_t ldo = (int64_t)a.G * a.M;
    for (int k = tid; k < BN * (BM / 8); k += 256) {
      const int px = k / (BM / 8), c = k % (BM / 8);
      const int64_t p = p0 + px;
      const int m = m0 + c * 8;
      if (p < P && m < a.M)
        *reinterpret_cast<uint4*>(a.out + p * ldo + (int64_t)g * a.M + m) =
            *reinterpret_cast<const uint4*>(smem + px * RS + c * 16);
    }
    return;
  }
  const int64_t HoWo = (int64_t)a.Ho * a.Wo;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int64_t p = p0 + (BN / 2) * wn + 32 * j + (lane & 31);
    if (p >= P) continue;
    const int64_t n = p / HoWo, pp = p - n * HoWo;
    bf16_t* ob = a.out + (n * a.G + g) * (int64_t)a.M * HoWo + pp;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + 64 * wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m >= a.M) continue;
        float v = acc[i][j][r];
        if (a.bias) v += bf2f(a.bias[g * a.M + m]);
        if (a.relu) v = fmaxf(v, 0.f);
        ob[(int64_t)m * HoWo] = f2bf(v);
      }
    }
  }
}

// ------------------------------------------------------------------------------- bwd-filter
struct WGradArgs {
  const bf16_t* dyt;  // [N][OH][OW][G][Kgp]
  const bf16_t* xt;   // [N][H][W][G][Cp]
  float* dw;          // [G*Kg][Cg][KH][KW] fp32, accumulated
  int N, G, Kg, Kgp, Cg, Cp, H, W, OH, OW, KH, KW, sh, sw, ph, pw;
  int splits;         // workgroups over the output pixels per output tile
};

// [rows][TC] bf16 image (TC = 64 or 128 channels per row): the attention kernels' swizzles,
// conflict-free for 16-B row writes and ds_read_b64_tr_b16 column reads
template <int TC>
__device__ __forceinline__ int offc(int row, int col) {
  const int sw = TC == 64 ? ((((row >> 1) & 1) << 2) | ((row >> 3) & 1) | (((row >> 4) & 1) << 1))
                          : (((row & 3) << 2) | ((row >> 2) & 3));
  return row * (TC * 2) + ((((col >> 3) ^ sw)) << 4) + ((col & 7) << 1);
}

// TC output channels x TC input channels of one (kh, kw) per workgroup, 64 output pixels per
// step; 4 waves in 2 x 2, each (TC/2)^2 = (TC/64)^2 MFMA tiles of 32 x 32
template <int TC>
__global__ void __launch_bounds__(256) conv_wgrad_kernel(WGradArgs a) {
  constexpr int BP = 64, TI = BP * TC * 2, NCH = TC / 8, LPT = BP * NCH / 256, MT = TC / 64;
  __shared__ __attribute__((aligned(16))) char smem[4 * TI];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  const int co0 = blockIdx.x * TC;
  const int ncb = (a.Cg + TC - 1) / TC;
  const int kpos = blockIdx.y / ncb, ci0 = (blockIdx.y % ncb) * TC;
  const int kh = kpos / a.KW, kw = kpos % a.KW;
  const int g = blockIdx.z / a.splits, split = blockIdx.z % a.splits;
  const int64_t P = (int64_t)a.N * a.OH * a.OW;
  const int64_t nsteps = (P + BP - 1) / BP;
  const int64_t s0 = nsteps * split / a.splits, s1 = nsteps * (split + 1) / a.splits;
  // this thread's LPT staging slots: pixel row, 16-B channel chunk; the pixel (n, oh, ow) of each
  // slot advances by 64 every step
  int srow[LPT], sch[LPT], on[LPT], ooh[LPT], oow[LPT];
#pragma unroll
  for (int i = 0; i < LPT; ++i) {
    const int id = tid + 256 * i;
    srow[i] = id / NCH;
    sch[i] = id % NCH;
    const int64_t p = s0 * BP + srow[i];
    on[i] = (int)(p / ((int64_t)a.OH * a.OW));
    const int rem = (int)(p - (int64_t)on[i] * a.OH * a.OW);
    ooh[i] = rem / a.OW;
    oow[i] = rem - ooh[i] * a.OW;
  }
  uint4 ry[LPT], rx[LPT];
  auto load = [&]() {
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      uint4 vy = make_uint4(0, 0, 0, 0), vx = make_uint4(0, 0, 0, 0);
      if (on[i] < a.N) {
        const int64_t p = ((int64_t)on[i] * a.OH + ooh[i]) * a.OW + oow[i];
        const int c = sch[i] * 8;
        if (co0 + c < a.Kgp) vy = *reinterpret_cast<const uint4*>(a.dyt + (p * a.G + g) * a.Kgp + co0 + c);
        const int ih = ooh[i] * a.sh - a.ph + kh, iw = oow[i] * a.sw - a.pw + kw;
        if (ih >= 0 && ih < a.H && iw >= 0 && iw < a.W && ci0 + c < a.Cp)
          vx = *reinterpret_cast<const uint4*>(a.xt + ((((int64_t)on[i] * a.H + ih) * a.W + iw) * a.G + g) * a.Cp +
                                               ci0 + c);
      }
      ry[i] = vy;
      rx[i] = vx;
      // next step: 64 pixels on
      oow[i] += BP;
      while (oow[i] >= a.OW) {
        oow[i] -= a.OW;
        if (++ooh[i] == a.OH) { ooh[i] = 0; ++on[i]; }
      }
    }
  };
  auto stash = [&](int buf) {
    char* ly = smem + buf * 2 * TI;
    char* lx = ly + TI;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      *reinterpret_cast<uint4*>(ly + offc<TC>(srow[i], sch[i] * 8)) = ry[i];
      *reinterpret_cast<uint4*>(lx + offc<TC>(srow[i], sch[i] * 8)) = rx[i];
    }
  };
  f32x16 acc[MT][MT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[i][j] = f32x16{};
  const int G4 = lane >> 4, qi = (lane & 15) >> 2, pi = lane & 3;
  if (s0 < s1) {
    load();
    stash(0);
  }
  __syncthreads();
  for (int64_t st = s0; st < s1; ++st) {
    const int buf = (int)((st - s0) & 1);
    const char* ly = smem + buf * 2 * TI;
    const char* lx = ly + TI;
    const bool more = st + 1 < s1;
    if (more) load();
#pragma unroll
    for (int ks = 0; ks < BP / 16; ++ks) {
      const int r0 = 16 * ks + 4 * h + qi;
      bf16x8 fa[MT], fb[MT];
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int col = (TC / 2) * wm + 32 * i + 16 * (G4 & 1) + 4 * pi;
        fa[i] = cat(trr(ly, offc<TC>(r0, col)), trr(ly, offc<TC>(r0 + 8, col)));
      }
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const int col = (TC / 2) * wn + 32 * j + 16 * (G4 & 1) + 4 * pi;
        fb[j] = cat(trr(lx, offc<TC>(r0, col)), trr(lx, offc<TC>(r0 + 8, col)));
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (more) stash(buf ^ 1);
    __syncthreads();
  }
  if (s0 >= s1) return;
  // acc[i][j]: row = output channel, column = input channel (lane & 31)
#pragma unroll
  for (int j = 0; j < MT; ++j) {
    const int ci = ci0 + (TC / 2) * wn + 32 * j + (lane & 31);
    if (ci >= a.Cg) continue;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + (TC / 2) * wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (co < a.Kg)
          atomicAdd(a.dw + ((((int64_t)(g * a.Kg + co) * a.Cg + ci) * a.KH + kh) * a.KW + kw), acc[i][j][r]);
      }
    }
  }
}

// ------------------------------------------------------------------------------- host
static int round8(int v) { return (v + 7) / 8 * 8; }
static int kpad(int KH, int KW, int redp) { return (KH * KW * redp + 31) / 32 * 32; }

// 128 x 128 tiles while they give at least two workgroups per CU, else 128 x 64 (twice the
// workgroups for the same work: the K loop is latency-bound at one workgroup per CU)
template <bool BWD>
static void launch_igemm(const IGemmArgs& a, int64_t P, int M, int G, hipStream_t st) {
  const int64_t t128 = ((P + 127) / 128) * ((M + 127) / 128) * G;
  if (t128 >= 512)
    hipLaunchKernelGGL((conv_igemm_kernel<BWD, 128>), dim3((unsigned)((P + 127) / 128), (M + 127) / 128, G), dim3(256),
                       0, st, a);
  else
    hipLaunchKernelGGL((conv_igemm_kernel<BWD, 64>), dim3((unsigned)((P + 63) / 64), (M + 127) / 128, G), dim3(256), 0,
                       st, a);
}

int64_t conv_ws_elems(int N, int C, int H, int W, int K, int OH, int OW, int KH, int KW, int G) {
  // bf16 elements: channel-last input + channel-last output gradient + packed weights (fwd / bwd)
  const int Cg = C / G, Kg = K / G, Cp = round8(Cg), Kgp = round8(Kg);
  const int64_t xt = (int64_t)N * H * W * G * Cp, yt = (int64_t)N * OH * OW * G * Kgp;
  const int64_t wf = (int64_t)G * Kg * kpad(KH, KW, Cp), wb = (int64_t)G * Cg * kpad(KH, KW, Kgp);
  return xt + yt + std::max(wf, wb) + 64;
}

void conv2d_fwd(const void* x, const void* w, const void* bias, void* y, void* ws, const int* geom, int relu,
                int x_nhwc, int y_nhwc, hipStream_t st) {
  const int N = geom[0], C = geom[1], H = geom[2], W = geom[3], K = geom[4], OH = geom[5], OW = geom[6];
  const int KH = geom[7], KW = geom[8], sh = geom[9], sw = geom[10], ph = geom[11], pw = geom[12], G = geom[13];
  const int Cg = C / G, Kg = K / G, Cp = round8(Cg);
  bf16_t* xt = (bf16_t*)ws;
  bf16_t* wp = xt + (int64_t)N * H * W * G * Cp + (int64_t)N * OH * OW * G * round8(Kg);
  const int Kp = kpad(KH, KW, Cp);
  // a channel-last input (Cg % 8 == 0, so Cp == Cg) is the implicit GEMM's B operand as it is
  const bf16_t* src = (const bf16_t*)x;
  if (!x_nhwc) {
    launch_nhwc((const bf16_t*)x, xt, N, G, Cg, H * W, Cp, st);
    src = xt;
  }
  hipLaunchKernelGGL(conv_pack_kernel, dim3(ew_grid((int64_t)G * Kg * Kp, 256)), dim3(256), 0, st, (const bf16_t*)w,
                     wp, G, Kg, Cg, KH, KW, Kp, 0);
  IGemmArgs a{wp, src, (bf16_t*)y, (const bf16_t*)bias, N, G, Kg, Kp, H, W, Cp, OH, OW, KH, KW, sh, sw, ph, pw, relu,
              y_nhwc};
  launch_igemm<false>(a, (int64_t)N * OH * OW, Kg, G, st);
}

void conv2d_bwd(const void* x, const void* w, const void* dy, void* dx, float* dw, void* ws, const int* geom,
                int need_dx, int x_nhwc, int dy_nhwc, hipStream_t st) {
  const int N = geom[0], C = geom[1], H = geom[2], W = geom[3], K = geom[4], OH = geom[5], OW = geom[6];
  const int KH = geom[7], KW = geom[8], sh = geom[9], sw = geom[10], ph = geom[11], pw = geom[12], G = geom[13];
  const int Cg = C / G, Kg = K / G, Cp = round8(Cg), Kgp = round8(Kg);
  bf16_t* xt = (bf16_t*)ws;
  bf16_t* yt = xt + (int64_t)N * H * W * G * Cp;
  bf16_t* wp = yt + (int64_t)N * OH * OW * G * Kgp;
  const bf16_t* ysrc = (const bf16_t*)dy;
  if (!dy_nhwc) {
    launch_nhwc((const bf16_t*)dy, yt, N, G, Kg, OH * OW, Kgp, st);
    ysrc = yt;
  }
  if (need_dx) {
    const int Kp = kpad(KH, KW, Kgp);
    hipLaunchKernelGGL(conv_pack_kernel, dim3(ew_grid((int64_t)G * Cg * Kp, 256)), dim3(256), 0, st, (const bf16_t*)w,
                       wp, G, Kg, Cg, KH, KW, Kp, 1);
    IGemmArgs a{wp, ysrc, (bf16_t*)dx, nullptr, N, G, Cg, Kp, OH, OW, Kgp, H, W, KH, KW, sh, sw, ph, pw, 0, x_nhwc};
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
    // 64-channel tiles (the 128-channel variant measured no faster); split the pixels so that
    // about 1k workgroups run, each over at least 16 steps of 64 pixels (2k workgroups of 8+
    // steps measured slower: more atomics, more prologues; scripts/conv_probe.py)
    const int TC = 64;
    const int tiles = ((Kg + TC - 1) / TC) * ((Cg + TC - 1) / TC) * KH * KW * G;
    const int64_t nsteps = ((int64_t)N * OH * OW + 63) / 64;
    const int splits = (int)std::max<int64_t>(1, std::min<int64_t>((nsteps + 15) / 16, (1024 + tiles - 1) / tiles));
    WGradArgs b{ysrc, xsrc, dw, N, G, Kg, Kgp, Cg, Cp, H, W, OH, OW, KH, KW, sh, sw, ph, pw, splits};
    const dim3 grid((Kg + TC - 1) / TC, ((Cg + TC - 1) / TC) * KH * KW, G * splits);
    if (TC == 128) hipLaunchKernelGGL(conv_wgrad_kernel<128>, grid, dim3(256), 0, st, b);
    else hipLaunchKernelGGL(conv_wgrad_kernel<64>, grid, dim3(256), 0, st, b);
  }
}

}  // namespace ffk

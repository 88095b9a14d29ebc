// Implicit-GEMM convolutions over the (B, C, H, W) STFT image (H = 3, or 1 for
// Conv1d) on gfx950 fp32 MFMA (v_mfma_f32_16x16x4_f32, exact fp32 FMA chains).
//
// Every conv on the TimeVQVAE path has KH in {1,3} with PH = KH/2 (so H_out == H_in),
// a W stride SW in {1,2} and PW = (KW-1)/2.  Three gather forms cover all of them:
//
//  F  out[b,n,h,wo] = sum_{c,kh,kw} Wt(n,c,kh,kw) * In[b,c,h+kh-PH, wo*SW+kw-PW]
//       Conv2d fwd (zero or replicate pad), ConvTranspose2d dgrad
//  T  out[b,n,h,wo] = sum_{c,kh,kw} Wt(n,c,kh,kw) * In[b,c,h-kh+PH, (wo-kw+PW)/SW]
//       Conv2d dgrad, ConvTranspose2d fwd (terms with a fractional/out-of-range
//       source are zero)
//  W  dW(n,c,kh,kw) = sum_{b,h,w} G[b,n,h,w] * In[b,c,h+kh-PH, w*SW+kw-PW]
//       Conv2d / ConvTranspose2d weight gradients (split over positions,
//       deterministic slab reduction)
//
// GEMM orientation: MFMA rows = output channels n (A = weights), MFMA columns =
// output positions (B = gathered input), so each accumulator register holds 16
// consecutive positions of one channel and the NCHW stores are 64-B segments.
// Tiles are staged global -> registers -> LDS with the next K-step's loads in
// flight during the current step's MFMAs.
#include "tvq_common.h"
#include "tvq_reduce.h"

namespace tvq {

struct FastDiv {  // q = n / d for 0 <= n < 2^30, d >= 1
  uint32_t d;
  uint64_t magic;
  uint32_t shift;
};
static FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.shift = 32 + s;
  f.magic = ((1ull << f.shift) + d - 1) / d;
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (uint32_t)(((uint64_t)n * f.magic) >> f.shift);
}

// Geometry of one conv launch.  "In" is the gathered tensor (reduction channels C),
// "out"/"G" has N channels at positions (b, h, w) with w in [0, Wo).
struct ConvGeom {
  int B, C, Hin, Win;  // gathered tensor
  int N, Hout, Wo;     // output / G positions
  int oph, opw;        // pad offsets: F: hi = h+kh-oph, wi = wo*SW+kw-opw;  T: hi = h-kh+oph, wn = wo-kw+opw
  int64_t wsn, wsc;    // weight strides for (n, c); (kh, kw) contiguous: kh*KW + kw
  FastDiv fd_wo, fd_hwo;
  int Kred;            // C*KH*KW
  int Mpos;            // B*Hout*Wo
};

enum { GATHER_F = 0, GATHER_T = 1 };

// gathered input value for reduction index k at output position (b, h, wo)
template <int MODE, int KH, int KW, int SW, bool REPL>
__device__ __forceinline__ float gather_in(const float* __restrict__ in, const ConvGeom& g,
                                           const float* inb, int h, int wo, int k) {
  constexpr int KK = KH * KW;
  const int c = k / KK;
  const int r = k - c * KK;
  const int kh = r / KW, kw = r - kh * KW;
  if (c >= g.C) return 0.f;
  int hi, wi;
  if (MODE == GATHER_F) {
    hi = h + kh - g.oph;
    wi = wo * SW + kw - g.opw;
    if (REPL) {
      hi = hi < 0 ? 0 : (hi >= g.Hin ? g.Hin - 1 : hi);
      wi = wi < 0 ? 0 : (wi >= g.Win ? g.Win - 1 : wi);
    } else if (hi < 0 || hi >= g.Hin || wi < 0 || wi >= g.Win) {
      return 0.f;
    }
  } else {
    hi = h - kh + g.oph;
    const int wn = wo - kw + g.opw;
    if (hi < 0 || hi >= g.Hin || wn < 0) return 0.f;
    if (SW == 2 && (wn & 1)) return 0.f;
    wi = wn / SW;
    if (wi >= g.Win) return 0.f;
  }
  return inb[((int64_t)c * g.Hin + hi) * g.Win + wi];
}

// Epilogue options for F/T launches
struct Epi {
  const float* bias;      // [N] or null
  const float* residual;  // same layout as out, or null: out = residual + v
  float drop_p;           // dropout on v (before the residual add)
  float drop_scale;
  const int64_t* seed_ptr;
  uint64_t offset;
};

template <int MODE, int KH, int KW, int SW, bool REPL, int TN, int TM, int WN, int WM>
__global__ __launch_bounds__(256) void conv_gemm_kernel(const float* __restrict__ in,
                                                       const float* __restrict__ wt,
                                                       float* __restrict__ out, ConvGeom g,
                                                       Epi e) {
  constexpr int BK = 16;
  constexpr int KK = KH * KW;
  constexpr int FN = TN / WN / 16;  // MFMA tiles per wave along channels
  constexpr int FM = TM / WM / 16;  // along positions
  constexpr int SA = ((TN + 31) / 32) * 32 + 16;
  constexpr int SB = ((TM + 31) / 32) * 32 + 16;
  constexpr int A_PER = TN * BK / 256;  // weight elements per thread per K-step
  constexpr int B_PER = TM * BK / 256;  // input elements per thread per K-step
  static_assert(A_PER >= 1 && B_PER >= 1, "tile too small");
  __shared__ float As[BK * SA];
  __shared__ float Bs[BK * SB];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid % WN, wm = wid / WN;
  const int n0 = blockIdx.y * TN;
  const int m0 = blockIdx.x * TM;

  // per-thread fixed position for the B (input) loads
  const int bm_local = tid % TM;
  const int bk_base = tid / TM;
  constexpr int BK_STEP = 256 / TM;
  const int mpos = m0 + bm_local;
  const bool mvalid = mpos < g.Mpos;
  int pb = 0, ph = 0, pw = 0;
  if (mvalid) {
    const uint32_t bh = fdiv((uint32_t)mpos, g.fd_wo);
    pw = mpos - (int)bh * g.Wo;
    pb = (int)fdiv((uint32_t)mpos, g.fd_hwo);
    ph = (int)bh - pb * g.Hout;
  }
  const float* inb = in + (int64_t)pb * g.C * g.Hin * g.Win;
  // per-thread fixed channel for the A (weight) loads
  const int an_local = tid % TN;
  const int ak_base = tid / TN;
  constexpr int AK_STEP = 256 / TN;
  const int an = n0 + an_local;

  float ra[A_PER], rb[B_PER];
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int j = 0; j < A_PER; ++j) {
      const int k = k0 + ak_base + j * AK_STEP;
      float v = 0.f;
      if (an < g.N && k < g.Kred) {
        const int c = k / KK, r = k - c * KK;
        v = wt[an * g.wsn + c * g.wsc + r];
      }
      ra[j] = v;
    }
#pragma unroll
    for (int j = 0; j < B_PER; ++j) {
      const int k = k0 + bk_base + j * BK_STEP;
      rb[j] = (mvalid && k < g.Kred) ? gather_in<MODE, KH, KW, SW, REPL>(in, g, inb, ph, pw, k) : 0.f;
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int j = 0; j < A_PER; ++j) As[(ak_base + j * AK_STEP) * SA + an_local] = ra[j];
#pragma unroll
    for (int j = 0; j < B_PER; ++j) Bs[(bk_base + j * BK_STEP) * SB + bm_local] = rb[j];
  };

  floatx4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int r16 = lane & 15, g4 = lane >> 4;
  load_tile(0);
  for (int k0 = 0; k0 < g.Kred; k0 += BK) {
    __syncthreads();
    store_tile();
    __syncthreads();
    if (k0 + BK < g.Kred) load_tile(k0 + BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      float af[FN], bf[FM];
#pragma unroll
      for (int i = 0; i < FN; ++i) af[i] = As[(kk + g4) * SA + (wn * FN + i) * 16 + r16];
#pragma unroll
      for (int j = 0; j < FM; ++j) bf[j] = Bs[(kk + g4) * SB + (wm * FM + j) * 16 + r16];
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = mfma16x16x4(af[i], bf[j], acc[i][j]);
    }
  }

  const uint64_t seed = e.drop_p > 0.f ? mix_seed(e.seed_ptr, e.offset) : 0ull;
  // epilogue: acc[i][j][r] -> channel n0 + (wn*FN+i)*16 + 4*g4 + r, position m0 + (wm*FM+j)*16 + r16
#pragma unroll
  for (int j = 0; j < FM; ++j) {
    const int m = m0 + (wm * FM + j) * 16 + r16;
    if (m >= g.Mpos) continue;
    const uint32_t bh = fdiv((uint32_t)m, g.fd_wo);
    const int w = m - (int)bh * g.Wo;
    const int b = (int)fdiv((uint32_t)m, g.fd_hwo);
    const int h = (int)bh - b * g.Hout;
#pragma unroll
    for (int i = 0; i < FN; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + (wn * FN + i) * 16 + 4 * g4 + r;
        if (n >= g.N) continue;
        const int64_t o = (((int64_t)b * g.N + n) * g.Hout + h) * g.Wo + w;
        float v = acc[i][j][r];
        if (e.bias) v += e.bias[n];
        if (e.drop_p > 0.f) v = (uniform01(seed, (uint64_t)o) >= e.drop_p) ? v * e.drop_scale : 0.f;
        if (e.residual) v += e.residual[o];
        out[o] = v;
      }
    }
  }
}

// Weight gradient: rows = n (channels of G), cols = k' = (c, kh, kw), reduction over
// positions.  blockIdx.z = split index over positions; partial results go to
// slab[z][n][k'] and are summed in split order by wgrad_reduce_kernel.
template <int KH, int KW, int SW, bool REPL, int TN, int TK, int WN, int WK>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(const float* __restrict__ G,
                                                        const float* __restrict__ in,
                                                        float* __restrict__ slab, ConvGeom g,
                                                        int pos_per_split, int kcols) {
  // kcols = Kred (+1: a column of ones whose result is the bias gradient sum_m G[n, m])
  constexpr int BK = 16;  // positions per K-step
  constexpr int KK = KH * KW;
  constexpr int FN = TN / WN / 16;
  constexpr int FK = TK / WK / 16;
  constexpr int SA = ((TN + 31) / 32) * 32 + 16;
  constexpr int SB = ((TK + 31) / 32) * 32 + 16;
  constexpr int A_PER = TN * BK / 256;
  constexpr int B_PER = TK * BK / 256;
  static_assert(A_PER >= 1 && B_PER >= 1, "tile too small");
  __shared__ float As[BK * SA];
  __shared__ float Bs[BK * SB];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid % WN, wk = wid / WN;
  const int n0 = blockIdx.y * TN;
  const int kp0 = blockIdx.x * TK;
  const int p_begin = blockIdx.z * pos_per_split;
  const int p_end = min(g.Mpos, p_begin + pos_per_split);

  const int kk_t = tid % BK;  // each thread owns one position slot of the K-step
  const int a_nbase = tid / BK;
  const int b_kbase = tid / BK;

  float ra[A_PER], rb[B_PER];
  auto load_tile = [&](int p0) {
    const int p = p0 + kk_t;
    const bool pv = p < p_end;
    int b = 0, h = 0, w = 0;
    if (pv) {
      const uint32_t bh = fdiv((uint32_t)p, g.fd_wo);
      w = p - (int)bh * g.Wo;
      b = (int)fdiv((uint32_t)p, g.fd_hwo);
      h = (int)bh - b * g.Hout;
    }
    const float* gb = G + (((int64_t)b * g.N) * g.Hout + h) * g.Wo + w;
#pragma unroll
    for (int j = 0; j < A_PER; ++j) {
      const int n = n0 + a_nbase + j * 16;
      ra[j] = (pv && n < g.N) ? gb[(int64_t)n * g.Hout * g.Wo] : 0.f;
    }
    const float* inb = in + (int64_t)b * g.C * g.Hin * g.Win;
#pragma unroll
    for (int j = 0; j < B_PER; ++j) {
      const int kp = kp0 + b_kbase + j * 16;
      float v = (pv && kp == g.Kred && kp < kcols) ? 1.0f : 0.f;
      if (pv && kp < g.Kred) {
        const int c = kp / KK, r = kp - c * KK;
        const int kh = r / KW, kw = r - kh * KW;
        int hi = h + kh - g.oph, wi = w * SW + kw - g.opw;
        bool ok = true;
        if (REPL) {
          hi = hi < 0 ? 0 : (hi >= g.Hin ? g.Hin - 1 : hi);
          wi = wi < 0 ? 0 : (wi >= g.Win ? g.Win - 1 : wi);
        } else {
          ok = hi >= 0 && hi < g.Hin && wi >= 0 && wi < g.Win;
        }
        if (ok) v = inb[((int64_t)c * g.Hin + hi) * g.Win + wi];
      }
      rb[j] = v;
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int j = 0; j < A_PER; ++j) As[kk_t * SA + a_nbase + j * 16] = ra[j];
#pragma unroll
    for (int j = 0; j < B_PER; ++j) Bs[kk_t * SB + b_kbase + j * 16] = rb[j];
  };

  floatx4 acc[FN][FK];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int r16 = lane & 15, g4 = lane >> 4;
  if (p_begin < p_end) {
    load_tile(p_begin);
    for (int p0 = p_begin; p0 < p_end; p0 += BK) {
      __syncthreads();
      store_tile();
      __syncthreads();
      if (p0 + BK < p_end) load_tile(p0 + BK);
#pragma unroll
      for (int kk = 0; kk < BK; kk += 4) {
        float af[FN], bf[FK];
#pragma unroll
        for (int i = 0; i < FN; ++i) af[i] = As[(kk + g4) * SA + (wn * FN + i) * 16 + r16];
#pragma unroll
        for (int j = 0; j < FK; ++j) bf[j] = Bs[(kk + g4) * SB + (wk * FK + j) * 16 + r16];
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
          for (int j = 0; j < FK; ++j) acc[i][j] = mfma16x16x4(af[i], bf[j], acc[i][j]);
      }
    }
  }
  float* sl = slab + (int64_t)blockIdx.z * g.N * kcols;
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + (wn * FN + i) * 16 + 4 * g4 + r;
        const int kp = kp0 + (wk * FK + j) * 16 + r16;
        if (n < g.N && kp < kcols) sl[(int64_t)n * kcols + kp] = acc[i][j][r];
      }
}

// Fold the gradient of a replicate-padded input (B,C,H+2PH,W+2PW) onto (B,C,H,W).
__global__ void replicate_fold_kernel(const float* __restrict__ dpad, int B, int C, int H, int W,
                                      int PH, int PW, float* __restrict__ dx) {
  const int Hp = H + 2 * PH, Wp = W + 2 * PW;
  const int64_t tot = (int64_t)B * C * H * W;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < tot;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int w = (int)(i % W);
    const int64_t t = i / W;
    const int h = (int)(t % H);
    const int64_t bc = t / H;
    const float* p = dpad + bc * Hp * Wp;
    const int hlo = h == 0 ? 0 : h + PH, hhi = h == H - 1 ? Hp - 1 : h + PH;
    const int wlo = w == 0 ? 0 : w + PW, whi = w == W - 1 ? Wp - 1 : w + PW;
    float s = 0.f;
    for (int hh = hlo; hh <= hhi; ++hh)
      for (int ww = wlo; ww <= whi; ++ww) s += p[hh * Wp + ww];
    dx[i] = s;
  }
}

// Per-channel sum over (B, HW) of a (B, C, HW) tensor: out[c] (+)= sum. Two stages,
// deterministic.  Stage 1: partial[c][chunk]; stage 2: fixed-order sum.
__global__ __launch_bounds__(256) void chan_sum_partial_kernel(const float* __restrict__ x, int B,
                                                               int C, int HW, int chunks,
                                                               float* __restrict__ part) {
  __shared__ float red[4];
  const int c = blockIdx.x, ch = blockIdx.y;
  const int64_t per = ((int64_t)B * HW + chunks - 1) / chunks;
  const int64_t lo = ch * per, hi = min((int64_t)B * HW, lo + per);
  float s = 0.f;
  for (int64_t i = lo + threadIdx.x; i < hi; i += 256) {
    const int64_t b = i / HW, p = i - b * HW;
    s += x[(b * C + c) * HW + p];
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[(int64_t)c * chunks + ch] = s;
}
__global__ void chan_sum_final_kernel(const float* __restrict__ part, int C, int chunks,
                                      float* __restrict__ out, int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int i = 0; i < chunks; ++i) s += part[(int64_t)c * chunks + i];
  out[c] = accumulate ? out[c] + s : s;
}

// ---------------------------------------------------------------- host dispatch
static ConvGeom make_geom(int B, int C, int Hin, int Win, int N, int Hout, int Wo, int KH, int KW,
                          int oph, int opw, int64_t wsn, int64_t wsc) {
  ConvGeom g;
  g.B = B; g.C = C; g.Hin = Hin; g.Win = Win; g.N = N; g.Hout = Hout; g.Wo = Wo;
  g.oph = oph; g.opw = opw;
  g.wsn = wsn; g.wsc = wsc;
  g.fd_wo = make_fastdiv((uint32_t)Wo);
  g.fd_hwo = make_fastdiv((uint32_t)(Hout * Wo));
  g.Kred = C * KH * KW;
  g.Mpos = B * Hout * Wo;
  return g;
}

template <int MODE, int KH, int KW, int SW, bool REPL>
static void launch_gemm(const float* in, const float* wt, float* out, const ConvGeom& g,
                        const Epi& e, hipStream_t st) {
  // channel tile by output channel count; position tile keeps >= ~2 waves of blocks
  if (g.N <= 16) {
    dim3 grid((g.Mpos + 255) / 256, (g.N + 15) / 16);
    hipLaunchKernelGGL((conv_gemm_kernel<MODE, KH, KW, SW, REPL, 16, 256, 1, 4>), grid, dim3(256),
                       0, st, in, wt, out, g, e);
  } else if (g.N <= 32) {
    dim3 grid((g.Mpos + 127) / 128, (g.N + 31) / 32);
    hipLaunchKernelGGL((conv_gemm_kernel<MODE, KH, KW, SW, REPL, 32, 128, 2, 2>), grid, dim3(256),
                       0, st, in, wt, out, g, e);
  } else {
    dim3 grid((g.Mpos + 127) / 128, (g.N + 63) / 64);
    hipLaunchKernelGGL((conv_gemm_kernel<MODE, KH, KW, SW, REPL, 64, 128, 2, 2>), grid, dim3(256),
                       0, st, in, wt, out, g, e);
  }
}

template <int KH, int KW, int SW, bool REPL>
static void launch_wgrad(const float* G, const float* in, float* slab, int splits, int pps,
                         const ConvGeom& g, int kcols, hipStream_t st) {
  if (g.N <= 16) {
    dim3 grid((kcols + 63) / 64, (g.N + 15) / 16, splits);
    hipLaunchKernelGGL((conv_wgrad_kernel<KH, KW, SW, REPL, 16, 64, 1, 4>), grid, dim3(256), 0, st,
                       G, in, slab, g, pps, kcols);
  } else {
    dim3 grid((kcols + 63) / 64, (g.N + 63) / 64, splits);
    hipLaunchKernelGGL((conv_wgrad_kernel<KH, KW, SW, REPL, 64, 64, 2, 2>), grid, dim3(256), 0, st,
                       G, in, slab, g, pps, kcols);
  }
}

// kind: 0 = 3x4 s2 (EncBlock / ConvT), 1 = 3x3 s1, 2 = 1x1, 3 = 1x3 s1 (Conv1d k3)
#define TVQ_DISPATCH_KIND(kind, repl, MACRO)                                  \
  switch (kind) {                                                             \
    case 0: if (repl) { MACRO(3, 4, 2, true) } else { MACRO(3, 4, 2, false) } break; \
    case 1: MACRO(3, 3, 1, false) break;                                      \
    case 2: MACRO(1, 1, 1, false) break;                                      \
    case 3: MACRO(1, 3, 1, false) break;                                      \
    default: set_error("conv: unsupported kernel kind %d", kind); return TVQ_ERR_ARG; \
  }

static int kind_of(int KH, int KW, int SW) {
  if (KH == 3 && KW == 4 && SW == 2) return 0;
  if (KH == 3 && KW == 3 && SW == 1) return 1;
  if (KH == 1 && KW == 1 && SW == 1) return 2;
  if (KH == 1 && KW == 3 && SW == 1) return 3;
  return -1;
}

static int wgrad_splits(const ConvGeom& g, int tiles, int* pps) {
  // aim for ~1024 blocks, each with >= 512 positions
  int splits = (1024 + tiles - 1) / tiles;
  const int maxs = (g.Mpos + 511) / 512;
  if (splits > maxs) splits = maxs;
  if (splits < 1) splits = 1;
  if (splits > 256) splits = 256;
  int per = (g.Mpos + splits - 1) / splits;
  per = (per + 15) / 16 * 16;
  splits = (g.Mpos + per - 1) / per;
  *pps = per;
  return splits;
}

}  // namespace tvq

using namespace tvq;

static Epi make_epi(const float* bias, const float* residual, float drop_p,
                    const int64_t* seed_ptr, uint64_t offset) {
  Epi e;
  e.bias = bias;
  e.residual = residual;
  e.drop_p = drop_p;
  e.drop_scale = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
  e.seed_ptr = seed_ptr;
  e.offset = offset;
  return e;
}

extern "C" int tvq_conv_out_width(int64_t Win, int64_t KW, int64_t SW, int64_t transposed) {
  const int64_t PW = (KW - 1) / 2;
  return (int)(transposed ? (Win - 1) * SW - 2 * PW + KW : (Win + 2 * PW - KW) / SW + 1);
}

#define PH_OF(KH) ((int)(KH) / 2)
#define PW_OF(KW) (((int)(KW) - 1) / 2)

extern "C" int tvq_conv2d_fwd(const float* x, int64_t B, int64_t Ci, int64_t H, int64_t Wi,
                              const float* w, const float* bias, int64_t Co, int64_t KH,
                              int64_t KW, int64_t SW, int64_t replicate, float* y,
                              const float* residual, float drop_p, const int64_t* seed_ptr,
                              uint64_t offset, tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && w && y && B > 0 && Ci > 0 && Co > 0, "tvq_conv2d_fwd: bad arguments");
  const int kind = kind_of((int)KH, (int)KW, (int)SW);
  TVQ_CHECK_ARG(kind >= 0, "tvq_conv2d_fwd: unsupported kernel %lldx%lld s%lld", (long long)KH,
                (long long)KW, (long long)SW);
  const int Wo = tvq_conv_out_width(Wi, KW, SW, 0);
  TVQ_CHECK_ARG(Wo > 0 && B * H * Wo < (1 << 30), "tvq_conv2d_fwd: bad geometry");
  ConvGeom g = make_geom((int)B, (int)Ci, (int)H, (int)Wi, (int)Co, (int)H, Wo, (int)KH, (int)KW,
                         PH_OF(KH), PW_OF(KW), Ci * KH * KW, KH * KW);
  Epi e = make_epi(bias, residual, drop_p, seed_ptr, offset);
  hipStream_t st = (hipStream_t)stream;
#define M_(a, b_, c, d) launch_gemm<GATHER_F, a, b_, c, d>(x, w, y, g, e, st);
  TVQ_DISPATCH_KIND(kind, replicate, M_)
#undef M_
  return launch_status("tvq_conv2d_fwd");
}

extern "C" int tvq_convT2d_fwd(const float* x, int64_t B, int64_t Ci, int64_t H, int64_t Wi,
                               const float* w, const float* bias, int64_t Co, int64_t KH,
                               int64_t KW, int64_t SW, float* y, const float* residual,
                               tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && w && y && B > 0 && Ci > 0 && Co > 0, "tvq_convT2d_fwd: bad arguments");
  const int kind = kind_of((int)KH, (int)KW, (int)SW);
  TVQ_CHECK_ARG(kind >= 0, "tvq_convT2d_fwd: unsupported kernel");
  const int Wo = tvq_conv_out_width(Wi, KW, SW, 1);
  // ConvTranspose2d weight (Ci, Co, KH, KW): reduction channel c = ci (first dim)
  ConvGeom g = make_geom((int)B, (int)Ci, (int)H, (int)Wi, (int)Co, (int)H, Wo, (int)KH, (int)KW,
                         PH_OF(KH), PW_OF(KW), KH * KW, Co * KH * KW);
  Epi e = make_epi(bias, residual, 0.f, nullptr, 0);
  hipStream_t st = (hipStream_t)stream;
#define M_(a, b_, c, d) launch_gemm<GATHER_T, a, b_, c, false>(x, w, y, g, e, st);
  TVQ_DISPATCH_KIND(kind, 0, M_)
#undef M_
  return launch_status("tvq_convT2d_fwd");
}

extern "C" int64_t tvq_conv2d_dgrad_workspace(int64_t B, int64_t Ci, int64_t H, int64_t Wi,
                                              int64_t KH, int64_t KW, int64_t replicate) {
  if (!replicate) return 0;
  return B * Ci * (H + 2 * PH_OF(KH)) * (Wi + 2 * PW_OF(KW));
}

extern "C" int tvq_conv2d_dgrad(const float* dy, int64_t B, int64_t Co, int64_t H, int64_t Wo,
                                const float* w, int64_t Ci, int64_t KH, int64_t KW, int64_t SW,
                                int64_t replicate, float* dx, int64_t Wi, float* workspace,
                                tvq_stream_t stream) {
  TVQ_CHECK_ARG(dy && w && dx && B > 0 && Ci > 0 && Co > 0, "tvq_conv2d_dgrad: bad arguments");
  const int kind = kind_of((int)KH, (int)KW, (int)SW);
  TVQ_CHECK_ARG(kind >= 0, "tvq_conv2d_dgrad: unsupported kernel");
  TVQ_CHECK_ARG(tvq_conv_out_width(Wi, KW, SW, 0) == Wo, "tvq_conv2d_dgrad: Wi/Wo mismatch");
  hipStream_t st = (hipStream_t)stream;
  Epi e = make_epi(nullptr, nullptr, 0.f, nullptr, 0);
  // conv weight (Co, Ci, KH, KW): reduction c = co (first dim), output channel n = ci
  if (!replicate) {
    ConvGeom g = make_geom((int)B, (int)Co, (int)H, (int)Wo, (int)Ci, (int)H, (int)Wi, (int)KH,
                           (int)KW, PH_OF(KH), PW_OF(KW), KH * KW, Ci * KH * KW);
#define M_(a, b_, c, d) launch_gemm<GATHER_T, a, b_, c, false>(dy, w, dx, g, e, st);
    TVQ_DISPATCH_KIND(kind, 0, M_)
#undef M_
    return launch_status("tvq_conv2d_dgrad");
  }
  // replicate pad: gradient of the padded canvas (H+2PH, Wi+2PW) with zero offsets,
  // then fold the pad rows/columns onto the edges.
  TVQ_CHECK_ARG(workspace, "tvq_conv2d_dgrad: replicate needs a workspace");
  const int Hp = (int)H + 2 * PH_OF(KH), Wp = (int)Wi + 2 * PW_OF(KW);
  ConvGeom g = make_geom((int)B, (int)Co, (int)H, (int)Wo, (int)Ci, Hp, Wp, (int)KH, (int)KW, 0, 0,
                         KH * KW, Ci * KH * KW);
#define M_(a, b_, c, d) launch_gemm<GATHER_T, a, b_, c, false>(dy, w, workspace, g, e, st);
  TVQ_DISPATCH_KIND(kind, 0, M_)
#undef M_
  const int64_t tot = B * Ci * H * Wi;
  const int blocks = (int)((tot + 255) / 256 < 8192 ? (tot + 255) / 256 : 8192);
  hipLaunchKernelGGL(replicate_fold_kernel, dim3(blocks), dim3(256), 0, st, workspace, (int)B,
                     (int)Ci, (int)H, (int)Wi, PH_OF(KH), PW_OF(KW), dx);
  return launch_status("tvq_conv2d_dgrad(replicate)");
}

extern "C" int tvq_convT2d_dgrad(const float* dy, int64_t B, int64_t Co, int64_t H, int64_t Wo,
                                 const float* w, int64_t Ci, int64_t KH, int64_t KW, int64_t SW,
                                 float* dx, int64_t Wi, tvq_stream_t stream) {
  TVQ_CHECK_ARG(dy && w && dx && B > 0 && Ci > 0 && Co > 0, "tvq_convT2d_dgrad: bad arguments");
  const int kind = kind_of((int)KH, (int)KW, (int)SW);
  TVQ_CHECK_ARG(kind >= 0, "tvq_convT2d_dgrad: unsupported kernel");
  TVQ_CHECK_ARG(tvq_conv_out_width(Wi, KW, SW, 1) == Wo, "tvq_convT2d_dgrad: Wi/Wo mismatch");
  // F-gather of dY with weight (Ci, Co, KH, KW) indexed (n = ci, c = co)
  ConvGeom g = make_geom((int)B, (int)Co, (int)H, (int)Wo, (int)Ci, (int)H, (int)Wi, (int)KH,
                         (int)KW, PH_OF(KH), PW_OF(KW), Co * KH * KW, KH * KW);
  Epi e = make_epi(nullptr, nullptr, 0.f, nullptr, 0);
  hipStream_t st = (hipStream_t)stream;
#define M_(a, b_, c, d) launch_gemm<GATHER_F, a, b_, c, false>(dy, w, dx, g, e, st);
  TVQ_DISPATCH_KIND(kind, 0, M_)
#undef M_
  return launch_status("tvq_convT2d_dgrad");
}

// Weight gradient workspace (floats): split slabs [splits][N][Kred+1].
static int64_t wgrad_ws(int64_t N, int64_t Kred, int64_t Mpos, int* splits_out, int* pps_out) {
  ConvGeom g;
  g.Mpos = (int)Mpos;
  const int64_t kc = Kred + 1;
  const int tiles = (int)(((kc + 63) / 64) * ((N + (N <= 16 ? 15 : 63)) / (N <= 16 ? 16 : 64)));
  int pps;
  const int splits = wgrad_splits(g, tiles, &pps);
  if (splits_out) *splits_out = splits;
  if (pps_out) *pps_out = pps;
  return (int64_t)splits * N * kc + reduce_rows_scratch(splits, N * kc);
}

extern "C" int64_t tvq_conv_wgrad_workspace(int64_t N, int64_t C, int64_t KH, int64_t KW,
                                            int64_t B, int64_t Hout, int64_t Wo) {
  return wgrad_ws(N, C * KH * KW, B * Hout * Wo, nullptr, nullptr);
}

static void wgrad_finish(float* slab, int splits, int64_t N, int64_t kcols, float* dw,
                         float* db, int accumulate, hipStream_t st) {
  // deterministic split sum; kcols = Kred+1 splits out the bias column.  The level-1
  // scratch follows the slab in the workspace.
  reduce_rows(slab, splits, N * kcols, N * kcols, dw, db, kcols > 0 && db ? kcols : 0, accumulate,
              slab + (int64_t)splits * N * kcols, st);
}

// Conv2d weight (+bias) gradient: dW[co,ci,kh,kw] (+)= sum dY[b,co,h,wo] X[b,ci,h+kh-PH, wo*SW+kw-PW],
// db[co] (+)= sum dY[b,co,h,wo] (db may be NULL)
extern "C" int tvq_conv2d_wgrad(const float* x, int64_t B, int64_t Ci, int64_t H, int64_t Wi,
                                const float* dy, int64_t Co, int64_t Wo, int64_t KH, int64_t KW,
                                int64_t SW, int64_t replicate, float* dw, float* db,
                                int64_t accumulate, float* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && dy && dw && workspace, "tvq_conv2d_wgrad: bad arguments");
  const int kind = kind_of((int)KH, (int)KW, (int)SW);
  TVQ_CHECK_ARG(kind >= 0, "tvq_conv2d_wgrad: unsupported kernel");
  ConvGeom g = make_geom((int)B, (int)Ci, (int)H, (int)Wi, (int)Co, (int)H, (int)Wo, (int)KH,
                         (int)KW, PH_OF(KH), PW_OF(KW), Ci * KH * KW, KH * KW);
  int splits, pps;
  wgrad_ws(Co, g.Kred, g.Mpos, &splits, &pps);
  const int kcols = g.Kred + (db ? 1 : 0);
  hipStream_t st = (hipStream_t)stream;
#define M_(a, b_, c, d) launch_wgrad<a, b_, c, d>(dy, x, workspace, splits, pps, g, kcols, st);
  TVQ_DISPATCH_KIND(kind, replicate, M_)
#undef M_
  wgrad_finish(workspace, splits, Co, kcols, dw, db, (int)accumulate, st);
  return launch_status("tvq_conv2d_wgrad");
}

// ConvTranspose2d weight gradient: dW[ci,co,kh,kw] (+)= sum X[b,ci,h,wi] dY[b,co,h+kh-PH, wi*SW+kw-PW]
extern "C" int tvq_convT2d_wgrad(const float* x, int64_t B, int64_t Ci, int64_t H, int64_t Wi,
                                 const float* dy, int64_t Co, int64_t Wo, int64_t KH, int64_t KW,
                                 int64_t SW, float* dw, int64_t accumulate, float* workspace,
                                 tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && dy && dw && workspace, "tvq_convT2d_wgrad: bad arguments");
  const int kind = kind_of((int)KH, (int)KW, (int)SW);
  TVQ_CHECK_ARG(kind >= 0, "tvq_convT2d_wgrad: unsupported kernel");
  // G = X (N = Ci channels at X's positions), In = dY gathered F-style (C = Co)
  ConvGeom g = make_geom((int)B, (int)Co, (int)H, (int)Wo, (int)Ci, (int)H, (int)Wi, (int)KH,
                         (int)KW, PH_OF(KH), PW_OF(KW), Co * KH * KW, KH * KW);
  int splits, pps;
  wgrad_ws(Ci, g.Kred, g.Mpos, &splits, &pps);
  hipStream_t st = (hipStream_t)stream;
#define M_(a, b_, c, d) launch_wgrad<a, b_, c, false>(x, dy, workspace, splits, pps, g, g.Kred, st);
  TVQ_DISPATCH_KIND(kind, 0, M_)
#undef M_
  wgrad_finish(workspace, splits, Ci, g.Kred, dw, nullptr, (int)accumulate, st);
  return launch_status("tvq_convT2d_wgrad");
}

extern "C" int64_t tvq_channel_sum_workspace(int64_t B, int64_t C, int64_t HW) {
  if (HW == 1) {
    const int64_t r = reduce_rows_scratch(B, C);
    return r > 0 ? r : 1;
  }
  int64_t chunks = (B * HW + 8191) / 8192;
  if (chunks > 64) chunks = 64;
  if (chunks < 1) chunks = 1;
  return C * chunks;
}

// out[c] (+)= sum_{b,p} x[b,c,p]   (bias gradients), deterministic
extern "C" int tvq_channel_sum(const float* x, int64_t B, int64_t C, int64_t HW, float* out,
                               int64_t accumulate, float* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && out && workspace && B > 0 && C > 0 && HW > 0, "tvq_channel_sum: bad args");
  if (HW == 1) {  // row-major (B, C): coalesced column sums
    reduce_rows(x, B, C, C, out, nullptr, 0, (int)accumulate, workspace, (hipStream_t)stream);
    return launch_status("tvq_channel_sum");
  }
  const int64_t chunks = tvq_channel_sum_workspace(B, C, HW) / C;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(chan_sum_partial_kernel, dim3((int)C, (int)chunks), dim3(256), 0, st, x,
                     (int)B, (int)C, (int)HW, (int)chunks, workspace);
  hipLaunchKernelGGL(chan_sum_final_kernel, dim3((int)((C + 127) / 128)), dim3(128), 0, st,
                     workspace, (int)C, (int)chunks, out, (int)accumulate);
  return launch_status("tvq_channel_sum");
}

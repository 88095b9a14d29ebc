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
#include "tvq_conv_internal.h"
#include "tvq_gemm.h"

#include <stdlib.h>

#include <map>
#include <vector>

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
  int64_t wsn, wsc, wst;  // weight strides for (n, c, tap = kh*KW + kw)
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
  // eval-mode BatchNorm (+ Snake) applied to conv + bias before the dropout / residual
  // (VQVAEDecBlock / ResBlock's conv -> BN -> Snake while sampling; null: off)
  const float* bn_w;
  const float* bn_b;
  const float* bn_rm;
  const float* bn_rv;
  const float* snake_a;
  float bn_eps;
  int gelu;  // GELU (erf form) on conv + bias before the BN (Upscale: Conv1d -> GELU -> BN)
  // training BatchNorm statistics of the stored output (the stride-2 kernels' STATS form,
  // tvq_conv2d_fwd_bnstats): per-block (sum, sum of squares) in fp64 at
  // bn_part[(n * gridDim.x + blockIdx.x) * 2 + k]; null: off
  double* bn_part;
};

// bn_eval_snake_kernel's BN arithmetic (tvq_norm.hip) for channel n: v -> v sc + sh, then
// Snake (a = 0: none) with its sin^2 from sin2_cw (within ~1e-7 relative of sinf's)
struct PostCh {
  float sc, sh, a;
};
__device__ __forceinline__ PostCh epi_post_ch(const Epi& e, int n) {
  PostCh p;
  const float inv = 1.0f / sqrtf(e.bn_rv[n] + e.bn_eps);
  p.sc = (e.bn_w ? e.bn_w[n] : 1.f) * inv;
  p.sh = (e.bn_b ? e.bn_b[n] : 0.f) - e.bn_rm[n] * p.sc;
  p.a = e.snake_a ? e.snake_a[n] : 0.f;
  return p;
}
__device__ __forceinline__ float epi_post_apply(const PostCh& p, float v, bool gelu) {
  if (gelu) v = gelu_as(v);  // branch-free erf (tvq_common.h), ~1e-7 of tvq_gelu_fwd's
  float s = fmaf(v, p.sc, p.sh);
  if (p.a != 0.f) s = s + (1.0f / p.a) * sin2_cw(p.a * s);
  return s;
}
__device__ __forceinline__ float epi_post(const Epi& e, float v, int n) {
  return e.bn_rv ? epi_post_apply(epi_post_ch(e, n), v, e.gelu != 0) : v;
}

// Set by the launch paths whose epilogue applied Epi's BN / Snake (tvq_conv2d_fwd_bn_eval
// launches the standalone eval BN after any other path)
static thread_local bool t_post_done = false;

// Epilogue helpers.  Every global load here is unconditional (clamped index) so the
// compiler issues them together instead of one load + wait per element.
template <int FN>
__device__ __forceinline__ void epi_load_bias(float (&bv)[FN][4], const float* __restrict__ bias,
                                              int nbase, int N) {
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = min(nbase + i * 16 + r, N - 1);
      bv[i][r] = bias ? bias[n] : 0.f;
    }
}

// a[i][r]: channel nbase + i*16 + r at flat offset ob + n*hw (ob for a clamped position
// when !pv, so every address is in bounds)
// POST kernels: the per-channel BN / Snake terms of a lane's FN x 4 channels, loaded once
// before the epilogue's position loop (as epi_load_bias does for the bias)
template <int FN>
struct PostTile {
  PostCh c[FN][4];
};
template <int FN>
__device__ __forceinline__ void epi_load_post(PostTile<FN>& pt, const Epi& e, int nbase, int N) {
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) pt.c[i][r] = epi_post_ch(e, min(nbase + i * 16 + r, N - 1));
}

template <int FN, bool POST = false>
__device__ __forceinline__ void epi_store(float* __restrict__ out, const Epi& e, uint64_t seed,
                                          const float (&bv)[FN][4], const floatx4 (&a)[FN],
                                          int64_t ob, int64_t hw, int nbase, int N, bool pv,
                                          bool wt = false, const PostTile<FN>* pt = nullptr) {
  float v[FN][4];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) v[i][r] = a[i][r] + bv[i][r];
  if constexpr (POST) {  // a separate instantiation: its terms would crowd every conv's epilogue
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[i][r] = epi_post_apply(pt->c[i][r], v[i][r], e.gelu != 0);
  }
  if (e.drop_p > 0.f) {
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint64_t o = (uint64_t)(ob + (int64_t)(nbase + i * 16 + r) * hw);
        v[i][r] = uniform01(seed, o) >= e.drop_p ? v[i][r] * e.drop_scale : 0.f;
      }
  }
  if (e.residual) {
    float rv[FN][4];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        rv[i][r] = e.residual[ob + (int64_t)min(nbase + i * 16 + r, N - 1) * hw];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[i][r] += rv[i][r];
  }
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = nbase + i * 16 + r;
      if (pv && n < N) {
        if (wt) st_wt(out + ob + (int64_t)n * hw, v[i][r]);  // split-K slab, last-block finish
        else out[ob + (int64_t)n * hw] = v[i][r];
      }
    }
}

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
        v = wt[an * g.wsn + c * g.wsc + r * g.wst];
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
  const int nbase = n0 + wn * FN * 16 + 4 * g4;
  float bv[FN][4];
  epi_load_bias<FN>(bv, e.bias, nbase, g.N);
  const int64_t hw = (int64_t)g.Hout * g.Wo;
#pragma unroll
  for (int j = 0; j < FM; ++j) {
    const int m = m0 + (wm * FM + j) * 16 + r16;
    const bool pv = m < g.Mpos;
    const int mc = pv ? m : 0;
    const uint32_t bh = fdiv((uint32_t)mc, g.fd_wo);
    const int w = mc - (int)bh * g.Wo;
    const int b = (int)fdiv((uint32_t)mc, g.fd_hwo);
    const int h = (int)bh - b * g.Hout;
    floatx4 a[FN];
#pragma unroll
    for (int i = 0; i < FN; ++i) a[i] = acc[i][j];
    epi_store<FN>(out, e, seed, bv, a, ((int64_t)b * g.N * g.Hout + h) * g.Wo + w, hw, nbase, g.N,
                  pv);
  }
}

// Tap-major variant for C % 16 == 0: the K loop runs over (tap, channel block), so a
// thread's spatial source (and its validity) is computed once per tap and every
// gathered element costs one multiply-add and one predicated load.
template <int MODE, int KH, int KW, int SW, bool REPL, int TN, int TM, int WN, int WM, int BK,
          bool POST = false>
__global__ __launch_bounds__(256) void conv_tap_kernel(const float* __restrict__ in,
                                                      const float* __restrict__ wt,
                                                      float* __restrict__ out, ConvGeom g, Epi e,
                                                      int steps_per_split, int64_t zstride,
                                                      int* __restrict__ cnt,
                                                      float* __restrict__ fout, Epi fe) {
  // split-K (gridDim.z > 1): block z covers K-steps [z*sps, (z+1)*sps) and stores raw
  // partial sums to out + z*zstride (the caller passes a slab and a raw Epi); with
  // `cnt` the last split block of the tile then sums the slabs in split order and
  // applies the real epilogue `fe` into `fout` (what conv_splitk_epi_kernel does)
  constexpr int KK = KH * KW;
  constexpr int FN = TN / WN / 16;
  constexpr int FM = TM / WM / 16;
  constexpr int SA = ((TN + 31) / 32) * 32 + 16;
  constexpr int SB = ((TM + 31) / 32) * 32 + 16;
  constexpr int A_PER = TN * BK / 256;
  constexpr int B_PER = TM * BK / 256;
  constexpr int BK_STEP = 256 / TM;
  constexpr int AK_STEP = 256 / TN;
  static_assert(A_PER >= 1 && B_PER >= 1 && BK_STEP >= 1 && AK_STEP >= 1, "tile");
  __shared__ float As[BK * SA];
  __shared__ float Bs[BK * SB];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid % WN, wm = wid / WN;
  const int n0 = blockIdx.y * TN;
  const int m0 = blockIdx.x * TM;
  const int bm_local = tid % TM, bk_base = tid / TM;
  const int mpos = m0 + bm_local;
  const bool mvalid = mpos < g.Mpos;
  int pb = 0, ph = 0, pw = 0;
  if (mvalid) {
    const uint32_t bh = fdiv((uint32_t)mpos, g.fd_wo);
    pw = mpos - (int)bh * g.Wo;
    pb = (int)fdiv((uint32_t)mpos, g.fd_hwo);
    ph = (int)bh - pb * g.Hout;
  }
  const int64_t plane = (int64_t)g.Hin * g.Win;
  const float* inb = in + (int64_t)pb * g.C * plane;
  float* const slab = out;
  const int an_local = tid % TN, ak_base = tid / TN;
  const int an = n0 + an_local;
  const float* wrow = wt + (int64_t)(an < g.N ? an : 0) * g.wsn;
  const int csteps = (g.C + BK - 1) / BK;
  const int kbeg = blockIdx.z * steps_per_split;
  const int nsteps = min(KK * csteps, kbeg + steps_per_split);
  out += (int64_t)blockIdx.z * zstride;

  float ra[A_PER], rb[B_PER];
  auto load_tile = [&](int step) {
    const int tap = step / csteps;
    const int c0 = (step - tap * csteps) * BK;
    const int kh = tap / KW, kw = tap - kh * KW;
    int hi, wi;
    bool ok = mvalid;
    if (MODE == GATHER_F) {
      hi = ph + kh - g.oph;
      wi = pw * SW + kw - g.opw;
      if (REPL) {
        hi = hi < 0 ? 0 : (hi >= g.Hin ? g.Hin - 1 : hi);
        wi = wi < 0 ? 0 : (wi >= g.Win ? g.Win - 1 : wi);
      } else {
        ok = ok && hi >= 0 && hi < g.Hin && wi >= 0 && wi < g.Win;
      }
    } else {
      hi = ph - kh + g.oph;
      const int wn_ = pw - kw + g.opw;
      ok = ok && hi >= 0 && hi < g.Hin && wn_ >= 0 && (SW == 1 || (wn_ & 1) == 0);
      wi = wn_ / SW;
      ok = ok && wi < g.Win;
    }
    const float* src = inb + (ok ? (int64_t)hi * g.Win + wi : 0);
#pragma unroll
    for (int j = 0; j < B_PER; ++j) {
      const int c = c0 + bk_base + j * BK_STEP;
      rb[j] = (ok && c < g.C) ? src[(int64_t)c * plane] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < A_PER; ++j) {
      const int c = c0 + ak_base + j * AK_STEP;
      ra[j] = (an < g.N && c < g.C) ? wrow[(int64_t)c * g.wsc + tap * g.wst] : 0.f;
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
  if (kbeg < nsteps) load_tile(kbeg);
  for (int step = kbeg; step < nsteps; ++step) {
    __syncthreads();
    store_tile();
    __syncthreads();
    if (step + 1 < nsteps) load_tile(step + 1);
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
  const int nbase = n0 + wn * FN * 16 + 4 * g4;
  float bv[FN][4];
  epi_load_bias<FN>(bv, e.bias, nbase, g.N);
  PostTile<FN> pt;
  if constexpr (POST) epi_load_post<FN>(pt, e, nbase, g.N);
  const int64_t hw = (int64_t)g.Hout * g.Wo;
#pragma unroll
  for (int j = 0; j < FM; ++j) {
    const int m = m0 + (wm * FM + j) * 16 + r16;
    const bool pv = m < g.Mpos;
    const int mc = pv ? m : 0;
    const uint32_t bh = fdiv((uint32_t)mc, g.fd_wo);
    const int w = mc - (int)bh * g.Wo;
    const int b = (int)fdiv((uint32_t)mc, g.fd_hwo);
    const int h = (int)bh - b * g.Hout;
    floatx4 a[FN];
#pragma unroll
    for (int i = 0; i < FN; ++i) a[i] = acc[i][j];
    epi_store<FN, POST>(out, e, seed, bv, a, ((int64_t)b * g.N * g.Hout + h) * g.Wo + w, hw, nbase,
                        g.N, pv, cnt != nullptr, &pt);
  }
  if (cnt && last_block(cnt + blockIdx.y * gridDim.x + blockIdx.x, (int)gridDim.z)) {
    const uint64_t fseed = fe.drop_p > 0.f ? mix_seed(fe.seed_ptr, fe.offset) : 0ull;
    for (int idx = tid; idx < TM * TN; idx += 256) {
      const int m = m0 + idx % TM, n = n0 + idx / TM;
      if (m >= g.Mpos || n >= g.N) continue;
      const uint32_t bh = fdiv((uint32_t)m, g.fd_wo);
      const int w = m - (int)bh * g.Wo;
      const int b = (int)fdiv((uint32_t)m, g.fd_hwo);
      const int h = (int)bh - b * g.Hout;
      const int64_t o = (((int64_t)b * g.N + n) * g.Hout + h) * g.Wo + w;
      float v = 0.f;
#pragma unroll 4
      for (int z = 0; z < (int)gridDim.z; ++z) v += ld_wt(slab + (int64_t)z * zstride + o);
      if (fe.bias) v += fe.bias[n];
      v = epi_post(fe, v, n);
      if (fe.drop_p > 0.f) v = uniform01(fseed, (uint64_t)o) >= fe.drop_p ? v * fe.drop_scale : 0.f;
      if (fe.residual) v += fe.residual[o];
      fout[o] = v;
    }
  }
}

// Wide-channel implicit GEMM on v_mfma_f32_32x32x2_f32 for the C, N >= 128-class convs
// (128->128 ResBlock convs at W 32, the Upscale Conv1d pair, their dgrads).  Block tile
// 128 channels x 96 positions: 4 waves x 32 channels, each wave three 32x32
// accumulators, so one block per CU covers the 24,576-position maps in 256 blocks
// without split-K.  K runs tap-major over 64-channel stages (packed weights
// [tap][c][n], n contiguous -> dwordx4 loads); the next stage is loaded into registers
// while the current one feeds 96 MFMAs per wave from the other half of a
// double-buffered LDS tile (112 KB), one barrier per stage.  Loads are raw buffer loads:
// per-thread offsets are three position bases + compile-time row steps, and an invalid
// (padding) source gets an offset past the buffer end, which the hardware returns as 0.
// Each output is the same k-ordered fma chain as conv_tap_kernel's unsplit path
// (tap-major, channel order within a stage), so the two kernels agree bit for bit.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0,
                                           (int)(bytes < 0x7fffffff ? bytes : 0x7fffffff),
                                           0x00020000);
}

// TN = channel tile (128, or 64 for the 64-channel LF convs, whose grids are too small
// for 128 x 96 tiles and otherwise need split-K); NWN = TN / 32 channel tiles.
// NW = waves per block: NWN (TN = 128 only: each wave 32 channels x 96 positions, three
// accumulators) or 3 NWN (each wave one 32x32 tile, up to 3 waves per SIMD so one wave's
// barrier / address work hides behind the others' MFMAs; the first NWN waves stage the
// weights, the other 2 NWN the input).  Same k order in every variant.
template <int MODE, int KH, int KW, int SW, bool REPL, int BK, int NW, int TN, bool POST = false>
__global__ __launch_bounds__(NW * 64) void conv_t32_kernel(const float* __restrict__ in,
                                                      const float* __restrict__ wt,
                                                      float* __restrict__ out, ConvGeom g,
                                                      Epi e) {
  constexpr int TM = 96, NWN = TN / 32;
  constexpr bool SPLIT = NW == 3 * NWN;     // one tile per wave, staging split A | B
  static_assert(SPLIT || (NW == 4 && TN == 128), "t32 variant");
  constexpr int ATH = SPLIT ? 64 * NWN : 64 * NW;       // threads loading A
  constexpr int LB = SPLIT ? 128 * NWN : 64 * NW;       // threads loading B
  constexpr int ROWF4 = TN / 4;             // dwordx4 per A row (one k)
  constexpr int APASS = ATH / ROWF4;        // A rows per pass (8)
  constexpr int PSTEP = LB % 96;            // position step between a thread's B rows
  constexpr int KSTEP = 3 * LB / 96;        // k step per 3 B elements
  constexpr int A4 = BK / APASS;            // dwordx4 A loads per A-loading thread
  constexpr int BL = TM * BK / LB;          // dword B loads per B-loading thread
  static_assert(BK % APASS == 0, "A rows");
  constexpr int BAD = 0x40000000;        // offset past any buffer end -> loads 0
  extern __shared__ float smem[];
  float* As = smem;                      // [2][BK][TN]
  float* Bs = smem + 2 * BK * TN;        // [2][BK][TM]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  constexpr int NJ = SPLIT ? 1 : 3;  // 32-position tiles per wave
  const bool aload = !SPLIT || tid < ATH;
  const bool bload = !SPLIT || tid >= ATH;
  const int bt = SPLIT ? tid - ATH : tid;  // index among the B-loading threads
  const int wch = wid % NWN, wpos = (wid / NWN) * NJ;
  const int n0 = blockIdx.y * TN, m0 = blockIdx.x * TM;
  const int csteps = g.C / BK;
  const int nsteps = KH * KW * csteps;
  const int plane = g.Hin * g.Win;
  const __amdgpu_buffer_rsrc_t rin = buf_rsrc(in, (int64_t)g.B * g.C * plane * 4);
  const __amdgpu_buffer_rsrc_t rwt = buf_rsrc(wt, (int64_t)KH * KW * g.C * g.N * 4);

  // B element i (< BL) of this thread: e = bt + LB i -> position (bt + PSTEP (i%3)) % 96,
  // row k = (bt + LB (i%3)) / 96 + KSTEP (i/3)
  static_assert(BK % 8 == 0 && (TM * BK) % (3 * LB) == 0, "stage rows");
  int pm_b[3], pm_h[3], pm_w[3], krow[3];
  bool pm_ok[3];
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int m = m0 + (bt + PSTEP * u) % TM;
    krow[u] = (bt + LB * u) / TM;
    pm_ok[u] = m < g.Mpos;
    const int mc = pm_ok[u] ? m : 0;
    const uint32_t bh = fdiv((uint32_t)mc, g.fd_wo);
    pm_w[u] = mc - (int)bh * g.Wo;
    pm_b[u] = (int)fdiv((uint32_t)mc, g.fd_hwo);
    pm_h[u] = (int)bh - pm_b[u] * g.Hout;
  }
  const int a_k = tid / ROWF4, a_n = n0 + (tid % ROWF4) * 4;
  float4 ra[A4];
  float rb[BL];
  auto load = [&](int step) {
    const int tap = step / csteps;
    const int c0 = (step - tap * csteps) * BK;
    const int kh = tap / KW, kw = tap - kh * KW;
    if (aload) {
      const int abase = (((tap * g.C + c0 + a_k) * g.N) + a_n) * 4;
#pragma unroll
      for (int i = 0; i < A4; ++i)
        ra[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                               rwt, abase, i * APASS * g.N * 4, 0));
    }
    if (!bload) return;
    int boff[3];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      int hi, wi;
      bool v = pm_ok[u];
      if (MODE == GATHER_F) {
        hi = pm_h[u] + kh - g.oph;
        wi = pm_w[u] * SW + kw - g.opw;
        if (REPL) {
          hi = hi < 0 ? 0 : (hi >= g.Hin ? g.Hin - 1 : hi);
          wi = wi < 0 ? 0 : (wi >= g.Win ? g.Win - 1 : wi);
        } else {
          v = v && hi >= 0 && hi < g.Hin && wi >= 0 && wi < g.Win;
        }
      } else {
        hi = pm_h[u] - kh + g.oph;
        const int wn = pm_w[u] - kw + g.opw;
        v = v && hi >= 0 && hi < g.Hin && wn >= 0 && (SW == 1 || (wn & 1) == 0);
        wi = wn / SW;
        v = v && wi < g.Win;
      }
      boff[u] = v ? (((pm_b[u] * g.C + c0 + krow[u]) * plane) + hi * g.Win + wi) * 4 : BAD;
    }
#pragma unroll
    for (int i = 0; i < BL; ++i)
      rb[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                            rin, boff[i % 3], (i / 3) * KSTEP * plane * 4, 0));
  };
  auto store = [&](int buf) {
    if (aload) {
      float* a = As + buf * BK * TN + a_k * TN + (tid % ROWF4) * 4;
#pragma unroll
      for (int i = 0; i < A4; ++i) *reinterpret_cast<float4*>(a + i * APASS * TN) = ra[i];
    }
    if (bload) {
      float* bb = Bs + buf * BK * TM;
#pragma unroll
      for (int i = 0; i < BL; ++i) {
        const int u = i % 3;
        bb[(krow[u] + KSTEP * (i / 3)) * TM + (bt + PSTEP * u) % TM] = rb[i];
      }
    }
  };

  floatx16 acc[NJ];
#pragma unroll
  for (int jb = 0; jb < NJ; ++jb)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[jb][r] = 0.f;
  const int r32 = lane & 31, hl = lane >> 5;
  load(0);
  store(0);
  __syncthreads();
  for (int step = 0; step < nsteps; ++step) {
    const int buf = step & 1;
    if (step + 1 < nsteps) load(step + 1);
    const float* a = As + buf * BK * TN + hl * TN + wch * 32 + r32;
    const float* bb = Bs + buf * BK * TM + hl * TM + wpos * 32 + r32;
    // fragments of FG k-pairs are read one group ahead of the MFMAs that use them, so
    // the LDS latency hides behind FG*3 MFMAs instead of stalling every one or two
    constexpr int FG = 4, NG = BK / 2 / FG;
    float fa[2][FG], fb[2][FG][NJ];
    auto fread = [&](int grp, int slot) {
#pragma unroll
      for (int u = 0; u < FG; ++u) {
        const int kp = grp * FG + u;
        fa[slot][u] = a[2 * kp * TN];
#pragma unroll
        for (int jb = 0; jb < NJ; ++jb) fb[slot][u][jb] = bb[2 * kp * TM + jb * 32];
      }
    };
    fread(0, 0);
#pragma unroll
    for (int grp = 0; grp < NG; ++grp) {
      if (grp + 1 < NG) fread(grp + 1, (grp + 1) & 1);
#pragma unroll
      for (int u = 0; u < FG; ++u)
#pragma unroll
        for (int jb = 0; jb < NJ; ++jb)
          acc[jb] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[grp & 1][u], fb[grp & 1][u][jb],
                                                         acc[jb], 0, 0, 0);
      // emit the next group's LDS reads ahead of this group's MFMAs (T19)
      __builtin_amdgcn_sched_group_barrier(0x100, (1 + NJ) * FG, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, NJ * FG, 0);
    }
    if (step + 1 < nsteps) store(buf ^ 1);
    __syncthreads();
  }

  // epilogue: acc[jb][reg] = (channel n0 + 32 wch + (reg & 3) + 8 (reg >> 2) + 4 hl,
  // position m0 + 32 (wpos + jb) + lane % 32); bias, dropout, residual as epi_store
  const uint64_t seed = e.drop_p > 0.f ? mix_seed(e.seed_ptr, e.offset) : 0ull;
  const int64_t hw = (int64_t)g.Hout * g.Wo;
  PostCh pc[POST ? 16 : 1];  // POST: this lane's 16 channels' BN / Snake terms
  if constexpr (POST) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
      pc[r] = epi_post_ch(e, min(n0 + wch * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl, g.N - 1));
  }
#pragma unroll
  for (int jb = 0; jb < NJ; ++jb) {
    const int m = m0 + (wpos + jb) * 32 + r32;
    const bool pv = m < g.Mpos;
    const int mc = pv ? m : 0;
    const uint32_t bh = fdiv((uint32_t)mc, g.fd_wo);
    const int w = mc - (int)bh * g.Wo;
    const int b = (int)fdiv((uint32_t)mc, g.fd_hwo);
    const int h = (int)bh - b * g.Hout;
    const int64_t ob = ((int64_t)b * g.N * g.Hout + h) * g.Wo + w;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int n = n0 + wch * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
      if (!pv || n >= g.N) continue;
      const int64_t o = ob + (int64_t)n * hw;
      float v = acc[jb][r] + (e.bias ? e.bias[n] : 0.f);
      if constexpr (POST) v = epi_post_apply(pc[r], v, e.gelu != 0);
      if (e.drop_p > 0.f) v = uniform01(seed, (uint64_t)o) >= e.drop_p ? v * e.drop_scale : 0.f;
      if (e.residual) v += e.residual[o];
      out[o] = v;
    }
  }
}

// LDS per block: 2 stages x BK x (128 + 96) floats.  With 12 waves per block, BK = 64
// (112 KB, 18 barriers for a 3x3 128-channel conv) runs the 128->128 conv at 78.7 us vs
// 86.7 us for BK = 32 (56 KB); in the joint step, where the LDS is shared with the
// concurrent streams' kernels, the two are within 0.5 % (7.29 vs 7.25 ms).
#ifndef TVQ_T32_BK
#define TVQ_T32_BK 64
#endif
static int g_t32_bk = TVQ_T32_BK;  // K-stage depth: 64, or 32 / 16 (tvq_conv_config bit 16 / 32)
static int g_t32_nw = 12;  // waves per block (12, or 4 with tvq_conv_config bit 64)
// 64-channel tile for narrow maps (tvq_conv_config bit 128 turns it on).  Off by default:
// at the LF band's 64->64 3x3 conv (6144 positions, 64 blocks) it takes 27.5 us against
// 23.4 us for the split-K tap kernel + epilogue -- 9 K-stages of 32 MFMAs per wave leave
// each stage's load latency exposed; the grid needs split-K or a deeper prefetch.
static int g_t32_n64 = 0;
static size_t t32_lds(int bk, int tn) { return (size_t)2 * bk * (tn + 96) * 4; }

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
  // the thread's k' columns are fixed for the whole launch: decompose them once
  int bc_off[B_PER], bkh[B_PER], bkw[B_PER];
  unsigned bmask = 0u, bones = 0u;
#pragma unroll
  for (int j = 0; j < B_PER; ++j) {
    const int kp = kp0 + b_kbase + j * 16;
    const int c = kp / KK, r = kp - c * KK;
    bkh[j] = r / KW - g.oph;
    bkw[j] = r - (r / KW) * KW - g.opw;
    bc_off[j] = (kp < g.Kred) ? c * g.Hin * g.Win : 0;
    if (kp < g.Kred) bmask |= 1u << j;
    if (kp == g.Kred && kp < kcols) bones |= 1u << j;
  }

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
      float v = (pv && (bones >> j & 1u)) ? 1.0f : 0.f;
      if (pv && (bmask >> j & 1u)) {
        int hi = h + bkh[j], wi = w * SW + bkw[j];
        bool ok = true;
        if (REPL) {
          hi = hi < 0 ? 0 : (hi >= g.Hin ? g.Hin - 1 : hi);
          wi = wi < 0 ? 0 : (wi >= g.Win ? g.Win - 1 : wi);
        } else {
          ok = hi >= 0 && hi < g.Hin && wi >= 0 && wi < g.Win;
        }
        if (ok) v = inb[bc_off[j] + (int64_t)hi * g.Win + wi];
      }
      rb[j] = v;
    }
  };
  // rows of 16 positions, columns XOR-swizzled by (row & 14) as in gemm_kernel: the row
  // pitches are 16 mod 32 store banks, so unswizzled a half-wave's stores land on 16
  // banks (and with (row & 12) still 2-way).  Layout only (same k order, same results).
  auto store_tile = [&]() {
#pragma unroll
    for (int j = 0; j < A_PER; ++j) As[kk_t * SA + ((a_nbase + j * 16) ^ (kk_t & 14))] = ra[j];
#pragma unroll
    for (int j = 0; j < B_PER; ++j) Bs[kk_t * SB + ((b_kbase + j * 16) ^ (kk_t & 14))] = rb[j];
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
        const int swz = r16 ^ ((kk & 12) | (g4 & 2));  // sw(kk + g4)
#pragma unroll
        for (int i = 0; i < FN; ++i) af[i] = As[(kk + g4) * SA + (wn * FN + i) * 16 + swz];
#pragma unroll
        for (int j = 0; j < FK; ++j) bf[j] = Bs[(kk + g4) * SB + (wk * FK + j) * 16 + swz];
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

// Per-channel sum over (B, HW) of a (B, C, HW) tensor: out[c] (+)= sum, deterministic.
// Stage 1: partial[c][chunk], chunk = `ipc` whole images of channel c (contiguous HW rows,
// float4 loads, 4 in flight per thread); stage 2 (fixed xor tree over <= 64 partials, one
// load per lane) in the last block of channel c when `cnt` is given, else
// chan_sum_final_kernel.
__device__ __forceinline__ void chan_sum_final_one(const float* part, int chunks, int c,
                                                   float* out, int accumulate) {
  float s = 0.f;
  for (int i = 0; i < chunks; ++i) s += ld_wt(part + (int64_t)c * chunks + i);
  out[c] = accumulate ? out[c] + s : s;
}
__global__ __launch_bounds__(256) void chan_sum_partial_kernel(const float* __restrict__ x, int B,
                                                               int C, int HW, int ipc, int chunks,
                                                               int vec, float* __restrict__ part,
                                                               int* __restrict__ cnt,
                                                               float* __restrict__ out,
                                                               int accumulate) {
  __shared__ float red[4];
  const int c = blockIdx.x, ch = blockIdx.y;
  const int b0 = ch * ipc, b1 = min(B, b0 + ipc);
  float s = 0.f;
  if (vec) {
    const int hw4 = HW >> 2, n4 = (b1 - b0) * hw4;
    for (int i0 = threadIdx.x; i0 < n4; i0 += 256 * 4) {
      floatx4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * 256;
        const int bb = b0 + (i < n4 ? i : 0) / hw4, q = (i < n4 ? i : 0) % hw4;
        v[u] = *reinterpret_cast<const floatx4*>(x + ((int64_t)bb * C + c) * HW + 4 * q);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i0 + u * 256 < n4) s += (v[u][0] + v[u][1]) + (v[u][2] + v[u][3]);
    }
  } else {
    const int n = (b1 - b0) * HW;
    for (int i = threadIdx.x; i < n; i += 256) {
      const int bb = b0 + i / HW, p = i % HW;
      s += x[((int64_t)bb * C + c) * HW + p];
    }
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) st_wt(part + (int64_t)c * chunks + ch, s);
  if (cnt && last_block(cnt + c, chunks) && threadIdx.x < 64) {
    float t = threadIdx.x < chunks ? ld_wt(part + (int64_t)c * chunks + threadIdx.x) : 0.f;
    t = wave_sum(t);
    if (threadIdx.x == 0) out[c] = accumulate ? out[c] + t : t;
  }
}
__global__ void chan_sum_final_kernel(const float* __restrict__ part, int C, int chunks,
                                      float* __restrict__ out, int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  chan_sum_final_one(part, chunks, c, out, accumulate);
}

// ---------------------------------------------------------------- host dispatch
static ConvGeom make_geom(int B, int C, int Hin, int Win, int N, int Hout, int Wo, int KH, int KW,
                          int oph, int opw, int64_t wsn, int64_t wsc) {
  ConvGeom g;
  g.B = B; g.C = C; g.Hin = Hin; g.Win = Win; g.N = N; g.Hout = Hout; g.Wo = Wo;
  g.oph = oph; g.opw = opw;
  g.wsn = wsn; g.wsc = wsc; g.wst = 1;
  g.fd_wo = make_fastdiv((uint32_t)Wo);
  g.fd_hwo = make_fastdiv((uint32_t)(Hout * Wo));
  g.Kred = C * KH * KW;
  g.Mpos = B * Hout * Wo;
  return g;
}

// ---------------------------------------------------------------- halo-tile path
// For convolutions whose padded input image (Cp x HP x WP) and a weight panel of NB
// output channels (K = Cp*KK columns) fit in LDS together -- the small-channel ResBlock,
// encoder and decoder convs -- one block takes one image b and NB channels: both
// tiles are loaded once (batched so many loads are in flight per thread, one sync),
// then every MFMA operand is an LDS read: A from the panel, B from the halo image at
// h*WP + w*SW + koff[k], koff[k] = c*PS + kh*WP + kw from a per-block table.  There is
// no per-K-step global round trip, which is what bounds the staged GEMM at these sizes
// (a few hundred positions per image, K <= 576).
//   F  out[n,h,w] = sum W(n,c,kh,kw) In[c, h+kh-oh, w*SW+kw-ow]         (halo = In, padded)
//   T  out[n,h,w] = sum W(n,c,kh,kw) D[c, h+KH-1-kh, w+KW-1-kw]          (D = In dilated by SW,
//      oh = KH-1-PH, ow = KW-1-PW: the transposed gather as a stride-1 conv, taps flipped)
// The weight panel keeps the raw (c, kh, kw) column order, so it is a straight copy of
// the weight rows.  KS = 4 splits K across the 4 waves when the image has <= 4 position
// tiles (partials reduced through LDS).
struct HaloGeom {
  Div16 dv_hw, dv_wp, dv_wo, dv_k;
  int C, Cp, Hin, Win, N, Hout, Wo;
  int oh, ow;          // halo (hp, wp) -> source row hp - oh, col (wp - ow) [/SW for T]
  int HP, WP, PS;      // halo rows / cols; channel-plane stride (== 16 mod 32)
  int P, MT;           // positions per image, 16-position tiles per image
  int KST;             // weight-panel row stride (== 2 mod 32)
  int64_t wsn, wsc;    // raw weight strides of (n, c); taps contiguous
};

static constexpr int HALO_U = 8;  // loads in flight per thread in the load phase

template <int MODE, int KH, int KW, int SW, bool REPL>
__device__ __forceinline__ void halo_fill(float* __restrict__ Hs, const float* __restrict__ inb,
                                          int C, int Cp, int Hin, int Win, int HP, int WP, int PS,
                                          int oh, int ow, const Div16& dv_hw, const Div16& dv_wp,
                                          int tid) {
  const int hw = HP * WP;
  const int total = Cp * hw;
  for (int base = tid; base < total; base += 256 * HALO_U) {
    float v[HALO_U];
    int dst[HALO_U];
#pragma unroll
    for (int u = 0; u < HALO_U; ++u) {
      const int idx = base + u * 256;
      v[u] = 0.f;
      dst[u] = -1;
      if (idx < total) {
        const int c = div16(idx, dv_hw);
        const int r = idx - c * hw;
        const int hp = div16(r, dv_wp);
        const int wp = r - hp * WP;
        dst[u] = c * PS + r;
        if (c < C) {
          int hi = hp - oh;
          if (MODE == GATHER_F) {
            int wi = wp - ow;
            if (REPL) {
              hi = hi < 0 ? 0 : (hi >= Hin ? Hin - 1 : hi);
              wi = wi < 0 ? 0 : (wi >= Win ? Win - 1 : wi);
              v[u] = inb[((int64_t)c * Hin + hi) * Win + wi];
            } else if (hi >= 0 && hi < Hin && wi >= 0 && wi < Win) {
              v[u] = inb[((int64_t)c * Hin + hi) * Win + wi];
            }
          } else {
            const int wn = wp - ow;
            const int wi = wn / SW;
            if (hi >= 0 && hi < Hin && wn >= 0 && wn - wi * SW == 0 && wi < Win)
              v[u] = inb[((int64_t)c * Hin + hi) * Win + wi];
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < HALO_U; ++u)
      if (dst[u] >= 0) Hs[dst[u]] = v[u];
  }
}

template <int MODE, int KH, int KW, int SW, bool REPL, int FN, int KS, bool POST = false>
__global__ __launch_bounds__(256) void conv_halo_kernel(const float* __restrict__ in,
                                                       const float* __restrict__ wt,
                                                       float* __restrict__ out, HaloGeom g,
                                                       Epi e) {
  constexpr int KK = KH * KW;
  constexpr int NB = FN * 16;
  constexpr int CSW = MODE == GATHER_F ? SW : 1;  // position stride inside the halo
  extern __shared__ float smem[];
  const int K = g.Cp * KK;
  float* Hs = smem;                                  // [Cp][PS]
  float* As = Hs + g.Cp * g.PS;                      // [NB][KST], columns (c, kh, kw)
  int* koff = reinterpret_cast<int*>(As + NB * g.KST);  // [K]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int b = blockIdx.x;
  const int n0 = blockIdx.y * NB;

  // ---- load phase
  halo_fill<MODE, KH, KW, SW, REPL>(Hs, in + (int64_t)b * g.C * g.Hin * g.Win, g.C, g.Cp, g.Hin,
                                    g.Win, g.HP, g.WP, g.PS, g.oh, g.ow, g.dv_hw, g.dv_wp, tid);
  {
    // panel element (nn, k = c*KK + t); walk the raw weight in its contiguous order
    const bool n_inner = g.wsn < g.wsc;  // dgrad / convT layouts: (c, n, t)
    const int total = NB * K;
    for (int base = tid; base < total; base += 256 * HALO_U) {
      float v[HALO_U];
      int dst[HALO_U];
#pragma unroll
      for (int u = 0; u < HALO_U; ++u) {
        const int idx = base + u * 256;
        v[u] = 0.f;
        dst[u] = -1;
        if (idx < total) {
          int nn, c, t;
          if (n_inner) {
            t = idx % KK;
            const int r = idx / KK;
            c = r / NB;
            nn = r - c * NB;
          } else {
            nn = div16(idx, g.dv_k);
            const int k = idx - nn * K;
            c = k / KK;
            t = k - c * KK;
          }
          dst[u] = nn * g.KST + c * KK + t;
          const int n = n0 + nn;
          if (n < g.N && c < g.C) v[u] = wt[(int64_t)n * g.wsn + (int64_t)c * g.wsc + t];
        }
      }
#pragma unroll
      for (int u = 0; u < HALO_U; ++u)
        if (dst[u] >= 0) As[dst[u]] = v[u];
    }
    for (int k = tid; k < K; k += 256) {
      const int c = k / KK, t = k - c * KK;
      const int tl = MODE == GATHER_F ? t : KK - 1 - t;
      koff[k] = c * g.PS + (tl / KW) * g.WP + (tl % KW);
    }
  }
  __syncthreads();

  const int j = lane & 15, kq = lane >> 4;
  const int Q = K / 4;
  const uint64_t seed = e.drop_p > 0.f ? mix_seed(e.seed_ptr, e.offset) : 0ull;

  auto run = [&](int mt0, int mstep, int fa, int qs, int qe, floatx4 (&acc)[FN][4]) {
    int base[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int p = (mt0 + f * mstep) * 16 + j;
      const int pp = p < g.P ? p : 0;
      const int h = div16(pp, g.dv_wo);
      const int w = pp - h * g.Wo;
      base[f] = h * g.WP + w * CSW;
    }
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int f = 0; f < 4; ++f) acc[i][f] = floatx4{0.f, 0.f, 0.f, 0.f};
    const float* ap = As + j * g.KST + kq;
    for (int q = qs; q < qe; ++q) {
      const int ko = koff[q * 4 + kq];
      float af[FN];
#pragma unroll
      for (int i = 0; i < FN; ++i) af[i] = ap[i * 16 * g.KST + q * 4];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        if (f < fa) {
          const float bf = Hs[base[f] + ko];
#pragma unroll
          for (int i = 0; i < FN; ++i) acc[i][f] = mfma16x16x4(af[i], bf, acc[i][f]);
        }
      }
    }
  };
  const int nbase = n0 + kq * 4;
  float bv[FN][4];
  epi_load_bias<FN>(bv, e.bias, nbase, g.N);
  PostTile<FN> pt;
  if constexpr (POST) epi_load_post<FN>(pt, e, nbase, g.N);
  const int64_t hwo = (int64_t)g.Hout * g.Wo;
  auto store = [&](int mt, const floatx4 (&a)[FN]) {
    const int p = mt * 16 + j;
    const bool pv = p < g.P;
    const int pp = pv ? p : 0;
    const int h = div16(pp, g.dv_wo);
    const int w = pp - h * g.Wo;
    epi_store<FN, POST>(out, e, seed, bv, a, ((int64_t)b * g.N * g.Hout + h) * g.Wo + w, hwo,
                        nbase, g.N, pv, false, &pt);
  };

  floatx4 acc[FN][4];
  if (KS == 1) {
    for (int mt0 = wid; mt0 < g.MT; mt0 += 16) {
      const int fa = min(4, (g.MT - mt0 + 3) / 4);
      run(mt0, 4, fa, 0, Q, acc);
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        if (f < fa) {
          floatx4 a[FN];
#pragma unroll
          for (int i = 0; i < FN; ++i) a[i] = acc[i][f];
          store(mt0 + 4 * f, a);
        }
      }
    }
  } else {
    // MT <= 4: every wave takes all position tiles over a quarter of K
    const int fa = g.MT;
    const int qs = wid * Q / 4, qe = (wid + 1) * Q / 4;
    run(0, 1, fa, qs, qe, acc);
    __syncthreads();  // all waves done with the tiles: reuse LDS for the partials
    floatx4* red = reinterpret_cast<floatx4*>(smem);
    if (wid > 0) {
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int f = 0; f < 4; ++f)
          if (f < fa) red[(((wid - 1) * FN + i) * 4 + f) * 64 + lane] = acc[i][f];
    }
    __syncthreads();
    if (wid == 0) {
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        if (f < fa) {
          floatx4 a[FN];
#pragma unroll
          for (int i = 0; i < FN; ++i) {
            a[i] = acc[i][f];
#pragma unroll
            for (int wv = 0; wv < 3; ++wv) {
              const floatx4 t = red[((wv * FN + i) * 4 + f) * 64 + lane];
              a[i][0] += t[0]; a[i][1] += t[1]; a[i][2] += t[2]; a[i][3] += t[3];
            }
          }
          store(f, a);
        }
      }
    }
  }
}

// Direct convolution for few channels on both sides (C, N <= 16): the stride-2 encoder /
// decoder convs and the decoders' ConvTranspose tail (12 <-> 4 / 12 channels at W up to
// 512), where an MFMA tile would be mostly padding and the staged GEMMs are latency-bound.
// One thread owns two adjacent output positions for all N channels (32 fp32 accumulators),
// the weights sit in LDS as [c][tap][16 n] (float4 broadcast reads), the input is read
// through L1/L2; for the T gather (stride-2 transposed) the taps whose source is fractional
// are skipped per output parity with wave-uniform branches.  Same epilogue as epi_store.
constexpr int SMALL_NB = 16;
template <int MODE, int KH, int KW, int SW, bool REPL, int NB>
__global__ __launch_bounds__(256) void conv_small_kernel(const float* __restrict__ in,
                                                         const float* __restrict__ wt,
                                                         float* __restrict__ out, ConvGeom g,
                                                         Epi e) {
  constexpr int KK = KH * KW;
  __shared__ floatx4 ws4[SMALL_NB * KK * NB / 4];  // [c][t][n], c < C <= 12 (dispatch)
  float* ws = reinterpret_cast<float*>(ws4);
  for (int i = threadIdx.x; i < g.C * KK * NB; i += 256) {
    const int n = i % NB, ct = i / NB;
    const int c = ct / KK, t = ct - c * KK;
    ws[i] = n < g.N ? wt[(int64_t)n * g.wsn + (int64_t)c * g.wsc + t] : 0.f;
  }
  __syncthreads();
  const int wo2 = (g.Wo + 1) >> 1;
  const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (tid >= (int64_t)g.B * g.Hout * wo2) return;
  const int j = (int)(tid % wo2);
  const int64_t bh = tid / wo2;
  const int h = (int)(bh % g.Hout), b = (int)(bh / g.Hout);
  const int wo0 = 2 * j;
  float acc[2][NB];
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int n = 0; n < NB; ++n) acc[p][n] = 0.f;
  const float* inb = in + (int64_t)b * g.C * g.Hin * g.Win;
  for (int c = 0; c < g.C; ++c) {
    const float* inc = inb + (int64_t)c * g.Hin * g.Win;
#pragma unroll
    for (int kh = 0; kh < KH; ++kh) {
      int hi = MODE == GATHER_F ? h + kh - g.oph : h - kh + g.oph;
      bool hv = hi >= 0 && hi < g.Hin;
      if (REPL) {
        hi = hi < 0 ? 0 : (hi >= g.Hin ? g.Hin - 1 : hi);
        hv = true;
      }
      const float* row = inc + (int64_t)(hv ? hi : 0) * g.Win;
#pragma unroll
      for (int kw = 0; kw < KW; ++kw) {
        const floatx4* w4 = ws4 + ((c * KK + kh * KW + kw) * NB) / 4;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int wo = wo0 + p;
          int wi;
          bool ok;
          if (MODE == GATHER_F) {
            wi = wo * SW + kw - g.opw;
            ok = wi >= 0 && wi < g.Win;
            if (REPL) {
              wi = wi < 0 ? 0 : (wi >= g.Win ? g.Win - 1 : wi);
              ok = true;
            }
          } else {
            const int wn = wo - kw + g.opw;
            if (SW == 2 && ((wn & 1) != 0)) continue;  // parity: uniform per (p, kw)
            wi = wn / SW;
            ok = wn >= 0 && wi < g.Win;
          }
          ok = ok && hv && wo < g.Wo;
          const float v = ok ? row[ok ? wi : 0] : 0.f;
#pragma unroll
          for (int q = 0; q < NB / 4; ++q) {
            const floatx4 w = w4[q];
            acc[p][4 * q + 0] = fmaf(w[0], v, acc[p][4 * q + 0]);
            acc[p][4 * q + 1] = fmaf(w[1], v, acc[p][4 * q + 1]);
            acc[p][4 * q + 2] = fmaf(w[2], v, acc[p][4 * q + 2]);
            acc[p][4 * q + 3] = fmaf(w[3], v, acc[p][4 * q + 3]);
          }
        }
      }
    }
  }
  const uint64_t seed = e.drop_p > 0.f ? mix_seed(e.seed_ptr, e.offset) : 0ull;
  const int64_t hw = (int64_t)g.Hout * g.Wo;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int wo = wo0 + p;
    if (wo >= g.Wo) continue;
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      if (n >= g.N) continue;
      const int64_t o = ((int64_t)b * g.N + n) * hw + (int64_t)h * g.Wo + wo;
      float v = acc[p][n] + (e.bias ? e.bias[n] : 0.f);
      if (e.drop_p > 0.f) v = uniform01(seed, (uint64_t)o) >= e.drop_p ? v * e.drop_scale : 0.f;
      if (e.residual) v += e.residual[o];
      out[o] = v;
    }
  }
}

// ---------------------------------------------------------------- stride-2 small-channel
// The 3x4 stride-2 convs with <= 16 channels on both sides at the bands' full widths: the
// EncBlock convs (F, replicate padding), the decoders' ConvTranspose tails (T) and the data
// gradients of both (T into the replicate canvas / F).  The staged GEMMs above ran them at
// 0.02-0.1 of peak: 9 K-steps of 16 with a branchy per-element gather and two barriers
// each.  Here a block owns one image's 64-wide output segment on every output row: the input
// rows it reads (C x rows x the segment's columns) are staged in LDS once, zero / replicate
// padding applied while staging, and each wave runs its 16-position tiles as 16x16x4 MFMA
// chains (rows = output channels, weights held in registers; columns = positions, read from
// the staged rows).  F: k = (c, kh) x kw on the lane groups, every tap of the window is a
// term.  T (stride-2 gather): the output parity fixes which two kw have an integer source,
// so each wave takes one parity and its K is c x kh x {two kw} (half the taps, no zero terms).
constexpr int S2_SEG = 64;                 // output positions per segment
constexpr int S2_XRF = 2 * S2_SEG + 2;     // F: staged columns (stride 2, 4 taps)
constexpr int S2_XRT = S2_SEG / 2 + 4;     // T: staged columns (source offsets -2..2)

// STATS epilogue of the stride-2 kernels (4 waves): lane (r16, g4) holds its positions' sums
// of channels 4 g4 + r in s1 / s2 (fp64); the 16 lanes of a g4 group are combined by a fixed
// xor tree, the 4 waves in wave order, and each channel's block partial is written for
// bn_apply_part_kernel (tvq_norm.hip), which finishes the statistics in the consumer.
// Replaces the BatchNorm's separate statistics pass over the conv output (bn_stats_partial).
__device__ __forceinline__ void s2_bn_stats_block(double (&s1)[4], double (&s2)[4], int nbase,
                                                  int N, double* __restrict__ part) {
  __shared__ double red[4][16][2];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      s1[r] += __shfl_xor(s1[r], o, 64);
      s2[r] += __shfl_xor(s2[r], o, 64);
    }
  if ((lane & 15) == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      red[wid][nbase + r][0] = s1[r];
      red[wid][nbase + r][1] = s2[r];
    }
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (t < 2 * N) {
    const int n = t >> 1, k = t & 1;
    part[((int64_t)n * gridDim.x + blockIdx.x) * 2 + k] =
        ((red[0][n][k] + red[1][n][k]) + red[2][n][k]) + red[3][n][k];
  }
}

// F: out[b,n,h,wo] = sum_{c,kh,kw} w(n,c,kh,kw) in[b,c,h+kh-1,2wo+kw-opw], H = 3
template <bool REPL, int CS, bool POST = false, bool STATS = false>
__global__ __launch_bounds__(256) void conv_s2f_kernel(const float* __restrict__ in,
                                                       const float* __restrict__ wt,
                                                       float* __restrict__ out, ConvGeom g, Epi e) {
  constexpr int NS = 3 * CS, RS = 5;  // K-steps (c, kh); staged rows hi = -1..3
  constexpr int XN = CS * RS * S2_XRF, XPER = (XN + 255) / 256;
  __shared__ float Xs[XN];
  const int tid = threadIdx.x, lane = tid & 63, r16 = lane & 15, g4 = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int segs = (g.Wo + S2_SEG - 1) / S2_SEG;
  const int b = blockIdx.x / segs, w0 = (blockIdx.x - b * segs) * S2_SEG;
  // weights of row n = r16, tap kw = g4, step s = (c, kh)
  float af[NS];
  const int nr = r16 < g.N ? r16 : 0;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int c = s / 3, kh = s - 3 * c;
    const int cc = c < g.C ? c : 0;
    af[s] = wt[nr * g.wsn + cc * g.wsc + (kh * 4 + g4) * g.wst];
  }
  const float* inb = in + (int64_t)b * g.C * g.Hin * g.Win;
  float xv[XPER];
  uint64_t okm = 0;
#pragma unroll
  for (int u = 0; u < XPER; ++u) {
    const int i = tid + 256 * u;
    const int ck = i / S2_XRF, j = i - ck * S2_XRF, c = ck / RS, r = ck - RS * c;
    int hi = r - 1, wi = 2 * w0 - g.opw + j;
    bool ok = i < XN && c < g.C;
    if (REPL) {
      hi = hi < 0 ? 0 : (hi >= g.Hin ? g.Hin - 1 : hi);
      wi = wi < 0 ? 0 : (wi >= g.Win ? g.Win - 1 : wi);
    } else {
      ok = ok && hi >= 0 && hi < g.Hin && wi >= 0 && wi < g.Win;
    }
    xv[u] = inb[ok ? ((int64_t)c * g.Hin + hi) * g.Win + wi : 0];
    okm |= (uint64_t)(ok ? 1 : 0) << u;
  }
#pragma unroll
  for (int u = 0; u < XPER; ++u) {
    const int i = tid + 256 * u;
    if (i < XN) Xs[i] = (okm >> u & 1) ? xv[u] : 0.f;
  }
  float bv[1][4];
  const int nbase = 4 * g4;
  epi_load_bias<1>(bv, e.bias, nbase, g.N);
  __syncthreads();
  // 12 tiles (3 rows x 4 position groups of 16), 3 per wave
  floatx4 acc[3];
  const float* xb[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int tile = wid * 3 + t, h = tile >> 2, p0 = (tile & 3) * 16;
    xb[t] = Xs + h * S2_XRF + 2 * (p0 + r16) + g4;
    acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int c = s / 3, kh = s - 3 * c, off = (c * RS + kh) * S2_XRF;
#pragma unroll
    for (int t = 0; t < 3; ++t) acc[t] = mfma16x16x4(af[s], xb[t][off], acc[t]);
  }
  const uint64_t seed = e.drop_p > 0.f ? mix_seed(e.seed_ptr, e.offset) : 0ull;
  const int64_t hw = (int64_t)g.Hout * g.Wo;
  PostTile<1> pt;
  if constexpr (POST) epi_load_post<1>(pt, e, nbase, g.N);
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int tile = wid * 3 + t, h = tile >> 2;
    const int wo = w0 + (tile & 3) * 16 + r16;
    const bool pv = wo < g.Wo;
    const floatx4 a[1] = {acc[t]};
    epi_store<1, POST>(out, e, seed, bv, a, ((int64_t)b * g.N * g.Hout + h) * g.Wo + (pv ? wo : 0),
                       hw, nbase, g.N, pv, false, &pt);
  }
  if constexpr (STATS) {  // (no dropout / residual on this path: the stored value is acc + b)
    double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int tile = wid * 3 + t;
      if (w0 + (tile & 3) * 16 + r16 >= g.Wo) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double v = (double)(acc[t][r] + bv[0][r]);
        s1[r] += v;
        s2[r] += v * v;
      }
    }
    s2_bn_stats_block(s1, s2, nbase, g.N, e.bn_part);
  }
}

// T: out[b,n,h,wo] = sum w(n,c,kh,kw) in[b,c,h-kh+oph,(wo-kw+opw)/2] over the integer
// sources, Hin = 3, HO = Hout (3, or 5 for the replicate canvas).  FOLD (the data gradient
// of a replicate-padded conv): the canvas (5 rows, Wo = Wx + 2 columns) is folded onto
// out = dx (3 rows, Wx columns) in the epilogue -- rows 0+1, 2, 3+4; canvas columns 0 / Wx+1
// onto dx columns 0 / Wx-1 through LDS -- instead of a canvas store and a fold launch.
template <int CS, int HO, bool FOLD = false, bool POST = false, bool STATS = false>
__global__ __launch_bounds__(256) void conv_s2t_kernel(const float* __restrict__ in,
                                                       const float* __restrict__ wt,
                                                       float* __restrict__ out, ConvGeom g, Epi e) {
  constexpr int NS = 6 * CS / 4, RS = 7;  // K-steps; staged rows hi = -2..4
  constexpr int XN = CS * RS * S2_XRT, XPER = (XN + 255) / 256;
  __shared__ float Xs[XN];
  const int tid = threadIdx.x, lane = tid & 63, r16 = lane & 15, g4 = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int par = wid & 1, mb = wid >> 1;  // this wave's output parity and 16-column group
  const int segs = (g.Wo + S2_SEG - 1) / S2_SEG;
  const int b = blockIdx.x / segs, w0 = (blockIdx.x - b * segs) * S2_SEG;
  const int m0 = w0 >> 1;  // staged column j <-> source column m0 - 2 + j
  // step s, lane group g4: k = 4s + g4 = (c, kh, e), kw = q + 2e with q = (par + opw) & 1
  float af[NS];
  int soff[NS];
  const int nr = r16 < g.N ? r16 : 0, q = (par + g.opw) & 1;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int k = 4 * s + g4, c = k / 6, rem = k - 6 * c, kh = rem >> 1, kw = q + 2 * (rem & 1);
    const int cc = c < g.C ? c : 0;
    af[s] = wt[nr * g.wsn + cc * g.wsc + (kh * 4 + kw) * g.wst];
    soff[s] = (c * RS - kh) * S2_XRT + ((par + g.opw - kw) >> 1);
  }
  const float* inb = in + (int64_t)b * g.C * g.Hin * g.Win;
  float xv[XPER];
  uint32_t okm = 0;
  static_assert(XPER <= 32, "staging mask");
#pragma unroll
  for (int u = 0; u < XPER; ++u) {
    const int i = tid + 256 * u;
    const int ck = i / S2_XRT, j = i - ck * S2_XRT, c = ck / RS, r = ck - RS * c;
    const int hi = r - 2, wi = m0 - 2 + j;
    const bool ok = i < XN && c < g.C && hi >= 0 && hi < g.Hin && wi >= 0 && wi < g.Win;
    xv[u] = inb[ok ? ((int64_t)c * g.Hin + hi) * g.Win + wi : 0];
    okm |= (uint32_t)(ok ? 1 : 0) << u;
  }
#pragma unroll
  for (int u = 0; u < XPER; ++u) {
    const int i = tid + 256 * u;
    if (i < XN) Xs[i] = (okm >> u & 1) ? xv[u] : 0.f;
  }
  float bv[1][4];
  const int nbase = 4 * g4;
  epi_load_bias<1>(bv, e.bias, nbase, g.N);
  __syncthreads();
  floatx4 acc[HO];
  const float* xb = Xs + (g.oph + 2) * S2_XRT + mb * 16 + r16 + 2;
#pragma unroll
  for (int h = 0; h < HO; ++h) acc[h] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int h = 0; h < HO; ++h) acc[h] = mfma16x16x4(af[s], xb[h * S2_XRT + soff[s]], acc[h]);
  const int wo = w0 + 2 * (mb * 16 + r16) + par;
  if constexpr (FOLD) {
    static_assert(HO == 5, "fold: replicate canvas");
    __shared__ floatx4 ex[2][3][4];
    const int Wx = g.Wo - 2;
    floatx4 y[3] = {acc[0] + acc[1], acc[2], acc[3] + acc[4]};
    if (wo == 0 || wo == Wx + 1) {
#pragma unroll
      for (int h = 0; h < 3; ++h) ex[wo == 0 ? 0 : 1][h][g4] = y[h];
    }
    __syncthreads();
    if (wo == 1) {
#pragma unroll
      for (int h = 0; h < 3; ++h) y[h] = ex[0][h][g4] + y[h];
    } else if (wo == Wx) {
#pragma unroll
      for (int h = 0; h < 3; ++h) y[h] = y[h] + ex[1][h][g4];
    }
    const bool pv = wo >= 1 && wo <= Wx;
#pragma unroll
    for (int h = 0; h < 3; ++h)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = nbase + r;
        if (pv && n < g.N) out[(((int64_t)b * g.N + n) * 3 + h) * Wx + wo - 1] = y[h][r];
      }
    return;
  }
  const uint64_t seed = e.drop_p > 0.f ? mix_seed(e.seed_ptr, e.offset) : 0ull;
  const int64_t hw = (int64_t)g.Hout * g.Wo;
  const bool pv = wo < g.Wo;
  PostTile<1> pt;
  if constexpr (POST) epi_load_post<1>(pt, e, nbase, g.N);
#pragma unroll
  for (int h = 0; h < HO; ++h) {
    const floatx4 a[1] = {acc[h]};
    epi_store<1, POST>(out, e, seed, bv, a, ((int64_t)b * g.N * g.Hout + h) * g.Wo + (pv ? wo : 0),
                       hw, nbase, g.N, pv, false, &pt);
  }
  if constexpr (STATS) {
    double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
    if (pv) {
#pragma unroll
      for (int h = 0; h < HO; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const double v = (double)(acc[h][r] + bv[0][r]);
          s1[r] += v;
          s2[r] += v * v;
        }
    }
    s2_bn_stats_block(s1, s2, nbase, g.N, e.bn_part);
  }
}

static int g_conv_s2 = 1;  // conv_s2f / conv_s2t enabled (tvq_conv_config bit 512 turns them off)

// which stride-2 small-channel kernel takes this launch: 0 none, 1 F, 2 T (Hout 3), 3 T (5)
static int s2_kind(int mode, const ConvGeom& g) {
  if (!g_conv_s2 || g.C > 16 || g.N > 16 || g.Hin != 3) return 0;
  if (mode == GATHER_F)
    return g.Hout == 3 && g.oph == 1 && g.opw >= 0 && g.opw <= 2 ? 1 : 0;
  if (g.opw < 0 || g.opw > 3) return 0;
  if (g.Hout == 3 && g.oph == 1) return 2;
  if (g.Hout == 5 && g.oph == 0) return 3;
  return 0;
}

template <bool REPL>
static void launch_s2(int kind, const float* in, const float* wt, float* out, const ConvGeom& g,
                      const Epi& e, hipStream_t st) {
  const dim3 grid((unsigned)(g.B * ((g.Wo + S2_SEG - 1) / S2_SEG)));
  const int cs = (g.C + 3) / 4;
  TVQ_PLAN("conv_s2%s cs%d hout%d%s", kind == 1 ? "f" : "t", 4 * cs, g.Hout,
           e.bn_part ? " bnstats" : "");
#define S2F(CSV)                                                                                \
  do {                                                                                          \
    if (e.bn_part)                                                                              \
      hipLaunchKernelGGL((conv_s2f_kernel<REPL, CSV, false, true>), grid, dim3(256), 0, st, in,  \
                         wt, out, g, e);                                                        \
    else if (e.bn_rv)                                                                           \
      hipLaunchKernelGGL((conv_s2f_kernel<REPL, CSV, true>), grid, dim3(256), 0, st, in, wt, out, \
                         g, e);                                                                 \
    else                                                                                        \
      hipLaunchKernelGGL((conv_s2f_kernel<REPL, CSV>), grid, dim3(256), 0, st, in, wt, out, g, e); \
  } while (0)
#define S2T(CSV, HOV)                                                                            \
  do {                                                                                           \
    if (e.bn_part)                                                                               \
      hipLaunchKernelGGL((conv_s2t_kernel<CSV, HOV, false, false, true>), grid, dim3(256), 0, st, \
                         in, wt, out, g, e);                                                     \
    else if (e.bn_rv)                                                                            \
      hipLaunchKernelGGL((conv_s2t_kernel<CSV, HOV, false, true>), grid, dim3(256), 0, st, in, wt, \
                         out, g, e);                                                             \
    else                                                                                         \
      hipLaunchKernelGGL((conv_s2t_kernel<CSV, HOV>), grid, dim3(256), 0, st, in, wt, out, g, e); \
  } while (0)
  t_post_done = e.bn_rv != nullptr;
  if (kind == 1) {
    if (cs == 1) S2F(4); else if (cs == 2) S2F(8); else if (cs == 3) S2F(12); else S2F(16);
    return;
  }
  if (kind == 2) {
    if (cs == 1) S2T(4, 3); else if (cs == 2) S2T(8, 3); else if (cs == 3) S2T(12, 3); else S2T(16, 3);
  } else {
    if (cs == 1) S2T(4, 5); else if (cs == 2) S2T(8, 5); else if (cs == 3) S2T(12, 5); else S2T(16, 5);
  }
#undef S2F
#undef S2T
}

// data gradient of a replicate-padded conv straight into dx (canvas geometry g, Wx = Wo - 2):
// the canvas columns Wx and Wx + 1 must share a segment
static bool s2_fold_fits(const ConvGeom& g) {
  return s2_kind(GATHER_T, g) == 3 && g.Wo >= 4 && (g.Wo - 1) % S2_SEG != 0;
}
static void launch_s2_fold(const float* in, const float* wt, float* dx, const ConvGeom& g,
                           hipStream_t st) {
  const dim3 grid((unsigned)(g.B * ((g.Wo + S2_SEG - 1) / S2_SEG)));
  const Epi e = {nullptr, nullptr, 0.f, 1.f, nullptr, 0};
  const int cs = (g.C + 3) / 4;
  TVQ_PLAN("conv_s2t_fold cs%d", 4 * cs);
#define S2T(CSV) hipLaunchKernelGGL((conv_s2t_kernel<CSV, 5, true>), grid, dim3(256), 0, st, in, wt, dx, g, e)
  if (cs == 1) S2T(4); else if (cs == 2) S2T(8); else if (cs == 3) S2T(12); else S2T(16);
#undef S2T
}

// Weight (+ bias) gradient of the same stride-2 small-channel convs, in the F-gather form
// both directions share (conv2d: G = dY, In = x;  ConvTranspose2d: G = x, In = dY):
//   dW[n][c,kh,kw] = sum_{b,h,w} G[b,n,h,w] In[b,c,h+kh-1,2w+kw-opw],  db[n] = sum G
// A block (8 waves) walks stages of one image's 64-wide G segment on all 3 rows: the G rows
// (16 x 192) and the input rows they read (C x 5 x 130, padding applied while staging) go
// through LDS with the next stage's loads in flight.  Wave w owns k' tiles w%4, w%4+4, ...
// of the N x (12C+1) slab row for half of the stage's positions (w/4), so a k-step is one
// G read shared by its tiles; each lane's column pointer is fixed once (window cell, a
// ones plane for the bias column, a zeros plane past it).  The position halves are summed
// in order at the end; blocks write slab rows (<= 256, one deferred ordered sum).
constexpr int W2_T = 512, W2_GS = 3 * S2_SEG + 4, W2_KP = 2 * S2_XRF + 2 * S2_SEG + 8;
struct W2Geom {
  int B, C, N, Win, Wo, Kred, kcols, segs, spr, opw;
};

template <bool REPL, int CS>
__global__ __launch_bounds__(W2_T) void conv_wgrad_s2_kernel(const float* __restrict__ G,
                                                            const float* __restrict__ X,
                                                            float* __restrict__ slab, W2Geom g) {
  constexpr int RS = 5, XN = CS * RS * S2_XRF, XPER = (XN + W2_T - 1) / W2_T;
  constexpr int GN = 16 * 3 * S2_SEG, GPER = GN / W2_T;
  constexpr int KT = (12 * CS + 1 + 15) / 16, TPW = (KT + 3) / 4;
  constexpr int RED = 4 * TPW * 256;
  static_assert(XPER <= 32 && GN % W2_T == 0, "staging");
  __shared__ float Xs[XN > RED ? XN : RED];  // after the stages: the second half's tiles
  __shared__ float Gs[16 * W2_GS];
  __shared__ float K1[2 * W2_KP];  // ones | zeros
  const int tid = threadIdx.x, lane = tid & 63, r16 = lane & 15, g4 = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tg = wid & 3, ph = wid >> 2;  // tile group, position half
  const int nst = g.B * g.segs, z = blockIdx.x;
  const int s_begin = z * g.spr, s_end = min(nst, s_begin + g.spr);
  for (int i = tid; i < 2 * W2_KP; i += W2_T) K1[i] = i < W2_KP ? 1.f : 0.f;
  // this lane's column pointer per tile (position offsets added per k-step)
  const float* bp[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int kc = (tg + 4 * t) * 16 + r16;
    const int k = kc < g.Kred ? kc : 0, c = k / 12, rem = k - 12 * c, kh = rem >> 2;
    bp[t] = (kc < g.Kred ? Xs + (c * RS + kh) * S2_XRF + (rem & 3)
                         : (kc == g.Kred && g.kcols > g.Kred ? K1 : K1 + W2_KP)) + 2 * g4;
  }
  const float* ap = Gs + r16 * W2_GS + g4;
  float xv[XPER], gv[GPER];
  uint32_t okm = 0, gok = 0;
  auto load = [&](int s) {
    const int b = s / g.segs, w0 = (s - b * g.segs) * S2_SEG;
    const float* xb = X + (int64_t)b * g.C * 3 * g.Win;
#pragma unroll
    for (int u = 0; u < XPER; ++u) {
      const int i = tid + W2_T * u;
      const int ck = i / S2_XRF, j = i - ck * S2_XRF, c = ck / RS, r = ck - RS * c;
      int hi = r - 1, wi = 2 * w0 - g.opw + j;
      bool ok = i < XN && c < g.C;
      if (REPL) {
        hi = hi < 0 ? 0 : (hi > 2 ? 2 : hi);
        wi = wi < 0 ? 0 : (wi >= g.Win ? g.Win - 1 : wi);
      } else {
        ok = ok && hi >= 0 && hi < 3 && wi >= 0 && wi < g.Win;
      }
      xv[u] = xb[ok ? ((int64_t)c * 3 + hi) * g.Win + wi : 0];
      okm = u == 0 ? (ok ? 1u : 0u) : (okm | (ok ? 1u : 0u) << u);
    }
    const float* gb = G + (int64_t)b * g.N * 3 * g.Wo;
#pragma unroll
    for (int u = 0; u < GPER; ++u) {
      const int i = tid + W2_T * u;
      const int n = i / (3 * S2_SEG), p = i - n * (3 * S2_SEG), h = p / S2_SEG, w = w0 + p - h * S2_SEG;
      const bool ok = n < g.N && w < g.Wo;
      gv[u] = gb[ok ? ((int64_t)n * 3 + h) * g.Wo + w : 0];
      gok = u == 0 ? (ok ? 1u : 0u) : (gok | (ok ? 1u : 0u) << u);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < XPER; ++u) {
      const int i = tid + W2_T * u;
      if (i < XN) Xs[i] = (okm >> u & 1u) ? xv[u] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < GPER; ++u) {
      const int i = tid + W2_T * u;
      const int n = i / (3 * S2_SEG), p = i - n * (3 * S2_SEG);
      Gs[n * W2_GS + p] = (gok >> u & 1u) ? gv[u] : 0.f;
    }
  };
  floatx4 acc[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  if (s_begin < s_end) load(s_begin);
  for (int s = s_begin; s < s_end; ++s) {
    __syncthreads();  // the previous stage's reads are done
    store();
    __syncthreads();
    if (s + 1 < s_end) load(s + 1);  // in flight during this stage's chains
    // this half's 24 k-steps: positions p = 96 ph + 4 i + g4 (row p / 64, column p % 64)
#pragma unroll
    for (int i = 0; i < 24; ++i) {
      const int p0 = 96 * ph + 4 * i, h = p0 / S2_SEG, w = p0 - h * S2_SEG;
      const float a = ap[p0];
      const int off = h * S2_XRF + 2 * w;
#pragma unroll
      for (int t = 0; t < TPW; ++t) acc[t] = mfma16x16x4(a, bp[t][off], acc[t]);
    }
  }
  __syncthreads();
  floatx4* red = reinterpret_cast<floatx4*>(Xs);
  if (ph == 1) {
#pragma unroll
    for (int t = 0; t < TPW; ++t) red[(tg * TPW + t) * 64 + lane] = acc[t];
  }
  __syncthreads();
  if (ph == 0) {
    float* sl = slab + (int64_t)z * g.N * g.kcols;
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const floatx4 o = red[(tg * TPW + t) * 64 + lane];
      const int kc = (tg + 4 * t) * 16 + r16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = 4 * g4 + r;
        const float v = acc[t][r] + o[r];
        if (n < g.N && kc < g.kcols) sl[(int64_t)n * g.kcols + kc] = v;
      }
    }
  }
}

static int g_conv_ws2 = 1;  // conv_wgrad_s2_kernel enabled (tvq_conv_config bit 1024 turns it off)

static bool ws2_fits(int64_t C, int64_t H, int64_t N, int64_t KH, int64_t KW, int64_t SW) {
  return g_conv_ws2 && KH == 3 && KW == 4 && SW == 2 && H == 3 && C <= 16 && N <= 16;
}
static void ws2_plan(int64_t B, int64_t Wo, int* S, int* spr) {
  const int64_t nst = B * ((Wo + S2_SEG - 1) / S2_SEG);
  const int64_t s = nst < RR_ONE_ROWS ? nst : RR_ONE_ROWS;
  const int64_t per = (nst + s - 1) / s;
  *spr = (int)per;
  *S = (int)((nst + per - 1) / per);
}
static int64_t ws2_ws(int64_t B, int64_t C, int64_t Wo, int64_t N) {
  int S, spr;
  ws2_plan(B, Wo, &S, &spr);
  const int64_t kc = C * 12 + 1;
  return (int64_t)S * N * kc + reduce_rows_scratch(S, N * kc);
}
// G (B, N, 3, Wo) against In (B, C, 3, Win) -> slab rows; returns the row count
static int ws2_launch(const float* G, const float* X, float* slab, int B, int C, int N, int Win,
                      int Wo, int kcols, bool repl, hipStream_t st) {
  W2Geom w;
  w.B = B; w.C = C; w.N = N; w.Win = Win; w.Wo = Wo; w.Kred = 12 * C; w.kcols = kcols;
  w.segs = (Wo + S2_SEG - 1) / S2_SEG; w.opw = 1;
  int S;
  ws2_plan(B, Wo, &S, &w.spr);
  const int cs = (C + 3) / 4;
  TVQ_PLAN("conv_wgrad_s2 cs%d S=%d spr=%d", 4 * cs, S, w.spr);
#define W2L(R, CSV) hipLaunchKernelGGL((conv_wgrad_s2_kernel<R, CSV>), dim3(S), dim3(W2_T), 0, st, G, X, slab, w)
  if (repl) {
    if (cs == 1) W2L(true, 4); else if (cs == 2) W2L(true, 8); else if (cs == 3) W2L(true, 12); else W2L(true, 16);
  } else {
    if (cs == 1) W2L(false, 4); else if (cs == 2) W2L(false, 8); else if (cs == 3) W2L(false, 12); else W2L(false, 16);
  }
#undef W2L
  return S;
}

static int g_conv_small = 1;  // conv_small_kernel enabled (tvq_conv_config bit 256 turns it off)

static constexpr int HALO_LDS_MAX = 64 * 1024;

struct HaloPlan {
  HaloGeom g;
  int FN, KS;
  size_t lds;
};

// mode F: (oh, ow) = (PH, PW) of the conv;  T: (KH-1-oph, KW-1-opw) of the T gather
static bool halo_plan(int mode, int B, int C, int Hin, int Win, int N, int Hout, int Wo, int KH,
                      int KW, int SW, int oh, int ow, int64_t wsn, int64_t wsc, HaloPlan* pl) {
  HaloGeom g;
  g.C = C; g.Cp = (C + 3) & ~3; g.Hin = Hin; g.Win = Win; g.N = N; g.Hout = Hout; g.Wo = Wo;
  g.oh = oh; g.ow = ow;
  g.HP = Hout + KH - 1;
  g.WP = mode == GATHER_F ? (Wo - 1) * SW + KW : Wo + KW - 1;
  const int hw = g.HP * g.WP;
  g.PS = hw + ((16 - hw % 32) + 32) % 32;
  g.P = Hout * Wo;
  g.MT = (g.P + 15) / 16;
  g.wsn = wsn; g.wsc = wsc;
  const int K = KH * KW * g.Cp;
  if (Wo < 2 || g.WP < 2 || K < 2 || g.P >= (1 << 16)) return false;
  g.dv_hw = make_div16(hw);
  g.dv_wp = make_div16(g.WP);
  g.dv_wo = make_div16(Wo);
  g.dv_k = make_div16(K);
  const int KST = K + ((2 - K % 32) + 32) % 32;
  const int fn_cover = N <= 16 ? 1 : (N <= 32 ? 2 : 4);
  for (int FN = fn_cover; FN >= 1; FN /= 2) {
    const int NB = FN * 16;
    if ((N + NB - 1) / NB > 4) break;  // the image would be re-staged by > 4 blocks
    const int KS = g.MT <= 4 ? 4 : 1;
    size_t fl = (size_t)g.Cp * g.PS + (size_t)NB * KST + K;
    const size_t red = KS > 1 ? (size_t)3 * FN * 4 * 64 * 4 : 0;
    if (red > fl) fl = red;
    if (fl * 4 <= (size_t)HALO_LDS_MAX) {
      g.KST = KST;
      pl->g = g;
      pl->FN = FN;
      pl->KS = KS;
      pl->lds = fl * 4;
      return true;
    }
  }
  (void)B;
  return false;
}

template <int MODE, int KH, int KW, int SW, bool REPL>
static void launch_halo(const float* in, const float* wt, float* out, const HaloPlan& pl, int B,
                        const Epi& e, hipStream_t st) {
  const dim3 grid(B, (pl.g.N + pl.FN * 16 - 1) / (pl.FN * 16));
  // the eval EncBlock (replicate 3x4 stride-2 conv -> BN -> Snake): an epilogue-fused instance
  if constexpr (MODE == GATHER_F && KH == 3 && KW == 4 && SW == 2 && REPL) {
    if (e.bn_rv) {
      t_post_done = true;
#define HP_(FN_, KS_)                                                                             \
  hipLaunchKernelGGL((conv_halo_kernel<MODE, KH, KW, SW, REPL, FN_, KS_, true>), grid, dim3(256), \
                     pl.lds, st, in, wt, out, pl.g, e)
      if (pl.KS == 4) {
        if (pl.FN == 1) HP_(1, 4); else if (pl.FN == 2) HP_(2, 4); else HP_(4, 4);
      } else {
        if (pl.FN == 1) HP_(1, 1); else if (pl.FN == 2) HP_(2, 1); else HP_(4, 1);
      }
#undef HP_
      return;
    }
  }
#define H_(FN_, KS_)                                                                          \
  hipLaunchKernelGGL((conv_halo_kernel<MODE, KH, KW, SW, REPL, FN_, KS_>), grid, dim3(256), \
                     pl.lds, st, in, wt, out, pl.g, e)
  if (pl.KS == 4) {
    if (pl.FN == 1) H_(1, 4); else if (pl.FN == 2) H_(2, 4); else H_(4, 4);
  } else {
    if (pl.FN == 1) H_(1, 1); else if (pl.FN == 2) H_(2, 1); else H_(4, 1);
  }
#undef H_
}

// Halo-tile weight gradient: dW[n, c, tap] = sum_{b,h,w} G[b,n,h,w] In[b,c, h+kh-oh, w*SW+kw-ow]
// (+ a ones column for the bias gradient).  Block (s, nb, cb) loops over the images of
// split s; per image the G tile (NB x P) and the halo of CB input channels are loaded
// with all loads in flight, then the MFMAs reduce over the image's positions from LDS.
// Partials go to slab[s][n][kcols] and are summed in split order (wgrad_finish).
struct WHaloGeom {
  Div16 dv_hw, dv_wp, dv_gst;
  int B, C, Hin, Win, N, Hout, Wo;
  int oh, ow, HP, WP, PS;
  int P, GST, CB;
  int Kred, kcols;   // kcols = Kred (+1: bias column)
  int ips;           // images per split
};

template <int KH, int KW, int SW, bool REPL, int FN>
__global__ __launch_bounds__(256) void conv_wgrad_halo_kernel(const float* __restrict__ G,
                                                             const float* __restrict__ in,
                                                             float* __restrict__ slab,
                                                             WHaloGeom g) {
  constexpr int KK = KH * KW;
  constexpr int NB = FN * 16;
  extern __shared__ float smem[];
  float* Gs = smem;                     // [NB][GST]
  float* Hs = smem + NB * g.GST;        // [CB][PS], then a plane of ones
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int s = blockIdx.x;
  const int n0 = blockIdx.y * NB;
  const int c0 = blockIdx.z * g.CB;
  const int cbn = min(g.CB, g.C - c0);
  const bool last_cb = c0 + g.CB >= g.C;
  const int kb = cbn * KK + ((last_cb && g.kcols > g.Kred) ? 1 : 0);  // columns of this block
  const int KT = (kb + 15) / 16;
  const int j = lane & 15, kq = lane >> 4;

  for (int idx = tid; idx < g.PS; idx += 256) Hs[g.CB * g.PS + idx] = 1.0f;
  int koff[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int kl = (wid + 4 * t) * 16 + j;
    const int c = kl / KK, tap = kl - c * KK;
    koff[t] = kl < cbn * KK ? c * g.PS + (tap / KW) * g.WP + (tap % KW) : g.CB * g.PS;
  }
  const int ktw = wid < KT ? (KT - wid + 3) / 4 : 0;  // k-tiles of this wave (<= 4)

  floatx4 acc[FN][4];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[i][t] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int b_begin = s * g.ips, b_end = min(g.B, b_begin + g.ips);
  for (int b = b_begin; b < b_end; ++b) {
    __syncthreads();  // previous image consumed
    const float* gb = G + ((int64_t)b * g.N + n0) * g.P;
    const int gtot = NB * g.GST;
    for (int base = tid; base < gtot; base += 256 * HALO_U) {
      float v[HALO_U];
#pragma unroll
      for (int u = 0; u < HALO_U; ++u) {
        const int idx = base + u * 256;
        const int nn = div16(idx, g.dv_gst), m = idx - nn * g.GST;
        v[u] = (idx < gtot && m < g.P && n0 + nn < g.N) ? gb[(int64_t)nn * g.P + m] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < HALO_U; ++u)
        if (base + u * 256 < gtot) Gs[base + u * 256] = v[u];
    }
    halo_fill<GATHER_F, KH, KW, SW, REPL>(Hs, in + ((int64_t)b * g.C + c0) * g.Hin * g.Win, cbn,
                                          cbn, g.Hin, g.Win, g.HP, g.WP, g.PS, g.oh, g.ow,
                                          g.dv_hw, g.dv_wp, tid);
    __syncthreads();
    // positions m0..m0+3 lie in one row (Wo % 4 == 0); lane group kq takes m0 + kq
    int h0 = 0, w0 = 0;
    for (int m0 = 0; m0 < g.P; m0 += 4) {
      const int base = h0 * g.WP + (w0 + kq) * SW;
      float af[FN];
#pragma unroll
      for (int i = 0; i < FN; ++i) af[i] = Gs[(i * 16 + j) * g.GST + m0 + kq];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (t < ktw) {
          const float bf = Hs[base + koff[t]];
#pragma unroll
          for (int i = 0; i < FN; ++i) acc[i][t] = mfma16x16x4(af[i], bf, acc[i][t]);
        }
      }
      w0 += 4;
      if (w0 == g.Wo) { w0 = 0; ++h0; }
    }
  }
  float* out = slab + (int64_t)s * g.N * g.kcols;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (t >= ktw) continue;
    const int kl = (wid + 4 * t) * 16 + j;
    int kg;
    if (kl < cbn * KK) kg = c0 * KK + kl;
    else if (kl == cbn * KK && kb > cbn * KK) kg = g.Kred;
    else continue;
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + i * 16 + kq * 4 + r;
        if (n < g.N) out[(int64_t)n * g.kcols + kg] = acc[i][t][r];
      }
  }
}

// Weight (+ bias) gradient of a 3x3, stride-1, zero-padded conv on narrow (B, C, 3, W)
// maps (instantiated for W = 8: the LF band's 64 / 128-channel ResBlock convs):
//   dW[n][c*9 + tap] (+ dB[n]) = sum_{b, p} dY[b, n, p] * X[b, c, window(p, tap)].
// conv_wgrad_halo_kernel staged one image per step and wrote one 64 x 577 slab per 1-3
// images (43 MB of HBM traffic per op for 3.3 MB of algorithmic bytes).  Here block
// (s, nb, cb) owns a 32-row x (CB*9 [+1]) column tile and W8_IMG images, walked in stages of
// 4 (one per wave) through two LDS buffers: stage s + 1's dY rows (16-B loads) and input
// halo rows are in registers while stage s multiplies, and are stored behind its MFMAs
// (round 5; loading all 16 images before the first MFMA left the MFMA pipe idle through the
// load and the memory idle through the MFMAs, one 86 KB block per CU).  Each wave reduces
// its images over all of the tile's columns (5 x 2 independent 16x16x4 MFMA chains), and
// the 4 partial tiles are summed in wave order through LDS.  One slab row per W8_IMG
// images: S = B / W8_IMG splits, summed in order by the deferred slab sum.
#ifndef TVQ_W8_IMG
#define TVQ_W8_IMG 16
#endif
constexpr int W8_IMG = TVQ_W8_IMG;
constexpr int W8_STG = 4;  // images per pipeline stage (one per wave)

// up to 4 problems of one shape in a launch, stacked on blockIdx.y (the fused ResBlocks'
// conv1 / conv2 weight gradients, tvq_resblock_w8.hip / tvq_resblock.hip)
struct W8Probs {
  const float* G[4];
  const float* X[4];
  float* slab[4];
};

template <int W, int CB>
__global__ __launch_bounds__(256) void conv_wgrad_w8_kernel(W8Probs pr, int B, int C, int N,
                                                           int kcols, int PS) {
  constexpr int P = 3 * W, WP = W + 2;
  constexpr int GST = P + 4;                         // dY row stride in LDS (16-B aligned)
  constexpr int KB = CB * 9 + 1, KT = (KB + 15) / 16;  // columns (+ bias), 16-col tiles
  constexpr int TW = KT * 16;                        // combine-buffer row length
  extern __shared__ float smem[];
  // W8_STG images per stage (one per wave), two stage buffers: stage s + 1's loads are in
  // registers while stage s multiplies, and its LDS stores follow the MFMAs
  constexpr int STG = W8_STG, NSTG = W8_IMG / STG;
  static_assert(STG == 4 && W8_IMG % STG == 0, "one image per wave and stage");
  const int hs_img = (CB + 1) * PS;
  const int gbuf = STG * 32 * GST, hbuf = STG * hs_img;
  float* Gs = smem;                                  // [2][STG][32][GST]
  float* Hs = smem + 2 * gbuf;                       // [2][STG][CB + 1][PS] (plane CB: ones)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int j = lane & 15, kq = lane >> 4;
  // a multi-problem launch (conv_wgrad_w8_pair, conv_wgrad_wn_multi) stacks the problems of
  // the same shape on blockIdx.y
  const int nty = (N + 31) / 32, pb = (int)blockIdx.y / nty;
  const float* __restrict__ G = pr.G[pb];
  const float* __restrict__ X = pr.X[pb];
  float* __restrict__ slab = pr.slab[pb];
  const int s = blockIdx.x, n0 = ((int)blockIdx.y - pb * nty) * 32, c0 = blockIdx.z * CB;
  const bool bias = c0 + CB >= C && kcols > C * 9;   // this block also owns the bias column
  const int b0 = s * W8_IMG;
  const int ni = min(W8_IMG, B - b0);
  constexpr int GQ = P / 4, GN = STG * 32 * GQ, GU = (GN + 255) / 256;
  constexpr int XQ = W / 4, XN = STG * CB * 3 * XQ, XU = (XN + 255) / 256;
  float4 gv[GU], xv[XU];
  auto load = [&](int sg) {  // stage sg's dY rows and input rows into registers
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      const int e = tid + u * 256;
      const int ii = e / (32 * GQ), r = (e / GQ) % 32, q = e % GQ, im = sg * STG + ii;
      gv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < GN && im < ni && n0 + r < N)
        gv[u] = *reinterpret_cast<const float4*>(G + ((int64_t)(b0 + im) * N + n0 + r) * P + 4 * q);
    }
#pragma unroll
    for (int u = 0; u < XU; ++u) {
      const int e = tid + u * 256;
      const int ii = e / (CB * 3 * XQ), c = (e / (3 * XQ)) % CB, hq = e % (3 * XQ), im = sg * STG + ii;
      xv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < XN && im < ni && c0 + c < C)
        xv[u] = *reinterpret_cast<const float4*>(X + ((int64_t)(b0 + im) * C + c0 + c) * P + 4 * hq);
    }
  };
  auto store = [&](int buf) {  // the registers into stage buffer buf (interior cells only)
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      const int e = tid + u * 256;
      if (e < GN) {
        const int ii = e / (32 * GQ), r = (e / GQ) % 32, q = e % GQ;
        *reinterpret_cast<float4*>(Gs + buf * gbuf + (ii * 32 + r) * GST + 4 * q) = gv[u];
      }
    }
#pragma unroll
    for (int u = 0; u < XU; ++u) {
      const int e = tid + u * 256;
      if (e < XN) {
        const int ii = e / (CB * 3 * XQ), c = (e / (3 * XQ)) % CB, hq = e % (3 * XQ);
        const int h = hq / XQ, q = hq % XQ;
        float* d = Hs + buf * hbuf + ii * hs_img + c * PS + (h + 1) * WP + 1 + 4 * q;
        d[0] = xv[u].x; d[1] = xv[u].y; d[2] = xv[u].z; d[3] = xv[u].w;
      }
    }
  };
  load(0);
  // zero padding and the ones planes of both buffers (the stores only write interiors)
  for (int e = tid; e < 2 * hbuf; e += 256) Hs[e] = (e % hs_img) >= CB * PS ? 1.f : 0.f;
  __syncthreads();
  store(0);
  __syncthreads();
  int koff[KT];
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    const int kl = t * 16 + j, c = kl / 9, tap = kl - 9 * c;
    koff[t] = kl < CB * 9 ? c * PS + (tap / 3) * WP + (tap % 3) : CB * PS;
  }
  floatx4 acc[2][KT];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < KT; ++t) acc[i][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  // wave w reduces images w, w + 4, ... (stage by stage), as the unstaged form did
  for (int sg = 0; sg < NSTG; ++sg) {
    const int cur = sg & 1;
    if (sg + 1 < NSTG) load(sg + 1);
    if (sg * STG + wid < ni) {
      const float* gb = Gs + cur * gbuf + wid * 32 * GST + j * GST + kq;
      const float* hb = Hs + cur * hbuf + wid * hs_img + kq;
#pragma unroll
      for (int m0 = 0; m0 < P; m0 += 4) {
        const int base = (m0 / W) * WP + (m0 % W);   // positions m0 .. m0+3: one row
        const float a0 = gb[m0], a1 = gb[16 * GST + m0];
#pragma unroll
        for (int t = 0; t < KT; ++t) {
          const float bv = hb[base + koff[t]];
          acc[0][t] = mfma16x16x4(a0, bv, acc[0][t]);
          acc[1][t] = mfma16x16x4(a1, bv, acc[1][t]);
        }
      }
    }
    // buffer cur ^ 1 was last read in stage sg - 1, before the previous barrier
    if (sg + 1 < NSTG) store(cur ^ 1);
    __syncthreads();
  }
  // the last stage's barrier: Gs / Hs reads done, the combine buffer aliases them
  float* red = smem;  // [4 waves][32 rows][TW]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[(wid * 32 + i * 16 + 4 * kq + r) * TW + t * 16 + j] = acc[i][t][r];
  __syncthreads();
  const int kb = CB * 9 + (bias ? 1 : 0);
  float* out = slab + (int64_t)s * N * kcols;
  for (int e = tid; e < 32 * kb; e += 256) {
    const int row = e / kb, col = e - row * kb;
    const int n = n0 + row;
    if (n >= N) continue;
    const float v = ((red[row * TW + col] + red[(32 + row) * TW + col]) +
                     red[(64 + row) * TW + col]) + red[(96 + row) * TW + col];
    const int kg = col < CB * 9 ? c0 * 9 + col : C * 9;
    out[(int64_t)n * kcols + kg] = v;
  }
}

template <int W, int CB>
static size_t w8_lds(int PS) {
  constexpr int P = 3 * W, GST = P + 4;
  const size_t a = (size_t)2 * W8_STG * 32 * GST + (size_t)2 * W8_STG * (CB + 1) * PS;
  const size_t red = (size_t)4 * 32 * (((CB * 9 + 1 + 15) / 16) * 16);
  return 4 * (a > red ? a : red);
}

// the shapes conv_wgrad_w8_kernel takes
static bool w8_on() { return true; }
static bool w8_fits(int64_t B, int64_t C, int64_t H, int64_t Wi, int64_t N, int64_t Wo, int64_t KH,
                    int64_t KW, int64_t SW, int64_t replicate) {
  return w8_on() && KH == 3 && KW == 3 && SW == 1 && !replicate && H == 3 && Wi == Wo &&
         Wi == 8 && N % 32 == 0 && C % 8 == 0 && B % W8_IMG == 0;
}
static int64_t w8_ws(int64_t B, int64_t N, int64_t C) {
  const int64_t S = B / W8_IMG, kc = C * 9 + 1;
  return S * N * kc + reduce_rows_scratch(S, N * kc);
}

// Two weight (+ bias) gradients of the same 3x3 shape on (B, C, 3, 8) maps in one launch:
// the fused LF ResBlock's conv1 and conv2 (tvq_resblock_w8.hip).  Each problem's slab goes
// to its own workspace (w8_ws floats) and its own ordered sum.
static void w8_pair_launch(const float* x0, const float* dy0, float* ws0, float* dw0, float* db0,
                           const float* x1, const float* dy1, float* ws1, float* dw1, float* db1,
                           int64_t B, int64_t C, int64_t N, int accumulate, hipStream_t st);

// ---------------------------------------------------------------- wide-map weight gradient
// Weight (+ bias) gradient of stride-1 "same" 3x3 / 1x3 convs on maps whose rows are a
// multiple of 32 wide, with >= 64 output channels -- the HF band's 128 -> 128 and
// 16 -> 128 3x3 convs on (256, C, 3, 32) and the HF prior's Upscale Conv1d k3 on
// (256, C, 1, 96), 7.25 / 4.8 GFLOP each, where the split 16x16x4 kernel with 16-position
// LDS steps ran at ~0.3 of the fp32 MFMA peak.  A block owns a 128 (n) x 128 (k' = c*KK +
// tap) tile of one split of the positions; positions go in stages of one 32-wide row
// segment (b, h, w0 .. w0+31): the stage's dY rows (128 x 32, 16-B loads) and the input rows
// its k' columns need (channels k0/KK .. (k0+127)/KK, KH rows, 34 floats with the zero
// halo) are staged in LDS, double-buffered (the next stage's loads are in flight while this
// one multiplies), and each of the 8 waves runs 2 interleaved v_mfma_f32_32x32x2_f32 chains
// (32 n rows x 2 x 32 k' columns) over the stage's 16 position pairs.  The bias column
// (k' = Kred) is summed by the k0 = 0 blocks from the staged dY rows.  Slabs summed in
// split order (wgrad_finish).
constexpr int WT_T = 512, WT_AP = 128 + 4;  // threads; staged dY pitch ([p][n], n fastest)
template <int KH, int KW>
struct WtCfg {
  static constexpr int KK = KH * KW, NCH = 128 / KK + 2;  // channels a 128-column tile spans
  static constexpr int XROW = 34, XCH = KH * XROW;        // staged row, floats per channel
  static constexpr int AS = 32 * WT_AP, XS = NCH * XCH;   // floats per stage buffer
  static constexpr int XPER = (XS + WT_T - 1) / WT_T;     // input loads per thread
  static_assert(XPER <= 32, "staging mask");
};

struct WtGeom {
  int B, C, N, H, W, Kred, kcols;
  int segs;    // 32-wide segments per row (W / 32)
  int spr;     // stages per split
  int ntiles;  // 128-row n tiles
};

__device__ __forceinline__ int wt_crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

template <int KH, int KW>
struct WtRegs {  // one stage's global loads, in flight until stored to LDS
  float4 ga[2];
  float xv[WtCfg<KH, KW>::XPER];
  uint32_t ok;
};

template <int KH, int KW>
__global__ __launch_bounds__(WT_T) void conv_wgrad_t32_kernel(const float* __restrict__ G,
                                                             const float* __restrict__ X,
                                                             float* __restrict__ slab, WtGeom g,
                                                             int ktiles) {
  using R = WtCfg<KH, KW>;
  using Regs = WtRegs<KH, KW>;
  constexpr int PH = KH / 2, PW = (KW - 1) / 2;
  __shared__ float As[2][R::AS];
  __shared__ float Xs[2][R::XS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wid & 3, wk = wid >> 2;
  // XCD-aware map (tvq_gemm.h xcd_tile): the k' / n tiles of one position split share an
  // XCD, so its dY rows are fetched into one L2 and re-read from there
  int z, tile;
  xcd_tile((int)blockIdx.x, ktiles * g.ntiles, &z, &tile);
  const int nst = g.B * g.H * g.segs;
  const int s_begin = z * g.spr, s_end = min(nst, s_begin + g.spr);
  if (s_begin >= nst) return;  // padding block of the XCD map (no split)
  const int k0 = (tile % ktiles) * 128, n0 = (tile / ktiles) * 128;
  const int c_lo = k0 / R::KK;
  // this lane's B-operand offsets into a stage's Xs: columns k' = k0 + 64 wk + 32 j + l % 32
  // (past Kred: a valid column, never stored)
  int boff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    int kp = k0 + wk * 64 + j * 32 + (lane & 31);
    kp = kp < g.Kred ? kp : g.Kred - 1;
    const int c = kp / R::KK, t = kp - c * R::KK, kh = t / KW, kw = t - kh * KW;
    boff[j] = (c - c_lo) * R::XCH + kh * R::XROW + kw;
  }
  auto load = [&](Regs& q, int s) {
    if (s >= s_end) return;
    const int row = s / g.segs, w0 = (s - row * g.segs) * 32;
    const int b = row / g.H, h = row - b * g.H;
#pragma unroll
    for (int j = 0; j < 2; ++j) {  // dY: 128 rows x 32 positions, 8 threads per row
      const int e = tid + j * WT_T, n = e >> 3, p4 = (e & 7) * 4;
      const int nn = n0 + n < g.N ? n0 + n : g.N - 1;
      q.ga[j] = *(const float4*)(G + ((int64_t)(b * g.N + nn) * g.H + h) * g.W + w0 + p4);
    }
    q.ok = 0u;
#pragma unroll
    for (int u = 0; u < R::XPER; ++u) {  // input rows: (channel, kh, 34 columns)
      const int e = tid + u * WT_T;
      const int c = e / R::XCH, r = e - c * R::XCH, kh = r / R::XROW, jj = r - kh * R::XROW;
      const int cc = c_lo + c, hi = h + kh - PH, wi = w0 - PW + jj;
      const bool ok = e < R::XS && cc < g.C && hi >= 0 && hi < g.H && wi >= 0 && wi < g.W;
      q.xv[u] = X[ok ? ((int64_t)(b * g.C + cc) * g.H + hi) * g.W + wi : 0];
      q.ok |= (ok ? 1u : 0u) << u;
    }
  };
  auto store = [&](const Regs& q, int buf) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int e = tid + j * WT_T, n = e >> 3, p4 = (e & 7) * 4;
      float* d = As[buf] + p4 * WT_AP + n;
      d[0] = q.ga[j].x;
      d[WT_AP] = q.ga[j].y;
      d[2 * WT_AP] = q.ga[j].z;
      d[3 * WT_AP] = q.ga[j].w;
    }
#pragma unroll
    for (int u = 0; u < R::XPER; ++u) {
      const int e = tid + u * WT_T;
      if (e < R::XS) Xs[buf][e] = (q.ok >> u & 1u) ? q.xv[u] : 0.f;
    }
  };
  floatx16 acc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  float bsum = 0.f;  // bias partial of row n0 + tid (k0 == 0 blocks, tid < 128)
  // stage i: LDS buffer i & 1; two stages' loads in flight ahead of the one multiplying
  auto body = [&](int s, const Regs& next, Regs& free) {
    const int buf = (s - s_begin) & 1;
    load(free, s + 2);
    const float* as = As[buf] + wn * 32 + (lane & 31);
    const float* xs = Xs[buf];
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      const int p = 2 * st + (lane >> 5);
      const float a = as[p * WT_AP];
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, xs[boff[j] + p], acc[j], 0, 0, 0);
    }
    if (k0 == 0 && tid < 128) {
#pragma unroll 8
      for (int p = 0; p < 32; ++p) bsum += As[buf][p * WT_AP + tid];
    }
    if (s + 1 < s_end) store(next, buf ^ 1);
    __syncthreads();
  };
  Regs r0, r1;
  load(r0, s_begin);
  load(r1, s_begin + 1);
  store(r0, 0);
  __syncthreads();
  for (int s = s_begin; s < s_end; s += 2) {
    body(s, r1, r0);                       // r1: stage s+1; r0 <- stage s+2
    if (s + 1 < s_end) body(s + 1, r0, r1);  // r0: stage s+2; r1 <- stage s+3
  }
  float* sl = slab + (int64_t)z * g.N * g.kcols;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int kp = k0 + wk * 64 + j * 32 + (lane & 31);
    if (kp >= g.Kred) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int n = n0 + wn * 32 + wt_crow(r, lane >> 5);
      if (n < g.N) sl[(int64_t)n * g.kcols + kp] = acc[j][r];
    }
  }
  if (k0 == 0 && tid < 128 && g.kcols > g.Kred && n0 + tid < g.N)
    sl[(int64_t)(n0 + tid) * g.kcols + g.Kred] = bsum;
}

// the shapes the wide-map weight-gradient kernel takes
static bool wt32_fits(int64_t B, int64_t C, int64_t H, int64_t Wi, int64_t N, int64_t Wo,
                      int64_t KH, int64_t KW, int64_t SW, int64_t replicate) {
  return SW == 1 && !replicate && KW == 3 && (KH == 1 || KH == 3) && Wi == Wo &&
         Wi % 32 == 0 && N >= 64 && C >= 64 && B * C * H * Wi < (1ll << 31) &&
         B * N * H * Wo < (1ll << 31);
}
static void wt32_plan(int64_t B, int64_t C, int64_t H, int64_t W, int64_t N, int64_t KK,
                      int* S, int* spr) {
  const int64_t kt = (C * KK + 127) / 128, nt = (N + 127) / 128;
  const int64_t nst = B * H * (W / 32);
  int64_t s = (512 + kt * nt - 1) / (kt * nt);  // ~2 blocks per CU
  if (s > 256) s = 256;
  if (s > nst) s = nst;
  if (s < 1) s = 1;
  const int64_t per = (nst + s - 1) / s;
  *spr = (int)per;
  *S = (int)((nst + per - 1) / per);
}
static int64_t wt32_ws(int64_t B, int64_t C, int64_t H, int64_t W, int64_t N, int64_t KK) {
  int S, spr;
  wt32_plan(B, C, H, W, N, KK, &S, &spr);
  const int64_t kc = C * KK + 1;
  return (int64_t)S * N * kc + reduce_rows_scratch(S, N * kc);
}

struct WHaloPlan {
  WHaloGeom g;
  int FN, S, nblk, cblk;
  size_t lds;
};

// slab floats cap of the halo weight gradient (8M: LF 64-ch leg 26 vs 30 us at 4M)
static int64_t whalo_slab_max() { return (int64_t)(8 << 20); }

// split count depends only on (N, C, KK, B) so the workspace query can reproduce it
static int whalo_splits(int64_t N, int64_t C, int KK, int64_t B, int nblk, int cblk) {
  const int64_t kc = C * KK + 1;
  int64_t S = 1024 / (nblk * cblk);
  const int64_t cap = whalo_slab_max() / (N * kc);
  if (S > cap) S = cap;
  if (S > B) S = B;
  if (S < 1) S = 1;
  const int64_t ips = (B + S - 1) / S;
  return (int)((B + ips - 1) / ips);
}

static void whalo_blocking(int64_t N, int64_t C, int KK, int* FN, int* CB) {
  *FN = N <= 16 ? 1 : (N <= 32 ? 2 : 4);
  int cb = 1;
  while (cb * 2 <= C && (cb * 2) * KK + 1 <= 256) cb *= 2;  // <= 16 k-tiles of 16
  if (cb > C) cb = (int)C;
  *CB = cb;
}

// Halo-plane stride of conv_wgrad_halo_kernel's image (>= hw): the B-operand read of a
// half-wave (lanes j = 0..15 over 16 consecutive reduction columns (c, tap), kq = 0..1 over
// 2 positions) is Hs[c*PS + toff(tap) + kq*SW + base]; its 32 addresses should fall on 32
// distinct (a/4) mod 32 banks.  The stride residue mod 32 that minimises the extra bank
// cycles over the kernel's column tiles is chosen on the host (layout only: same sums).
static int whalo_plane_stride(int hw, int KK, int KW, int WP, int SW, int CB) {
  int best = hw + ((16 - hw % 32) + 32) % 32, best_cost = 1 << 30;
  const int ncols = CB * KK;
  for (int pad = 0; pad < 32; ++pad) {
    const int PS = hw + pad;
    int cost = 0;
    for (int t0 = 0; t0 < ncols; t0 += 16) {
      int hits[32][2];  // per bank: distinct addresses seen (up to 2 tracked) and count
      int cnt[32] = {0};
      for (int l = 0; l < 32; ++l) {
        const int j = l & 15, kq = l >> 4;
        const int kl = t0 + j;
        if (kl >= ncols) continue;
        const int c = kl / KK, tap = kl - c * KK;
        const int a = c * PS + (tap / KW) * WP + (tap % KW) + kq * SW;
        const int bank = ((a % 32) + 32) % 32;
        bool dup = false;
        for (int q = 0; q < cnt[bank] && q < 2; ++q) dup |= hits[bank][q] == a;
        if (dup) continue;
        if (cnt[bank] < 2) hits[bank][cnt[bank]] = a;
        ++cnt[bank];
      }
      int worst = 0;
      for (int b = 0; b < 32; ++b) worst = cnt[b] > worst ? cnt[b] : worst;
      cost += worst > 1 ? worst - 1 : 0;
    }
    if (cost < best_cost) {
      best_cost = cost;
      best = PS;
    }
  }
  return best;
}

static bool whalo_plan(int B, int C, int Hin, int Win, int N, int Hout, int Wo, int KH, int KW,
                       int SW, int oh, int ow, int kcols, WHaloPlan* pl) {
  if (Wo % 4 != 0) return false;
  // long images with many channels (the Upscale Conv1d) and the 128x128 ResBlock convs
  // run better on the split GEMM (tools/conv_shapes_bench.py: 148 vs 178 us at W 32)
  if (Hout * Wo > 128 && C > 64) return false;
  if ((int64_t)C * N >= 128 * 128) return false;
  WHaloGeom g;
  g.B = B; g.C = C; g.Hin = Hin; g.Win = Win; g.N = N; g.Hout = Hout; g.Wo = Wo;
  g.oh = oh; g.ow = ow;
  g.HP = Hout + KH - 1;
  g.WP = (Wo - 1) * SW + KW;
  const int hw = g.HP * g.WP;
  g.P = Hout * Wo;
  g.GST = g.P + ((2 - g.P % 32) + 32) % 32;
  if (g.WP < 2 || g.P >= (1 << 16)) return false;
  g.dv_hw = make_div16(hw);
  g.dv_wp = make_div16(g.WP);
  g.dv_gst = make_div16(g.GST);
  const int KK = KH * KW;
  int FN, CB;
  whalo_blocking(N, C, KK, &FN, &CB);
  g.PS = whalo_plane_stride(hw, KK, KW, g.WP, SW, CB);
  g.CB = CB;
  g.Kred = C * KK;
  g.kcols = kcols;
  const size_t fl = (size_t)FN * 16 * g.GST + (size_t)(CB + 1) * g.PS;
  if (fl * 4 > (size_t)HALO_LDS_MAX) return false;
  pl->nblk = (N + FN * 16 - 1) / (FN * 16);
  pl->cblk = (C + CB - 1) / CB;
  pl->S = whalo_splits(N, C, KK, B, pl->nblk, pl->cblk);
  g.ips = (B + pl->S - 1) / pl->S;
  pl->g = g;
  pl->FN = FN;
  pl->lds = fl * 4;
  return true;
}

template <int KH, int KW, int SW, bool REPL>
static void launch_wgrad_halo(const float* G, const float* in, float* slab, const WHaloPlan& pl,
                              hipStream_t st) {
  const dim3 grid(pl.S, pl.nblk, pl.cblk);
#define W_(FN_)                                                                              \
  hipLaunchKernelGGL((conv_wgrad_halo_kernel<KH, KW, SW, REPL, FN_>), grid, dim3(256), pl.lds, \
                     st, G, in, slab, pl.g)
  if (pl.FN == 1) W_(1); else if (pl.FN == 2) W_(2); else W_(4);
#undef W_
}

// out[o] = epi(sum_z slab[z][o]) in split order; channel n = (o / HW) % N.  The dropout
// mask depends on (seed, offset, o) only, so it matches the unsplit epilogue exactly.
__global__ __launch_bounds__(256) void conv_splitk_epi_kernel(const float* __restrict__ slab,
                                                             int splits, int n_out, int N,
                                                             Div16 dhw, Epi e,
                                                             float* __restrict__ out) {
  const uint64_t seed = e.drop_p > 0.f ? mix_seed(e.seed_ptr, e.offset) : 0ull;
  // eval BN / Snake terms once per channel (N <= 256 here: tvq_conv2d_fwd_bn_eval's shapes)
  __shared__ PostCh pcs[256];
  const bool post = e.bn_rv != nullptr && N <= 256;
  if (post) {
    for (int n = threadIdx.x; n < N; n += 256) pcs[n] = epi_post_ch(e, n);
    __syncthreads();
  }
  for (int o = blockIdx.x * 256 + threadIdx.x; o < n_out; o += gridDim.x * 256) {
    float v = 0.f;
#pragma unroll 4
    for (int z = 0; z < splits; ++z) v += slab[(int64_t)z * n_out + o];
    const int n = div16(o, dhw) % N;
    if (e.bias) v += e.bias[n];
    if (post) v = epi_post_apply(pcs[n], v, e.gelu != 0);
    else v = epi_post(e, v, n);
    if (e.drop_p > 0.f) v = uniform01(seed, (uint64_t)o) >= e.drop_p ? v * e.drop_scale : 0.f;
    if (e.residual) v += e.residual[o];
    out[o] = v;
  }
}

// Repack a weight seen as (n, c, tap) with strides (wsn, wsc, 1) into [tap][c][n] so the
// A-operand loads of a K-step read TN consecutive floats (one or two cache lines) instead
// of TN rows a whole filter apart.
__global__ void conv_pack_weight_kernel(const float* __restrict__ w, int N, int C, int KK,
                                        int64_t wsn, int64_t wsc, float* __restrict__ out) {
  const int64_t total = (int64_t)N * C * KK;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int n = (int)(i % N);
    const int64_t r = i / N;
    const int c = (int)(r % C);
    const int tap = (int)(r / C);
    out[i] = w[n * wsn + c * wsc + tap];
  }
}

// Per-step weight-pack cache (tvq_conv_packcache_*).  Inside a scope, the first time a
// (weight, view) is packed it gets a slot in the caller's arena and is recorded; at the
// next scope's begin every recorded entry is repacked from the current weights by a few
// batched launches, and the convs of the scope read their slot without packing again.
// The scope must not contain weight updates (a trainer opens it around forward+backward,
// the optimizer step is outside).  Entries belong to one cache id (one arena); several ids
// keep their entries side by side, so two step segments captured as separate graphs (the
// DP trainer's stage1 and stage2) each repack only their own weights.  An id's entries are
// dropped by tvq_conv_packcache_release (its owner is freed) or when the id begins with
// another arena.
struct PackEntry {
  const float* src;
  int N, C, KK;
  int64_t wsn, wsc, off;
};
struct PackCacheState {
  std::vector<PackEntry> entries;
  float* arena = nullptr;
  int64_t cap = 0, used = 0;
};
static std::map<int64_t, PackCacheState> g_pcs;
static PackCacheState* g_pc_cur = nullptr;  // the open scope's cache (null: no scope)
static int64_t g_pc_last = -1;              // id of the last scope (entries query)
// deferred weight-gradient split sums (see wgrad_finish), each with the stream its producer
// ran on: the flush issues each stream's records as one batch on that stream (ordered after
// that stream's producers), so a backward spread over several streams (a branch's side
// stream) defers its reductions too
struct RdRec {
  RrJob job;
  hipStream_t st;
};
static std::vector<RdRec> g_rd;
static bool g_rd_on = false, g_rd_paused = false;

// one launch repacks a whole step's weights (a stage1 + stage2 step records ~70): 36 bytes
// per entry keep PACK_BATCH of them inside a 4 KB kernel-argument block
constexpr int PACK_BATCH = 96;
struct PackBatch {
  const float* src[PACK_BATCH];
  int64_t off[PACK_BATCH];
  int wsn[PACK_BATCH], wsc[PACK_BATCH];
  int N[PACK_BATCH], C[PACK_BATCH], KK[PACK_BATCH];
};
static_assert(sizeof(PackBatch) <= 3900, "pack batch kernel arguments");

// blockIdx.y = entry; blocks stride over the entry's N*C*KK elements ([tap][c][n] order)
__global__ void conv_pack_multi_kernel(PackBatch b, float* __restrict__ arena) {
  const int j = blockIdx.y;
  const int N = b.N[j], C = b.C[j];
  const int64_t total = (int64_t)N * C * b.KK[j];
  const float* w = b.src[j];
  float* out = arena + b.off[j];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int n = (int)(i % N);
    const int64_t r = i / N;
    const int c = (int)(r % C);
    const int tap = (int)(r / C);
    out[i] = w[(int64_t)n * b.wsn[j] + (int64_t)c * b.wsc[j] + tap];
  }
}

static void pack_launch(const float* wt, int N, int C, int KK, int64_t wsn, int64_t wsc,
                        float* dst, hipStream_t st) {
  const int64_t total = (int64_t)N * C * KK;
  const int blocks = (int)((total + 255) / 256 < 2048 ? (total + 255) / 256 : 2048);
  hipLaunchKernelGGL(conv_pack_weight_kernel, dim3(blocks), dim3(256), 0, st, wt, N, C, KK, wsn,
                     wsc, dst);
}

// Pack `wt` into `ws` (N*C*KK floats) when given -- or serve it from the active pack cache
// -- and retarget the geometry's weight strides.
static const float* pack_weight(const float* wt, ConvGeom& g, int KK, float* ws, hipStream_t st) {
  if (!ws) return wt;
  const int64_t total = (int64_t)g.N * g.C * KK;
  float* dst = ws;
  bool need = true;
  if (PackCacheState* pc = g_pc_cur) {
    for (const PackEntry& p : pc->entries)
      if (p.src == wt && p.N == g.N && p.C == g.C && p.KK == KK && p.wsn == g.wsn &&
          p.wsc == g.wsc) {
        dst = pc->arena + p.off;
        need = false;  // repacked at this scope's begin
        break;
      }
    const int64_t slot = (total + 63) / 64 * 64;
    if (need && pc->used + slot <= pc->cap) {
      pc->entries.push_back({wt, g.N, g.C, KK, g.wsn, g.wsc, pc->used});
      dst = pc->arena + pc->used;
      pc->used += slot;
    }
  }
  if (need) pack_launch(wt, g.N, g.C, KK, g.wsn, g.wsc, dst, st);
  g.wsn = 1;
  g.wsc = g.N;
  g.wst = (int64_t)g.N * g.C;
  return dst;
}

// A (weight, view) packed [tap][c][n] for a kernel outside the conv engine (the fused LF
// ResBlock): from the open pack-cache scope (recorded and repacked at each scope's begin like
// the engine's own), else packed into `ws`, else (no scope, no ws) the unpacked weight.
// Returns the pointer and the view's strides (n, c, tap) in *sn / *sc / *st.
const float* conv_pack_view(const float* w, int N, int C, int KK, int64_t wsn, int64_t wsc,
                            float* ws, hipStream_t st, int64_t* sn, int64_t* sc, int64_t* stp) {
  ConvGeom g = {};
  g.N = N;
  g.C = C;
  g.wsn = wsn;
  g.wsc = wsc;
  g.wst = 1;
  float* dst = ws;
  if (PackCacheState* pc = g_pc_cur) {
    for (const PackEntry& p : pc->entries)
      if (p.src == w && p.N == N && p.C == C && p.KK == KK && p.wsn == wsn && p.wsc == wsc) {
        *sn = 1; *sc = N; *stp = (int64_t)N * C;
        return pc->arena + p.off;
      }
    const int64_t slot = ((int64_t)N * C * KK + 63) / 64 * 64;
    if (pc->used + slot <= pc->cap) {
      pc->entries.push_back({w, N, C, KK, wsn, wsc, pc->used});
      dst = pc->arena + pc->used;
      pc->used += slot;
    }
  }
  if (!dst) {
    *sn = wsn; *sc = wsc; *stp = 1;
    return w;
  }
  pack_launch(w, N, C, KK, wsn, wsc, dst, st);
  *sn = 1; *sc = N; *stp = (int64_t)N * C;
  return dst;
}

static void tap_tile(int N, int* TN, int* TM) {
  if (N <= 16) { *TN = 16; *TM = 256; }
  else if (N <= 32) { *TN = 32; *TM = 128; }
  else { *TN = 64; *TM = 128; }
}

// split-K factor for the tap-major GEMM: only when the grid is small and K is deep
static int tap_splits(const ConvGeom& g, int KK, int* sps) {
  const int BK = g.C % 32 == 0 ? 32 : 16;
  int TN, TM;
  tap_tile(g.N, &TN, &TM);
  const int tiles = ((g.Mpos + TM - 1) / TM) * ((g.N + TN - 1) / TN);
  const int ksteps = KK * ((g.C + BK - 1) / BK);
  int s = 1;
  if (g.C % 16 == 0 && tiles < 512 && ksteps >= 8) {
    s = (1024 + tiles - 1) / tiles;
    if (s > ksteps / 4) s = ksteps / 4;
    if (s > 16) s = 16;
    if (s < 1) s = 1;
  }
  const int per = (ksteps + s - 1) / s;
  *sps = per;
  return (ksteps + per - 1) / per;
}

template <int MODE, int KH, int KW, int SW, bool REPL, int BK>
static void launch_tap(const float* in, const float* wt, float* out, const ConvGeom& g,
                       const Epi& e, int splits, int sps, int64_t zstride, hipStream_t st,
                       int* cnt = nullptr, float* fout = nullptr, const Epi* fe = nullptr) {
  int TN, TM;
  tap_tile(g.N, &TN, &TM);
  dim3 grid((g.Mpos + TM - 1) / TM, (g.N + TN - 1) / TN, splits);
  const Epi fin = fe ? *fe : e;
  // the eval conv -> BN -> Snake shapes (ResBlock 3x3 / 1x1, DecBlock ConvT, Upscale Conv1d)
  // have epilogue-fused variants; the split-K finish applies `fin`'s BN itself
  constexpr bool post_kind = (MODE == GATHER_F && ((KH == 3 && KW == 3) || (KH == 1 && KW == 3 && !REPL) ||
                                                   (KH == 1 && KW == 1) ||
                                                   (KH == 3 && KW == 4 && SW == 2 && REPL))) ||
                             (MODE == GATHER_T && KH == 3 && KW == 4 && SW == 2);
  if constexpr (post_kind) {
    if (splits == 1 && e.bn_rv) {
      t_post_done = true;
      if (TN == 16)
        hipLaunchKernelGGL((conv_tap_kernel<MODE, KH, KW, SW, REPL, 16, 256, 1, 4, BK, true>), grid,
                           dim3(256), 0, st, in, wt, out, g, e, sps, zstride, cnt, fout, fin);
      else if (TN == 32)
        hipLaunchKernelGGL((conv_tap_kernel<MODE, KH, KW, SW, REPL, 32, 128, 2, 2, BK, true>), grid,
                           dim3(256), 0, st, in, wt, out, g, e, sps, zstride, cnt, fout, fin);
      else
        hipLaunchKernelGGL((conv_tap_kernel<MODE, KH, KW, SW, REPL, 64, 128, 2, 2, BK, true>), grid,
                           dim3(256), 0, st, in, wt, out, g, e, sps, zstride, cnt, fout, fin);
      return;
    }
  }
  if (cnt && fin.bn_rv) t_post_done = true;
  if (TN == 16)
    hipLaunchKernelGGL((conv_tap_kernel<MODE, KH, KW, SW, REPL, 16, 256, 1, 4, BK>), grid,
                       dim3(256), 0, st, in, wt, out, g, e, sps, zstride, cnt, fout, fin);
  else if (TN == 32)
    hipLaunchKernelGGL((conv_tap_kernel<MODE, KH, KW, SW, REPL, 32, 128, 2, 2, BK>), grid,
                       dim3(256), 0, st, in, wt, out, g, e, sps, zstride, cnt, fout, fin);
  else
    hipLaunchKernelGGL((conv_tap_kernel<MODE, KH, KW, SW, REPL, 64, 128, 2, 2, BK>), grid,
                       dim3(256), 0, st, in, wt, out, g, e, sps, zstride, cnt, fout, fin);
}

static int g_conv_t32 = 1;  // conv_t32_kernel enabled (tvq_conv_config bit 8 turns it off)
static int g_conv_n16 = 1;  // conv_n16_kernel enabled (tvq_conv_config bit 2048 turns it off)

// ---------------------------------------------------------------- direct path
// Convolutions of narrow maps with >= 32 channels on both sides -- the LF band's 64 /
// 128-channel convs on (256, C, 3, 8), 6,144 positions, and their neighbours (the 1x1
// projections, the 32 -> 64 EncBlock, the 64 -> 32 DecBlock): the staged paths give them
// 48-96 blocks (so split-K + an epilogue launch, 21 + 5 us per 3x3 64-channel conv at 0.13
// of the fp32 MFMA peak).  Here a block owns a 32-channel x 32-position output tile and its
// NW waves split the reduction by input-channel ranges (each wave: its C / NW channels for
// every tap), so the LF 64-channel convs run as 384 blocks of short MFMA chains with no LDS
// staging: every operand goes global (L2) -> registers.  Per step a lane supplies one
// packed weight w[tap][c][n0 + l % 32] (coalesced) and one gathered input value at its
// position (gather_in's index rules: zero / replicate padding, the stride-2 transposed
// parity skip); the wave runs one v_mfma_f32_32x32x2_f32 per 2 channels.  Up to ~144
// floats of loads (every tap of a 64-channel 3x3 conv) are in flight before the first MFMA.  The partial tiles are added in
// LDS in a fixed pairwise order; bias, dropout (the same counter hash) and residual as
// epi_store.  Replaced: split-K tap + epilogue, 6.12 -> 5.92 ms per joint step.
template <int MODE, int KH, int KW, int SW, bool REPL, int CW, int NW>
__global__ __launch_bounds__(64 * NW) void conv_d32_kernel(const float* __restrict__ in,
                                                          const float* __restrict__ wt,
                                                          float* __restrict__ out, ConvGeom g,
                                                          Epi e, int mtiles) {
  constexpr int KK = KH * KW;
  __shared__ float red[NW][16][64];
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hl = lane >> 5;
  const int mt = (int)blockIdx.x % mtiles, nt = (int)blockIdx.x / mtiles;
  const int m0 = mt * 32, n0 = nt * 32;
  // this lane's output position (B operand column) and output channel (A operand row)
  const int m = m0 + r32;
  const bool pv = m < g.Mpos;
  const int mc = pv ? m : 0;
  const uint32_t bh = fdiv((uint32_t)mc, g.fd_wo);
  const int ww = mc - (int)bh * g.Wo;
  const int b = (int)fdiv((uint32_t)mc, g.fd_hwo);
  const int hh = (int)bh - b * g.Hout;
  const int HW = g.Hin * g.Win;
  const int c0 = wid * CW;  // this wave's input channels [c0, c0 + CW)
  const float* inb = in + ((int64_t)b * g.C + c0 + hl) * HW;
  const float* wl = wt + (int64_t)(c0 + hl) * g.wsc + min(n0 + r32, g.N - 1);
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  constexpr int ST = CW / 2;  // MFMA steps per tap
  // PD taps' loads in flight (a ring of PD register buffers, ~144 floats): every tap of a
  // 64-channel conv is requested before the first MFMA, so the block pays one L2 round
  // trip instead of one per tap (9 x ~1 us with one tap of prefetch)
  constexpr int PD0 = 144 / CW, PD = PD0 < 1 ? 1 : (PD0 > KK ? KK : PD0);
  float fa[PD][ST], fb[PD][ST];
  auto load = [&](int buf, int tap) {
    const int kh = tap / KW, kw = tap - KW * kh;
    int hi, wi;
    bool ok = pv;
    if (MODE == GATHER_F) {
      hi = hh + kh - g.oph;
      wi = ww * SW + kw - g.opw;
      if (REPL) {
        hi = hi < 0 ? 0 : (hi >= g.Hin ? g.Hin - 1 : hi);
        wi = wi < 0 ? 0 : (wi >= g.Win ? g.Win - 1 : wi);
      } else {
        ok = ok && hi >= 0 && hi < g.Hin && wi >= 0 && wi < g.Win;
      }
    } else {
      hi = hh - kh + g.oph;
      const int wn = ww - kw + g.opw;
      ok = ok && hi >= 0 && hi < g.Hin && wn >= 0 && (SW == 1 || (wn & 1) == 0);
      wi = wn / SW;
      ok = ok && wi < g.Win;
    }
    const int o = ok ? hi * g.Win + wi : 0;
    const float* wtap = wl + (int64_t)tap * g.wst;
#pragma unroll
    for (int u = 0; u < ST; ++u) {
      fa[buf][u] = wtap[(int64_t)(2 * u) * g.wsc];
      const float v = inb[(int64_t)(2 * u) * HW + o];
      fb[buf][u] = ok ? v : 0.f;
    }
  };
#pragma unroll
  for (int t = 0; t < PD; ++t) load(t, t);
#pragma unroll
  for (int tap = 0; tap < KK; ++tap) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < ST; ++u)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[tap % PD][u], fb[tap % PD][u], acc, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    if (tap + PD < KK) load(tap % PD, tap + PD);
  }
  // partial tiles -> LDS, summed pairwise ((w0 + w1) + (w2 + w3)) + ...; thread t then owns
  // tile elements t, t + 64 NW, ... with the channel slowest (row-major [n][m]: the stores
  // coalesce along m)
#pragma unroll
  for (int r = 0; r < 16; ++r) red[wid][r][lane] = acc[r];
  __syncthreads();
  const uint64_t seed = e.drop_p > 0.f ? mix_seed(e.seed_ptr, e.offset) : 0ull;
#pragma unroll
  for (int q = 0; q < 1024 / (64 * NW); ++q) {
    const int el = tid + 64 * NW * q, nr = el >> 5, mr = el & 31;
    // acc r of lane l: row (n) 8 (r / 4) + 4 (l / 32) + r % 4, column (m) l % 32
    const int ln = mr + 32 * ((nr >> 2) & 1), r = (nr & 3) + 4 * (nr >> 3);
    float part[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) part[w] = red[w][r][ln];
#pragma unroll
    for (int span = 1; span < NW; span *= 2)
#pragma unroll
      for (int w = 0; w + span < NW; w += 2 * span) part[w] += part[w + span];
    const int n = n0 + nr, mm = m0 + mr;
    if (n >= g.N || mm >= g.Mpos) continue;
    const uint32_t bh2 = fdiv((uint32_t)mm, g.fd_wo);
    const int w2 = mm - (int)bh2 * g.Wo;
    const int b2 = (int)fdiv((uint32_t)mm, g.fd_hwo);
    const int h2 = (int)bh2 - b2 * g.Hout;
    const int64_t o = (((int64_t)b2 * g.N + n) * g.Hout + h2) * g.Wo + w2;
    float v = epi_post(e, part[0] + (e.bias ? e.bias[n] : 0.f), n);
    if (e.drop_p > 0.f) v = uniform01(seed, (uint64_t)o) >= e.drop_p ? v * e.drop_scale : 0.f;
    if (e.residual) v += e.residual[o];
    out[o] = v;
  }
}

// the largest position count the direct narrow-map conv takes (the LF maps, 6,144
// positions) and its waves per block
static int d32_max_pos() { return 8192; }
static int d32_nw() { return 4; }

template <int MODE, int KH, int KW, int SW, bool REPL, int NW>
static bool launch_d32_nw(const float* in, const float* wt, float* out, const ConvGeom& g,
                          const Epi& e, int mtiles, unsigned grid, hipStream_t st) {
#define TVQ_D32(CWV)                                                                         \
  hipLaunchKernelGGL((conv_d32_kernel<MODE, KH, KW, SW, REPL, CWV, NW>), dim3(grid),        \
                     dim3(64 * NW), 0, st, in, wt, out, g, e, mtiles);                        \
  return true;
  switch (g.C / NW) {
    case 4: if (NW == 8) { TVQ_D32(4) } return false;
    case 8: TVQ_D32(8)
    case 16: TVQ_D32(16)
    case 24: TVQ_D32(24)
    case 32: TVQ_D32(32)
    default: return false;
  }
#undef TVQ_D32
}

template <int MODE, int KH, int KW, int SW, bool REPL>
static bool launch_d32(const float* in, const float* wt, float* out, const ConvGeom& g,
                       const Epi& e, hipStream_t st) {
  // off with the 32x32-MFMA tiles (tvq_conv_config bit 8: the tap kernel alone)
  if (!g_conv_t32 || g.Mpos > d32_max_pos()) return false;
  if (g.wsn != 1 || g.N < 32 || g.C < 32 || g.C > 128) return false;
  const int nw = d32_nw() == 8 ? 8 : 4;
  if (g.C % (2 * nw) != 0) return false;
  const int mtiles = (g.Mpos + 31) / 32, ntiles = (g.N + 31) / 32;
  const unsigned grid = (unsigned)(mtiles * ntiles);
  return nw == 8 ? launch_d32_nw<MODE, KH, KW, SW, REPL, 8>(in, wt, out, g, e, mtiles, grid, st)
                 : launch_d32_nw<MODE, KH, KW, SW, REPL, 4>(in, wt, out, g, e, mtiles, grid, st);
}

// Weight (+ bias) gradient of the same narrow-map convs (conv2d only): slab[z][n][k'] =
// sum over split z's positions of dY[n][pos] X[c][pos + tap] (k' = c KK + tap; k' = Kred:
// the bias column, X = 1).  A block owns a 32 (n) x 32 (k') tile of one split; its 4 waves
// take quarters of the split's positions, each position pair one 32x32x2 MFMA step (lane
// l: dY at channel n0 + l % 32 and X gathered at column k0 + l % 32, position 2 s + l / 32),
// 16 steps' loads in flight ahead of the previous 16 steps' MFMAs.  Quarter tiles added in
// LDS in the order (w0 + w1) + (w2 + w3); slabs summed in split order by wgrad_finish.
// Measured slower than conv_wgrad_halo_kernel in the step (see tvq_conv2d_wgrad): off by
// default, kept for A/B (TVQ_CONV_WD32=1).
constexpr int WD32_KC = 16;

template <int KH, int KW, int SW, bool REPL>
__global__ __launch_bounds__(256) void conv_wgrad_d32_kernel(const float* __restrict__ dy,
                                                             const float* __restrict__ x,
                                                             float* __restrict__ slab, ConvGeom g,
                                                             int pps, int kcols, int ntiles,
                                                             int ctiles) {
  constexpr int KK = KH * KW;
  __shared__ float red[4][16][64];
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hl = lane >> 5;
  int bid = (int)blockIdx.x;
  const int tc = bid % ctiles;
  bid /= ctiles;
  const int tn = bid % ntiles, z = bid / ntiles;
  const int n0 = tn * 32, k0 = tc * 32;
  // this lane's A row (output channel) and B column (c, tap) / bias / padding column
  const int n = min(n0 + r32, g.N - 1);
  const int col = k0 + r32;
  const bool bias_col = col == g.Kred, real_col = col < g.Kred;
  const int c = real_col ? col / KK : 0, tap = real_col ? col - (col / KK) * KK : 0;
  const int dh = tap / KW - g.oph, dw = tap - (tap / KW) * KW - g.opw;
  const int64_t HWo = (int64_t)g.Hout * g.Wo, HWi = (int64_t)g.Hin * g.Win;
  const int q = pps >> 2;  // positions per wave (even)
  const int pb = z * pps + wid * q, pe = min(g.Mpos, pb + q);
  const int steps = pb < pe ? (pe - pb + 1) >> 1 : 0;
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float fa[2][WD32_KC], fb[2][WD32_KC];
  auto load = [&](int buf, int s0) {
#pragma unroll
    for (int u = 0; u < WD32_KC; ++u) {
      const int pos = pb + 2 * (s0 + u) + hl;
      const bool pv = pos < pe;
      const int pc = pv ? pos : pb;
      const uint32_t bh = fdiv((uint32_t)pc, g.fd_wo);
      const int wo = pc - (int)bh * g.Wo;
      const int b = (int)fdiv((uint32_t)pc, g.fd_hwo);
      const int h = (int)bh - b * g.Hout;
      const float av = dy[((int64_t)b * g.N + n) * HWo + (int64_t)h * g.Wo + wo];
      int hi = h + dh, wi = wo * SW + dw;
      bool ok = real_col;
      if (REPL) {
        hi = hi < 0 ? 0 : (hi >= g.Hin ? g.Hin - 1 : hi);
        wi = wi < 0 ? 0 : (wi >= g.Win ? g.Win - 1 : wi);
      } else {
        ok = ok && hi >= 0 && hi < g.Hin && wi >= 0 && wi < g.Win;
      }
      const float xv = x[((int64_t)b * g.C + c) * HWi + (ok ? hi * g.Win + wi : 0)];
      fa[buf][u] = pv ? av : 0.f;
      fb[buf][u] = ok ? xv : (bias_col ? 1.f : 0.f);
    }
  };
  const int nch = (steps + WD32_KC - 1) / WD32_KC;
  if (nch > 0) load(0, 0);
  for (int ch = 0; ch < nch; ch += 2) {
    load(1, (ch + 1) * WD32_KC);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < WD32_KC; ++u)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[0][u], fb[0][u], acc, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    if (ch + 1 >= nch) break;
    load(0, (ch + 2) * WD32_KC);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < WD32_KC; ++u)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[1][u], fb[1][u], acc, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) red[wid][r][lane] = acc[r];
  __syncthreads();
  float* sz = slab + (int64_t)z * g.N * kcols;
#pragma unroll
  for (int qq = 0; qq < 4; ++qq) {
    const int el = tid + 256 * qq, nr = el >> 5, cr = el & 31;
    const int ln = cr + 32 * ((nr >> 2) & 1), r = (nr & 3) + 4 * (nr >> 3);
    const float v = (red[0][r][ln] + red[1][r][ln]) + (red[2][r][ln] + red[3][r][ln]);
    const int nn = n0 + nr, cc = k0 + cr;
    if (nn < g.N && cc < kcols) sz[(int64_t)nn * kcols + cc] = v;
  }
}

static bool wd32_on() { return false; }  // measured slower than the halo kernel (below)

// the direct weight gradient's split count (<= max_s, the workspace's slab count)
static int wd32_splits(const ConvGeom& g, int kcols, int max_s, int* pps) {
  const int tiles = ((g.N + 31) / 32) * ((kcols + 31) / 32);
  int s = (768 + tiles / 2) / tiles;
  if (s > max_s) s = max_s;
  if (s < 1) s = 1;
  int p = (g.Mpos + s - 1) / s;
  p = (p + 7) / 8 * 8;
  *pps = p;
  return (g.Mpos + p - 1) / p;
}

// the 16 / 48-channel convs into 128 on the 32x32-MFMA tile with a 16 / 32-wide K stage
// instead of the halo tile: HF 16 -> 128 3x3 forward and the 128 -> 16 conv's data gradient
// 32.2 / 30.9 -> 22.1 / 20.3 us, step -30 us (tools/gpu_t32s_ab.sh)
static bool t32_smallc() { return true; }

// staged GEMM; `slab` (nullable) enables split-K with splits*N*Mpos floats of partials
template <int MODE, int KH, int KW, int SW, bool REPL>
static void launch_gemm(const float* in, const float* wt, float* out, const ConvGeom& g,
                        const Epi& e, float* slab, hipStream_t st) {
  if (g.C % 16 == 0) {
    // wide channels: 32x32 MFMA tile, no split-K (needs packed weights).  128-channel
    // tiles on a full grid; 64-channel tiles (6 waves) for N % 64 maps too small for it
    // (the LF band's 64-channel convs), which otherwise run split-K + an epilogue launch.
    const bool t32_ok = g_conv_t32 && g.wsn == 1 && g.wsc == g.N &&
                        (int64_t)g.B * g.C * g.Hin * g.Win < (1ll << 29) &&
                        (int64_t)KH * KW * g.C * g.N < (1ll << 29);
    const int64_t mt = (g.Mpos + 95) / 96;
    // K stage: the configured BK where the channels divide it, else 32 / 16 (C = 16 / 48:
    // the HF band's 16 -> 128 convs, when t32_smallc() routes them here)
    const int bk = g.C % g_t32_bk == 0 ? g_t32_bk : (g.C % 32 == 0 ? 32 : 16);
    const bool wide128 = t32_ok && (g.C % g_t32_bk == 0 || t32_smallc()) && g.N % 128 == 0 &&
                         mt * (g.N / 128) >= 192;
    const bool wide64 = !wide128 && t32_ok && g_t32_n64 && g.C % 64 == 0 && g.N % 64 == 0 &&
                        mt >= 32;
    if (wide128 || wide64) {
      static bool lds_set = false;  // > 64 KB of dynamic LDS must be opted into once
      if (!lds_set) {
        (void)hipFuncSetAttribute(
            reinterpret_cast<const void*>(&conv_t32_kernel<MODE, KH, KW, SW, REPL, 64, 4, 128>),
            hipFuncAttributeMaxDynamicSharedMemorySize, (int)t32_lds(64, 128));
        (void)hipFuncSetAttribute(
            reinterpret_cast<const void*>(&conv_t32_kernel<MODE, KH, KW, SW, REPL, 64, 12, 128>),
            hipFuncAttributeMaxDynamicSharedMemorySize, (int)t32_lds(64, 128));
        (void)hipFuncSetAttribute(
            reinterpret_cast<const void*>(&conv_t32_kernel<MODE, KH, KW, SW, REPL, 64, 6, 64>),
            hipFuncAttributeMaxDynamicSharedMemorySize, (int)t32_lds(64, 64));
        lds_set = true;
      }
#define TVQ_T32(BKV, NWV, TNV)                                                             \
  hipLaunchKernelGGL((conv_t32_kernel<MODE, KH, KW, SW, REPL, BKV, NWV, TNV>),             \
                     dim3((unsigned)mt, g.N / TNV), dim3(64 * NWV), t32_lds(BKV, TNV), st, in, \
                     wt, out, g, e)
      // eval conv -> BN (-> Snake / after GELU): the epilogue-fused instance (12 waves, 128
      // channels; Upscale's Conv1d, the 128-channel ResBlock convs)
      constexpr bool t32_post = MODE == GATHER_F && !REPL &&
                                ((KH == 1 && KW == 3) || (KH == 3 && KW == 3));
      if constexpr (t32_post) {
        if (e.bn_rv && !wide64 && g_t32_nw == 12) {
          static bool lds_post = false;
          if (!lds_post) {
            (void)hipFuncSetAttribute(
                reinterpret_cast<const void*>(
                    &conv_t32_kernel<MODE, KH, KW, SW, REPL, 64, 12, 128, true>),
                hipFuncAttributeMaxDynamicSharedMemorySize, (int)t32_lds(64, 128));
            lds_post = true;
          }
          TVQ_PLAN("conv_t32 bk%d nw12 tn128 post", bk);
          if (bk == 64)
            hipLaunchKernelGGL((conv_t32_kernel<MODE, KH, KW, SW, REPL, 64, 12, 128, true>),
                               dim3((unsigned)mt, g.N / 128), dim3(64 * 12), t32_lds(64, 128), st,
                               in, wt, out, g, e);
          else if (bk == 32)
            hipLaunchKernelGGL((conv_t32_kernel<MODE, KH, KW, SW, REPL, 32, 12, 128, true>),
                               dim3((unsigned)mt, g.N / 128), dim3(64 * 12), t32_lds(32, 128), st,
                               in, wt, out, g, e);
          else  // the 16-channel -> 128 convs (HF encoder's last ResBlock)
            hipLaunchKernelGGL((conv_t32_kernel<MODE, KH, KW, SW, REPL, 16, 12, 128, true>),
                               dim3((unsigned)mt, g.N / 128), dim3(64 * 12), t32_lds(16, 128), st,
                               in, wt, out, g, e);
          t_post_done = true;
          return;
        }
      }
      TVQ_PLAN("conv_t32 bk%d nw%d tn%d", wide64 ? 64 : bk, wide64 ? 6 : g_t32_nw,
               wide64 ? 64 : 128);
      if (wide64) {
        TVQ_T32(64, 6, 64);
      } else if (g_t32_nw == 12) {
        if (bk == 64) TVQ_T32(64, 12, 128);
        else if (bk == 16) TVQ_T32(16, 12, 128);
        else TVQ_T32(32, 12, 128);
      } else {
        if (bk == 64) TVQ_T32(64, 4, 128);
        else if (bk == 16) TVQ_T32(16, 4, 128);
        else TVQ_T32(32, 4, 128);
      }
#undef TVQ_T32
      return;
    }
    if (launch_d32<MODE, KH, KW, SW, REPL>(in, wt, out, g, e, st)) {
      t_post_done = e.bn_rv != nullptr;
      TVQ_PLAN("conv_d32");
      return;
    }
    int sps;
    const int splits = slab ? tap_splits(g, KH * KW, &sps) : 1;
    if (!slab) sps = KH * KW * ((g.C + 31) / 16);  // >= all K-steps
    TVQ_PLAN("conv_tap splits%d", splits);
    if (splits > 1) {
      const int64_t n_out = (int64_t)g.Mpos * g.N;
      const Epi raw = {nullptr, nullptr, 0.f, 1.f, nullptr, 0};
      int TN, TM;
      tap_tile(g.N, &TN, &TM);
      int* cnt = counters((int64_t)((g.Mpos + TM - 1) / TM) * ((g.N + TN - 1) / TN), FIN_CONV);
      if (g.C % 32 == 0)
        launch_tap<MODE, KH, KW, SW, REPL, 32>(in, wt, slab, g, raw, splits, sps, n_out, st, cnt,
                                               out, &e);
      else
        launch_tap<MODE, KH, KW, SW, REPL, 16>(in, wt, slab, g, raw, splits, sps, n_out, st, cnt,
                                               out, &e);
      if (cnt) return;
      int blocks = (int)((n_out + 255) / 256);
      if (blocks > 8192) blocks = 8192;
      hipLaunchKernelGGL(conv_splitk_epi_kernel, dim3(blocks), dim3(256), 0, st, slab, splits,
                         (int)n_out, g.N, make_div16((int64_t)g.Hout * g.Wo), e, out);
      t_post_done = e.bn_rv != nullptr;
      return;
    }
    if (g.C % 32 == 0)
      launch_tap<MODE, KH, KW, SW, REPL, 32>(in, wt, out, g, e, 1, sps, 0, st);
    else
      launch_tap<MODE, KH, KW, SW, REPL, 16>(in, wt, out, g, e, 1, sps, 0, st);
    return;
  }
  // small channel counts: flat (c, kh, kw) K order keeps the K-steps full
  TVQ_PLAN("conv_gemm n%d", g.N);
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

// tvq_conv_config bits: 1 = halo fwd/dgrad, 2 = halo wgrad, 4 = halo fwd/dgrad wherever
// it fits (ignore halo_preferred; tests)
static int g_conv_halo = 3;

// Measured per shape on MI355X (tools/conv_shapes_bench.py, halo vs staged GEMM at the
// step's shapes): the halo tile wins while the gathered channel count is small (its
// per-image restaging of the weight panel grows with C), loses to the tap-major GEMM
// for 1x1 convs, for C >= 32, and for the stride-2 transposed gathers.  A register-
// resident-weight variant (whole reduction row per wave in VGPRs) was 1.5-4x slower
// than both (1 wave/SIMD, uncoalesced weight loads) and was dropped.
static bool halo_preferred(int mode, int C, int KK, int SW, int N, int64_t Mpos) {
  if (g_conv_halo & 4) return true;
  if (KK == 1 || C >= 32) return false;
  // 16 / 48 channels into >= 128 on a full grid: the 32x32-MFMA tile with a 16-wide K stage
  if (t32_smallc() && g_conv_t32 && C % 16 == 0 && N % 128 == 0 && (Mpos + 95) / 96 * (N / 128) >= 192)
    return false;
  if (mode == GATHER_T && SW == 2) return false;
  return true;
}

// ---------------------------------------------------------------- few outputs, wide input
// The HF band's 128 -> <= 16 channel convs on (B, 128, 3, 32): ResBlock(128, 16)'s 3x3 conv1
// and 1x1 projection forward (the decoder's first block), ResBlock(16, 128)'s data gradients
// (the encoder's last block) -- a 24,576 x 16 output with a 1,152- (or 128-) deep reduction.
// The tap-major GEMM gave them 96 blocks of a 16-row tile (0.11 of the fp32 peak, 51 us for
// the 3x3 at B = 256).  Here one 8-wave block owns one image: its C x 3 x 32 input is staged
// once into zero-padded LDS halo planes (C x 5 x 34), every B operand of the
// v_mfma_f32_16x16x4_f32 chains is an LDS read at an immediate offset from the lane's base
// (the reduction is tap-major, k = tap * C + c, so a step never crosses a tap), and the A
// operand comes straight from the [tap][c][n]-packed weight (a wave's 64 lanes read 256
// contiguous bytes per step).  Wave w takes input channels 32 (w & 3) .. for every tap (72
// steps for 3x3) and position tiles 3 (w >> 2) .. + 2 (3 chains sharing each weight value);
// the 4 channel splits are summed in LDS in split order.
constexpr int N16_H = 3, N16_W = 32, N16_P = 96, N16_WPD = 34, N16_PS = 176, N16_T = 512;
static bool n16_geom_ok(int mode, const ConvGeom& g, int KH, int KW, int SW, bool repl) {
  return SW == 1 && !repl && g.N <= 16 && g.C == 128 && g.Hin == N16_H && g.Hout == N16_H &&
         g.Win == N16_W && g.Wo == N16_W && g.oph == KH / 2 && g.opw == (KW - 1) / 2 &&
         ((KH == 3 && KW == 3) || (KH == 1 && KW == 1)) && (mode == GATHER_F || mode == GATHER_T);
}
constexpr size_t N16_LDS = 4 * ((size_t)128 * N16_PS + 4 * 16 * N16_P);

template <int MODE, int KH, int KW, bool POST>
__global__ __launch_bounds__(N16_T) void conv_n16_kernel(const float* __restrict__ in,
                                                         const float* __restrict__ wp,
                                                         float* __restrict__ out, ConvGeom g,
                                                         Epi e) {
  constexpr int C = 128, KK = KH * KW, SPT = 8;  // 8 steps of 4 channels per tap and split
  extern __shared__ float n16_smem[];
  float* Pl = n16_smem;               // [C][PS] halo planes
  float* red = n16_smem + C * N16_PS;  // [4 splits][16 rows][96 positions]
  const int tid = threadIdx.x, lane = tid & 63, j = lane & 15, kq = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ks = w & 3, pg = w >> 2, b = blockIdx.x, N = g.N;
  // the image's values (24 per thread in flight) and this wave's weights
  const float* inb = in + (int64_t)b * C * N16_P;
  float xv[C * N16_P / N16_T];
#pragma unroll
  for (int i = 0; i < C * N16_P / N16_T; ++i) xv[i] = inb[tid + N16_T * i];
  const int nn = j < N ? j : N - 1;
  float a[KK][SPT];
#pragma unroll
  for (int t = 0; t < KK; ++t)
#pragma unroll
    for (int s = 0; s < SPT; ++s) a[t][s] = wp[((int64_t)t * C + 32 * ks + 4 * s + kq) * N + nn];
  for (int i = tid; i < C * N16_PS; i += N16_T) Pl[i] = 0.f;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < C * N16_P / N16_T; ++i) {
    const int el = tid + N16_T * i, c = el / N16_P, p = el - c * N16_P;
    Pl[c * N16_PS + (p / N16_W + 1) * N16_WPD + p % N16_W + 1] = xv[i];
  }
  __syncthreads();
  // lane base: channel 32 ks + kq, the window centre of position 16 tile + j of row tile / 2
  const float* sp = Pl + (32 * ks + kq) * N16_PS + N16_WPD + 1 + j;
  floatx4 acc[3];
#pragma unroll
  for (int f = 0; f < 3; ++f) acc[f] = floatx4{0.f, 0.f, 0.f, 0.f};
  int pb[3];
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    const int tile = 3 * pg + f;  // 16 positions of row tile / 2
    pb[f] = (tile >> 1) * N16_WPD + 16 * (tile & 1);
  }
#pragma unroll
  for (int t = 0; t < KK; ++t) {
    const int kh = t / KW, kw = t % KW;
    const int dr = MODE == GATHER_F ? kh - KH / 2 : KH / 2 - kh;
    const int dc = MODE == GATHER_F ? kw - (KW - 1) / 2 : (KW - 1) / 2 - kw;
    const int off = dr * N16_WPD + dc;
#pragma unroll
    for (int s = 0; s < SPT; ++s)
#pragma unroll
      for (int f = 0; f < 3; ++f)
        acc[f] = mfma16x16x4(a[t][s], sp[pb[f] + 4 * s * N16_PS + off], acc[f]);
  }
#pragma unroll
  for (int f = 0; f < 3; ++f)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[(ks * 16 + 4 * kq + r) * N16_P + 16 * (3 * pg + f) + j] = acc[f][r];
  __syncthreads();
  const uint64_t seed = e.drop_p > 0.f ? mix_seed(e.seed_ptr, e.offset) : 0ull;
  for (int el = tid; el < N * N16_P; el += N16_T) {
    const int n = el / N16_P, p = el - n * N16_P;
    float v = red[n * N16_P + p];
#pragma unroll
    for (int k = 1; k < 4; ++k) v += red[(k * 16 + n) * N16_P + p];
    v += e.bias ? e.bias[n] : 0.f;
    if (POST) v = epi_post(e, v, n);
    const int64_t o = ((int64_t)b * N + n) * N16_P + p;
    if (e.drop_p > 0.f) v = uniform01(seed, (uint64_t)o) >= e.drop_p ? v * e.drop_scale : 0.f;
    if (e.residual) v += e.residual[o];
    out[o] = v;
  }
}

template <int MODE, int KH, int KW>
static void launch_n16(const float* in, const float* wt, float* out, const ConvGeom& g,
                       const Epi& e, hipStream_t st) {
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)conv_n16_kernel<MODE, KH, KW, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)N16_LDS);
    (void)hipFuncSetAttribute((const void*)conv_n16_kernel<MODE, KH, KW, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)N16_LDS);
    return true;
  }();
  (void)attr;
  TVQ_PLAN("conv_n16 k%dx%d mode%d n%d", KH, KW, MODE, g.N);
  if (e.bn_rv) {
    t_post_done = true;
    hipLaunchKernelGGL((conv_n16_kernel<MODE, KH, KW, true>), dim3(g.B), dim3(N16_T), N16_LDS, st,
                       in, wt, out, g, e);
  } else {
    hipLaunchKernelGGL((conv_n16_kernel<MODE, KH, KW, false>), dim3(g.B), dim3(N16_T), N16_LDS,
                       st, in, wt, out, g, e);
  }
}

// halo path when the image + weight panel fit in LDS, else the staged GEMM
// workspace (nullable) = [packed weight N*C*KK][split-K slab]; see conv_gemm_ws
template <int MODE, int KH, int KW, int SW, bool REPL>
static void launch_conv(const float* in, const float* wt, float* out, ConvGeom g, float* ws,
                        const Epi& e, hipStream_t st) {
  // measured per shape (tools/conv_shapes_bench.py, r02): the direct kernel wins for the
  // stride-2 transposed gathers with <= 12 channels on both sides (the decoders' ConvT tail
  // and DecBlocks 8->4, the EncBlocks' data gradients), loses to the halo / staged paths
  // elsewhere
  if constexpr (KH == 3 && KW == 4 && SW == 2) {
    const int k2 = s2_kind(MODE, g);
    if (k2) {
      launch_s2<REPL>(k2, in, wt, out, g, e, st);
      return;
    }
  }
  if (g_conv_small && MODE == GATHER_T && SW == 2 && g.C <= 12 && g.N <= 12) {
    const int64_t th = (int64_t)g.B * g.Hout * ((g.Wo + 1) / 2);
    // outputs per thread rounded up to 4 (every channel's sum in the same order)
    const dim3 grid((unsigned)((th + 255) / 256));
    TVQ_PLAN("conv_small n%d", g.N);
    if (g.N <= 4)
      hipLaunchKernelGGL((conv_small_kernel<MODE, KH, KW, SW, REPL, 4>), grid, dim3(256), 0, st, in, wt, out, g, e);
    else if (g.N <= 8)
      hipLaunchKernelGGL((conv_small_kernel<MODE, KH, KW, SW, REPL, 8>), grid, dim3(256), 0, st, in, wt, out, g, e);
    else if (g.N <= 12)
      hipLaunchKernelGGL((conv_small_kernel<MODE, KH, KW, SW, REPL, 12>), grid, dim3(256), 0, st, in, wt, out, g, e);
    else
      hipLaunchKernelGGL((conv_small_kernel<MODE, KH, KW, SW, REPL, 16>), grid, dim3(256), 0, st, in, wt, out, g, e);
    return;
  }
  if constexpr (SW == 1 && !REPL && ((KH == 3 && KW == 3) || (KH == 1 && KW == 1))) {
    if (ws && g_conv_n16 && n16_geom_ok(MODE, g, KH, KW, SW, REPL)) {
      wt = pack_weight(wt, g, KH * KW, ws, st);  // [tap][c][n]
      launch_n16<MODE, KH, KW>(in, wt, out, g, e, st);
      return;
    }
  }
  HaloPlan pl;
  const int oh = MODE == GATHER_F ? g.oph : KH - 1 - g.oph;
  const int ow = MODE == GATHER_F ? g.opw : KW - 1 - g.opw;
  if ((g_conv_halo & 1) && halo_preferred(MODE, g.C, KH * KW, SW, g.N, g.Mpos) && halo_plan(MODE, g.B, g.C, g.Hin, g.Win, g.N, g.Hout, g.Wo, KH, KW, SW, oh,
                               ow, g.wsn, g.wsc, &pl)) {
    TVQ_PLAN("conv_halo");
    launch_halo<MODE, KH, KW, SW, REPL>(in, wt, out, pl, g.B, e, st);
    return;
  }
  float* slab = nullptr;
  if (ws && g.C % 16 == 0) {
    wt = pack_weight(wt, g, KH * KW, ws, st);
    slab = ws + (int64_t)g.N * g.C * KH * KW;
  }
  launch_gemm<MODE, KH, KW, SW, REPL>(in, wt, out, g, e, slab, st);
}

// floats of workspace launch_conv may use for this geometry (pack + split-K slab)
static int64_t conv_gemm_ws(const ConvGeom& g, int KK) {
  if (g.C % 16 != 0) return 0;
  int sps;
  const int s = tap_splits(g, KK, &sps);
  return (int64_t)g.N * g.C * KK + (s > 1 ? (int64_t)s * g.N * g.Mpos : 0);
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
    case 3: if (repl) { MACRO(1, 3, 1, true) } else { MACRO(1, 3, 1, false) } break; \
    case 4: MACRO(1, 7, 1, false) break;                                      \
    case 5: MACRO(1, 4, 2, false) break;                                      \
    default: set_error("conv: unsupported kernel kind %d", kind); return TVQ_ERR_ARG; \
  }

static int kind_of(int KH, int KW, int SW) {
  if (KH == 3 && KW == 4 && SW == 2) return 0;
  if (KH == 3 && KW == 3 && SW == 1) return 1;
  if (KH == 1 && KW == 1 && SW == 1) return 2;
  if (KH == 1 && KW == 3 && SW == 1) return 3;
  if (KH == 1 && KW == 7 && SW == 1) return 4;  // FidelityEnhancer init conv (k7, pad 3)
  if (KH == 1 && KW == 4 && SW == 2) return 5;  // FidelityEnhancer Downsample (k4, s2, pad 1)
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
  Epi e = {};
  e.bias = bias;
  e.residual = residual;
  e.drop_p = drop_p;
  e.drop_scale = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
  e.seed_ptr = seed_ptr;
  e.offset = offset;
  return e;
}

extern "C" int tvq_conv_packcache_begin(int64_t id, float* arena, int64_t cap_floats,
                                        tvq_stream_t stream) {
  TVQ_CHECK_ARG(id >= 0 && arena && cap_floats > 0, "tvq_conv_packcache_begin: bad arguments");
  TVQ_CHECK_ARG(!g_pc_cur, "tvq_conv_packcache_begin: a scope is already open");
  PackCacheState& pc = g_pcs[id];
  if (arena != pc.arena || cap_floats != pc.cap) {
    pc.entries.clear();
    pc.arena = arena;
    pc.cap = cap_floats;
    pc.used = 0;
  }
  hipStream_t st = (hipStream_t)stream;
  for (size_t i0 = 0; i0 < pc.entries.size(); i0 += PACK_BATCH) {
    PackBatch b;
    int n = 0;
    int64_t most = 0;
    for (size_t i = i0; i < pc.entries.size() && n < PACK_BATCH; ++i, ++n) {
      const PackEntry& p = pc.entries[i];
      b.src[n] = p.src; b.wsn[n] = (int)p.wsn; b.wsc[n] = (int)p.wsc; b.off[n] = p.off;
      b.N[n] = p.N; b.C[n] = p.C; b.KK[n] = p.KK;
      const int64_t t = (int64_t)p.N * p.C * p.KK;
      most = t > most ? t : most;
    }
    const int bx = (int)((most + 255) / 256 < 512 ? (most + 255) / 256 : 512);
    hipLaunchKernelGGL(conv_pack_multi_kernel, dim3(bx, n), dim3(256), 0, st, b, pc.arena);
  }
  g_pc_cur = &pc;
  g_pc_last = id;
  return launch_status("tvq_conv_packcache_begin");
}

extern "C" int tvq_conv_packcache_end(void) {
  g_pc_cur = nullptr;
  return TVQ_OK;
}

// pause(1): convs run without the open scope's cache (weights computed inside the scope,
// e.g. folded per call, must not be recorded: the cache repacks at the NEXT scope's begin,
// before such a weight is recomputed); pause(0) resumes it
static PackCacheState* g_pc_paused = nullptr;
extern "C" int tvq_conv_packcache_pause(int64_t on) {
  if (on) {
    TVQ_CHECK_ARG(!g_pc_paused, "tvq_conv_packcache_pause: already paused");
    g_pc_paused = g_pc_cur;
    g_pc_cur = nullptr;
  } else {
    g_pc_cur = g_pc_paused;
    g_pc_paused = nullptr;
  }
  return TVQ_OK;
}

extern "C" int tvq_conv_packcache_release(int64_t id) {
  auto it = g_pcs.find(id);
  if (it == g_pcs.end()) return TVQ_OK;
  TVQ_CHECK_ARG(g_pc_cur != &it->second, "tvq_conv_packcache_release: the cache's scope is open");
  g_pcs.erase(it);
  return TVQ_OK;
}

extern "C" int64_t tvq_conv_packcache_entries(void) {
  auto it = g_pcs.find(g_pc_last);
  return it == g_pcs.end() ? 0 : (int64_t)it->second.entries.size();
}

extern "C" int tvq_conv_wgrad_defer_begin(void) {
  TVQ_CHECK_ARG(!g_rd_on, "tvq_conv_wgrad_defer_begin: a scope is already open");
  g_rd.clear();
  g_rd_on = true;
  return TVQ_OK;
}

// kept for the ABI: every record now carries its own stream, so this is begin()
extern "C" int tvq_wgrad_defer_begin_stream(tvq_stream_t stream) {
  (void)stream;
  return tvq_conv_wgrad_defer_begin();
}

extern "C" int tvq_conv_wgrad_defer_pause(int64_t paused) {
  g_rd_paused = paused != 0;
  return TVQ_OK;
}

extern "C" int tvq_conv_wgrad_defer_flush(tvq_stream_t stream) {
  g_rd_on = false;
  g_rd_paused = false;
  // one batch per producing stream, in first-record order ((void)stream: kept for the ABI)
  (void)stream;
  std::vector<RrJob> jobs;
  while (!g_rd.empty()) {
    const hipStream_t st = g_rd.front().st;
    jobs.clear();
    std::vector<RdRec> rest;
    int64_t bytes = 0;
    for (const RdRec& r : g_rd) {
      if (r.st == st) {
        jobs.push_back(r.job);
        bytes += r.job.P * r.job.N * 4;
        TVQ_PLAN("wgrad_flush_job st=%p P=%lld N=%lld", (void*)st, (long long)r.job.P,
                 (long long)r.job.N);
      } else {
        rest.push_back(r);
      }
    }
    TVQ_PLAN("wgrad_flush st=%p jobs=%d MB=%.1f", (void*)st, (int)jobs.size(), bytes / 1e6);
    reduce_rows_batch(jobs.data(), (int)jobs.size(), st);
    g_rd.swap(rest);
  }
  return launch_status("tvq_conv_wgrad_defer_flush");
}

extern "C" int tvq_conv_config(int64_t halo) {
  const int prev = g_conv_halo | (g_conv_t32 ? 0 : 8) | (g_t32_bk == 32 ? 16 : 0) |
                   (g_t32_bk == 16 ? 32 : 0) | (g_t32_nw == 4 ? 64 : 0) |
                   (g_t32_n64 ? 128 : 0) | (g_conv_small ? 0 : 256) | (g_conv_s2 ? 0 : 512) |
                   (g_conv_ws2 ? 0 : 1024) | (g_conv_n16 ? 0 : 2048);
  if (halo >= 0) {
    g_conv_halo = (int)(halo & 7);
    g_conv_t32 = (halo & 8) ? 0 : 1;
    g_t32_bk = (halo & 16) ? 32 : ((halo & 32) ? 16 : 64);
    g_t32_nw = (halo & 64) ? 4 : 12;
    g_t32_n64 = (halo & 128) ? 1 : 0;
    g_conv_small = (halo & 256) ? 0 : 1;
    g_conv_s2 = (halo & 512) ? 0 : 1;
    g_conv_ws2 = (halo & 1024) ? 0 : 1;
    g_conv_n16 = (halo & 2048) ? 0 : 1;
  }
  return prev;
}

extern "C" int tvq_conv_out_width(int64_t Win, int64_t KW, int64_t SW, int64_t transposed) {
  const int64_t PW = (KW - 1) / 2;
  return (int)(transposed ? (Win - 1) * SW - 2 * PW + KW : (Win + 2 * PW - KW) / SW + 1);
}

#define PH_OF(KH) ((int)(KH) / 2)
#define PW_OF(KW) (((int)(KW) - 1) / 2)

// ---- geometry of each op as one F/T gather launch
static ConvGeom geom_conv_fwd(int64_t B, int64_t Ci, int64_t H, int64_t Wi, int64_t Co, int64_t KH,
                              int64_t KW, int64_t SW) {
  const int Wo = tvq_conv_out_width(Wi, KW, SW, 0);
  return make_geom((int)B, (int)Ci, (int)H, (int)Wi, (int)Co, (int)H, Wo, (int)KH, (int)KW,
                   PH_OF(KH), PW_OF(KW), Ci * KH * KW, KH * KW);
}
// ConvTranspose2d weight (Ci, Co, KH, KW): reduction channel c = ci (first dim)
static ConvGeom geom_convT_fwd(int64_t B, int64_t Ci, int64_t H, int64_t Wi, int64_t Co,
                               int64_t KH, int64_t KW, int64_t SW) {
  const int Wo = tvq_conv_out_width(Wi, KW, SW, 1);
  return make_geom((int)B, (int)Ci, (int)H, (int)Wi, (int)Co, (int)H, Wo, (int)KH, (int)KW,
                   PH_OF(KH), PW_OF(KW), KH * KW, Co * KH * KW);
}
// conv weight (Co, Ci, KH, KW): reduction c = co, output channel n = ci.  Replicate pad:
// gradient of the padded canvas (H+2PH, Wi+2PW) with zero offsets, folded afterwards.
static ConvGeom geom_conv_dgrad(int64_t B, int64_t Ci, int64_t H, int64_t Wi, int64_t Co,
                                int64_t KH, int64_t KW, int64_t SW, int64_t replicate) {
  const int Wo = tvq_conv_out_width(Wi, KW, SW, 0);
  if (!replicate)
    return make_geom((int)B, (int)Co, (int)H, Wo, (int)Ci, (int)H, (int)Wi, (int)KH, (int)KW,
                     PH_OF(KH), PW_OF(KW), KH * KW, Ci * KH * KW);
  return make_geom((int)B, (int)Co, (int)H, Wo, (int)Ci, (int)H + 2 * PH_OF(KH),
                   (int)Wi + 2 * PW_OF(KW), (int)KH, (int)KW, 0, 0, KH * KW, Ci * KH * KW);
}
// F-gather of dY with weight (Ci, Co, KH, KW) indexed (n = ci, c = co)
static ConvGeom geom_convT_dgrad(int64_t B, int64_t Ci, int64_t H, int64_t Wi, int64_t Co,
                                 int64_t KH, int64_t KW, int64_t SW) {
  const int Wo = tvq_conv_out_width(Wi, KW, SW, 1);
  return make_geom((int)B, (int)Co, (int)H, Wo, (int)Ci, (int)H, (int)Wi, (int)KH, (int)KW,
                   PH_OF(KH), PW_OF(KW), Co * KH * KW, KH * KW);
}

static int64_t canvas_floats(const ConvGeom& g) { return (int64_t)g.B * g.N * g.Hout * g.Wo; }

static bool geom_ok(const ConvGeom& g) {
  return g.Wo > 0 && g.Win > 0 && (int64_t)g.B * g.Hout * g.Wo < (1 << 30) &&
         (int64_t)g.B * g.N * g.Hout * g.Wo < (1ll << 31);
}

extern "C" int tvq_conv2d_fwd(const float* x, int64_t B, int64_t Ci, int64_t H, int64_t Wi,
                              const float* w, const float* bias, int64_t Co, int64_t KH,
                              int64_t KW, int64_t SW, int64_t replicate, float* y,
                              const float* residual, float drop_p, const int64_t* seed_ptr,
                              uint64_t offset, float* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && w && y && B > 0 && Ci > 0 && Co > 0, "tvq_conv2d_fwd: bad arguments");
  const int kind = kind_of((int)KH, (int)KW, (int)SW);
  TVQ_CHECK_ARG(kind >= 0, "tvq_conv2d_fwd: unsupported kernel %lldx%lld s%lld", (long long)KH,
                (long long)KW, (long long)SW);
  ConvGeom g = geom_conv_fwd(B, Ci, H, Wi, Co, KH, KW, SW);
  TVQ_CHECK_ARG(geom_ok(g), "tvq_conv2d_fwd: bad geometry");
  Epi e = make_epi(bias, residual, drop_p, seed_ptr, offset);
  hipStream_t st = (hipStream_t)stream;
#define M_(a, b_, c, d) launch_conv<GATHER_F, a, b_, c, d>(x, w, y, g, workspace, e, st);
  TVQ_DISPATCH_KIND(kind, replicate, M_)
#undef M_
  return launch_status("tvq_conv2d_fwd");
}

extern "C" int tvq_convT2d_fwd(const float* x, int64_t B, int64_t Ci, int64_t H, int64_t Wi,
                               const float* w, const float* bias, int64_t Co, int64_t KH,
                               int64_t KW, int64_t SW, float* y, const float* residual,
                               float* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && w && y && B > 0 && Ci > 0 && Co > 0, "tvq_convT2d_fwd: bad arguments");
  const int kind = kind_of((int)KH, (int)KW, (int)SW);
  TVQ_CHECK_ARG(kind >= 0, "tvq_convT2d_fwd: unsupported kernel");
  ConvGeom g = geom_convT_fwd(B, Ci, H, Wi, Co, KH, KW, SW);
  TVQ_CHECK_ARG(geom_ok(g), "tvq_convT2d_fwd: bad geometry");
  Epi e = make_epi(bias, residual, 0.f, nullptr, 0);
  hipStream_t st = (hipStream_t)stream;
#define M_(a, b_, c, d) launch_conv<GATHER_T, a, b_, c, false>(x, w, y, g, workspace, e, st);
  TVQ_DISPATCH_KIND(kind, 0, M_)
#undef M_
  return launch_status("tvq_convT2d_fwd");
}

// The training EncBlock / DecBlock conv with its BatchNorm's statistics in the epilogue
// (reference vq_vae.py:65-121: Conv2d / ConvTranspose2d (3x4, stride (1,2)) -> BatchNorm2d):
// tvq_conv_bnstats_blocks gives the number of per-block partials per channel (0: this shape
// does not take the stride-2 kernels, use tvq_conv2d_fwd + tvq_bn_train_fwd); part holds
// Co x blocks x 2 doubles for tvq_bn_train_apply_part.
static bool bnstats_geom(int64_t B, int64_t Ci, int64_t H, int64_t Wi, int64_t Co, int64_t KH,
                         int64_t KW, int64_t SW, int64_t transposed, ConvGeom* gout) {
  if (B <= 0 || Ci <= 0 || Co <= 0 || Wi <= 0 || kind_of((int)KH, (int)KW, (int)SW) != 0)
    return false;
  const ConvGeom g = transposed ? geom_convT_fwd(B, Ci, H, Wi, Co, KH, KW, SW)
                                : geom_conv_fwd(B, Ci, H, Wi, Co, KH, KW, SW);
  if (!geom_ok(g) || s2_kind(transposed ? GATHER_T : GATHER_F, g) != (transposed ? 2 : 1))
    return false;
  *gout = g;
  return true;
}

extern "C" int64_t tvq_conv_bnstats_blocks(int64_t B, int64_t Ci, int64_t H, int64_t Wi,
                                           int64_t Co, int64_t KH, int64_t KW, int64_t SW,
                                           int64_t transposed) {
  ConvGeom g;
  if (!bnstats_geom(B, Ci, H, Wi, Co, KH, KW, SW, transposed, &g)) return 0;
  return (int64_t)g.B * ((g.Wo + S2_SEG - 1) / S2_SEG);
}

extern "C" int tvq_conv2d_fwd_bnstats(const float* x, int64_t B, int64_t Ci, int64_t H,
                                      int64_t Wi, const float* w, const float* bias, int64_t Co,
                                      int64_t KH, int64_t KW, int64_t SW, int64_t replicate,
                                      int64_t transposed, float* y, double* part,
                                      tvq_stream_t stream) {
  ConvGeom g;
  TVQ_CHECK_ARG(x && w && y && part &&
                    bnstats_geom(B, Ci, H, Wi, Co, KH, KW, SW, transposed, &g) &&
                    !(transposed && replicate),
                "tvq_conv2d_fwd_bnstats: unsupported (see tvq_conv_bnstats_blocks)");
  Epi e = make_epi(bias, nullptr, 0.f, nullptr, 0);
  e.bn_part = part;
  hipStream_t st = (hipStream_t)stream;
  if (transposed)
    launch_s2<false>(2, x, w, y, g, e, st);
  else if (replicate)
    launch_s2<true>(1, x, w, y, g, e, st);
  else
    launch_s2<false>(1, x, w, y, g, e, st);
  return launch_status("tvq_conv2d_fwd_bnstats");
}

// Eval-mode conv -> BatchNorm(running statistics) -> Snake in one launch: the BN affine
// and the Snake are the conv epilogue's (epi_post), no (B, Co, H, W) round trip through
// HBM between them.  The same function as tvq_conv2d_fwd + tvq_bn_eval_fwd within ~1e-7
// relative, not bit for bit: the epilogue's GELU is the branch-free A&S erf (gelu_as) and its
// Snake sin^2 a Cody-Waite / polynomial form, where the separate launches call erff / sinf
// (tests/test_conv_bn_eval.py: 1e-6 of the two-launch path).
extern "C" int tvq_conv2d_fwd_bn_eval(const float* x, int64_t B, int64_t Ci, int64_t H,
                                      int64_t Wi, const float* w, const float* bias, int64_t Co,
                                      int64_t KH, int64_t KW, int64_t SW, int64_t replicate,
                                      int64_t pre_gelu, const float* bn_w, const float* bn_b,
                                      const float* running_mean, const float* running_var,
                                      float eps, const float* snake_a, float* y,
                                      float* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && w && y && running_mean && running_var && B > 0 && Ci > 0 && Co > 0,
                "tvq_conv2d_fwd_bn_eval: bad arguments");
  const int kind = kind_of((int)KH, (int)KW, (int)SW);
  TVQ_CHECK_ARG(kind >= 0, "tvq_conv2d_fwd_bn_eval: unsupported kernel");
  ConvGeom g = geom_conv_fwd(B, Ci, H, Wi, Co, KH, KW, SW);
  TVQ_CHECK_ARG(geom_ok(g), "tvq_conv2d_fwd_bn_eval: bad geometry");
  Epi e = make_epi(bias, nullptr, 0.f, nullptr, 0);
  e.bn_w = bn_w;
  e.bn_b = bn_b;
  e.bn_rm = running_mean;
  e.bn_rv = running_var;
  e.bn_eps = eps;
  e.snake_a = snake_a;
  e.gelu = pre_gelu != 0;
  hipStream_t st = (hipStream_t)stream;
  TVQ_PLAN("conv_bn_eval");
  t_post_done = false;
#define M_(a, b_, c, d) launch_conv<GATHER_F, a, b_, c, d>(x, w, y, g, workspace, e, st);
  TVQ_DISPATCH_KIND(kind, replicate, M_)
#undef M_
  if (!t_post_done) {  // this shape's conv path has no fused epilogue: the eval BN after it
    TVQ_PLAN("bn_eval separate");
    if (pre_gelu) {
      const int rg = tvq_gelu_fwd(y, B * Co * g.Hout * g.Wo, y, stream);
      if (rg != TVQ_OK) return rg;
    }
    const int rc = tvq_bn_eval_fwd(y, B, Co, (int64_t)g.Hout * g.Wo, bn_w, bn_b, running_mean,
                                   running_var, eps, snake_a, y, y, stream);
    if (rc != TVQ_OK) return rc;
  }
  return launch_status("tvq_conv2d_fwd_bn_eval");
}

extern "C" int tvq_convT2d_fwd_bn_eval(const float* x, int64_t B, int64_t Ci, int64_t H,
                                       int64_t Wi, const float* w, const float* bias, int64_t Co,
                                       int64_t KH, int64_t KW, int64_t SW, const float* bn_w,
                                       const float* bn_b, const float* running_mean,
                                       const float* running_var, float eps,
                                       const float* snake_a, float* y, float* workspace,
                                       tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && w && y && running_mean && running_var && B > 0 && Ci > 0 && Co > 0,
                "tvq_convT2d_fwd_bn_eval: bad arguments");
  const int kind = kind_of((int)KH, (int)KW, (int)SW);
  TVQ_CHECK_ARG(kind >= 0, "tvq_convT2d_fwd_bn_eval: unsupported kernel");
  ConvGeom g = geom_convT_fwd(B, Ci, H, Wi, Co, KH, KW, SW);
  TVQ_CHECK_ARG(geom_ok(g), "tvq_convT2d_fwd_bn_eval: bad geometry");
  Epi e = make_epi(bias, nullptr, 0.f, nullptr, 0);
  e.bn_w = bn_w;
  e.bn_b = bn_b;
  e.bn_rm = running_mean;
  e.bn_rv = running_var;
  e.bn_eps = eps;
  e.snake_a = snake_a;
  hipStream_t st = (hipStream_t)stream;
  TVQ_PLAN("convT_bn_eval");
  t_post_done = false;
#define M_(a, b_, c, d) launch_conv<GATHER_T, a, b_, c, false>(x, w, y, g, workspace, e, st);
  TVQ_DISPATCH_KIND(kind, 0, M_)
#undef M_
  if (!t_post_done) {  // this shape's conv path has no fused epilogue: the eval BN after it
    TVQ_PLAN("bn_eval separate");
    const int rc = tvq_bn_eval_fwd(y, B, Co, (int64_t)g.Hout * g.Wo, bn_w, bn_b, running_mean,
                                   running_var, eps, snake_a, y, y, stream);
    if (rc != TVQ_OK) return rc;
  }
  return launch_status("tvq_convT2d_fwd_bn_eval");
}

// workspace: [replicate canvas][pack + split-K slab]; required when replicate
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
  ConvGeom g = geom_conv_dgrad(B, Ci, H, Wi, Co, KH, KW, SW, replicate);
  TVQ_CHECK_ARG(geom_ok(g), "tvq_conv2d_dgrad: bad geometry");
  if (!replicate) {
#define M_(a, b_, c, d) launch_conv<GATHER_T, a, b_, c, false>(dy, w, dx, g, workspace, e, st);
    TVQ_DISPATCH_KIND(kind, 0, M_)
#undef M_
    return launch_status("tvq_conv2d_dgrad");
  }
  if (KH == 3 && KW == 4 && SW == 2 && s2_fold_fits(g)) {
    launch_s2_fold(dy, w, dx, g, st);
    return launch_status("tvq_conv2d_dgrad(replicate, s2)");
  }
  TVQ_CHECK_ARG(workspace, "tvq_conv2d_dgrad: replicate needs a workspace");
  float* canvas = workspace;
  float* rest = workspace + canvas_floats(g);
#define M_(a, b_, c, d) launch_conv<GATHER_T, a, b_, c, false>(dy, w, canvas, g, rest, e, st);
  TVQ_DISPATCH_KIND(kind, 0, M_)
#undef M_
  const int64_t tot = B * Ci * H * Wi;
  const int blocks = (int)((tot + 255) / 256 < 8192 ? (tot + 255) / 256 : 8192);
  hipLaunchKernelGGL(replicate_fold_kernel, dim3(blocks), dim3(256), 0, st, canvas, (int)B,
                     (int)Ci, (int)H, (int)Wi, PH_OF(KH), PW_OF(KW), dx);
  return launch_status("tvq_conv2d_dgrad(replicate)");
}

extern "C" int tvq_convT2d_dgrad(const float* dy, int64_t B, int64_t Co, int64_t H, int64_t Wo,
                                 const float* w, int64_t Ci, int64_t KH, int64_t KW, int64_t SW,
                                 float* dx, int64_t Wi, float* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(dy && w && dx && B > 0 && Ci > 0 && Co > 0, "tvq_convT2d_dgrad: bad arguments");
  const int kind = kind_of((int)KH, (int)KW, (int)SW);
  TVQ_CHECK_ARG(kind >= 0, "tvq_convT2d_dgrad: unsupported kernel");
  TVQ_CHECK_ARG(tvq_conv_out_width(Wi, KW, SW, 1) == Wo, "tvq_convT2d_dgrad: Wi/Wo mismatch");
  ConvGeom g = geom_convT_dgrad(B, Ci, H, Wi, Co, KH, KW, SW);
  TVQ_CHECK_ARG(geom_ok(g), "tvq_convT2d_dgrad: bad geometry");
  Epi e = make_epi(nullptr, nullptr, 0.f, nullptr, 0);
  hipStream_t st = (hipStream_t)stream;
#define M_(a, b_, c, d) launch_conv<GATHER_F, a, b_, c, false>(dy, w, dx, g, workspace, e, st);
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

static int64_t whalo_ws(int64_t N, int64_t C, int64_t KH, int64_t KW, int64_t B) {
  int FN, CB;
  const int KK = (int)(KH * KW);
  whalo_blocking(N, C, KK, &FN, &CB);
  const int nblk = (int)((N + FN * 16 - 1) / (FN * 16)), cblk = (int)((C + CB - 1) / CB);
  const int S = whalo_splits(N, C, KK, B, nblk, cblk);
  const int64_t kc = C * KK + 1;
  return (int64_t)S * N * kc + reduce_rows_scratch(S, N * kc);
}

static int64_t conv_wgrad_ws(int64_t N, int64_t C, int64_t KH, int64_t KW, int64_t B,
                             int64_t Hout, int64_t Wo) {
  const int64_t a = wgrad_ws(N, C * KH * KW, B * Hout * Wo, nullptr, nullptr);
  const int64_t h = whalo_ws(N, C, KH, KW, B);
  const int64_t w = (KH == 3 && KW == 3 && B % W8_IMG == 0) ? w8_ws(B, N, C) : 0;
  const int64_t t = wt32_fits(B, C, Hout, Wo, N, Wo, KH, KW, 1, 0)
                        ? wt32_ws(B, C, Hout, Wo, N, KH * KW) : 0;
  // conv_wgrad_s2 (Wo: the width of G)
  const int64_t s2 = (KH == 3 && KW == 4 && C <= 16 && N <= 16) ? ws2_ws(B, C, Wo, N) : 0;
  return std::max(std::max(std::max(a, t), std::max(h, w)), s2);
}

// op: 0 conv2d fwd, 1 convT2d fwd, 2 conv2d dgrad, 3 convT2d dgrad, 4 conv2d wgrad,
// 5 convT2d wgrad.  (Ci, Co, Wi) are the layer's input channels, output channels and
// input width.  Returns floats (>= 1).
extern "C" int64_t tvq_conv_workspace(int64_t op, int64_t B, int64_t Ci, int64_t H, int64_t Wi,
                                      int64_t Co, int64_t KH, int64_t KW, int64_t SW,
                                      int64_t replicate) {
  int64_t r = 0;
  const int KK = (int)(KH * KW);
  switch (op) {
    case 0: r = conv_gemm_ws(geom_conv_fwd(B, Ci, H, Wi, Co, KH, KW, SW), KK); break;
    case 1: r = conv_gemm_ws(geom_convT_fwd(B, Ci, H, Wi, Co, KH, KW, SW), KK); break;
    case 2: {
      const ConvGeom g = geom_conv_dgrad(B, Ci, H, Wi, Co, KH, KW, SW, replicate);
      r = (replicate ? canvas_floats(g) : 0) + conv_gemm_ws(g, KK);
      break;
    }
    case 3: r = conv_gemm_ws(geom_convT_dgrad(B, Ci, H, Wi, Co, KH, KW, SW), KK); break;
    case 4:
      r = conv_wgrad_ws(Co, Ci, KH, KW, B, H, tvq_conv_out_width(Wi, KW, SW, 0));
      break;
    case 5: r = conv_wgrad_ws(Ci, Co, KH, KW, B, H, Wi); break;
    default: return -1;
  }
  return r > 0 ? r : 1;
}

// Deferred weight-gradient split sums (tvq_conv_wgrad_defer_*): inside a scope the
// slabs' reductions are recorded and run by a few batched launches at the flush instead
// of one launch per conv (the caller keeps the workspaces alive until then).

static bool rd_records(int64_t rows) {
  return g_rd_on && !g_rd_paused && rows <= RR_ONE_ROWS;
}

static void wgrad_finish(float* slab, int splits, int64_t N, int64_t kcols, float* dw,
                         float* db, int accumulate, hipStream_t st) {
  // deterministic split sum; kcols = Kred+1 splits out the bias column.  The level-1
  // scratch follows the slab in the workspace.
  const int64_t L = kcols > 0 && db ? kcols : 0;
  if (rd_records(splits)) {  // the single-level case: batched at the flush
    g_rd.push_back({{slab, dw, db, splits, N * kcols, L, accumulate}, st});
    return;
  }
  reduce_rows(slab, splits, N * kcols, N * kcols, dw, db, L, accumulate,
              slab + (int64_t)splits * N * kcols, st);
}

// out[0..N) (+)= sum of the P contiguous rows of `in` (a parameter gradient only the
// optimizer reads): joins the open deferral scope's batch, else reduce_rows now
void tvq::param_rows_finish(const float* in, int64_t P, int64_t N, float* out, int accumulate,
                            float* scratch, hipStream_t st) {
  if (rd_records(P)) {
    g_rd.push_back({{in, out, nullptr, P, N, 0, accumulate}, st});
    return;
  }
  reduce_rows(in, P, N, N, out, nullptr, 0, accumulate, scratch, st);
}

void tvq::conv_wgrad_finish(float* slab, int splits, int64_t N, int64_t kcols, float* dw, float* db,
                       int accumulate, hipStream_t st) {
  wgrad_finish(slab, splits, N, kcols, dw, db, accumulate, st);
}

// Conv2d weight (+bias) gradient: dW[co,ci,kh,kw] (+)= sum dY[b,co,h,wo] X[b,ci,h+kh-PH, wo*SW+kw-PW],
// db[co] (+)= sum dY[b,co,h,wo] (db may be NULL)
namespace tvq {
static void w8_pair_launch(const float* x0, const float* dy0, float* ws0, float* dw0, float* db0,
                           const float* x1, const float* dy1, float* ws1, float* dw1, float* db1,
                           int64_t B, int64_t C, int64_t N, int accumulate, hipStream_t st) {
  const int S = (int)(B / W8_IMG);
  const int PS = whalo_plane_stride(5 * (8 + 2), 9, 3, 8 + 2, 1, 8);
  const dim3 grid((unsigned)S, (unsigned)(2 * (N / 32)), (unsigned)(C / 8));
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_wgrad_w8_kernel<8, 8>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
    attr = true;
  }
  const int kcols = (int)(C * 9 + 1);
  TVQ_PLAN("conv_wgrad_w8 pair S=%d", S);
  const W8Probs pr = {{dy0, dy1, nullptr, nullptr}, {x0, x1, nullptr, nullptr}, {ws0, ws1, nullptr, nullptr}};
  hipLaunchKernelGGL((conv_wgrad_w8_kernel<8, 8>), grid, dim3(256), (w8_lds<8, 8>(PS)), st, pr,
                     (int)B, (int)C, (int)N, kcols, PS);
  wgrad_finish(ws0, S, N, kcols, dw0, db0, accumulate, st);
  wgrad_finish(ws1, S, N, kcols, dw1, db1, accumulate, st);
}

// n <= 4 weight (+ bias) gradients of 3x3 stride-1 zero-padded convs of one shape on
// (B, C, 3, 16) maps in one launch (conv_wgrad_w8_kernel<16, 8>: the fused RB<32, 16>
// ResBlocks' conv1 / conv2, tvq_resblock.hip): problem i reduces dy[i] against x[i] into its
// S = B / 16 slab rows ws[i] (S * N * (9 C + 1) floats), summed in order by the deferred slab
// sum into dw[i] / db[i].
int64_t conv_wgrad_w16_slab_floats(int64_t B, int64_t C, int64_t N) {
  return (B / W8_IMG) * N * (C * 9 + 1);
}
bool conv_wgrad_w16_fits(int64_t B, int64_t C, int64_t N) {
  return B % W8_IMG == 0 && C % 8 == 0 && N % 32 == 0 && B > 0;
}
void conv_wgrad_w16_multi(int n, const float* const* x, const float* const* dy, float* const* ws,
                          float* const* dw, float* const* db, int64_t B, int64_t C, int64_t N,
                          int accumulate, hipStream_t st) {
  const int S = (int)(B / W8_IMG);
  const int PS = whalo_plane_stride(5 * (16 + 2), 9, 3, 16 + 2, 1, 8);
  const dim3 grid((unsigned)S, (unsigned)(n * (N / 32)), (unsigned)(C / 8));
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_wgrad_w8_kernel<16, 8>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
    attr = true;
  }
  W8Probs pr = {};
  for (int i = 0; i < n; ++i) {
    pr.G[i] = dy[i];
    pr.X[i] = x[i];
    pr.slab[i] = ws[i];
  }
  const int kcols = (int)(C * 9 + 1);
  TVQ_PLAN("conv_wgrad_w16 n=%d S=%d", n, S);
  hipLaunchKernelGGL((conv_wgrad_w8_kernel<16, 8>), grid, dim3(256), (w8_lds<16, 8>(PS)), st, pr,
                     (int)B, (int)C, (int)N, kcols, PS);
  for (int i = 0; i < n; ++i) wgrad_finish(ws[i], S, N, kcols, dw[i], db[i], accumulate, st);
}
// n <= 4 weight (+ bias) gradients of 3x3 stride-1 zero-padded C -> N convs on (B, C, 3, 8)
// maps in one conv_wgrad_w8_kernel<8, 8> launch (the LF ResBlock pair's four convs):
// problem i into its slab ws[i], each summed in order into dw[i] / db[i] (bit for bit the
// sums of one launch per problem)
bool conv_wgrad_w8_fits(int64_t B, int64_t C, int64_t N) {
  return w8_fits(B, C, 3, 8, N, 8, 3, 3, 1, 0);
}
void conv_wgrad_w8_multi(int n, const float* const* x, const float* const* dy, float* const* ws,
                         float* const* dw, float* const* db, int64_t B, int64_t C, int64_t N,
                         int accumulate, hipStream_t st) {
  const int S = (int)(B / W8_IMG);
  const int PS = whalo_plane_stride(5 * (8 + 2), 9, 3, 8 + 2, 1, 8);
  const dim3 grid((unsigned)S, (unsigned)(n * (N / 32)), (unsigned)(C / 8));
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_wgrad_w8_kernel<8, 8>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
    attr = true;
  }
  W8Probs pr = {};
  for (int i = 0; i < n; ++i) {
    pr.G[i] = dy[i];
    pr.X[i] = x[i];
    pr.slab[i] = ws[i];
  }
  const int kcols = (int)(C * 9 + 1);
  TVQ_PLAN("conv_wgrad_w8 n=%d S=%d", n, S);
  hipLaunchKernelGGL((conv_wgrad_w8_kernel<8, 8>), grid, dim3(256), (w8_lds<8, 8>(PS)), st, pr,
                     (int)B, (int)C, (int)N, kcols, PS);
  for (int i = 0; i < n; ++i) wgrad_finish(ws[i], S, N, kcols, dw[i], db[i], accumulate, st);
}
bool conv_wgrad_w8_pair(const float* x0, const float* dy0, float* ws0, float* dw0, float* db0,
                        const float* x1, const float* dy1, float* ws1, float* dw1, float* db1,
                        int64_t B, int64_t C, int64_t N, int accumulate, hipStream_t st) {
  if (!w8_fits(B, C, 3, 8, N, 8, 3, 3, 1, 0)) return false;
  w8_pair_launch(x0, dy0, ws0, dw0, db0, x1, dy1, ws1, dw1, db1, B, C, N, accumulate, st);
  return true;
}
}  // namespace tvq

extern "C" int tvq_conv2d_wgrad(const float* x, int64_t B, int64_t Ci, int64_t H, int64_t Wi,
                                const float* dy, int64_t Co, int64_t Wo, int64_t KH, int64_t KW,
                                int64_t SW, int64_t replicate, float* dw, float* db,
                                int64_t accumulate, float* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && dy && dw && workspace, "tvq_conv2d_wgrad: bad arguments");
  const int kind = kind_of((int)KH, (int)KW, (int)SW);
  TVQ_CHECK_ARG(kind >= 0, "tvq_conv2d_wgrad: unsupported kernel");
  ConvGeom g = make_geom((int)B, (int)Ci, (int)H, (int)Wi, (int)Co, (int)H, (int)Wo, (int)KH,
                         (int)KW, PH_OF(KH), PW_OF(KW), Ci * KH * KW, KH * KW);
  const int kcols = g.Kred + (db ? 1 : 0);
  hipStream_t st = (hipStream_t)stream;
  if (ws2_fits(Ci, H, Co, KH, KW, SW)) {
    const int S = ws2_launch(dy, x, workspace, (int)B, (int)Ci, (int)Co, (int)Wi, (int)Wo, kcols,
                             replicate != 0, st);
    wgrad_finish(workspace, S, Co, kcols, dw, db, (int)accumulate, st);
    return launch_status("tvq_conv2d_wgrad(s2)");
  }
  if (wt32_fits(B, Ci, H, Wi, Co, Wo, KH, KW, SW, replicate)) {
    WtGeom t;
    t.B = (int)B; t.C = (int)Ci; t.N = (int)Co; t.H = (int)H; t.W = (int)Wi;
    t.Kred = g.Kred; t.kcols = kcols; t.segs = (int)(Wi / 32);
    int S;
    wt32_plan(B, Ci, H, Wi, Co, KH * KW, &S, &t.spr);
    const int kt = (g.Kred + 127) / 128;
    t.ntiles = (int)((Co + 127) / 128);
    const dim3 grid(xcd_grid(S, kt * t.ntiles));
    TVQ_PLAN("conv_wgrad_t32 S=%d", S);
    if (KH == 3)
      hipLaunchKernelGGL((conv_wgrad_t32_kernel<3, 3>), grid, dim3(WT_T), 0, st, dy, x, workspace, t,
                         kt);
    else
      hipLaunchKernelGGL((conv_wgrad_t32_kernel<1, 3>), grid, dim3(WT_T), 0, st, dy, x, workspace, t,
                         kt);
    wgrad_finish(workspace, S, Co, kcols, dw, db, (int)accumulate, st);
    return launch_status("tvq_conv2d_wgrad(t32)");
  }
  if (w8_fits(B, Ci, H, Wi, Co, Wo, KH, KW, SW, replicate)) {
    const int S = (int)(B / W8_IMG);
    const int PS = whalo_plane_stride(5 * ((int)Wi + 2), 9, 3, (int)Wi + 2, 1, 8);
    const dim3 grid((unsigned)S, (unsigned)(Co / 32), (unsigned)(Ci / 8));
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_wgrad_w8_kernel<8, 8>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
      attr = true;
    }
    const size_t lds = w8_lds<8, 8>(PS);
    TVQ_PLAN("conv_wgrad_w8 S=%d", S);
    const W8Probs pr = {{dy, nullptr, nullptr, nullptr}, {x, nullptr, nullptr, nullptr},
                        {workspace, nullptr, nullptr, nullptr}};
    hipLaunchKernelGGL((conv_wgrad_w8_kernel<8, 8>), grid, dim3(256), lds, st, pr, (int)B, (int)Ci,
                       (int)Co, kcols, PS);
    wgrad_finish(workspace, S, Co, kcols, dw, db, (int)accumulate, st);
    return launch_status("tvq_conv2d_wgrad(w8)");
  }
  WHaloPlan pl;
  const bool halo = (g_conv_halo & 2) && whalo_plan((int)B, (int)Ci, (int)H, (int)Wi, (int)Co,
                                                    (int)H, (int)Wo, (int)KH, (int)KW, (int)SW,
                                                    PH_OF(KH), PW_OF(KW), kcols, &pl);
  // narrow maps with >= 32 channels: the direct kernel, into the slabs of the halo plan or
  // of the split GEMM (the workspace holds either)
  // (off by default: measured 6.06 vs 5.84 ms per joint step -- the per-step position
  // decode and gather address math of every lane outweigh the MFMA; the halo kernel stages
  // the image in LDS instead.  TVQ_CONV_WD32=1 turns it on.)
  if (wd32_on() && g_conv_t32 && g.Mpos <= d32_max_pos() && Co >= 32 && Ci >= 8 &&
      g.Kred >= 32) {
    int gs, gpps;
    wgrad_ws(Co, g.Kred, g.Mpos, &gs, &gpps);
    int pps;
    const int S = wd32_splits(g, kcols, halo && pl.S > gs ? pl.S : gs, &pps);
    const int ntiles = (int)((Co + 31) / 32), ctiles = (kcols + 31) / 32;
    const unsigned grid = (unsigned)(S * ntiles * ctiles);
    TVQ_PLAN("conv_wgrad_d32 S=%d", S);
#define M_(a, b_, c, d)                                                                        \
  hipLaunchKernelGGL((conv_wgrad_d32_kernel<a, b_, c, d>), dim3(grid), dim3(256), 0, st, dy, x, \
                     workspace, g, pps, kcols, ntiles, ctiles);
    TVQ_DISPATCH_KIND(kind, replicate, M_)
#undef M_
    wgrad_finish(workspace, S, Co, kcols, dw, db, (int)accumulate, st);
    return launch_status("tvq_conv2d_wgrad(direct)");
  }
  if (halo) {
    TVQ_PLAN("conv_wgrad_halo S=%d", pl.S);
#define M_(a, b_, c, d) launch_wgrad_halo<a, b_, c, d>(dy, x, workspace, pl, st);
    TVQ_DISPATCH_KIND(kind, replicate, M_)
#undef M_
    wgrad_finish(workspace, pl.S, Co, kcols, dw, db, (int)accumulate, st);
    return launch_status("tvq_conv2d_wgrad(halo)");
  }
  int splits, pps;
  wgrad_ws(Co, g.Kred, g.Mpos, &splits, &pps);
  TVQ_PLAN("conv_wgrad split=%d", splits);
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
  hipStream_t st = (hipStream_t)stream;
  if (ws2_fits(Co, H, Ci, KH, KW, SW)) {
    const int S = ws2_launch(x, dy, workspace, (int)B, (int)Co, (int)Ci, (int)Wo, (int)Wi, g.Kred,
                             false, st);
    wgrad_finish(workspace, S, Ci, g.Kred, dw, nullptr, (int)accumulate, st);
    return launch_status("tvq_convT2d_wgrad(s2)");
  }
  WHaloPlan pl;
  if ((g_conv_halo & 2) && whalo_plan((int)B, (int)Co, (int)H, (int)Wo, (int)Ci, (int)H, (int)Wi,
                                      (int)KH, (int)KW, (int)SW, PH_OF(KH), PW_OF(KW), g.Kred,
                                      &pl)) {
    TVQ_PLAN("conv_wgrad_halo S=%d", pl.S);
#define M_(a, b_, c, d) launch_wgrad_halo<a, b_, c, false>(x, dy, workspace, pl, st);
    TVQ_DISPATCH_KIND(kind, 0, M_)
#undef M_
    wgrad_finish(workspace, pl.S, Ci, g.Kred, dw, nullptr, (int)accumulate, st);
    return launch_status("tvq_convT2d_wgrad(halo)");
  }
  int splits, pps;
  wgrad_ws(Ci, g.Kred, g.Mpos, &splits, &pps);
  TVQ_PLAN("conv_wgrad split=%d", splits);
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
  int* cnt = counters(C, FIN_REDUCE);
  // whole images per chunk (at most the workspace's `chunks`, which is <= 64)
  const int64_t ipc = (B + chunks - 1) / chunks;
  const int64_t nch = (B + ipc - 1) / ipc;
  TVQ_CHECK_ARG(ipc * HW < (1ll << 31), "tvq_channel_sum: bad geometry");
  const int vec = (HW & 3) == 0 && ((uintptr_t)x & 15) == 0;
  hipLaunchKernelGGL(chan_sum_partial_kernel, dim3((int)C, (int)nch), dim3(256), 0, st, x,
                     (int)B, (int)C, (int)HW, (int)ipc, (int)nch, vec, workspace, cnt, out,
                     (int)accumulate);
  if (!cnt)
    hipLaunchKernelGGL(chan_sum_final_kernel, dim3((int)((C + 127) / 128)), dim3(128), 0, st,
                       workspace, (int)C, (int)nch, out, (int)accumulate);
  return launch_status("tvq_channel_sum");
}



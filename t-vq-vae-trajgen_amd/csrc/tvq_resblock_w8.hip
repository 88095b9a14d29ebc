// Fused ResBlock(64, 64) of the LF band on its (B, 64, 3, 8) maps (reference
// vq_vae.py:13-62; the last two encoder and first two decoder ResBlocks of the LF VQ-VAE):
//
//   y = x + Dropout_p(conv2(Snake_a2(BN(conv1(Snake_a1(x)) + b1))) + b2)
//
// The small-channel fused ResBlocks (tvq_resblock.hip) keep the whole 3x3 weight panel in
// LDS; a 64-channel panel is 147 KB, so here the weights stream from L2 as the MFMA A
// operand (packed [tap][c][n] by the step's pack cache: one coalesced 128-B row per half-wave
// and step) while the image -- 64 channels x 3 x 8, a 20 KB halo-plane stack -- is staged in
// LDS once per conv.  One 8-wave block per image (256 images = one block per CU); wave w
// owns output tile w & 1 (32 channels) and input-channel chunk w >> 1 (16 channels): 9 taps
// x 8 v_mfma_f32_32x32x2_f32 steps, its 72 weight values loaded before the first MFMA; the
// 4 chunk partials of a tile are summed in LDS in chunk order.  The 24 positions of an image
// fill 24 of the tile's 32 columns.
//
//   w8_fwd1  s1 = Snake_a1(x) staged (and stored: the conv1 weight gradient's input) ->
//            h = conv1(s1) + b1 -> store h; per-image fp64 BN partial sums
//   (bn_stats_final_kernel: 64 one-wave blocks reduce the partials in a fixed order to the
//            batch mean / invstd / affine form and the running statistics)
//   w8_fwd2  s2 = Snake_a2(BN(h)) staged (and stored) -> y = x + Dropout(conv2(s2) + b2)
//   w8_bwd2  g2 = Dropout'(dy) staged (and stored) -> ds2 = conv2^T(g2) -> du = ds2 *
//            Snake'(u) (u = BN(h) recomputed) -> store du; per-image (sum du, sum du xhat,
//            Snake a2 term)
//   (bn_bwd_final_kernel: those partials -> the BN backward coefficients, the BN weight /
//            bias and Snake a2 gradients)
//   w8_bwd1  dh = BN'(du) staged (and stored) -> ds1 = conv1^T(dh) -> dx = ds1 * Snake'(x)
//            + dy; the Snake a1 term (a slab row)
// Reducing the 256 images' partials in every consumer block (as the small-channel kernels
// do) read 256 KB of partials per block and held them in 128 VGPRs: 24 us per fwd2 / bwd1
// launch (round 5); the one-wave-per-channel finish launch is ~3 us.
//   weight gradients: (s2, g2) and (s1, dh) in one launch of the image-batched
//            conv_wgrad_w8 kernel (a 64 x 577 slab row per image would be 148 KB)
//   w8_eval  both convs in one launch with BN from the running statistics (the frozen
//            encoder of stage2, the LF decoder while sampling)
//
// Replaces, per ResBlock: tvq_snake_fwd, two conv launches, the whole-channel BN kernel, and
// in the backward the dropout, snake and BN kernels and two data-gradient convs.  Arithmetic
// is the per-op kernels' (Snake, BN affine / backward formulas, the dropout hash at the flat
// NCHW index) up to the summation order, which is fixed.
#include "tvq_bn.h"
#include "tvq_common.h"
#include "tvq_conv_internal.h"
#include "tvq_reduce.h"

namespace tvq {
namespace w8 {

constexpr int C = 64, W = 8, P = 3 * W, NW = 8, T = 64 * NW;
constexpr int WP = W + 2;      // halo row stride
constexpr int PS = 80;         // halo plane stride (5 x 10 cells, padded; == 16 mod 32)
constexpr int PLANE = C * PS;  // floats
constexpr int CPC = 16;        // input channels per wave chunk
constexpr int RED = NW * 16 * 64;
constexpr int K = 9 * C;

struct WView {  // element (row n, reduction channel c, tap t) at w[n*sn + c*sc + t*st]
  const float* w;
  int64_t sn, sc, st;
};

struct Args {
  const float *x, *h, *dy, *du_in;
  const float *a1, *b1, *a2, *b2;
  const float *bn_w, *bn_b, *rmean, *rvar;  // eval / BN backward
  const float* save;                         // mean | invstd | scale | shift
  const float* coef;                         // BN backward (sum du, sum du xhat) per channel
  WView w1, w2;                              // forward views (eval / fwd) or data-gradient views
  float *h_out, *s_out, *y, *du, *dx, *g_out, *slabda;
  double* part;
  float eps, drop_p, drop_scale, invN;
  const int64_t* seed_ptr;
  uint64_t offset;
  int B, accumulate;
  BNFinal fin;
  BNBwdFinal bfin;
};

__device__ __forceinline__ int wid_() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// halo cell of position p (the 3x3 window's centre)
__device__ __forceinline__ int cell(int c, int p) { return c * PS + WP + 1 + (p / W) * WP + p % W; }

// zero the border cells of the 64 halo planes
__device__ __forceinline__ void border(float* __restrict__ S) {
  for (int i = threadIdx.x; i < C * 26; i += T) {
    const int c = i / 26, r = i - 26 * c;
    int o;
    if (r < WP) o = r;
    else if (r < 2 * WP) o = 4 * WP + (r - WP);
    else {
      const int k = r - 2 * WP;
      o = (1 + (k >> 1)) * WP + ((k & 1) ? W + 1 : 0);
    }
    S[c * PS + o] = 0.f;
  }
}

// Elementwise layout: wave w, iteration j -> channel 8w + 2j + (lane >> 5), position lane & 31
// (valid below 24); a channel's 24 positions sit in one 32-lane half.
__device__ __forceinline__ int el_c(int j) { return 8 * wid_() + 2 * j + ((threadIdx.x & 63) >> 5); }
__device__ __forceinline__ int el_p() { return threadIdx.x & 31; }

// sum over the lane's 32-lane half (fixed xor tree)
__device__ __forceinline__ double half_sum_d(double v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// This lane's 72 weight values of the block's conv: a[t][u] = W(row 32 (w & 1) + (l & 31),
// reduction channel 16 (w >> 1) + (l >> 5) + 2u, tap t).  Issued at the kernel's start (the
// weights do not depend on the staged image), so their L2 round trip overlaps the prologue;
// the scheduling barrier keeps the compiler from sinking them next to their MFMAs.
__device__ __forceinline__ void load_w(const WView wv, float (&a)[9][8]) {
  const int lane = threadIdx.x & 63, wid = wid_();
  const int r32 = lane & 31, hl = lane >> 5;
  const int nt = wid & 1, c0 = (wid >> 1) * CPC;
  const float* wp = wv.w + (int64_t)(32 * nt + r32) * wv.sn + (int64_t)(c0 + hl) * wv.sc;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int u = 0; u < 8; ++u) a[t][u] = wp[(int64_t)(2 * u) * wv.sc + (int64_t)t * wv.st];
  __builtin_amdgcn_sched_barrier(0);
}

// The block's conv of the staged planes S: D[row][pos] for rows 32 (w & 1) .. and input
// chunk w >> 1 (weights `a` from load_w), partial tile to red[w][16][64].  FLIP: the data
// gradient (taps mirrored).
template <bool FLIP>
__device__ __forceinline__ void conv(const float (&a)[9][8], const float* __restrict__ S,
                                     float* __restrict__ red) {
  const int lane = threadIdx.x & 63, wid = wid_();
  const int r32 = lane & 31, hl = lane >> 5;
  const int c0 = (wid >> 1) * CPC;
  const int m = r32 < P ? r32 : 0;
  const float* sp = S + (c0 + hl) * PS + (m / W) * WP + (m % W);
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int tt = FLIP ? 8 - t : t, off = (tt / 3) * WP + tt % 3;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t][u], sp[2 * u * PS + off], acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) red[(wid * 16 + r) * 64 + lane] = acc[r];
}

// conv result (row n, position p): the 4 chunk partials of tile n / 32 summed in order
__device__ __forceinline__ float conv_at(const float* __restrict__ red, int n, int p) {
  const int nt = n >> 5, i = n & 31, h = (i >> 2) & 1, r = (i & 3) + 4 * (i >> 3);
  const int l = p + 32 * h;
  float s = red[(nt * 16 + r) * 64 + l];
#pragma unroll
  for (int ch = 1; ch < 4; ++ch) s += red[((nt + 2 * ch) * 16 + r) * 64 + l];
  return s;
}

// ---------------------------------------------------------------- kernels
// The kernels' bodies take the block's LDS, the weight registers and, for a fused pair of
// consecutive ResBlocks (w8_fwd21 / w8_bwd12 below), the activation handed over in
// registers (every kernel has the same elementwise layout) with the next body's weights
// already loaded (issued right after the first body's last MFMA).
__device__ __forceinline__ void fwd1_body(const Args& a, float* sm, float (&wa)[9][8],
                                          const float (*xin)[4]) {
  float* S = sm;
  float* red = sm + PLANE;
  const int b = blockIdx.x, p = el_p();
  const int64_t img0 = (int64_t)b * C * P;
  float xv[4], av[4], bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    xv[j] = xin ? (*xin)[j] : a.x[img0 + el_c(j) * P + (p < P ? p : 0)];
    av[j] = a.a1[el_c(j)];
    bv[j] = a.b1[el_c(j)];
  }
  // after the staging operands: their wait leaves the weights in flight (a pair's second
  // body has them already)
  if (!xin) load_w(a.w1, wa);
  border(S);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = el_c(j);
    if (p >= P) continue;
    const float s = snake_f(xv[j], av[j], 1.0f / av[j]);
    S[cell(c, p)] = s;
    a.s_out[img0 + c * P + p] = s;
  }
  __syncthreads();
  conv<false>(wa, S, red);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = el_c(j);
    double s0 = 0.0, s1 = 0.0;
    if (p < P) {
      const float v = conv_at(red, c, p) + bv[j];
      a.h_out[img0 + c * P + p] = v;
      s0 = (double)v;
      s1 = (double)v * (double)v;
    }
    s0 = half_sum_d(s0);
    s1 = half_sum_d(s1);
    if ((threadIdx.x & 31) == 0) {  // [c][image][2]: bn_stats_final_kernel's chunk layout
      a.part[((int64_t)c * a.B + b) * 2 + 0] = s0;
      a.part[((int64_t)c * a.B + b) * 2 + 1] = s1;
    }
  }
}

__global__ __launch_bounds__(T) void w8_fwd1_kernel(Args a) {
  extern __shared__ float sm[];
  float wa[9][8];
  fwd1_body(a, sm, wa, nullptr);
}

// next: the following body's weights, loaded into wa once this conv is done with them
__device__ __forceinline__ void fwd2_body(const Args& a, float* sm, float (&wa)[9][8],
                                          float (&yout)[4], const WView* next) {
  float* S = sm;
  float* red = sm + PLANE;
  const int b = blockIdx.x, p = el_p();
  const int64_t img0 = (int64_t)b * C * P;
  float hv[4], xv[4], av[4], bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t gi = img0 + el_c(j) * P + (p < P ? p : 0);
    hv[j] = a.h[gi];
    xv[j] = a.x[gi];
    av[j] = a.a2[el_c(j)];
    bv[j] = a.b2[el_c(j)];
  }
  float sc[4], sh[4];  // the batch statistics' affine form (bn_stats_final_kernel's)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    sc[j] = a.save[2 * C + el_c(j)];
    sh[j] = a.save[3 * C + el_c(j)];
  }
  load_w(a.w2, wa);
  border(S);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = el_c(j);
    if (p >= P) continue;
    const float s = snake_f(fmaf(hv[j], sc[j], sh[j]), av[j], 1.0f / av[j]);
    S[cell(c, p)] = s;
    a.s_out[img0 + c * P + p] = s;
  }
  __syncthreads();
  conv<false>(wa, S, red);
  if (next) load_w(*next, wa);
  __syncthreads();
  const uint64_t seed = a.drop_p > 0.f ? mix_seed(a.seed_ptr, a.offset) : 0ull;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = el_c(j);
    yout[j] = 0.f;
    if (p >= P) continue;
    const int64_t gi = img0 + c * P + p;
    float v = conv_at(red, c, p) + bv[j];
    if (a.drop_p > 0.f) v = uniform01(seed, (uint64_t)gi) >= a.drop_p ? v * a.drop_scale : 0.f;
    yout[j] = xv[j] + v;
    a.y[gi] = yout[j];
  }
}

__global__ __launch_bounds__(T) void w8_fwd2_kernel(Args a) {
  extern __shared__ float sm[];
  float wa[9][8], y[4];
  fwd2_body(a, sm, wa, y, nullptr);
}

// fwd2 of ResBlock 1 and fwd1 of ResBlock 2 (its input = ResBlock 1's output) in one launch
__global__ __launch_bounds__(T) void w8_fwd21_kernel(Args a1, Args a2) {
  extern __shared__ float sm[];
  float wa[9][8], y[4];
  fwd2_body(a1, sm, wa, y, &a2.w1);
  __syncthreads();  // LDS reused
  fwd1_body(a2, sm, wa, &y);
}

__global__ __launch_bounds__(T) void w8_eval_kernel(Args a) {
  extern __shared__ float sm[];
  float* S = sm;
  float* red = sm + PLANE;
  const int b = blockIdx.x, p = el_p();
  const int64_t img0 = (int64_t)b * C * P;
  float wa[9][8], xv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) xv[j] = a.x[img0 + el_c(j) * P + (p < P ? p : 0)];
  load_w(a.w1, wa);
  border(S);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = el_c(j);
    if (p >= P) continue;
    const float av = a.a1[c];
    S[cell(c, p)] = snake_f(xv[j], av, 1.0f / av);
  }
  __syncthreads();
  conv<false>(wa, S, red);
  load_w(a.w2, wa);  // conv2's weights in flight during conv1's epilogue
  __syncthreads();
  float s2[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {  // BN from the running statistics (bn_eval's affine form)
    const int c = el_c(j);
    const float inv = 1.0f / sqrtf(a.rvar[c] + a.eps);
    const float scv = (a.bn_w ? a.bn_w[c] : 1.f) * inv;
    const float shv = (a.bn_b ? a.bn_b[c] : 0.f) - a.rmean[c] * scv;
    const float av = a.a2[c];
    s2[j] = snake_f(fmaf(conv_at(red, c, p < P ? p : 0) + a.b1[c], scv, shv), av, 1.0f / av);
  }
  __syncthreads();  // conv1's partials read; S free
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (p < P) S[cell(el_c(j), p)] = s2[j];
  __syncthreads();
  conv<false>(wa, S, red);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = el_c(j);
    if (p < P) a.y[img0 + c * P + p] = xv[j] + (conv_at(red, c, p) + a.b2[c]);
  }
}

__device__ __forceinline__ void bwd2_body(const Args& a, float* sm, float (&wa)[9][8],
                                          const float (*dyin)[4]) {
  float* G = sm;
  float* red = sm + PLANE;
  const int b = blockIdx.x, p = el_p();
  const int64_t img0 = (int64_t)b * C * P;
  float gv[4], hv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t gi = img0 + el_c(j) * P + (p < P ? p : 0);
    gv[j] = dyin ? (*dyin)[j] : a.dy[gi];
    hv[j] = a.h[gi];
  }
  if (!dyin) load_w(a.w2, wa);
  border(G);
  const uint64_t seed = a.drop_p > 0.f ? mix_seed(a.seed_ptr, a.offset) : 0ull;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = el_c(j);
    if (p >= P) continue;
    const int64_t gi = img0 + c * P + p;
    float d = gv[j];
    if (a.drop_p > 0.f) d = uniform01(seed, (uint64_t)gi) >= a.drop_p ? d * a.drop_scale : 0.f;
    G[cell(c, p)] = d;
    a.g_out[gi] = d;
  }
  __syncthreads();
  conv<true>(wa, G, red);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = el_c(j);
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    if (p < P) {
      const float av = a.a2[c], inv_a = 1.0f / av;
      const float sc = a.save[2 * C + c], sh = a.save[3 * C + c];
      const float mu = a.save[c], is = a.save[C + c];
      const float gs = conv_at(red, c, p);  // d loss / d s2
      const float uu = fmaf(hv[j], sc, sh);
      float sn, cs;
      sincosf(av * uu, &sn, &cs);
      const float tt = 2.0f * sn * cs;
      const float d = gs + gs * inv_a * tt * av;  // d loss / d u (bn_bwd_partial_kernel)
      const float xhat = (hv[j] - mu) * is;
      a.du[img0 + c * P + p] = d;
      s0 = d;
      s1 = (double)d * xhat;
      s2 = (double)(gs * inv_a * tt * uu) - (double)(gs * (sn * sn) * inv_a * inv_a);
    }
    s0 = half_sum_d(s0);
    s1 = half_sum_d(s1);
    s2 = half_sum_d(s2);
    if ((threadIdx.x & 31) == 0) {  // [c][image][3]: bn_bwd_final_kernel's chunk layout
      double* pp = a.part + ((int64_t)c * a.B + b) * 3;
      pp[0] = s0;
      pp[1] = s1;
      pp[2] = s2;
    }
  }
}

__global__ __launch_bounds__(T) void w8_bwd2_kernel(Args a) {
  extern __shared__ float sm[];
  float wa[9][8];
  bwd2_body(a, sm, wa, nullptr);
}

__device__ __forceinline__ void bwd1_body(const Args& a, float* sm, float (&wa)[9][8],
                                          float (&dxout)[4], const WView* next) {
  float* G = sm;
  float* red = sm + PLANE;
  const int b = blockIdx.x, p = el_p();
  const int64_t img0 = (int64_t)b * C * P;
  float dv[4], hv[4], xv[4], yv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t gi = img0 + el_c(j) * P + (p < P ? p : 0);
    dv[j] = a.du_in[gi];
    hv[j] = a.h[gi];
    xv[j] = a.x[gi];  // the epilogue's operands, requested with the prologue's
    yv[j] = a.dy[gi];
  }
  float md[4], mx[4];  // the BN backward coefficients (bn_bwd_final_kernel's sums)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    md[j] = a.coef[2 * el_c(j)] * a.invN;
    mx[j] = a.coef[2 * el_c(j) + 1] * a.invN;
  }
  load_w(a.w1, wa);
  border(G);
  // dh = w * invstd * (du - mean(du) - xhat * mean(du * xhat))  (bn_bwd_apply_kernel)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = el_c(j);
    if (p >= P) continue;
    const float mu = a.save[c], is = a.save[C + c], bw = a.bn_w ? a.bn_w[c] : 1.f;
    const float xhat = (hv[j] - mu) * is;
    const float g = bw * is * (dv[j] - md[j] - xhat * mx[j]);
    G[cell(c, p)] = g;
    a.g_out[img0 + c * P + p] = g;
  }
  __syncthreads();
  conv<true>(wa, G, red);
  if (next) load_w(*next, wa);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = el_c(j);
    double s0 = 0.0;
    dxout[j] = 0.f;
    if (p < P) {
      const int64_t gi = img0 + c * P + p;
      const float av = a.a1[c], inv_a = 1.0f / av;
      const float gs = conv_at(red, c, p);  // d loss / d s1
      float sn, cs;
      sincosf(av * xv[j], &sn, &cs);
      const float tt = 2.0f * sn * cs;
      // snake_bwd_kernel, plus the identity skip's gradient
      dxout[j] = (gs + gs * inv_a * tt * av) + yv[j];
      a.dx[gi] = dxout[j];
      s0 = (double)(gs * inv_a * tt * xv[j]) - (double)(gs * (sn * sn) * inv_a * inv_a);
    }
    s0 = half_sum_d(s0);
    if ((threadIdx.x & 31) == 0) a.slabda[(int64_t)b * C + c] = (float)s0;
  }
}

__global__ __launch_bounds__(T) void w8_bwd1_kernel(Args a) {
  extern __shared__ float sm[];
  float wa[9][8], dx[4];
  bwd1_body(a, sm, wa, dx, nullptr);
}

// bwd1 of ResBlock 2 and bwd2 of ResBlock 1 (its output gradient = ResBlock 2's input
// gradient) in one launch
__global__ __launch_bounds__(T) void w8_bwd12_kernel(Args a2, Args a1) {
  extern __shared__ float sm[];
  float wa[9][8], d[4];
  bwd1_body(a2, sm, wa, d, &a1.w2);
  __syncthreads();  // LDS reused
  bwd2_body(a1, sm, wa, &d);
}

constexpr size_t LDS = 4 * (size_t)(PLANE + RED);

static void set_lds() {
  static bool done = false;
  if (done) return;
  const void* ks[] = {(const void*)&w8_fwd1_kernel, (const void*)&w8_fwd2_kernel,
                      (const void*)&w8_eval_kernel, (const void*)&w8_bwd2_kernel,
                      (const void*)&w8_bwd1_kernel, (const void*)&w8_fwd21_kernel,
                      (const void*)&w8_bwd12_kernel};
  for (const void* k : ks)
    (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS);
  done = true;
}

static size_t al(size_t n) { return (n + 255) & ~(size_t)255; }

struct Ws {  // workspace layout (bytes)
  size_t part, slabda1, slabda2, g2, dh, du, wg1, wg2, pk, total;
};
static Ws ws_layout(int64_t B) {
  Ws w;
  const size_t img = (size_t)B * C * P * 4;
  const size_t slabd = (size_t)(B * C + reduce_rows_scratch(B, C)) * 4;
  const size_t wg = (size_t)tvq_conv_workspace(4, B, C, 3, W, C, 3, 3, 1, 0) * 4;
  w.part = 0;
  w.slabda1 = w.part + al((size_t)B * C * 3 * 8);
  w.slabda2 = w.slabda1 + al(slabd);
  w.g2 = w.slabda2 + al(slabd);
  w.dh = w.g2 + al(img);
  w.du = w.dh + al(img);
  w.wg1 = w.du + al(img);
  w.wg2 = w.wg1 + al(wg);
  w.pk = w.wg2 + al(wg);
  w.total = w.pk + al((size_t)4 * K * C * 4);  // w1, w2 forward and data-gradient packs
  return w;
}

static WView view(const float* w, bool transposed, float* ws, hipStream_t st) {
  WView v;
  // forward: rows = output channels n (stride K), reduction = input channels c (stride 9);
  // data gradient: rows = input channels, reduction = output channels
  v.w = conv_pack_view(w, C, C, 9, transposed ? 9 : K, transposed ? K : 9, ws, st, &v.sn,
                       &v.sc, &v.st);
  return v;
}

}  // namespace w8

bool w8_supported(int64_t B, int64_t C, int64_t H, int64_t W) {
  return C == w8::C && H == 3 && W == w8::W && B >= 1 && B * C * 3 * W < (1ll << 31);
}
int64_t w8_workspace(int64_t B) { return (int64_t)w8::ws_layout(B).total; }
int64_t w8_saved_floats(int64_t B) { return 3 * B * w8::C * w8::P; }  // h | s1 | s2

int w8_train_fwd(const float* x, int64_t B, const float* a1, const float* w1, const float* b1,
                 const float* bn_w, const float* bn_b, float* running_mean, float* running_var,
                 int64_t* nbt, float momentum, float eps, const float* a2, const float* w2,
                 const float* b2, float drop_p, const int64_t* seed_ptr, uint64_t offset,
                 float* saved, float* y, float* save, void* workspace, hipStream_t st) {
  using namespace w8;
  set_lds();
  const Ws L = ws_layout(B);
  char* ws = (char*)workspace;
  float* pk = (float*)(ws + L.pk);
  const int64_t img = B * C * P;
  Args a = {};
  a.x = x; a.a1 = a1; a.b1 = b1; a.a2 = a2; a.b2 = b2;
  a.w1 = view(w1, false, pk, st);
  a.w2 = view(w2, false, pk + K * C, st);
  a.h_out = saved; a.h = saved; a.y = y;
  a.part = (double*)(ws + L.part);
  a.B = (int)B;
  a.drop_p = drop_p;
  a.drop_scale = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
  a.seed_ptr = seed_ptr; a.offset = offset;
  a.fin = {C, (int)B, B * P, eps, momentum, bn_w, bn_b, running_mean, running_var, nbt,
           save, save + C, save + 2 * C, save + 3 * C};
  TVQ_PLAN("w8_fwd1 C%d W%d B%lld", C, W, (long long)B);
  a.s_out = saved + img;  // s1
  hipLaunchKernelGGL(w8_fwd1_kernel, dim3((unsigned)B), dim3(T), LDS, st, a);
  a.fin.chunks = (int)B;  // the per-image partials -> save, running statistics
  bn_stats_final_launch(a.part, a.fin, st);
  a.save = save;
  TVQ_PLAN("w8_fwd2 C%d W%d B%lld", C, W, (long long)B);
  a.s_out = saved + 2 * img;  // s2
  hipLaunchKernelGGL(w8_fwd2_kernel, dim3((unsigned)B), dim3(T), LDS, st, a);
  return launch_status("tvq_resblock_train_fwd");
}

int w8_eval_fwd(const float* x, int64_t B, const float* a1, const float* w1, const float* b1,
                const float* bn_w, const float* bn_b, const float* running_mean,
                const float* running_var, float eps, const float* a2, const float* w2,
                const float* b2, float* y, hipStream_t st) {
  using namespace w8;
  set_lds();
  Args a = {};
  a.x = x; a.a1 = a1; a.b1 = b1; a.a2 = a2; a.b2 = b2;
  a.bn_w = bn_w; a.bn_b = bn_b; a.rmean = running_mean; a.rvar = running_var; a.eps = eps;
  // no workspace: the open pack-cache scope's packs, else the weights as they are
  a.w1 = view(w1, false, nullptr, st);
  a.w2 = view(w2, false, nullptr, st);
  a.y = y; a.B = (int)B;
  TVQ_PLAN("w8_eval C%d W%d B%lld packed=%d", C, W, (long long)B, (int)(a.w1.sn == 1));
  hipLaunchKernelGGL(w8_eval_kernel, dim3((unsigned)B), dim3(T), LDS, st, a);
  return launch_status("tvq_resblock_eval_fwd");
}

int w8_bwd(const float* dy, const float* x, const float* saved, int64_t B, const float* a1,
           const float* w1, const float* bn_w, const float* save, const float* a2,
           const float* w2, float drop_p, const int64_t* seed_ptr, uint64_t offset, float* dx,
           float* da1, float* dw1, float* db1, float* dbn_w, float* dbn_b, float* da2, float* dw2,
           float* db2, int64_t accumulate, void* workspace, hipStream_t st) {
  using namespace w8;
  set_lds();
  const Ws L = ws_layout(B);
  char* ws = (char*)workspace;
  float* pk = (float*)(ws + L.pk);
  const int64_t img = B * C * P;
  const float* h = saved;
  const float* s1 = saved + img;
  const float* s2 = saved + 2 * img;
  float* g2 = (float*)(ws + L.g2);
  float* dh = (float*)(ws + L.dh);
  float* du = (float*)(ws + L.du);
  float* slabda1 = (float*)(ws + L.slabda1);
  Args a = {};
  a.x = x; a.h = h; a.dy = dy; a.du_in = du;
  a.a1 = a1; a.a2 = a2; a.bn_w = bn_w; a.save = save;
  a.w1 = view(w1, true, pk + 2 * K * C, st);
  a.w2 = view(w2, true, pk + 3 * K * C, st);
  a.du = du; a.dx = dx;
  a.part = (double*)(ws + L.part);
  a.B = (int)B; a.accumulate = (int)accumulate;
  a.drop_p = drop_p;
  a.drop_scale = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
  a.seed_ptr = seed_ptr; a.offset = offset;
  a.invN = 1.0f / (float)(B * P);
  float* coef = (float*)(ws + L.slabda2);  // 2C floats
  a.bfin = {C, (int)B, coef, dbn_w, dbn_b, da2, (int)accumulate};
  a.coef = coef;
  TVQ_PLAN("w8_bwd2 C%d W%d B%lld", C, W, (long long)B);
  a.g_out = g2;
  hipLaunchKernelGGL(w8_bwd2_kernel, dim3((unsigned)B), dim3(T), LDS, st, a);
  int rc = launch_status("tvq_resblock_bwd");
  if (rc) return rc;
  // per-image partials -> the BN backward coefficients, BN weight / bias and Snake a2 gradients
  bn_bwd_final_launch(a.part, a.bfin, st);
  TVQ_PLAN("w8_bwd1 C%d W%d B%lld", C, W, (long long)B);
  a.g_out = dh; a.slabda = slabda1;
  hipLaunchKernelGGL(w8_bwd1_kernel, dim3((unsigned)B), dim3(T), LDS, st, a);
  rc = launch_status("tvq_resblock_bwd");
  if (rc) return rc;
  // both convs' weight gradients, (s2, g2) and (s1, dh), in one launch
  if (!conv_wgrad_w8_pair(s2, g2, (float*)(ws + L.wg2), dw2, db2, s1, dh, (float*)(ws + L.wg1),
                          dw1, db1, B, C, C, (int)accumulate, st)) {
    rc = tvq_conv2d_wgrad(s2, B, C, 3, W, g2, C, W, 3, 3, 1, 0, dw2, db2, accumulate,
                          (float*)(ws + L.wg2), st);
    if (rc) return rc;
    rc = tvq_conv2d_wgrad(s1, B, C, 3, W, dh, C, W, 3, 3, 1, 0, dw1, db1, accumulate,
                          (float*)(ws + L.wg1), st);
    if (rc) return rc;
  }
  conv_wgrad_finish(slabda1, (int)B, C, 1, da1, nullptr, (int)accumulate, st);
  return launch_status("tvq_resblock_bwd");
}

// Two consecutive ResBlock(64, 64)s (tvq_resblock_pair_train_fwd / _bwd): p = {a1, w1, b1,
// bn_w, bn_b, a2, w2, b2}, rs = {running_mean, running_var}; 5 launches forward instead of 6
// (w8_fwd21 = block 1's fwd2 + block 2's fwd1), 4 + weight gradients backward instead of 5.
int w8_pair_train_fwd(const float* x, int64_t B, const float* const* p1, const float* const* p2,
                      float* const* rs1, float* const* rs2, int64_t* nbt1, int64_t* nbt2,
                      float momentum, float eps, float drop_p, const int64_t* seed_ptr,
                      uint64_t off1, uint64_t off2, float* saved1, float* y1, float* save1,
                      float* saved2, float* y2, float* save2, void* ws1, void* ws2,
                      hipStream_t st) {
  using namespace w8;
  set_lds();
  const int64_t img = B * C * P;
  Args A[2];
  const float* const* ps[2] = {p1, p2};
  float* const* rss[2] = {rs1, rs2};
  int64_t* nbts[2] = {nbt1, nbt2};
  const float* xs[2] = {x, y1};
  float* saveds[2] = {saved1, saved2};
  float* ys[2] = {y1, y2};
  float* saves[2] = {save1, save2};
  void* wss[2] = {ws1, ws2};
  const uint64_t offs[2] = {off1, off2};
  for (int i = 0; i < 2; ++i) {
    const Ws L = ws_layout(B);
    char* ws = (char*)wss[i];
    float* pk = (float*)(ws + L.pk);
    const float* const* p = ps[i];
    Args& a = A[i];
    a = Args{};
    a.x = xs[i]; a.a1 = p[0]; a.b1 = p[2]; a.a2 = p[5]; a.b2 = p[7];
    a.w1 = view(p[1], false, pk, st);
    a.w2 = view(p[6], false, pk + K * C, st);
    a.h_out = saveds[i]; a.h = saveds[i]; a.y = ys[i];
    a.part = (double*)(ws + L.part);
    a.B = (int)B;
    a.drop_p = drop_p;
    a.drop_scale = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
    a.seed_ptr = seed_ptr; a.offset = offs[i];
    float* sv = saves[i];
    a.fin = {C, (int)B, B * P, eps, momentum, p[3], p[4], rss[i][0], rss[i][1], nbts[i],
             sv, sv + C, sv + 2 * C, sv + 3 * C};
    a.fin.chunks = (int)B;
    a.save = sv;
  }
  TVQ_PLAN("w8_fwd1 C%d W%d B%lld", C, W, (long long)B);
  A[0].s_out = saved1 + img;  // s1 of block 1
  hipLaunchKernelGGL(w8_fwd1_kernel, dim3((unsigned)B), dim3(T), LDS, st, A[0]);
  bn_stats_final_launch(A[0].part, A[0].fin, st);
  TVQ_PLAN("w8_fwd21 C%d W%d B%lld", C, W, (long long)B);
  A[0].s_out = saved1 + 2 * img;  // s2 of block 1
  A[1].s_out = saved2 + img;      // s1 of block 2
  hipLaunchKernelGGL(w8_fwd21_kernel, dim3((unsigned)B), dim3(T), LDS, st, A[0], A[1]);
  bn_stats_final_launch(A[1].part, A[1].fin, st);
  TVQ_PLAN("w8_fwd2 C%d W%d B%lld", C, W, (long long)B);
  A[1].s_out = saved2 + 2 * img;
  hipLaunchKernelGGL(w8_fwd2_kernel, dim3((unsigned)B), dim3(T), LDS, st, A[1]);
  return launch_status("tvq_resblock_pair_train_fwd");
}

// q = {a1, w1, bn_w, save, a2, w2}, g = {da1, dw1, db1, dbn_w, dbn_b, da2, dw2, db2}
int w8_pair_bwd(const float* dy, const float* x, int64_t B, const float* const* q1,
                const float* const* q2, const float* saved1, const float* y1,
                const float* saved2, float drop_p, const int64_t* seed_ptr, uint64_t off1,
                uint64_t off2, float* dx, float* dy1, float* const* g1, float* const* g2,
                int64_t accumulate, void* ws1, void* ws2, hipStream_t st) {
  using namespace w8;
  set_lds();
  const Ws L = ws_layout(B);
  const int64_t img = B * C * P;
  // index 0: block 2 (runs first), 1: block 1
  const float* const* qs[2] = {q2, q1};
  float* const* gs[2] = {g2, g1};
  const float* dys[2] = {dy, dy1};
  const float* xs[2] = {y1, x};
  const float* saveds[2] = {saved2, saved1};
  float* dxs[2] = {dy1, dx};
  void* wss[2] = {ws2, ws1};
  const uint64_t offs[2] = {off2, off1};
  Args A[2];
  for (int i = 0; i < 2; ++i) {
    char* ws = (char*)wss[i];
    float* pk = (float*)(ws + L.pk);
    const float* const* q = qs[i];
    float* const* g = gs[i];
    Args& a = A[i];
    a = Args{};
    a.x = xs[i]; a.h = saveds[i]; a.dy = dys[i]; a.du_in = (float*)(ws + L.du);
    a.a1 = q[0]; a.a2 = q[4]; a.bn_w = q[2]; a.save = q[3];
    a.w1 = view(q[1], true, pk + 2 * K * C, st);
    a.w2 = view(q[5], true, pk + 3 * K * C, st);
    a.du = (float*)(ws + L.du); a.dx = dxs[i];
    a.part = (double*)(ws + L.part);
    a.B = (int)B; a.accumulate = (int)accumulate;
    a.drop_p = drop_p;
    a.drop_scale = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
    a.seed_ptr = seed_ptr; a.offset = offs[i];
    a.invN = 1.0f / (float)(B * P);
    float* coef = (float*)(ws + L.slabda2);
    a.bfin = {C, (int)B, coef, g[3], g[4], g[5], (int)accumulate};
    a.coef = coef;
  }
  auto ws_of = [&](int i, size_t off) { return (float*)((char*)wss[i] + off); };
  TVQ_PLAN("w8_bwd2 C%d W%d B%lld", C, W, (long long)B);
  A[0].g_out = ws_of(0, L.g2);
  hipLaunchKernelGGL(w8_bwd2_kernel, dim3((unsigned)B), dim3(T), LDS, st, A[0]);
  int rc = launch_status("tvq_resblock_pair_bwd");
  if (rc) return rc;
  bn_bwd_final_launch(A[0].part, A[0].bfin, st);
  TVQ_PLAN("w8_bwd12 C%d W%d B%lld", C, W, (long long)B);
  A[0].g_out = ws_of(0, L.dh); A[0].slabda = ws_of(0, L.slabda1);
  A[1].g_out = ws_of(1, L.g2);
  hipLaunchKernelGGL(w8_bwd12_kernel, dim3((unsigned)B), dim3(T), LDS, st, A[0], A[1]);
  rc = launch_status("tvq_resblock_pair_bwd");
  if (rc) return rc;
  bn_bwd_final_launch(A[1].part, A[1].bfin, st);
  TVQ_PLAN("w8_bwd1 C%d W%d B%lld", C, W, (long long)B);
  A[1].g_out = ws_of(1, L.dh); A[1].slabda = ws_of(1, L.slabda1);
  hipLaunchKernelGGL(w8_bwd1_kernel, dim3((unsigned)B), dim3(T), LDS, st, A[1]);
  rc = launch_status("tvq_resblock_pair_bwd");
  if (rc) return rc;
  if (conv_wgrad_w8_fits(B, C, C)) {  // the pair's four weight gradients in one launch
    const float* x[4];
    const float* dy[4];
    float* wsl[4];
    float* dw[4];
    float* db[4];
    for (int i = 0; i < 2; ++i) {
      float* const* g = gs[i];
      x[2 * i] = saveds[i] + 2 * img;  // conv2: (s2, g2)
      dy[2 * i] = ws_of(i, L.g2);
      wsl[2 * i] = ws_of(i, L.wg2);
      dw[2 * i] = g[6];
      db[2 * i] = g[7];
      x[2 * i + 1] = saveds[i] + img;  // conv1: (s1, dh)
      dy[2 * i + 1] = ws_of(i, L.dh);
      wsl[2 * i + 1] = ws_of(i, L.wg1);
      dw[2 * i + 1] = g[1];
      db[2 * i + 1] = g[2];
    }
    conv_wgrad_w8_multi(4, x, dy, wsl, dw, db, B, C, C, (int)accumulate, st);
    for (int i = 0; i < 2; ++i)
      conv_wgrad_finish(ws_of(i, L.slabda1), (int)B, C, 1, gs[i][0], nullptr, (int)accumulate, st);
    return launch_status("tvq_resblock_pair_bwd");
  }
  for (int i = 0; i < 2; ++i) {
    float* const* g = gs[i];
    const float* s1 = saveds[i] + img;
    const float* s2 = saveds[i] + 2 * img;
    float* g2b = ws_of(i, L.g2);
    float* dh = ws_of(i, L.dh);
    if (!conv_wgrad_w8_pair(s2, g2b, ws_of(i, L.wg2), g[6], g[7], s1, dh, ws_of(i, L.wg1), g[1],
                            g[2], B, C, C, (int)accumulate, st)) {
      rc = tvq_conv2d_wgrad(s2, B, C, 3, W, g2b, C, W, 3, 3, 1, 0, g[6], g[7], accumulate,
                            ws_of(i, L.wg2), st);
      if (rc) return rc;
      rc = tvq_conv2d_wgrad(s1, B, C, 3, W, dh, C, W, 3, 3, 1, 0, g[1], g[2], accumulate,
                            ws_of(i, L.wg1), st);
      if (rc) return rc;
    }
    conv_wgrad_finish(ws_of(i, L.slabda1), (int)B, C, 1, g[0], nullptr, (int)accumulate, st);
  }
  return launch_status("tvq_resblock_pair_bwd");
}

}  // namespace tvq

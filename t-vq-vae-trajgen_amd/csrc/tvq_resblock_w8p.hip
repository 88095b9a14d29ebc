// Fused projection ResBlock on the LF band's W = 8 maps (reference vq_vae.py:13-62 with
// in_channels != out_channels): the encoder's last block ResBlock(64, 128) and the decoder's
// first ResBlock(128, 64), both on (B, C, 3, 8) images,
//
//   y = proj(x) + Dropout_p(conv2(Snake_a2(BN(conv1(Snake_a1(x)) + b1))) + b2),
//   proj = the 1x1 Conv2d(Ci, Co) on the raw input,
//
// on the w8 scheme (csrc/tvq_resblock_w8.hip): one 8-wave block per image (256 images = one
// block per CU), every conv of the block on v_mfma_f32_32x32x2_f32 with the staged halo
// planes in LDS as the B operand and the weights, read from L2 (packed [tap][c][n] by the
// pack cache when a scope is open), as the A operand.  A conv of NCI -> NCO channels runs
// NCO / 32 output tiles x (NCI / 16) input-channel chunks over the 8 waves: wave w owns tile
// w % (NCO/32) and a contiguous run of chunks, whose 72 weight values per chunk it requests
// a chunk ahead of their MFMAs (two register buffers); the chunk-group partial tiles are
// summed in LDS in group order.
//
//   w8p_fwd1  s1 = Snake_a1(x) staged (and stored: the conv1 weight gradient's input) ->
//             h = conv1(s1) + b1 -> store h; per-image fp64 BN partial sums
//   (bn_stats_final_kernel: the partials -> batch mean / invstd / affine form, running
//             statistics)
//   w8p_fwd2  s2 = Snake_a2(BN(h)) staged (and stored) -> v = Dropout(conv2(s2) + b2); raw x
//             restaged -> y = (proj(x) + bp) + v
//   w8p_bwd2  g2 = Dropout'(dy) staged (and stored) -> ds2 = conv2^T(g2) -> du = ds2 *
//             Snake'(u) -> store du; per-image (sum du, sum du xhat, Snake a2 term)
//   (bn_bwd_final_kernel: -> BN backward coefficients, BN weight / bias and a2 gradients)
//   w8p_bwd1  dh = BN'(du) staged (and stored) -> ds1 = conv1^T(dh); dy restaged ->
//             dx = ds1 * Snake'(x) + proj^T(dy); the Snake a1 term (a slab row)
//   weight gradients: conv2 (s2, g2) and conv1 (s1, dh) by the image-batched
//             conv_wgrad_w8 kernel, proj (x, dy) by the 1x1 weight-gradient path
//   w8p_eval  the three convs in one launch, BN from the running statistics
//
// Replaces per block: tvq_snake_fwd, three conv launches and the whole-channel BN kernel
// forward; the dropout, BN and Snake kernels and three data-gradient convs backward.
// Arithmetic is the per-op kernels' (Snake, BN affine / backward formulas, the dropout hash
// at the flat NCHW index of the output) up to the summation order, which is fixed.
#include "tvq_bn.h"
#include "tvq_common.h"
#include "tvq_conv_internal.h"
#include "tvq_reduce.h"

namespace tvq {
namespace w8p {

constexpr int W = 8, P = 3 * W, NW = 8, T = 64 * NW;
constexpr int WP = W + 2;          // halo row stride
constexpr int PS = 80;             // halo plane stride (5 x 10 cells, padded)
constexpr int MAXC = 128;          // planes staged at most
constexpr int RED = NW * 16 * 64;  // one partial 32 x 32 tile per wave

struct WView {  // element (row n, reduction channel c, tap t) at w[n*sn + c*sc + t*st]
  const float* w;
  int64_t sn, sc, st;
};

struct Args {
  const float *x, *h, *dy, *du_in;
  const float *a1, *b1, *a2, *b2, *bp;
  const float *bn_w, *bn_b, *rmean, *rvar;  // eval / BN backward
  const float* save;                         // mean | invstd | scale | shift
  const float* coef;                         // BN backward (sum du, sum du xhat) per channel
  WView w1, w2, wp;                          // forward views (eval / fwd) or data-gradient views
  float *h_out, *s_out, *y, *du, *dx, *g_out, *slabda;
  double* part;
  float eps, drop_p, drop_scale, invN;
  const int64_t* seed_ptr;
  uint64_t offset;
  int B;
};

__device__ __forceinline__ int wid_() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// halo cell of position p (the 3x3 window's centre)
__device__ __forceinline__ int cell(int c, int p) { return c * PS + WP + 1 + (p / W) * WP + p % W; }

// zero the border cells of NC halo planes
template <int NC>
__device__ __forceinline__ void border(float* __restrict__ S) {
  for (int i = threadIdx.x; i < NC * 26; i += T) {
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

// Elementwise layout of NC channels: wave w, iteration j < NC / 16 -> channel
// (NC / 8) w + 2 j + (lane >> 5), position lane & 31 (valid below 24); a channel's 24
// positions sit in one 32-lane half.
template <int NC>
__device__ __forceinline__ int el_c(int j) {
  return (NC / 8) * wid_() + 2 * j + ((threadIdx.x & 63) >> 5);
}
__device__ __forceinline__ int el_p() { return threadIdx.x & 31; }

__device__ __forceinline__ double half_sum_d(double v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Conv geometry of NCI -> NCO: NTO output tiles of 32 rows, NCG chunk groups of CPW chunks
// of 16 input channels; wave w owns tile w % NTO and chunks (w / NTO) * CPW + i.
template <int NCI, int NCO>
struct Geo {
  static constexpr int NTO = NCO / 32, NCG = NW / NTO, NCH = NCI / 16, CPW = NCH / NCG;
  static_assert(NCO % 32 == 0 && NW % NTO == 0 && NCI % 16 == 0 && NCH % NCG == 0 && CPW >= 1,
                "unsupported conv geometry");
};

// this lane's TAPS x 8 weights of chunk ch: W(row 32 nt + (l & 31), reduction channel
// 16 ch + (l >> 5) + 2u, tap t)
template <int NCI, int NCO, int TAPS>
__device__ __forceinline__ void load_chunk(const WView wv, int ch, float (&a)[TAPS][8]) {
  using G = Geo<NCI, NCO>;
  const int lane = threadIdx.x & 63, wid = wid_();
  const int nt = wid % G::NTO;
  const float* wp = wv.w + (int64_t)(32 * nt + (lane & 31)) * wv.sn +
                    (int64_t)(16 * ch + (lane >> 5)) * wv.sc;
#pragma unroll
  for (int t = 0; t < TAPS; ++t)
#pragma unroll
    for (int u = 0; u < 8; ++u) a[t][u] = wp[(int64_t)(2 * u) * wv.sc + (int64_t)t * wv.st];
}

// the wave's first chunk, issued ahead (at kernel start / before an epilogue): the
// scheduling barrier keeps the loads from sinking next to their MFMAs
template <int NCI, int NCO, int TAPS>
__device__ __forceinline__ void preload(const WView wv, float (&a)[TAPS][8]) {
  using G = Geo<NCI, NCO>;
  load_chunk<NCI, NCO, TAPS>(wv, (wid_() / G::NTO) * G::CPW, a);
  __builtin_amdgcn_sched_barrier(0);
}

// The block's conv of the staged planes S (NCI of them) into red[w][16][64]; a0 holds the
// first chunk's weights (preload).  FLIP: data gradient (taps mirrored).  TAPS = 1: the 1x1
// conv (centre cells).
template <int NCI, int NCO, int TAPS, bool FLIP>
__device__ __forceinline__ void conv(const WView wv, float (&a0)[TAPS][8],
                                     const float* __restrict__ S, float* __restrict__ red) {
  using G = Geo<NCI, NCO>;
  const int lane = threadIdx.x & 63, wid = wid_();
  const int r32 = lane & 31, hl = lane >> 5;
  const int ch0 = (wid / G::NTO) * G::CPW;
  const int m = r32 < P ? r32 : 0;
  const float* sp0 = S + hl * PS + (m / W) * WP + (m % W) + (TAPS == 1 ? WP + 1 : 0);
  float a1[TAPS][8];
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
  for (int i = 0; i < G::CPW; ++i) {
    float(&cur)[TAPS][8] = (i & 1) ? a1 : a0;
    float(&nxt)[TAPS][8] = (i & 1) ? a0 : a1;
    if (i + 1 < G::CPW) load_chunk<NCI, NCO, TAPS>(wv, ch0 + i + 1, nxt);
    __builtin_amdgcn_sched_barrier(0);
    const float* sp = sp0 + (16 * (ch0 + i)) * PS;
#pragma unroll
    for (int t = 0; t < TAPS; ++t) {
      const int tt = FLIP ? TAPS - 1 - t : t, off = TAPS == 1 ? 0 : (tt / 3) * WP + tt % 3;
#pragma unroll
      for (int u = 0; u < 8; ++u)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[t][u], sp[2 * u * PS + off], acc, 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) red[(wid * 16 + r) * 64 + lane] = acc[r];
}

// conv result (row n, position p): the NCG chunk-group partials of tile n / 32, group order
template <int NCI, int NCO>
__device__ __forceinline__ float conv_at(const float* __restrict__ red, int n, int p) {
  using G = Geo<NCI, NCO>;
  const int nt = n >> 5, i = n & 31, h = (i >> 2) & 1, r = (i & 3) + 4 * (i >> 3);
  const int l = p + 32 * h;
  float s = red[(nt * 16 + r) * 64 + l];
#pragma unroll
  for (int g = 1; g < G::NCG; ++g) s += red[((nt + G::NTO * g) * 16 + r) * 64 + l];
  return s;
}

// ---------------------------------------------------------------- kernels
template <int CI, int CO>
__global__ __launch_bounds__(T) void w8p_fwd1_kernel(Args a) {
  extern __shared__ float sm[];
  float* S = sm;
  float* red = sm + MAXC * PS;
  constexpr int JI = CI / 16, JO = CO / 16;
  const int b = blockIdx.x, p = el_p(), pp = p < P ? p : 0;
  const int64_t i0 = (int64_t)b * CI * P, o0 = (int64_t)b * CO * P;
  float xv[JI], av[JI], bv[JO];
#pragma unroll
  for (int j = 0; j < JI; ++j) {
    xv[j] = a.x[i0 + el_c<CI>(j) * P + pp];
    av[j] = a.a1[el_c<CI>(j)];
  }
#pragma unroll
  for (int j = 0; j < JO; ++j) bv[j] = a.b1[el_c<CO>(j)];
  float wa[9][8];
  preload<CI, CO, 9>(a.w1, wa);
  border<CI>(S);
#pragma unroll
  for (int j = 0; j < JI; ++j) {
    const int c = el_c<CI>(j);
    if (p >= P) continue;
    const float s = snake_f(xv[j], av[j], 1.0f / av[j]);
    S[cell(c, p)] = s;
    a.s_out[i0 + c * P + p] = s;
  }
  __syncthreads();
  conv<CI, CO, 9, false>(a.w1, wa, S, red);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < JO; ++j) {
    const int c = el_c<CO>(j);
    double s0 = 0.0, s1 = 0.0;
    if (p < P) {
      const float v = conv_at<CI, CO>(red, c, p) + bv[j];
      a.h_out[o0 + c * P + p] = v;
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

template <int CI, int CO>
__global__ __launch_bounds__(T) void w8p_fwd2_kernel(Args a) {
  extern __shared__ float sm[];
  float* S = sm;
  float* red = sm + MAXC * PS;
  constexpr int JI = CI / 16, JO = CO / 16;
  const int b = blockIdx.x, p = el_p(), pp = p < P ? p : 0;
  const int64_t i0 = (int64_t)b * CI * P, o0 = (int64_t)b * CO * P;
  float hv[JO], xv[JI], av[JO], sc[JO], sh[JO];
#pragma unroll
  for (int j = 0; j < JO; ++j) {
    const int c = el_c<CO>(j);
    hv[j] = a.h[o0 + c * P + pp];
    av[j] = a.a2[c];
    sc[j] = a.save[2 * CO + c];  // the batch statistics' affine form (bn_stats_final_kernel's)
    sh[j] = a.save[3 * CO + c];
  }
#pragma unroll
  for (int j = 0; j < JI; ++j) xv[j] = a.x[i0 + el_c<CI>(j) * P + pp];
  float wa[9][8], wq[1][8];
  preload<CO, CO, 9>(a.w2, wa);
  preload<CI, CO, 1>(a.wp, wq);
  border<CO>(S);
#pragma unroll
  for (int j = 0; j < JO; ++j) {
    const int c = el_c<CO>(j);
    if (p >= P) continue;
    const float s = snake_f(fmaf(hv[j], sc[j], sh[j]), av[j], 1.0f / av[j]);
    S[cell(c, p)] = s;
    a.s_out[o0 + c * P + p] = s;
  }
  __syncthreads();
  conv<CO, CO, 9, false>(a.w2, wa, S, red);
  __syncthreads();
  const uint64_t seed = a.drop_p > 0.f ? mix_seed(a.seed_ptr, a.offset) : 0ull;
  float v2[JO];
#pragma unroll
  for (int j = 0; j < JO; ++j) {
    const int c = el_c<CO>(j);
    float v = conv_at<CO, CO>(red, c, pp) + a.b2[c];
    if (a.drop_p > 0.f)
      v = uniform01(seed, (uint64_t)(o0 + c * P + pp)) >= a.drop_p ? v * a.drop_scale : 0.f;
    v2[j] = v;
  }
  __syncthreads();  // red and S read: the projection's input and partials reuse them
#pragma unroll
  for (int j = 0; j < JI; ++j)
    if (p < P) S[cell(el_c<CI>(j), p)] = xv[j];
  __syncthreads();
  conv<CI, CO, 1, false>(a.wp, wq, S, red);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < JO; ++j) {
    const int c = el_c<CO>(j);
    if (p < P) a.y[o0 + c * P + p] = (conv_at<CI, CO>(red, c, p) + a.bp[c]) + v2[j];
  }
}

template <int CI, int CO>
__global__ __launch_bounds__(T) void w8p_eval_kernel(Args a) {
  extern __shared__ float sm[];
  float* S = sm;
  float* red = sm + MAXC * PS;
  constexpr int JI = CI / 16, JO = CO / 16;
  const int b = blockIdx.x, p = el_p(), pp = p < P ? p : 0;
  const int64_t i0 = (int64_t)b * CI * P, o0 = (int64_t)b * CO * P;
  float xv[JI];
#pragma unroll
  for (int j = 0; j < JI; ++j) xv[j] = a.x[i0 + el_c<CI>(j) * P + pp];
  float wa[9][8];
  preload<CI, CO, 9>(a.w1, wa);
  border<CI>(S);
#pragma unroll
  for (int j = 0; j < JI; ++j) {
    const int c = el_c<CI>(j);
    if (p >= P) continue;
    const float av = a.a1[c];
    S[cell(c, p)] = snake_f(xv[j], av, 1.0f / av);
  }
  __syncthreads();
  conv<CI, CO, 9, false>(a.w1, wa, S, red);
  preload<CO, CO, 9>(a.w2, wa);  // conv2's first weights in flight during conv1's epilogue
  __syncthreads();
  float s2[JO];
#pragma unroll
  for (int j = 0; j < JO; ++j) {  // BN from the running statistics (bn_eval's affine form)
    const int c = el_c<CO>(j);
    const float inv = 1.0f / sqrtf(a.rvar[c] + a.eps);
    const float scv = (a.bn_w ? a.bn_w[c] : 1.f) * inv;
    const float shv = (a.bn_b ? a.bn_b[c] : 0.f) - a.rmean[c] * scv;
    const float av = a.a2[c];
    s2[j] = snake_f(fmaf(conv_at<CI, CO>(red, c, pp) + a.b1[c], scv, shv), av, 1.0f / av);
  }
  __syncthreads();  // conv1's partials read; S free
  if (CO > CI) border<CO>(S);  // planes CI .. CO - 1 have no zero border yet
#pragma unroll
  for (int j = 0; j < JO; ++j)
    if (p < P) S[cell(el_c<CO>(j), p)] = s2[j];
  __syncthreads();
  conv<CO, CO, 9, false>(a.w2, wa, S, red);
  float wq[1][8];
  preload<CI, CO, 1>(a.wp, wq);
  __syncthreads();
  float v2[JO];
#pragma unroll
  for (int j = 0; j < JO; ++j) v2[j] = conv_at<CO, CO>(red, el_c<CO>(j), pp) + a.b2[el_c<CO>(j)];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < JI; ++j)
    if (p < P) S[cell(el_c<CI>(j), p)] = xv[j];
  __syncthreads();
  conv<CI, CO, 1, false>(a.wp, wq, S, red);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < JO; ++j) {
    const int c = el_c<CO>(j);
    if (p < P) a.y[o0 + c * P + p] = (conv_at<CI, CO>(red, c, p) + a.bp[c]) + v2[j];
  }
}

template <int CI, int CO>
__global__ __launch_bounds__(T) void w8p_bwd2_kernel(Args a) {
  extern __shared__ float sm[];
  float* G = sm;
  float* red = sm + MAXC * PS;
  constexpr int JO = CO / 16;
  const int b = blockIdx.x, p = el_p(), pp = p < P ? p : 0;
  const int64_t o0 = (int64_t)b * CO * P;
  float gv[JO], hv[JO];
#pragma unroll
  for (int j = 0; j < JO; ++j) {
    const int64_t gi = o0 + el_c<CO>(j) * P + pp;
    gv[j] = a.dy[gi];
    hv[j] = a.h[gi];
  }
  float wa[9][8];
  preload<CO, CO, 9>(a.w2, wa);
  border<CO>(G);
  const uint64_t seed = a.drop_p > 0.f ? mix_seed(a.seed_ptr, a.offset) : 0ull;
#pragma unroll
  for (int j = 0; j < JO; ++j) {
    const int c = el_c<CO>(j);
    if (p >= P) continue;
    const int64_t gi = o0 + c * P + p;
    float d = gv[j];
    if (a.drop_p > 0.f) d = uniform01(seed, (uint64_t)gi) >= a.drop_p ? d * a.drop_scale : 0.f;
    G[cell(c, p)] = d;
    a.g_out[gi] = d;
  }
  __syncthreads();
  conv<CO, CO, 9, true>(a.w2, wa, G, red);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < JO; ++j) {
    const int c = el_c<CO>(j);
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    if (p < P) {
      const float av = a.a2[c], inv_a = 1.0f / av;
      const float sc = a.save[2 * CO + c], sh = a.save[3 * CO + c];
      const float mu = a.save[c], is = a.save[CO + c];
      const float gs = conv_at<CO, CO>(red, c, p);  // d loss / d s2
      const float uu = fmaf(hv[j], sc, sh);
      float sn, cs;
      sincosf(av * uu, &sn, &cs);
      const float tt = 2.0f * sn * cs;
      const float d = gs + gs * inv_a * tt * av;  // d loss / d u (bn_bwd_partial_kernel)
      const float xhat = (hv[j] - mu) * is;
      a.du[o0 + c * P + p] = d;
      s0 = d;
      s1 = (double)d * xhat;
      s2 = (double)(gs * inv_a * tt * uu) - (double)(gs * (sn * sn) * inv_a * inv_a);
    }
    s0 = half_sum_d(s0);
    s1 = half_sum_d(s1);
    s2 = half_sum_d(s2);
    if ((threadIdx.x & 31) == 0) {  // [c][image][3]: bn_bwd_final_kernel's chunk layout
      double* q = a.part + ((int64_t)c * a.B + b) * 3;
      q[0] = s0;
      q[1] = s1;
      q[2] = s2;
    }
  }
}

template <int CI, int CO>
__global__ __launch_bounds__(T) void w8p_bwd1_kernel(Args a) {
  extern __shared__ float sm[];
  float* G = sm;
  float* red = sm + MAXC * PS;
  constexpr int JI = CI / 16, JO = CO / 16;
  const int b = blockIdx.x, p = el_p(), pp = p < P ? p : 0;
  const int64_t i0 = (int64_t)b * CI * P, o0 = (int64_t)b * CO * P;
  float dv[JO], hv[JO], yv[JO], xv[JI];
#pragma unroll
  for (int j = 0; j < JO; ++j) {
    const int64_t gi = o0 + el_c<CO>(j) * P + pp;
    dv[j] = a.du_in[gi];
    hv[j] = a.h[gi];
    yv[j] = a.dy[gi];  // the projection's input gradient, requested with the prologue's
  }
#pragma unroll
  for (int j = 0; j < JI; ++j) xv[j] = a.x[i0 + el_c<CI>(j) * P + pp];
  float md[JO], mx[JO];  // the BN backward coefficients (bn_bwd_final_kernel's sums)
#pragma unroll
  for (int j = 0; j < JO; ++j) {
    md[j] = a.coef[2 * el_c<CO>(j)] * a.invN;
    mx[j] = a.coef[2 * el_c<CO>(j) + 1] * a.invN;
  }
  // data gradients: conv1^T is CO -> CI (rows = input channels), proj^T likewise
  float wa[9][8], wq[1][8];
  preload<CO, CI, 9>(a.w1, wa);
  preload<CO, CI, 1>(a.wp, wq);
  border<CO>(G);
  // dh = w * invstd * (du - mean(du) - xhat * mean(du * xhat))  (bn_bwd_apply_kernel)
#pragma unroll
  for (int j = 0; j < JO; ++j) {
    const int c = el_c<CO>(j);
    if (p >= P) continue;
    const float mu = a.save[c], is = a.save[CO + c], bw = a.bn_w ? a.bn_w[c] : 1.f;
    const float xhat = (hv[j] - mu) * is;
    const float g = bw * is * (dv[j] - md[j] - xhat * mx[j]);
    G[cell(c, p)] = g;
    a.g_out[o0 + c * P + p] = g;
  }
  __syncthreads();
  conv<CO, CI, 9, true>(a.w1, wa, G, red);
  __syncthreads();
  float gs1[JI];
#pragma unroll
  for (int j = 0; j < JI; ++j) gs1[j] = conv_at<CO, CI>(red, el_c<CI>(j), pp);
  __syncthreads();  // red and G read: the projection's input and partials reuse them
#pragma unroll
  for (int j = 0; j < JO; ++j)
    if (p < P) G[cell(el_c<CO>(j), p)] = yv[j];
  __syncthreads();
  conv<CO, CI, 1, false>(a.wp, wq, G, red);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < JI; ++j) {
    const int c = el_c<CI>(j);
    double s0 = 0.0;
    if (p < P) {
      const float av = a.a1[c], inv_a = 1.0f / av;
      const float gs = gs1[j];  // d loss / d s1
      float sn, cs;
      sincosf(av * xv[j], &sn, &cs);
      const float tt = 2.0f * sn * cs;
      // snake_bwd_kernel, plus the projection's input gradient
      a.dx[i0 + c * P + p] = (gs + gs * inv_a * tt * av) + conv_at<CO, CI>(red, c, p);
      s0 = (double)(gs * inv_a * tt * xv[j]) - (double)(gs * (sn * sn) * inv_a * inv_a);
    }
    s0 = half_sum_d(s0);
    if ((threadIdx.x & 31) == 0) a.slabda[(int64_t)b * CI + c] = (float)s0;
  }
}

constexpr size_t LDS = 4 * (size_t)(MAXC * PS + RED);

template <int CI, int CO>
static void set_lds() {
  static bool done = false;
  if (done) return;
  const void* ks[] = {(const void*)&w8p_fwd1_kernel<CI, CO>, (const void*)&w8p_fwd2_kernel<CI, CO>,
                      (const void*)&w8p_eval_kernel<CI, CO>, (const void*)&w8p_bwd2_kernel<CI, CO>,
                      (const void*)&w8p_bwd1_kernel<CI, CO>};
  for (const void* k : ks)
    (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS);
  done = true;
}

static size_t al(size_t n) { return (n + 255) & ~(size_t)255; }

struct Ws {  // workspace layout (bytes)
  size_t part, slabda1, coef, g2, dh, du, wg1, wg2, wgp, pk, total;
};
static Ws ws_layout(int64_t B, int64_t CI, int64_t CO) {
  Ws w;
  const size_t img = (size_t)B * CO * P * 4;
  const size_t slabd = (size_t)(B * CI + reduce_rows_scratch(B, CI)) * 4;
  w.part = 0;
  w.slabda1 = w.part + al((size_t)B * CO * 3 * 8);
  w.coef = w.slabda1 + al(slabd);
  w.g2 = w.coef + al((size_t)2 * CO * 4);
  w.dh = w.g2 + al(img);
  w.du = w.dh + al(img);
  w.wg1 = w.du + al(img);
  w.wg2 = w.wg1 + al((size_t)tvq_conv_workspace(4, B, CI, 3, W, CO, 3, 3, 1, 0) * 4);
  w.wgp = w.wg2 + al((size_t)tvq_conv_workspace(4, B, CO, 3, W, CO, 3, 3, 1, 0) * 4);
  w.pk = w.wgp + al((size_t)tvq_conv_workspace(4, B, CI, 3, W, CO, 1, 1, 1, 0) * 4);
  // packs: w1, w2, wp forward and data-gradient views
  w.total = w.pk + al((size_t)2 * (9 * CI * CO + 9 * CO * CO + CI * CO) * 4);
  return w;
}

// forward: rows = the conv's output channels, reduction = its input channels; data
// gradient (transposed): rows = input channels, reduction = output channels
static WView view(const float* w, int64_t cin, int64_t cout, int KK, bool transposed, float* ws,
                  hipStream_t st) {
  WView v;
  if (transposed)
    v.w = conv_pack_view(w, (int)cin, (int)cout, KK, KK, cin * KK, ws, st, &v.sn, &v.sc, &v.st);
  else
    v.w = conv_pack_view(w, (int)cout, (int)cin, KK, cin * KK, KK, ws, st, &v.sn, &v.sc, &v.st);
  return v;
}

static bool shape_ok(int64_t B, int64_t CI, int64_t CO, int64_t H, int64_t Wd) {
  return H == 3 && Wd == W && B >= 1 && ((CI == 64 && CO == 128) || (CI == 128 && CO == 64)) &&
         B * 128 * P < (1ll << 31);
}

// the body (variadic: it holds commas) for the two instantiated shapes
#define W8P_DISPATCH(CI_, CO_, ...)             \
  if ((CI_) == 64 && (CO_) == 128) {           \
    constexpr int CI = 64, CO = 128;           \
    __VA_ARGS__                                \
  } else {                                     \
    constexpr int CI = 128, CO = 64;           \
    __VA_ARGS__                                \
  }

}  // namespace w8p
}  // namespace tvq

using namespace tvq;
using namespace tvq::w8p;

extern "C" int64_t tvq_resblock_proj_workspace(int64_t B, int64_t Ci, int64_t Co, int64_t H,
                                               int64_t Wd) {
  if (!shape_ok(B, Ci, Co, H, Wd)) return 0;
  return (int64_t)ws_layout(B, Ci, Co).total;
}

extern "C" int64_t tvq_resblock_proj_saved_floats(int64_t B, int64_t Ci, int64_t Co, int64_t H,
                                                  int64_t Wd) {
  if (!shape_ok(B, Ci, Co, H, Wd)) return 0;
  return B * P * (2 * Co + Ci);  // h | s1 | s2
}

extern "C" int tvq_resblock_proj_train_fwd(
    const float* x, int64_t B, int64_t Ci, int64_t Co, int64_t H, int64_t Wd, const float* a1,
    const float* w1, const float* b1, const float* bn_w, const float* bn_b, float* running_mean,
    float* running_var, int64_t* nbt, float momentum, float eps, const float* a2, const float* w2,
    const float* b2, const float* wp, const float* bp, float drop_p, const int64_t* seed_ptr,
    uint64_t offset, float* saved, float* y, float* save, void* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(shape_ok(B, Ci, Co, H, Wd), "tvq_resblock_proj_train_fwd: unsupported shape");
  TVQ_CHECK_ARG(x && a1 && w1 && b1 && running_mean && running_var && a2 && w2 && b2 && wp && bp &&
                    saved && y && save && workspace && (drop_p == 0.f || seed_ptr),
                "tvq_resblock_proj_train_fwd: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  const Ws L = ws_layout(B, Ci, Co);
  char* ws = (char*)workspace;
  float* pk = (float*)(ws + L.pk);
  Args a = {};
  a.x = x; a.a1 = a1; a.b1 = b1; a.a2 = a2; a.b2 = b2; a.bp = bp;
  a.w1 = view(w1, Ci, Co, 9, false, pk, st);
  a.w2 = view(w2, Co, Co, 9, false, pk + 9 * Ci * Co, st);
  a.wp = view(wp, Ci, Co, 1, false, pk + 9 * Ci * Co + 9 * Co * Co, st);
  a.h_out = saved; a.h = saved; a.y = y;
  a.part = (double*)(ws + L.part);
  a.B = (int)B;
  a.drop_p = drop_p;
  a.drop_scale = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
  a.seed_ptr = seed_ptr; a.offset = offset;
  BNFinal fin = {(int)Co, (int)B, B * P, eps, momentum, bn_w, bn_b, running_mean, running_var,
                 nbt, save, save + Co, save + 2 * Co, save + 3 * Co};
  TVQ_PLAN("w8p_fwd Ci%lld Co%lld B%lld packed=%d", (long long)Ci, (long long)Co, (long long)B,
           (int)(a.w1.sn == 1));
  W8P_DISPATCH(Ci, Co, {
    set_lds<CI, CO>();
    a.s_out = saved + B * P * CO;  // s1
    hipLaunchKernelGGL((w8p_fwd1_kernel<CI, CO>), dim3((unsigned)B), dim3(T), LDS, st, a);
    bn_stats_final_launch(a.part, fin, st);  // the per-image partials -> save, running stats
    a.save = save;
    a.s_out = saved + B * P * (CO + CI);  // s2
    hipLaunchKernelGGL((w8p_fwd2_kernel<CI, CO>), dim3((unsigned)B), dim3(T), LDS, st, a);
  })
  return launch_status("tvq_resblock_proj_train_fwd");
}

extern "C" int tvq_resblock_proj_eval_fwd(const float* x, int64_t B, int64_t Ci, int64_t Co,
                                          int64_t H, int64_t Wd, const float* a1, const float* w1,
                                          const float* b1, const float* bn_w, const float* bn_b,
                                          const float* running_mean, const float* running_var,
                                          float eps, const float* a2, const float* w2,
                                          const float* b2, const float* wp, const float* bp,
                                          float* y, tvq_stream_t stream) {
  TVQ_CHECK_ARG(shape_ok(B, Ci, Co, H, Wd), "tvq_resblock_proj_eval_fwd: unsupported shape");
  TVQ_CHECK_ARG(x && a1 && w1 && b1 && running_mean && running_var && a2 && w2 && b2 && wp && bp &&
                    y, "tvq_resblock_proj_eval_fwd: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  Args a = {};
  a.x = x; a.a1 = a1; a.b1 = b1; a.a2 = a2; a.b2 = b2; a.bp = bp;
  a.bn_w = bn_w; a.bn_b = bn_b; a.rmean = running_mean; a.rvar = running_var; a.eps = eps;
  // no workspace: the open pack-cache scope's packs, else the weights as they are
  a.w1 = view(w1, Ci, Co, 9, false, nullptr, st);
  a.w2 = view(w2, Co, Co, 9, false, nullptr, st);
  a.wp = view(wp, Ci, Co, 1, false, nullptr, st);
  a.y = y; a.B = (int)B;
  TVQ_PLAN("w8p_eval Ci%lld Co%lld B%lld packed=%d", (long long)Ci, (long long)Co, (long long)B,
           (int)(a.w1.sn == 1));
  W8P_DISPATCH(Ci, Co, {
    set_lds<CI, CO>();
    hipLaunchKernelGGL((w8p_eval_kernel<CI, CO>), dim3((unsigned)B), dim3(T), LDS, st, a);
  })
  return launch_status("tvq_resblock_proj_eval_fwd");
}

extern "C" int tvq_resblock_proj_bwd(
    const float* dy, const float* x, const float* saved, int64_t B, int64_t Ci, int64_t Co,
    int64_t H, int64_t Wd, const float* a1, const float* w1, const float* bn_w, const float* save,
    const float* a2, const float* w2, const float* wp, float drop_p, const int64_t* seed_ptr,
    uint64_t offset, float* dx, float* da1, float* dw1, float* db1, float* dbn_w, float* dbn_b,
    float* da2, float* dw2, float* db2, float* dwp, float* dbp, int64_t accumulate,
    void* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(shape_ok(B, Ci, Co, H, Wd), "tvq_resblock_proj_bwd: unsupported shape");
  TVQ_CHECK_ARG(dy && x && saved && a1 && w1 && save && a2 && w2 && wp && dx && da1 && dw1 &&
                    db1 && da2 && dw2 && db2 && dwp && dbp && workspace &&
                    (drop_p == 0.f || seed_ptr),
                "tvq_resblock_proj_bwd: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  const Ws L = ws_layout(B, Ci, Co);
  char* ws = (char*)workspace;
  float* pk = (float*)(ws + L.pk) + 9 * Ci * Co + 9 * Co * Co + Ci * Co;  // the transposed packs
  const float* h = saved;
  const float* s1 = saved + B * P * Co;
  const float* s2 = saved + B * P * (Co + Ci);
  float* g2 = (float*)(ws + L.g2);
  float* dh = (float*)(ws + L.dh);
  float* du = (float*)(ws + L.du);
  float* slabda1 = (float*)(ws + L.slabda1);
  float* coef = (float*)(ws + L.coef);
  Args a = {};
  a.x = x; a.h = h; a.dy = dy; a.du_in = du;
  a.a1 = a1; a.a2 = a2; a.bn_w = bn_w; a.save = save;
  a.w1 = view(w1, Ci, Co, 9, true, pk, st);
  a.w2 = view(w2, Co, Co, 9, true, pk + 9 * Ci * Co, st);
  a.wp = view(wp, Ci, Co, 1, true, pk + 9 * Ci * Co + 9 * Co * Co, st);
  a.du = du; a.dx = dx;
  a.part = (double*)(ws + L.part);
  a.B = (int)B;
  a.drop_p = drop_p;
  a.drop_scale = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
  a.seed_ptr = seed_ptr; a.offset = offset;
  a.invN = 1.0f / (float)(B * P);
  a.coef = coef;
  BNBwdFinal bfin = {(int)Co, (int)B, coef, dbn_w, dbn_b, da2, (int)accumulate};
  TVQ_PLAN("w8p_bwd Ci%lld Co%lld B%lld", (long long)Ci, (long long)Co, (long long)B);
  W8P_DISPATCH(Ci, Co, {
    set_lds<CI, CO>();
    a.g_out = g2;
    hipLaunchKernelGGL((w8p_bwd2_kernel<CI, CO>), dim3((unsigned)B), dim3(T), LDS, st, a);
    // per-image partials -> BN backward coefficients, BN weight / bias and Snake a2 gradients
    bn_bwd_final_launch(a.part, bfin, st);
    a.g_out = dh; a.slabda = slabda1;
    hipLaunchKernelGGL((w8p_bwd1_kernel<CI, CO>), dim3((unsigned)B), dim3(T), LDS, st, a);
  })
  int rc = launch_status("tvq_resblock_proj_bwd");
  if (rc) return rc;
  // weight gradients: conv2 (s2, g2), conv1 (s1, dh), proj (x, dy)
  rc = tvq_conv2d_wgrad(s2, B, Co, 3, W, g2, Co, W, 3, 3, 1, 0, dw2, db2, accumulate,
                        (float*)(ws + L.wg2), stream);
  if (rc) return rc;
  rc = tvq_conv2d_wgrad(s1, B, Ci, 3, W, dh, Co, W, 3, 3, 1, 0, dw1, db1, accumulate,
                        (float*)(ws + L.wg1), stream);
  if (rc) return rc;
  rc = tvq_conv2d_wgrad(x, B, Ci, 3, W, dy, Co, W, 1, 1, 1, 0, dwp, dbp, accumulate,
                        (float*)(ws + L.wgp), stream);
  if (rc) return rc;
  conv_wgrad_finish(slabda1, (int)B, Ci, 1, da1, nullptr, (int)accumulate, st);
  return launch_status("tvq_resblock_proj_bwd");
}

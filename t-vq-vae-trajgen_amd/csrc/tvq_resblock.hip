// Fused small-channel ResBlock (reference vq_vae.py:13-62) for C_in == C_out = C in
// {8, 16, 32} on the (B, C, 3, W) STFT image, W in {16, 32, 64} -- the ResBlocks after the
// strided encoder / decoder blocks of both bands.  At these sizes one kernel per op is
// pure latency (a few MB per launch, ~10 us each); here one block per image keeps the image
// and its conv halos in LDS through several ops, so a ResBlock is 2 launches forward (1 in
// eval) and 2 backward (+ the weight-gradient slab sums, batched into the step's deferred
// reduction launch) instead of ~6 and ~13.
//
//   y = x + Dropout_p(conv2(Snake_a2(BN(conv1(Snake_a1(x)) + b1))) + b2)
//
//   rb_fwd1   s1 = Snake_a1(x) staged into LDS -> h = conv1(s1) + b1 -> store h; per-image
//             BN partial sums (fp64) -> the last block: batch mean / invstd, running stats,
//             scale / shift (bn_final_channel, as tvq_bn_train_fwd)
//   rb_fwd2   s2 = Snake_a2(h*scale + shift) staged -> y = x + Dropout(conv2(s2) + b2)
//   rb_eval   both convs in one block with BN from the running statistics (s2 in LDS)
//   rb_bwd2   g2 = Dropout'(dy) (same counter-hash mask) -> dW2 | db2 per-image slab row;
//             ds2 = conv2^T(g2) -> du = ds2 * Snake'(u), u = h*scale + shift recomputed
//             -> store du; per-image (sum du, sum du*xhat, da2 term) -> last block: BN
//             backward coefficients, BN weight / bias grads, da2 (bn_bwd_final_channel)
//   rb_bwd1   dh = BN'(du) staged -> dW1 | db1 slab row; ds1 = conv1^T(dh) ->
//             dx = ds1 * Snake'(x) + dy (identity skip); da1 partials -> last block
//
// Convs are v_mfma_f32_16x16x4_f32 tiles, MFMA rows = channels (16-row tiles, zero-padded),
// columns = 16 positions, both operands from LDS: the forward gathers the halo plane at
// koff[c*9+t] = c*PS + toff(t); the data gradient is the same gather over the gradient
// planes with transposed weights and flipped taps; the weight gradient reduces over the
// image's positions with a ones column for the bias.  Everything is compile-time in (C, W)
// so the K loops unroll and their LDS reads pipeline; every kernel issues all its global
// loads (image, weights, per-channel parameters, epilogue operands) before it waits on
// any.  Arithmetic is the unfused kernels' (Snake, BN affine / backward formulas, dropout
// hash) up to the summation order.
#include <algorithm>

#include "tvq_bn.h"
#include "tvq_common.h"
#include "tvq_conv_internal.h"
#include "tvq_reduce.h"

namespace tvq {

constexpr int RB_T = 256;  // 4 waves per block, one image per block

template <int C_, int W_>
struct RB {
  static constexpr int C = C_, W = W_;
  static constexpr int P = 3 * W, MT = P / 16;       // positions, 16-position tiles
  static constexpr int NR = (C + 15) / 16, CT = 16 * NR;  // 16-row channel tiles
  static constexpr int WP = W + 2, HW = 5 * WP;      // halo row length, halo plane cells
  static constexpr int PS = HW + ((2 - HW % 32) + 32) % 32;  // plane stride == 2 mod 32
  static constexpr int K = 9 * C;                    // conv reduction length
  static constexpr int KST = K + ((2 - K % 32) + 32) % 32;  // panel row stride == 2 mod 32
  static constexpr int KC = K + 1, KT = (KC + 15) / 16;     // wgrad columns (+bias), tiles
  static constexpr int NT = MT * NR, WT = NR * KT;   // conv / wgrad output tiles
  static constexpr int TPW = (NT + 3) / 4;           // conv tiles per wave
  static constexpr int NE = C * P, UE = (NE + RB_T - 1) / RB_T;  // image elements
  static constexpr int NB = 2 * WP + 6;              // border cells per halo plane
  static constexpr int PLANE = C * PS, PANEL = CT * KST;
  static constexpr int NPAN = CT * K, UP = (NPAN + RB_T - 1) / RB_T;  // panel loads
  static_assert(P % 16 == 0 && TPW <= 3, "unsupported ResBlock geometry");
};

struct RBArgs {  // every pointer / scalar a fused ResBlock kernel reads or writes
  const float *x, *h, *dy;
  const float *a1, *w1, *b1, *a2, *w2, *b2;
  const float *bn_w, *bn_b, *rmean, *rvar;  // eval
  const float* save;                         // mean | invstd | scale | shift (C each)
  const float* coef;                         // 2C: (sum du, sum du*xhat) of the backward
  float *h_out, *y, *du, *dx, *slab1, *slab2, *da1;
  double *part, *part1;
  int* cnt;
  float eps, drop_p, drop_scale, invN;
  const int64_t* seed_ptr;
  uint64_t offset;
  int B, accumulate;
  BNFinal fin;
  BNBwdFinal bfin;
  unsigned long long* tbuf;  // RB_TIMING builds: per-block phase timestamps
};

#ifdef RB_TIMING
#define RB_MARK(i)                                                                  \
  do {                                                                              \
    if (a.tbuf && threadIdx.x == 0) a.tbuf[(size_t)blockIdx.x * 16 + (i)] = wall_clock64(); \
  } while (0)
#else
#define RB_MARK(i) \
  do {             \
  } while (0)
#endif

__device__ __forceinline__ int rb_toff(int t, int WP) {
  const int kh = t / 3;
  return kh * WP + (t - 3 * kh);
}

// halo offset of position p's top-left window cell
template <class R>
__device__ __forceinline__ int rb_pos(int p) {
  const int h = p / R::W;
  return h * R::WP + (p - h * R::W);
}

// this thread's elements e = tid + u*RB_T of the image (all loads issued, none waited on;
// consecutive lanes read consecutive addresses and write consecutive LDS cells)
template <class R>
__device__ __forceinline__ void rb_load_img(const float* __restrict__ src, int64_t img0,
                                            float (&v)[R::UE]) {
#pragma unroll
  for (int u = 0; u < R::UE; ++u) {
    const int e = threadIdx.x + u * RB_T;
    v[u] = src[img0 + (e < R::NE ? e : 0)];
  }
}

// dst[c*PS + halo(h,w)] = f(c, element e of the image, v[, v2]) for this thread's elements
template <class R, class F>
__device__ __forceinline__ void rb_put_img(float* __restrict__ dst, const float (&v)[R::UE],
                                           const float (&v2)[R::UE], F f) {
#pragma unroll
  for (int u = 0; u < R::UE; ++u) {
    const int e = threadIdx.x + u * RB_T;
    if (e < R::NE) {
      const int c = e / R::P, r = e - c * R::P;
      dst[c * R::PS + R::WP + 1 + rb_pos<R>(r)] = f(c, e, v[u], v2[u]);
    }
  }
}

// zero border of C halo planes (the zero padding of a conv input)
template <class R>
__device__ __forceinline__ void rb_border(float* __restrict__ dst) {
  for (int i = threadIdx.x; i < R::C * R::NB; i += RB_T) {
    const int c = i / R::NB, r = i - c * R::NB;
    int o;
    if (r < R::WP) {
      o = r;
    } else if (r < 2 * R::WP) {
      o = 4 * R::WP + (r - R::WP);
    } else {
      const int k = r - 2 * R::WP;
      o = (1 + (k >> 1)) * R::WP + ((k & 1) ? R::WP - 1 : 0);
    }
    dst[c * R::PS + o] = 0.f;
  }
}

// weight panel values of this thread: TRANS = false: A[n][k] = w[n*K + k] (rows = output
// channels); TRANS: A[c][n*9+t] = w[n*K + c*9 + t] (rows = input channels, data gradient)
template <class R, bool TRANS>
__device__ __forceinline__ void rb_load_panel(const float* __restrict__ w, float (&v)[R::UP]) {
#pragma unroll
  for (int u = 0; u < R::UP; ++u) {
    const int i = threadIdx.x + u * RB_T;
    const int row = i / R::K, k = i - row * R::K;
    float val = 0.f;
    if (i < R::NPAN && row < R::C) {
      if (TRANS) {
        const int n = k / 9, t = k - 9 * n;
        val = w[n * R::K + row * 9 + t];
      } else {
        val = w[i];
      }
    }
    v[u] = val;
  }
}

template <class R>
__device__ __forceinline__ void rb_put_panel(float* __restrict__ A, const float (&v)[R::UP]) {
#pragma unroll
  for (int u = 0; u < R::UP; ++u) {
    const int i = threadIdx.x + u * RB_T;
    if (i < R::NPAN) {
      const int row = i / R::K, k = i - row * R::K;
      A[row * R::KST + k] = v[u];
    }
  }
}

// this lane's conv output tiles t = wid + 4f: channel tile nr, position p, halo base
template <class R>
struct RBTiles {
  int nt;  // tiles of this wave
  int nr[3], p[3], base[3];
  __device__ __forceinline__ RBTiles() {
    const int wid = threadIdx.x >> 6, j = threadIdx.x & 15;
    nt = wid < R::NT ? (R::NT - wid + 3) / 4 : 0;
#pragma unroll
    for (int f = 0; f < 3; ++f) {
      const int t = f < nt ? wid + 4 * f : 0;
      nr[f] = t / R::MT;
      p[f] = (t - nr[f] * R::MT) * 16 + j;
      base[f] = rb_pos<R>(p[f]);
    }
  }
  // channel of accumulator register r of tile f
  __device__ __forceinline__ int chan(int f, int r) const {
    return nr[f] * 16 + 4 * ((threadIdx.x & 63) >> 4) + r;
  }
};

// gather offset of reduction index k = c*9 + t: c*PS + toff(t) (FLIP: toff(8 - t))
template <class R, bool FLIP>
__device__ __forceinline__ int rb_koff(int k) {
  const int c = k / 9, t0 = k - 9 * c;
  const int t = FLIP ? 8 - t0 : t0;
  const int kh = t / 3;
  return c * R::PS + kh * R::WP + (t - 3 * kh);
}

// acc[f] = A (channel tile nr[f]: 16 x K) x S gathered at base[f] + koff(k), f < 3 (a wave
// with fewer tiles runs dummies on valid addresses: no branch in the loop)
template <class R, bool FLIP>
__device__ __forceinline__ void rb_mma(const float* __restrict__ A, const float* __restrict__ S,
                                       const RBTiles<R>& tl, floatx4 (&acc)[3]) {
  const int l = threadIdx.x & 63, j = l & 15, kq = l >> 4;
  const float* ap[3];
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    ap[f] = A + ((R::NR == 1 ? 0 : tl.nr[f]) * 16 + j) * R::KST + kq;
    acc[f] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll 12
  for (int q = 0; q < R::K; q += 4) {
    const int ko = rb_koff<R, FLIP>(q + kq);
    float av[3];
    av[0] = ap[0][q];
#pragma unroll
    for (int f = 1; f < 3; ++f) av[f] = R::NR == 1 ? av[0] : ap[f][q];
#pragma unroll
    for (int f = 0; f < 3; ++f) acc[f] = mfma16x16x4(av[f], S[tl.base[f] + ko], acc[f]);
  }
}

// Weight gradient of one image into its slab row: D[n][kc] = sum_p G[n][p] * B[p][kc],
// B[p][kc] = S[koff(kc) + pos(p)] (kc < K), 1 (kc == K: bias), 0 beyond; rows n >= C are 0.
// Wave wid takes tiles wid, wid+4, ... in groups of 3 interleaved chains; every load is
// unconditional (clamped) so the position loop has no branch.
template <class R>
__device__ __forceinline__ void rb_wgrad(const float* __restrict__ G, const float* __restrict__ S,
                                         float* __restrict__ slab_row) {
  const int l = threadIdx.x & 63, wid = threadIdx.x >> 6, j = l & 15, kq = l >> 4;
  for (int t0 = wid; t0 < R::WT; t0 += 12) {
    int gofs[3], ko[3], kc[3], n0[3];
    float cst[3];
    bool colv[3], rowv[3];
#pragma unroll
    for (int f = 0; f < 3; ++f) {
      const int t = t0 + 4 * f < R::WT ? t0 + 4 * f : t0;
      const int nr = t / R::KT;
      kc[f] = (t0 + 4 * f < R::WT ? t - nr * R::KT : R::KT) * 16 + j;  // dead tile: kc >= KC
      n0[f] = nr * 16;
      colv[f] = kc[f] < R::K;
      ko[f] = rb_koff<R, false>(colv[f] ? kc[f] : 0);
      cst[f] = kc[f] == R::K ? 1.f : 0.f;
      const int n = nr * 16 + j;
      rowv[f] = n < R::C;
      gofs[f] = (rowv[f] ? n : 0) * R::PS + R::WP + 1;
    }
    floatx4 acc[3];
#pragma unroll
    for (int f = 0; f < 3; ++f) acc[f] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int p0 = 0; p0 < R::P; p0 += 4) {
      const int po = (p0 / R::W) * R::WP + (p0 % R::W) + kq;  // 4 | W: same row
#pragma unroll
      for (int f = 0; f < 3; ++f) {
        const float ga = G[gofs[f] + po];
        const float sb = S[ko[f] + po];
        acc[f] = mfma16x16x4(rowv[f] ? ga : 0.f, colv[f] ? sb : cst[f], acc[f]);
      }
    }
#pragma unroll
    for (int f = 0; f < 3; ++f) {
      if (kc[f] >= R::KC) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0[f] + 4 * kq + r;
        if (n < R::C) slab_row[n * R::KC + kc[f]] = acc[f][r];
      }
    }
  }
}

// s[i][f][r]: this lane's partials of channel tl.chan(f, r) (0 for dead tiles / channels)
// -> summed over the lane's tiles of one channel tile, staged in LDS (red: NR*4*64*4*NS
// doubles) -> thread (n, i) sums its channel's 64 lane values in a fixed order ->
// part[(n*B + b)*NS + i] (write-through, for the last block)
template <class R, int NS>
__device__ __forceinline__ void rb_channel_partials(double (&s)[NS][3][4], const RBTiles<R>& tl,
                                                    double* red, int B, int b, double* part) {
  const int l = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int nr = 0; nr < R::NR; ++nr) {
    double v[NS][4];
#pragma unroll
    for (int i = 0; i < NS; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double t = 0.0;
#pragma unroll
        for (int f = 0; f < 3; ++f)
          if (f < tl.nt && tl.nr[f] == nr) t += s[i][f][r];
        v[i][r] = t;
      }
    double* dst = red + ((size_t)(nr * 4 + wid) * 64 + l) * 4 * NS;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int i = 0; i < NS; ++i) dst[r * NS + i] = v[i][r];
  }
  __syncthreads();
  if (threadIdx.x < R::C * NS) {
    const int n = threadIdx.x / NS, i = threadIdx.x - n * NS;
    const int nr = n >> 4, kq = (n & 15) >> 2, r = n & 3;
    double t = 0.0;
    for (int wv = 0; wv < 4; ++wv) {
      const double* src = red + ((size_t)(nr * 4 + wv) * 64 + kq * 16) * 4 * NS + r * NS + i;
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) t += src[jj * 4 * NS];
    }
    st_wt(part + ((int64_t)n * B + b) * NS + i, t);
  }
}

// ---------------------------------------------------------------- kernels
template <class R>
__global__ __launch_bounds__(RB_T) void rb_fwd1_kernel(RBArgs a) {
  extern __shared__ double rb_smem[];
  float* prm = reinterpret_cast<float*>(rb_smem);  // a1 | b1
  float* S = prm + 2 * R::CT;
  float* A = S + R::PLANE;
  // the channel-partial staging [NR][4][64][4][2] doubles reuses the S / A region once
  // the conv is done (rb_lds: the max of the two, not their sum -> more blocks per CU)
  double* red = reinterpret_cast<double*>(S);
  const int b = blockIdx.x, l = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t img0 = (int64_t)b * R::C * R::P;
  RB_MARK(0);
  float v[R::UE];
  float pv[R::UP];
  rb_load_img<R>(a.x, img0, v);
  rb_load_panel<R, false>(a.w1, pv);
  if (threadIdx.x < R::C) {
    prm[threadIdx.x] = a.a1[threadIdx.x];
    prm[R::CT + threadIdx.x] = a.b1 ? a.b1[threadIdx.x] : 0.f;
  }
  rb_border<R>(S);
  rb_put_panel<R>(A, pv);
  __syncthreads();
  RB_MARK(1);
  rb_put_img<R>(S, v, v, [&](int c, int, float x, float) {
    const float al = prm[c];
    return snake_f(x, al, 1.0f / al);
  });
  __syncthreads();
  RB_MARK(2);
  const RBTiles<R> tl;
  floatx4 acc[3];
  rb_mma<R, false>(A, S, tl, acc);
  RB_MARK(3);
  double s[2][3][4] = {};
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    if (f >= tl.nt) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = tl.chan(f, r);
      if (n < R::C) {
        const float val = acc[f][r] + prm[R::CT + n];
        a.h_out[img0 + (int64_t)n * R::P + tl.p[f]] = val;
        s[0][f][r] = (double)val;
        s[1][f][r] = (double)val * (double)val;
      }
    }
  }
  RB_MARK(4);
  __syncthreads();  // every wave's S / A reads are done before red overwrites them
  rb_channel_partials<R, 2>(s, tl, red, a.B, b, a.part);
  RB_MARK(5);
  if (a.cnt && last_block(a.cnt, a.B))
    for (int c = wid; c < R::C; c += 4) bn_final_channel(a.part, c, l, a.fin);
  RB_MARK(6);
}

template <class R>
__global__ __launch_bounds__(RB_T) void rb_fwd2_kernel(RBArgs a) {
  extern __shared__ double rb_smem[];
  float* prm = reinterpret_cast<float*>(rb_smem);  // a2 | scale | shift | b2
  float* S = prm + 4 * R::CT;
  float* A = S + R::PLANE;
  const int b = blockIdx.x;
  const int64_t img0 = (int64_t)b * R::C * R::P;
  RB_MARK(0);
  float v[R::UE];
  float pv[R::UP];
  rb_load_img<R>(a.h, img0, v);
  rb_load_panel<R, false>(a.w2, pv);
  const RBTiles<R> tl;
  float xr[3][4];  // the residual at this lane's outputs
#pragma unroll
  for (int f = 0; f < 3; ++f)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = tl.chan(f, r);
      xr[f][r] = a.x[img0 + (int64_t)(n < R::C ? n : 0) * R::P + tl.p[f]];
    }
  if (threadIdx.x < R::C) {
    const int c = threadIdx.x;
    prm[c] = a.a2[c];
    prm[R::CT + c] = a.save[2 * R::C + c];
    prm[2 * R::CT + c] = a.save[3 * R::C + c];
    prm[3 * R::CT + c] = a.b2 ? a.b2[c] : 0.f;
  }
  rb_border<R>(S);
  rb_put_panel<R>(A, pv);
  __syncthreads();
  RB_MARK(1);
  rb_put_img<R>(S, v, v, [&](int c, int, float hv, float) {
    const float al = prm[c];
    return snake_f(fmaf(hv, prm[R::CT + c], prm[2 * R::CT + c]), al, 1.0f / al);
  });
  __syncthreads();
  RB_MARK(2);
  floatx4 acc[3];
  rb_mma<R, false>(A, S, tl, acc);
  RB_MARK(3);
  const uint64_t seed = a.drop_p > 0.f ? mix_seed(a.seed_ptr, a.offset) : 0ull;
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    if (f >= tl.nt) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = tl.chan(f, r);
      if (n < R::C) {
        const int64_t gi = img0 + (int64_t)n * R::P + tl.p[f];
        float val = acc[f][r] + prm[3 * R::CT + n];
        if (a.drop_p > 0.f)
          val = uniform01(seed, (uint64_t)gi) >= a.drop_p ? val * a.drop_scale : 0.f;
        a.y[gi] = xr[f][r] + val;
      }
    }
  }
}

template <class R>
__global__ __launch_bounds__(RB_T) void rb_eval_kernel(RBArgs a) {
  extern __shared__ double rb_smem[];
  float* prm = reinterpret_cast<float*>(rb_smem);  // a1 | b1 | scale | shift | a2 | b2
  float* S1 = prm + 6 * R::CT;
  float* S2 = S1 + R::PLANE;
  float* A1 = S2 + R::PLANE;  // conv1's panel, then conv2's (one panel of LDS: more blocks
                              // per CU; conv2's weights wait in registers meanwhile)
  const int b = blockIdx.x;
  const int64_t img0 = (int64_t)b * R::C * R::P;
  float v[R::UE];
  float pv1[R::UP], pv2[R::UP];
  rb_load_img<R>(a.x, img0, v);
  rb_load_panel<R, false>(a.w1, pv1);
  rb_load_panel<R, false>(a.w2, pv2);
  const RBTiles<R> tl;
  float xr[3][4];
#pragma unroll
  for (int f = 0; f < 3; ++f)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = tl.chan(f, r);
      xr[f][r] = a.x[img0 + (int64_t)(n < R::C ? n : 0) * R::P + tl.p[f]];
    }
  if (threadIdx.x < R::C) {
    const int c = threadIdx.x;
    // bn_eval_prep_kernel's affine form (then Snake, affine_snake_kernel)
    const float inv = 1.0f / sqrtf(a.rvar[c] + a.eps);
    const float sc = (a.bn_w ? a.bn_w[c] : 1.f) * inv;
    prm[c] = a.a1[c];
    prm[R::CT + c] = a.b1 ? a.b1[c] : 0.f;
    prm[2 * R::CT + c] = sc;
    prm[3 * R::CT + c] = (a.bn_b ? a.bn_b[c] : 0.f) - a.rmean[c] * sc;
    prm[4 * R::CT + c] = a.a2[c];
    prm[5 * R::CT + c] = a.b2 ? a.b2[c] : 0.f;
  }
  rb_border<R>(S1);
  rb_border<R>(S2);
  rb_put_panel<R>(A1, pv1);
  __syncthreads();
  rb_put_img<R>(S1, v, v, [&](int c, int, float x, float) {
    const float al = prm[c];
    return snake_f(x, al, 1.0f / al);
  });
  __syncthreads();
  floatx4 acc[3];
  rb_mma<R, false>(A1, S1, tl, acc);
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    if (f >= tl.nt) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = tl.chan(f, r);
      if (n < R::C) {
        const float al = prm[4 * R::CT + n];
        const float u = fmaf(acc[f][r] + prm[R::CT + n], prm[2 * R::CT + n], prm[3 * R::CT + n]);
        S2[n * R::PS + tl.base[f] + R::WP + 1] = snake_f(u, al, 1.0f / al);
      }
    }
  }
  __syncthreads();  // S2 complete; every wave is done reading conv1's panel
  rb_put_panel<R>(A1, pv2);
  __syncthreads();
  rb_mma<R, false>(A1, S2, tl, acc);
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    if (f >= tl.nt) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = tl.chan(f, r);
      if (n < R::C)
        a.y[img0 + (int64_t)n * R::P + tl.p[f]] = xr[f][r] + (acc[f][r] + prm[5 * R::CT + n]);
    }
  }
}

template <class R>
__global__ __launch_bounds__(RB_T) void rb_bwd2_kernel(RBArgs a) {
  extern __shared__ double rb_smem[];
  float* prm = reinterpret_cast<float*>(rb_smem);  // a2|scale|shift|mean|invstd
  float* G = prm + 5 * R::CT;                      // g2 planes
  float* S = G + R::PLANE;                         // s2 planes
  float* A = S + R::PLANE;                         // transposed w2
  double* red = reinterpret_cast<double*>(G);      // [NR][4][64][4][3], after the convs
  const int b = blockIdx.x, l = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t img0 = (int64_t)b * R::C * R::P;
  RB_MARK(0);
  float vg[R::UE], vh[R::UE];
  float pv[R::UP];
  rb_load_img<R>(a.dy, img0, vg);
  rb_load_img<R>(a.h, img0, vh);
  rb_load_panel<R, true>(a.w2, pv);
  const RBTiles<R> tl;
  float hr[3][4];
#pragma unroll
  for (int f = 0; f < 3; ++f)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = tl.chan(f, r);
      hr[f][r] = a.h[img0 + (int64_t)(n < R::C ? n : 0) * R::P + tl.p[f]];
    }
  if (threadIdx.x < R::C) {
    const int c = threadIdx.x;
    prm[c] = a.a2[c];
    prm[R::CT + c] = a.save[2 * R::C + c];
    prm[2 * R::CT + c] = a.save[3 * R::C + c];
    prm[3 * R::CT + c] = a.save[c];
    prm[4 * R::CT + c] = a.save[R::C + c];
  }
  rb_border<R>(G);
  rb_border<R>(S);
  rb_put_panel<R>(A, pv);
  __syncthreads();
  RB_MARK(1);
  const uint64_t seed = a.drop_p > 0.f ? mix_seed(a.seed_ptr, a.offset) : 0ull;
  rb_put_img<R>(G, vg, vg, [&](int, int e, float d, float) {
    if (a.drop_p > 0.f)
      return uniform01(seed, (uint64_t)(img0 + e)) >= a.drop_p ? d * a.drop_scale : 0.f;
    return d;
  });
  rb_put_img<R>(S, vh, vh, [&](int c, int, float hv, float) {
    const float al = prm[c];
    return snake_f(fmaf(hv, prm[R::CT + c], prm[2 * R::CT + c]), al, 1.0f / al);
  });
  __syncthreads();
  RB_MARK(2);
  rb_wgrad<R>(G, S, a.slab2 + (int64_t)b * R::C * R::KC);
  RB_MARK(3);
  floatx4 acc[3];
  rb_mma<R, true>(A, G, tl, acc);
  RB_MARK(4);
  double s[3][3][4] = {};
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    if (f >= tl.nt) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = tl.chan(f, r);
      if (n >= R::C) continue;
      const float av = prm[n], inv_a = 1.0f / av;
      const float hv = hr[f][r];
      const float gs = acc[f][r];  // d loss / d s2
      const float u = fmaf(hv, prm[R::CT + n], prm[2 * R::CT + n]);
      float sn, cs;
      sincosf(av * u, &sn, &cs);
      const float t = 2.0f * sn * cs;
      const float d = gs + gs * inv_a * t * av;  // d loss / d u (bn_bwd_partial_kernel)
      const float xhat = (hv - prm[3 * R::CT + n]) * prm[4 * R::CT + n];
      s[0][f][r] = d;
      s[1][f][r] = (double)d * xhat;
      s[2][f][r] = (double)(gs * inv_a * t * u) - (double)(gs * (sn * sn) * inv_a * inv_a);
      a.du[img0 + (int64_t)n * R::P + tl.p[f]] = d;
    }
  }
  RB_MARK(5);
  __syncthreads();  // G / S / A reads done before red overwrites them
  rb_channel_partials<R, 3>(s, tl, red, a.B, b, a.part);
  RB_MARK(6);
  if (a.cnt && last_block(a.cnt, a.B))
    for (int c = wid; c < R::C; c += 4) bn_bwd_final_channel(a.part, c, l, a.bfin);
  RB_MARK(7);
}

template <class R>
__global__ __launch_bounds__(RB_T) void rb_bwd1_kernel(RBArgs a) {
  extern __shared__ double rb_smem[];
  float* prm = reinterpret_cast<float*>(rb_smem);  // a1|mean|invstd|w|mds|mdsx
  float* G = prm + 6 * R::CT;                      // dh planes
  float* S = G + R::PLANE;                         // s1 planes
  float* A = S + R::PLANE;                         // transposed w1
  double* red = reinterpret_cast<double*>(G);      // [NR][4][64][4][1], after the convs
  const int b = blockIdx.x;
  const int64_t img0 = (int64_t)b * R::C * R::P;
  float vd[R::UE], vh[R::UE], vx[R::UE];
  float pv[R::UP];
  rb_load_img<R>(a.du, img0, vd);
  rb_load_img<R>(a.h, img0, vh);
  rb_load_img<R>(a.x, img0, vx);
  rb_load_panel<R, true>(a.w1, pv);
  const RBTiles<R> tl;
  float xr[3][4], gr[3][4];
#pragma unroll
  for (int f = 0; f < 3; ++f)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = tl.chan(f, r);
      const int64_t gi = img0 + (int64_t)(n < R::C ? n : 0) * R::P + tl.p[f];
      xr[f][r] = a.x[gi];
      gr[f][r] = a.dy[gi];
    }
  if (threadIdx.x < R::C) {
    const int c = threadIdx.x;
    prm[c] = a.a1[c];
    prm[R::CT + c] = a.save[c];
    prm[2 * R::CT + c] = a.save[R::C + c];
    prm[3 * R::CT + c] = a.bn_w ? a.bn_w[c] : 1.f;
    prm[4 * R::CT + c] = a.coef[2 * c] * a.invN;
    prm[5 * R::CT + c] = a.coef[2 * c + 1] * a.invN;
  }
  rb_border<R>(G);
  rb_border<R>(S);
  rb_put_panel<R>(A, pv);
  __syncthreads();
  // dh = w*invstd*(du - mean(du) - xhat*mean(du*xhat))  (bn_bwd_apply_kernel)
  rb_put_img<R>(G, vd, vh, [&](int c, int, float d, float hv) {
    const float is = prm[2 * R::CT + c];
    const float xhat = (hv - prm[R::CT + c]) * is;
    return prm[3 * R::CT + c] * is * (d - prm[4 * R::CT + c] - xhat * prm[5 * R::CT + c]);
  });
  rb_put_img<R>(S, vx, vx, [&](int c, int, float x, float) {
    const float al = prm[c];
    return snake_f(x, al, 1.0f / al);
  });
  __syncthreads();
  rb_wgrad<R>(G, S, a.slab1 + (int64_t)b * R::C * R::KC);
  floatx4 acc[3];
  rb_mma<R, true>(A, G, tl, acc);
  double s[1][3][4] = {};
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    if (f >= tl.nt) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = tl.chan(f, r);
      if (n >= R::C) continue;
      const float av = prm[n], inv_a = 1.0f / av;
      const float xv = xr[f][r];
      const float gs = acc[f][r];  // d loss / d s1
      float sn, cs;
      sincosf(av * xv, &sn, &cs);
      const float t = 2.0f * sn * cs;
      // snake_bwd_kernel, plus the identity skip's gradient
      a.dx[img0 + (int64_t)n * R::P + tl.p[f]] = (gs + gs * inv_a * t * av) + gr[f][r];
      s[0][f][r] = (double)(gs * inv_a * t * xv) - (double)(gs * (sn * sn) * inv_a * inv_a);
    }
  }
  __syncthreads();  // G / S / A reads done before red overwrites them
  rb_channel_partials<R, 1>(s, tl, red, a.B, b, a.part1);
  if (a.cnt && last_block(a.cnt, a.B) && threadIdx.x < 64)
    for (int c = 0; c < R::C; ++c)
      snake_bwd_final_channel(a.part1, R::C, a.B, c, a.da1, a.accumulate);
}

// ---------------------------------------------------------------- host side
template <class R>
static size_t rb_lds(int kind) {
  const size_t CT = R::CT, PL = R::PLANE, PA = R::PANEL, RD = (size_t)R::NR * 1024 * 8;
  switch (kind) {
    // fwd1 / bwd2 / bwd1: the double channel-partial staging (n RD) aliases the conv
    // region that follows the per-channel parameters
    case 0: return 4 * 2 * CT + std::max(2 * RD, 4 * (PL + PA));       // fwd1
    case 1: return 4 * (4 * CT + PL + PA);                              // fwd2
    case 2: return 4 * (6 * CT + 2 * PL + PA);                          // eval
    case 3: return 4 * 5 * CT + std::max(3 * RD, 4 * (2 * PL + PA));   // bwd2
    default: return 4 * 6 * CT + std::max(RD, 4 * (2 * PL + PA));      // bwd1
  }
}

constexpr size_t RB_LDS_MAX = 160 * 1024;

template <class R>
static void rb_launch(int kind, const RBArgs& a, hipStream_t st) {
  static bool attr = false;
  if (!attr) {  // more than 64 KB of dynamic LDS must be opted into once per kernel
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&rb_fwd1_kernel<R>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)rb_lds<R>(0));
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&rb_fwd2_kernel<R>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)rb_lds<R>(1));
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&rb_eval_kernel<R>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)rb_lds<R>(2));
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&rb_bwd2_kernel<R>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)rb_lds<R>(3));
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&rb_bwd1_kernel<R>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)rb_lds<R>(4));
    attr = true;
  }
  const dim3 grid(a.B), block(RB_T);
  const size_t lds = rb_lds<R>(kind);
  switch (kind) {
    case 0: hipLaunchKernelGGL(rb_fwd1_kernel<R>, grid, block, lds, st, a); break;
    case 1: hipLaunchKernelGGL(rb_fwd2_kernel<R>, grid, block, lds, st, a); break;
    case 2: hipLaunchKernelGGL(rb_eval_kernel<R>, grid, block, lds, st, a); break;
    case 3: hipLaunchKernelGGL(rb_bwd2_kernel<R>, grid, block, lds, st, a); break;
    default: hipLaunchKernelGGL(rb_bwd1_kernel<R>, grid, block, lds, st, a); break;
  }
#ifdef RB_TIMING
  (void)0;
#endif
}

// the (C, W) instantiations: C in {8, 16, 32}, W in {16, 32, 64}, C*W <= 1024
#define RB_SHAPES(X) X(8, 16) X(8, 32) X(8, 64) X(16, 16) X(16, 32) X(16, 64) X(32, 16) X(32, 32)

static unsigned long long* g_rb_tbuf = nullptr;  // RB_TIMING builds (tvq_rb_timing)

static bool rb_dispatch(int C, int W, int kind, const RBArgs* a_in, hipStream_t st,
                        size_t* lds_max) {
  RBArgs a_local;
  const RBArgs* a = a_in;
  if (a_in && g_rb_tbuf) {
    a_local = *a_in;
    a_local.tbuf = g_rb_tbuf + (size_t)kind * a_in->B * 16;
    a = &a_local;
  }
#define RB_CASE(CC, WW)                                                         \
  if (C == CC && W == WW) {                                                     \
    using R = RB<CC, WW>;                                                       \
    if (lds_max) {                                                              \
      size_t m = 0;                                                             \
      for (int k = 0; k < 5; ++k) m = rb_lds<R>(k) > m ? rb_lds<R>(k) : m;      \
      *lds_max = m;                                                             \
    }                                                                           \
    if (a) rb_launch<R>(kind, *a, st);                                          \
    return true;                                                                \
  }
  RB_SHAPES(RB_CASE)
#undef RB_CASE
  return false;
}

static bool rb_supported(int64_t B, int64_t C, int64_t H, int64_t W) {
  if (B < 1 || H != 3 || (int64_t)B * C * 3 * W >= (1ll << 31)) return false;
  size_t m = 0;
  return rb_dispatch((int)C, (int)W, 0, nullptr, nullptr, &m) && m <= RB_LDS_MAX;
}

static size_t rb_align(size_t n) { return (n + 255) & ~(size_t)255; }

struct RBWs {  // workspace layout (bytes)
  size_t part, part1, coef, slab2, slab1, du, total;
};
static RBWs rb_ws(int64_t B, int64_t C, int64_t W) {
  RBWs w;
  const int64_t kc = 9 * C + 1;
  const size_t slab = (size_t)(B * C * kc + reduce_rows_scratch(B, C * kc));
  w.part = 0;
  w.part1 = w.part + rb_align((size_t)B * C * 3 * 8);
  w.coef = w.part1 + rb_align((size_t)B * C * 8);
  w.slab2 = w.coef + rb_align((size_t)2 * C * 4);
  w.slab1 = w.slab2 + rb_align(slab * 4);
  w.du = w.slab1 + rb_align(slab * 4);
  w.total = w.du + rb_align((size_t)B * C * 3 * W * 4);
  return w;
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace tvq

using namespace tvq;

#ifdef RB_TIMING
// timing builds only: per-block phase timestamps of the next launches into buf
// (5 kernels x B blocks x 16 slots of wall_clock64)
extern "C" int tvq_rb_timing(unsigned long long* buf) {
  g_rb_tbuf = buf;
  return 0;
}
#endif

extern "C" int64_t tvq_resblock_workspace(int64_t B, int64_t C, int64_t H, int64_t W) {
  if (!rb_supported(B, C, H, W)) return -1;
  return (int64_t)rb_ws(B, C, W).total;
}

extern "C" int tvq_resblock_train_fwd(const float* x, int64_t B, int64_t C, int64_t H, int64_t W,
                                      const float* a1, const float* w1, const float* b1,
                                      const float* bn_w, const float* bn_b, float* running_mean,
                                      float* running_var, int64_t* num_batches_tracked,
                                      float momentum, float eps, const float* a2, const float* w2,
                                      const float* b2, float drop_p, const int64_t* seed_ptr,
                                      uint64_t offset, float* h, float* y, float* save,
                                      void* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(rb_supported(B, C, H, W), "tvq_resblock_train_fwd: unsupported shape");
  TVQ_CHECK_ARG(x && a1 && w1 && a2 && w2 && h && y && save && workspace && running_mean &&
                    running_var && aligned16(x) && aligned16(h),
                "tvq_resblock_train_fwd: bad arguments");
  TVQ_CHECK_ARG(drop_p >= 0.f && drop_p < 1.f && (drop_p == 0.f || seed_ptr),
                "tvq_resblock_train_fwd: bad dropout");
  hipStream_t st = (hipStream_t)stream;
  RBArgs a = {};
  a.x = x; a.h = h; a.a1 = a1; a.w1 = w1; a.b1 = b1; a.a2 = a2; a.w2 = w2; a.b2 = b2;
  a.save = save; a.h_out = h; a.y = y;
  a.part = (double*)workspace;
  a.B = (int)B;
  a.drop_p = drop_p;
  a.drop_scale = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
  a.seed_ptr = seed_ptr;
  a.offset = offset;
  a.fin = {(int)C, (int)B, B * 3 * W, eps, momentum, bn_w, bn_b, running_mean, running_var,
           num_batches_tracked, save, save + C, save + 2 * C, save + 3 * C};
  a.cnt = counters(1, FIN_NORM);
  rb_dispatch((int)C, (int)W, 0, &a, st, nullptr);
  if (!a.cnt) bn_stats_final_launch(a.part, a.fin, st);
  rb_dispatch((int)C, (int)W, 1, &a, st, nullptr);
  return launch_status("tvq_resblock_train_fwd");
}

extern "C" int tvq_resblock_eval_fwd(const float* x, int64_t B, int64_t C, int64_t H, int64_t W,
                                     const float* a1, const float* w1, const float* b1,
                                     const float* bn_w, const float* bn_b,
                                     const float* running_mean, const float* running_var,
                                     float eps, const float* a2, const float* w2, const float* b2,
                                     float* y, tvq_stream_t stream) {
  TVQ_CHECK_ARG(rb_supported(B, C, H, W), "tvq_resblock_eval_fwd: unsupported shape");
  TVQ_CHECK_ARG(x && a1 && w1 && a2 && w2 && y && running_mean && running_var && aligned16(x),
                "tvq_resblock_eval_fwd: bad arguments");
  RBArgs a = {};
  a.x = x; a.a1 = a1; a.w1 = w1; a.b1 = b1; a.bn_w = bn_w; a.bn_b = bn_b;
  a.rmean = running_mean; a.rvar = running_var; a.eps = eps;
  a.a2 = a2; a.w2 = w2; a.b2 = b2; a.y = y; a.B = (int)B;
  rb_dispatch((int)C, (int)W, 2, &a, (hipStream_t)stream, nullptr);
  return launch_status("tvq_resblock_eval_fwd");
}

extern "C" int tvq_resblock_bwd(const float* dy, const float* x, const float* h, int64_t B,
                                int64_t C, int64_t H, int64_t W, const float* a1, const float* w1,
                                const float* bn_w, const float* save, const float* a2,
                                const float* w2, float drop_p, const int64_t* seed_ptr,
                                uint64_t offset, float* dx, float* da1, float* dw1, float* db1,
                                float* dbn_w, float* dbn_b, float* da2, float* dw2, float* db2,
                                int64_t accumulate, void* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(rb_supported(B, C, H, W), "tvq_resblock_bwd: unsupported shape");
  TVQ_CHECK_ARG(dy && x && h && a1 && w1 && save && a2 && w2 && dx && da1 && dw1 && db1 && da2 &&
                    dw2 && db2 && workspace && aligned16(dy) && aligned16(x) && aligned16(h),
                "tvq_resblock_bwd: bad arguments");
  TVQ_CHECK_ARG(drop_p >= 0.f && drop_p < 1.f && (drop_p == 0.f || seed_ptr),
                "tvq_resblock_bwd: bad dropout");
  hipStream_t st = (hipStream_t)stream;
  const RBWs w = rb_ws(B, C, W);
  char* ws = (char*)workspace;
  float* coef = (float*)(ws + w.coef);
  float* slab2 = (float*)(ws + w.slab2);
  float* slab1 = (float*)(ws + w.slab1);
  RBArgs a = {};
  a.x = x; a.h = h; a.dy = dy; a.a1 = a1; a.w1 = w1; a.a2 = a2; a.w2 = w2; a.bn_w = bn_w;
  a.save = save; a.coef = coef;
  a.du = (float*)(ws + w.du); a.dx = dx; a.slab1 = slab1; a.slab2 = slab2; a.da1 = da1;
  a.part = (double*)(ws + w.part); a.part1 = (double*)(ws + w.part1);
  a.B = (int)B; a.accumulate = (int)accumulate;
  a.drop_p = drop_p;
  a.drop_scale = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
  a.seed_ptr = seed_ptr; a.offset = offset;
  a.invN = 1.0f / (float)(B * 3 * W);
  a.bfin = {(int)C, (int)B, coef, dbn_w, dbn_b, da2, (int)accumulate};
  a.cnt = counters(1, FIN_NORM);
  rb_dispatch((int)C, (int)W, 3, &a, st, nullptr);
  if (!a.cnt) bn_bwd_final_launch(a.part, a.bfin, st);
  a.cnt = counters(1, FIN_NORM);
  rb_dispatch((int)C, (int)W, 4, &a, st, nullptr);
  if (!a.cnt) snake_da_final_launch(a.part1, (int)C, (int)B, da1, (int)accumulate, st);
  const int64_t kc = 9 * C + 1;
  conv_wgrad_finish(slab2, (int)B, C, kc, dw2, db2, (int)accumulate, st);
  conv_wgrad_finish(slab1, (int)B, C, kc, dw1, db1, (int)accumulate, st);
  return launch_status("tvq_resblock_bwd");
}

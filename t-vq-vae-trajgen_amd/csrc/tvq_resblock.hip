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
//             BN partial sums (fp64)
//   rb_fwd2   every block reduces the partials (same fixed order) to the batch mean /
//             invstd -> scale / shift (bn_final_channel's arithmetic; block 0 writes them
//             and the running statistics); s2 = Snake_a2(h*scale + shift) staged ->
//             y = x + Dropout(conv2(s2) + b2)
//   rb_eval   both convs in one block with BN from the running statistics (s2 in LDS)
//   rb_bwd2   g2 = Dropout'(dy) (same counter-hash mask) -> dW2 | db2 per-image slab row;
//             ds2 = conv2^T(g2) -> du = ds2 * Snake'(u), u = h*scale + shift recomputed
//             -> store du; per-image (sum du, sum du*xhat, da2 term)
//   rb_bwd1   every block reduces those partials to the BN backward coefficients (block 0
//             writes the BN weight / bias and Snake a2 gradients);
//             dh = BN'(du) staged -> dW1 | db1 slab row; ds1 = conv1^T(dh) ->
//             dx = ds1 * Snake'(x) + dy (identity skip); per-image da1 terms -> a slab
//             row, summed over the images with the weight-gradient slabs
//
// Work split inside a block (RB_NW = 8 waves, one image; 256 images = 256 blocks = 2 waves
// per SIMD, where 4-wave blocks left each SIMD one wave and nothing to hide latency with):
//   * elementwise phases (staging the conv inputs, epilogues) run channel-per-wave: wave w
//     takes channels w, w + 8, ... and its lanes that channel's positions, so global loads
//     and stores are lane-contiguous and every per-channel sum is one fixed xor tree;
//   * a conv: each wave owns one (16-channel row tile, input-channel chunk of CPC) pair and
//     a set of 16-position tiles, run as interleaved v_mfma_f32_16x16x4_f32 chains that
//     read each weight fragment once; the chunk partials go to LDS and the epilogue sums
//     them in chunk order;
//   * a weight gradient: each wave owns a position chunk and a set of 16-column tiles of
//     the C x (9C+1) slab row, its chains sharing the dY and input-window fragments; the
//     chunk partials are summed in order into the image's slab row.
// Both operands of every MFMA come from LDS: the conv gathers the halo plane at
// c*PS + toff(t) (the data gradient: transposed weights, flipped taps), the weight gradient
// reduces over the image's positions with a ones column for the bias.  Arithmetic is the
// unfused kernels' (Snake, BN affine / backward formulas, dropout hash) up to the
// summation order, which is fixed.
#include <algorithm>

#include "tvq_bn.h"
#include "tvq_common.h"
#include "tvq_conv_internal.h"
#include "tvq_reduce.h"

namespace tvq {

#ifndef RB_NW
#define RB_NW 8
#endif
constexpr int RB_T = 64 * RB_NW;  // one image per block

template <int C_, int W_>
struct RB {
  static constexpr int C = C_, W = W_;
  static constexpr int P = 3 * W, MT = P / 16;       // positions, 16-position tiles
  static constexpr int NR = (C + 15) / 16, CT = 16 * NR;  // 16-row channel tiles
  // Halo planes (LDS bank map: MI355X_MICROARCH.md §LDS, ds_read_b32 bank = dword mod 32):
  // row stride WP = W + 2, plane stride PS == 2 mod 32.  (Round 4 measured a bank-linear
  // layout -- WP == 3, PS == 9 mod 32, permuted reduction order -- that cut
  // SQ_LDS_BANK_CONFLICT of rb_bwd1/2<16,32> 482K -> 62K per launch but ran slower, fused
  // fwd+bwd 66.8 -> 69.2 us: these kernels are bound by their global-memory phases, not
  // the LDS; it was removed in round 5.)
  static constexpr int WP = W + 2;
  static constexpr int HW = 5 * WP;                  // halo plane cells
  static constexpr int PS = HW + ((2 - HW % 32) + 32) % 32;  // plane stride
  static constexpr int K = 9 * C;                    // conv reduction length
  static constexpr int KST = K + ((2 - K % 32) + 32) % 32;  // panel row stride == 2 mod 32
  static constexpr int KC = K + 1, KT = (KC + 15) / 16;     // wgrad columns (+bias), tiles
  // conv: the waves are NR x NCH (row tile, input-channel chunk of CPC) combos times CMS
  // position groups; a wave runs CNF 16-position tiles of its combo as interleaved chains
  // that share the weight operand (1 + CNF LDS reads per CNF MFMAs)
  static constexpr int NCH0 = (C / 4) < (RB_NW / NR) ? C / 4 : RB_NW / NR;
  static constexpr int NCH = NCH0 < 4 ? NCH0 : 4;  // chunk partials stay within the LDS
  static constexpr int CPC = C / NCH;
  static constexpr int NCHK = 9 * CPC, NSTEP = NCHK / 4;  // a chunk's reductions, MFMA steps
  static constexpr int CMS = RB_NW / (NR * NCH), CNF = (MT + CMS - 1) / CMS;
  static constexpr int PR = P + ((4 - P % 8) + 8) % 8;  // conv partial row stride == 4 mod 8
  // weight gradient: the KT column tiles dealt over WKG wave groups, the positions split
  // into WPS chunks (WKG x WPS = RB_NW); a wave runs NR x WNF chains sharing the row (dY)
  // and column (input window) operands (NR + WNF LDS reads per NR x WNF MFMAs)
  static constexpr int PSTEPS = P / 4;
  static constexpr int WPS0 = C >= 32 ? 1 : (C == 8 && W >= 32) ? 8 : 4;
  static constexpr int WPS = WPS0 < RB_NW ? WPS0 : RB_NW;
  static constexpr int WKG = RB_NW / WPS, WNF = (KT + WKG - 1) / WKG;
  static constexpr int WSTEPS = PSTEPS / WPS;
  static constexpr int KCR = KC + ((4 - KC % 8) + 8) % 8;  // wgrad partial row stride
  // elementwise phases: channels per wave, positions per lane
  static constexpr int CPW = (C + RB_NW - 1) / RB_NW, PPL = (P + 63) / 64;
  static constexpr int NB = 2 * WP + 6;              // border cells per halo plane
  static constexpr int PLANE = C * PS, PANEL = CT * KST;
  static constexpr int NPAN = CT * K, UP = (NPAN + RB_T - 1) / RB_T;  // panel loads
  static constexpr int PARTC = NCH * C * PR;         // conv chunk partials (floats)
  static constexpr int PARTW = WPS > 1 ? WPS * C * KCR : 0;  // wgrad chunk partials
  // backward kernels' LDS: G planes | S planes | panel | conv partials | wgrad partials |
  // ones plane K1 | zeros plane K0 = K1 + PS
  // the weight-gradient partials are summed (rb_wgrad_sum) before the conv items write
  // theirs, so the two share one region (round 5: RB<16,32>'s backward 99 -> 74 KB, two
  // blocks per CU beside the other streams' kernels)
  static constexpr int PARTCW = PARTC > PARTW ? PARTC : PARTW;
  static constexpr int K1OFF = 2 * PLANE + PANEL + PARTCW;
  static constexpr int CONSTP = 2 * PS;  // ones plane + zeros plane
  // external weight gradients (C = 32 at W = 16): the backward kernels write the conv
  // operands (g and s planes) and conv_wgrad_w16_multi reduces them over images in one
  // launch per ResBlock (pair), instead of a C x (9C + 1) slab row per image (37 KB, 12x the
  // image's activations); taken when RBArgs::wext is set (B % 16 == 0)
  static constexpr bool WEXT = C_ == 32 && W_ == 16;
  static_assert(P % 16 == 0 && W % 4 == 0 && C % NCH == 0 && CPC % 4 == 0 &&
                    RB_NW % (NR * NCH) == 0 && RB_NW % WPS == 0 && PSTEPS % WPS == 0,
                "unsupported ResBlock geometry");
};

struct RBArgs {  // every pointer / scalar a fused ResBlock kernel reads or writes
  const float *x, *h, *dy;
  const float *a1, *w1, *b1, *a2, *w2, *b2;
  const float *bn_w, *bn_b, *rmean, *rvar;  // eval
  const float* save;                         // mean | invstd | scale | shift (C each)
  float *h_out, *y, *du, *dx, *slab1, *slab2, *slabda, *slabda2;
  // RB::WEXT shapes with wext set: the (B, C, 3, W) conv operand planes the backward writes
  // (conv1: g = dh, s = Snake_a1(x); conv2: g = Dropout'(dy), s = Snake_a2(BN(h))) and the
  // small slabs conv_wgrad_w16_multi reduces them into
  float *gp1, *sp1, *gp2, *sp2, *wsl1, *wsl2;
  int wext;
  double* part;
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

// halo offset of position p's top-left window cell
template <class R>
__device__ __forceinline__ int rb_pos(int p) {
  const int h = p / R::W;
  return h * R::WP + (p - h * R::W);
}

__device__ __forceinline__ int rb_wid() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// channel-per-wave element layout: element (u, v) of this lane is channel
// c = wid + RB_NW * u, position p = lane + 64 * v
template <class R>
struct RBElems {
  int c[R::CPW];
  int p[R::PPL];
  __device__ __forceinline__ RBElems() {
    const int wid = rb_wid(), l = threadIdx.x & 63;
#pragma unroll
    for (int u = 0; u < R::CPW; ++u) c[u] = wid + RB_NW * u;
#pragma unroll
    for (int v = 0; v < R::PPL; ++v) p[v] = l + 64 * v;
  }
  __device__ __forceinline__ bool ok(int u, int v) const { return c[u] < R::C && p[v] < R::P; }
  __device__ __forceinline__ int64_t gi(int64_t img0, int u, int v) const {
    return img0 + (int64_t)(c[u] < R::C ? c[u] : 0) * R::P + (p[v] < R::P ? p[v] : 0);
  }
  __device__ __forceinline__ int cell(int u, int v) const {  // halo-plane cell
    return c[u] * R::PS + R::WP + 1 + rb_pos<R>(p[v]);
  }
};

// every element of this lane's layout (loads issued, none waited on)
template <class R>
__device__ __forceinline__ void rb_load(const float* __restrict__ src, int64_t img0,
                                        const RBElems<R>& el, float (&v)[R::CPW][R::PPL]) {
#pragma unroll
  for (int u = 0; u < R::CPW; ++u)
#pragma unroll
    for (int q = 0; q < R::PPL; ++q) v[u][q] = src[el.gi(img0, u, q)];
}

// a per-channel parameter at this lane's channels (0 beyond C)
template <class R>
__device__ __forceinline__ void rb_param(const float* __restrict__ src, const RBElems<R>& el,
                                         float (&v)[R::CPW], float dflt = 0.f) {
#pragma unroll
  for (int u = 0; u < R::CPW; ++u) v[u] = src ? src[el.c[u] < R::C ? el.c[u] : 0] : dflt;
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
      o = (1 + (k >> 1)) * R::WP + ((k & 1) ? R::W + 1 : 0);
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

// TRANS: the panel of the data gradient (rows = input channels, k = n*9 + t)
template <class R, bool TRANS = false>
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

// Conv of the staged plane(s) S with the panel A.  Wave w owns output-row tile nr, input
// channel chunk ch (CPC channels) and position tiles mt = m, m + CMS, ...: CNF interleaved
// 16 x 16 chains that read each weight fragment once.  The chunk partial of tile (nr, mt)
// goes to Pc[(ch*C + n)*PR + p].  A dead chain (mt >= MT, wave-uniform) recomputes tile m
// on valid addresses and stores nothing, so the loop has no branch.  FLIP: data gradient
// (taps flipped).
template <class R, bool FLIP>
__device__ __forceinline__ void rb_conv_items(const float* __restrict__ A,
                                              const float* __restrict__ S, float* __restrict__ Pc) {
  const int l = threadIdx.x & 63, j = l & 15, kq = l >> 4, wid = rb_wid();
  const int m = wid % R::CMS, combo = wid / R::CMS, ch = combo % R::NCH, nr = combo / R::NCH;
  // gather offsets of the 9 MFMA steps of a 4-channel group, relative to its first channel:
  // step s reads reduction index k = 4s + kq = c*9 + t
  int roff[9];
#pragma unroll
  for (int s = 0; s < 9; ++s) {
    const int k = 4 * s + kq, c = k / 9, t0 = k - 9 * c, t = FLIP ? 8 - t0 : t0;
    const int kh = t / 3;
    roff[s] = c * R::PS + kh * R::WP + (t - 3 * kh);
  }
  const float* ap = A + (nr * 16 + j) * R::KST + ch * R::CPC * 9 + kq;
  const float* sp[R::CNF];
#pragma unroll
  for (int f = 0; f < R::CNF; ++f) {
    const int mt = m + R::CMS * f;
    sp[f] = S + rb_pos<R>((mt < R::MT ? mt : m) * 16 + j) + ch * R::CPC * R::PS;
  }
  floatx4 acc[R::CNF];
#pragma unroll
  for (int f = 0; f < R::CNF; ++f) acc[f] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int g = 0; g < R::CPC / 4; ++g)
#pragma unroll
    for (int s = 0; s < 9; ++s) {
      const float a = ap[g * 36 + 4 * s];
#pragma unroll
      for (int f = 0; f < R::CNF; ++f)
        acc[f] = mfma16x16x4(a, sp[f][g * 4 * R::PS + roff[s]], acc[f]);
    }
#pragma unroll
  for (int f = 0; f < R::CNF; ++f) {
    const int mt = m + R::CMS * f;
    if (mt >= R::MT) continue;  // wave-uniform
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = nr * 16 + 4 * kq + r;  // channel of this register
      if (n < R::C) Pc[(ch * R::C + n) * R::PR + mt * 16 + j] = acc[f][r];
    }
  }
}

// conv result at this lane's element (u, v): the chunk partials summed in chunk order
template <class R>
__device__ __forceinline__ float rb_conv_at(const float* __restrict__ Pc, const RBElems<R>& el,
                                            int u, int v) {
  const int c = el.c[u] < R::C ? el.c[u] : 0, p = el.p[v] < R::P ? el.p[v] : 0;
  float s = Pc[c * R::PR + p];
#pragma unroll
  for (int ch = 1; ch < R::NCH; ++ch) s += Pc[(ch * R::C + c) * R::PR + p];
  return s;
}

// Weight gradient of one image: D[n][kc] = sum_p G[n][p] * B[p][kc], B[p][kc] =
// S[koff(kc) + pos(p)] (kc < K), 1 (kc == K: bias), 0 beyond; rows n >= C are 0.  Wave w
// owns position chunk pc = w / WKG and column tiles kt = w % WKG + WKG*f; each lane's
// operand pointers are chosen once (the window cell of its column, the ones plane for the
// bias column, the zeros plane for padding columns and rows), so every MFMA step is two
// unconditional LDS reads and no branch.  WPS == 1: straight into the slab row, else the
// chunk partials to Pw[(pc*C + n)*KCR + kc] (rb_wgrad_sum adds them in chunk order).
template <class R>
__device__ __forceinline__ void rb_wgrad_items(const float* __restrict__ G,
                                               const float* __restrict__ S,
                                               const float* __restrict__ K1,
                                               float* __restrict__ Pw,
                                               float* __restrict__ slab_row) {
  const int l = threadIdx.x & 63, j = l & 15, kq = l >> 4, wid = rb_wid();
  const int kg = wid % R::WKG, pc = wid / R::WKG;
  const float* K0 = K1 + R::PS;  // zeros plane
  const float* gp[R::NR];
#pragma unroll
  for (int nr = 0; nr < R::NR; ++nr) {
    const int n = nr * 16 + j;
    gp[nr] = (n < R::C ? G + n * R::PS : K0) + R::WP + 1;
  }
  const float* sp[R::WNF];
#pragma unroll
  for (int f = 0; f < R::WNF; ++f) {
    const int kc = (kg + R::WKG * f) * 16 + j;
    const int k = kc < R::K ? kc : 0, c = k / 9, t = k - 9 * c, kh = t / 3;
    sp[f] = kc < R::K ? S + c * R::PS + kh * R::WP + (t - 3 * kh) : kc == R::K ? K1 : K0;
  }
  floatx4 acc[R::NR][R::WNF];
#pragma unroll
  for (int nr = 0; nr < R::NR; ++nr)
#pragma unroll
    for (int f = 0; f < R::WNF; ++f) acc[nr][f] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int pbase = pc * R::WSTEPS * 4;
#pragma unroll
  for (int s = 0; s < R::WSTEPS; ++s) {
    const int p0 = pbase + 4 * s;                         // 4 | W: one row
    const int po = p0 + 2 * (p0 / R::W) + kq;            // (p0 / W) * WP + p0 % W + kq
    float ga[R::NR], sb[R::WNF];
#pragma unroll
    for (int nr = 0; nr < R::NR; ++nr) ga[nr] = gp[nr][po];
#pragma unroll
    for (int f = 0; f < R::WNF; ++f) sb[f] = sp[f][po];
#pragma unroll
    for (int nr = 0; nr < R::NR; ++nr)
#pragma unroll
      for (int f = 0; f < R::WNF; ++f) acc[nr][f] = mfma16x16x4(ga[nr], sb[f], acc[nr][f]);
  }
#pragma unroll
  for (int f = 0; f < R::WNF; ++f) {
    const int kt = kg + R::WKG * f;
    if (kt >= R::KT) continue;  // wave-uniform
    const int kc = kt * 16 + j;
    if (kc >= R::KC) continue;
#pragma unroll
    for (int nr = 0; nr < R::NR; ++nr)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = nr * 16 + 4 * kq + r;
        if (n >= R::C) continue;
        if (R::WPS == 1)
          slab_row[n * R::KC + kc] = acc[nr][f][r];
        else
          Pw[(pc * R::C + n) * R::KCR + kc] = acc[nr][f][r];
      }
  }
}

// the ones plane (bias column) and zeros plane (padding) the weight-gradient items read
template <class R>
__device__ __forceinline__ void rb_const_planes(float* __restrict__ K1) {
  for (int i = threadIdx.x; i < 2 * R::PS; i += RB_T) K1[i] = i < R::PS ? 1.f : 0.f;
}

template <class R>
__device__ __forceinline__ void rb_wgrad_sum(const float* __restrict__ Pw,
                                             float* __restrict__ slab_row) {
  if (R::WPS == 1) return;
  for (int e = threadIdx.x; e < R::C * R::KC; e += RB_T) {
    const int n = e / R::KC, kc = e - n * R::KC;
    float s = Pw[n * R::KCR + kc];
#pragma unroll
    for (int pc = 1; pc < R::WPS; ++pc) s += Pw[(pc * R::C + n) * R::KCR + kc];
    slab_row[e] = s;
  }
}

// per-channel fp64 sums of this lane's element values s[0..NS) (fixed order: over v, then
// the xor tree) -> lane 0 stores part[(c*NS + i)*B + b] (image-fastest: the consumer's
// lanes read consecutive images)
template <class R, int NS, int NT>
__device__ __forceinline__ void rb_channel_sums(double (&s)[NT][R::CPW][R::PPL],
                                                const RBElems<R>& el, int B, int b,
                                                double* part) {
#pragma unroll
  for (int u = 0; u < R::CPW; ++u) {
    if (el.c[u] >= R::C) continue;  // wave-uniform
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      double t = s[i][u][0];
#pragma unroll
      for (int v = 1; v < R::PPL; ++v) t += s[i][u][v];
      t = wave_sum_d(t);
      if ((threadIdx.x & 63) == 0) part[((int64_t)el.c[u] * NS + i) * B + b] = t;
    }
  }
}

// one image's per-channel total of s[i] (same order) -> its row of a float slab, summed
// over the images in order by the deferred slab reduction (the Snake a gradients)
template <class R, int NT>
__device__ __forceinline__ void rb_slab_row_sums(double (&s)[NT][R::CPW][R::PPL], int i,
                                                 const RBElems<R>& el, int b, float* slab) {
#pragma unroll
  for (int u = 0; u < R::CPW; ++u) {
    if (el.c[u] >= R::C) continue;  // wave-uniform
    double t = s[i][u][0];
#pragma unroll
    for (int v = 1; v < R::PPL; ++v) t += s[i][u][v];
    t = wave_sum_d(t);
    if ((threadIdx.x & 63) == 0) slab[(int64_t)b * R::C + el.c[u]] = (float)t;
  }
}

// Batch totals of NS per-image fp64 partials part[(c*NS + i)*B + b] for this wave's
// channels.  Every block of the consuming kernel reduces them itself in the same fixed
// order (each lane its images in increasing b, then the xor tree -- wave_chunk_sums' order),
// so the blocks agree bit for bit and the producing kernel needs no last block.
// rb_batch_issue loads the first 64*RB_UB images' values (issued with the block's other
// prologue loads, so they share one round trip); rb_batch_sums adds them and any further
// images in order.
constexpr int RB_UB = 4;
template <class R, int NS>
__device__ __forceinline__ void rb_batch_issue(const double* __restrict__ part, int B,
                                               const RBElems<R>& el,
                                               double (&v)[R::CPW][RB_UB][NS]) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int u = 0; u < R::CPW; ++u) {
    const int c = el.c[u] < R::C ? el.c[u] : 0;
#pragma unroll
    for (int k = 0; k < RB_UB; ++k)
#pragma unroll
      for (int i = 0; i < NS; ++i)
        v[u][k][i] = l + 64 * k < B ? part[((int64_t)c * NS + i) * B + l + 64 * k] : 0.0;
  }
}

template <class R, int NS>
__device__ __forceinline__ void rb_batch_sums(const double* __restrict__ part, int B,
                                              const RBElems<R>& el,
                                              const double (&v)[R::CPW][RB_UB][NS],
                                              double (&t)[R::CPW][NS]) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int u = 0; u < R::CPW; ++u) {
    const int c = el.c[u] < R::C ? el.c[u] : 0;
#pragma unroll
    for (int i = 0; i < NS; ++i) t[u][i] = 0.0;
#pragma unroll
    for (int k = 0; k < RB_UB; ++k)
#pragma unroll
      for (int i = 0; i < NS; ++i) t[u][i] += v[u][k][i];
    for (int b = l + 64 * RB_UB; b < B; b += 64)  // B > 256 only
#pragma unroll
      for (int i = 0; i < NS; ++i) t[u][i] += part[((int64_t)c * NS + i) * B + b];
#pragma unroll
    for (int i = 0; i < NS; ++i) t[u][i] = wave_sum_d(t[u][i]);
  }
}

// ---------------------------------------------------------------- kernels
// The kernels' bodies take the block's LDS and, for the fused pairs of consecutive
// ResBlocks (rb_fwd21 / rb_bwd12 below), the activation handed over in registers: the
// elementwise layout (RBElems) is the same in every kernel of a shape, so each lane hands
// over exactly the elements it consumes next.
template <class R>
using RBRegs = float[R::CPW][R::PPL];

template <class R, bool XREG>
__device__ __forceinline__ void rb_fwd1_body(const RBArgs& a, double* rb_smem,
                                             const RBRegs<R>& xin) {
  float* S = reinterpret_cast<float*>(rb_smem);
  float* A = S + R::PLANE;
  float* Pc = A + R::PANEL;
  const int b = blockIdx.x;
  const int64_t img0 = (int64_t)b * R::C * R::P;
  RB_MARK(0);
  const RBElems<R> el;
  float v[R::CPW][R::PPL], pv[R::UP], a1[R::CPW], b1[R::CPW];
  rb_load_panel<R, false>(a.w1, pv);  // first: the panel store waits for these alone
  if constexpr (XREG) {
#pragma unroll
    for (int u = 0; u < R::CPW; ++u)
#pragma unroll
      for (int q = 0; q < R::PPL; ++q) v[u][q] = xin[u][q];
  } else {
    rb_load<R>(a.x, img0, el, v);
  }
  rb_param<R>(a.a1, el, a1);
  rb_param<R>(a.b1, el, b1);
  rb_border<R>(S);
  rb_put_panel<R>(A, pv);
  RB_MARK(1);
#pragma unroll
  for (int u = 0; u < R::CPW; ++u)
#pragma unroll
    for (int q = 0; q < R::PPL; ++q)
      if (el.ok(u, q)) S[el.cell(u, q)] = snake_f(v[u][q], a1[u], 1.0f / a1[u]);
  __syncthreads();
  RB_MARK(2);
  rb_conv_items<R, false>(A, S, Pc);
  __syncthreads();
  RB_MARK(3);
  double s[2][R::CPW][R::PPL];
#pragma unroll
  for (int u = 0; u < R::CPW; ++u)
#pragma unroll
    for (int q = 0; q < R::PPL; ++q) {
      s[0][u][q] = s[1][u][q] = 0.0;
      if (!el.ok(u, q)) continue;
      const float val = rb_conv_at<R>(Pc, el, u, q) + b1[u];
      a.h_out[el.gi(img0, u, q)] = val;
      s[0][u][q] = (double)val;
      s[1][u][q] = (double)val * (double)val;
    }
  RB_MARK(4);
  rb_channel_sums<R, 2>(s, el, a.B, b, a.part);
  RB_MARK(5);
}

template <class R>
__global__ __launch_bounds__(RB_T) void rb_fwd1_kernel(RBArgs a) {
  extern __shared__ double rb_smem[];
  RBRegs<R> none;
  rb_fwd1_body<R, false>(a, rb_smem, none);
}

// yout: this lane's y elements (the next block's input in a fused pair)
template <class R>
__device__ __forceinline__ void rb_fwd2_body(const RBArgs& a, double* rb_smem, RBRegs<R>& yout) {
  float* S = reinterpret_cast<float*>(rb_smem);
  float* A = S + R::PLANE;
  float* Pc = A + R::PANEL;
  const int b = blockIdx.x;
  const int64_t img0 = (int64_t)b * R::C * R::P;
  RB_MARK(0);
  const RBElems<R> el;
  float v[R::CPW][R::PPL], xr[R::CPW][R::PPL], pv[R::UP];
  float a2[R::CPW], sc[R::CPW], sh[R::CPW], b2[R::CPW];
  rb_load_panel<R, false>(a.w2, pv);
  rb_load<R>(a.h, img0, el, v);
  rb_load<R>(a.x, img0, el, xr);
  rb_param<R>(a.a2, el, a2);
  rb_param<R>(a.b2, el, b2);
  double bv[R::CPW][RB_UB][2], bs[R::CPW][2];
  rb_batch_issue<R, 2>(a.part, a.B, el, bv);
  rb_border<R>(S);
  rb_put_panel<R>(A, pv);
  rb_batch_sums<R, 2>(a.part, a.B, el, bv, bs);
  // the batch statistics (bn_final_channel's arithmetic); block 0 publishes them (save,
  // running statistics, num_batches_tracked)
  const bool pub = b == 0 && (threadIdx.x & 63) == 0;
  if (pub && threadIdx.x == 0 && a.fin.nbt) a.fin.nbt[0] += 1;
#pragma unroll
  for (int u = 0; u < R::CPW; ++u) {
    const int c = el.c[u] < R::C ? el.c[u] : 0;
    bn_final_from_sums(bs[u][0], bs[u][1], c, a.fin, pub && el.c[u] < R::C, sc[u], sh[u]);
  }
  RB_MARK(1);
#pragma unroll
  for (int u = 0; u < R::CPW; ++u)
#pragma unroll
    for (int q = 0; q < R::PPL; ++q)
      if (el.ok(u, q)) S[el.cell(u, q)] = snake_f(fmaf(v[u][q], sc[u], sh[u]), a2[u], 1.0f / a2[u]);
  __syncthreads();
  RB_MARK(2);
  rb_conv_items<R, false>(A, S, Pc);
  __syncthreads();
  RB_MARK(3);
  const uint64_t seed = a.drop_p > 0.f ? mix_seed(a.seed_ptr, a.offset) : 0ull;
#pragma unroll
  for (int u = 0; u < R::CPW; ++u)
#pragma unroll
    for (int q = 0; q < R::PPL; ++q) {
      yout[u][q] = 0.f;
      if (!el.ok(u, q)) continue;
      const int64_t gi = el.gi(img0, u, q);
      float val = rb_conv_at<R>(Pc, el, u, q) + b2[u];
      if (a.drop_p > 0.f)
        val = uniform01(seed, (uint64_t)gi) >= a.drop_p ? val * a.drop_scale : 0.f;
      yout[u][q] = xr[u][q] + val;
      a.y[gi] = yout[u][q];
    }
}

template <class R>
__global__ __launch_bounds__(RB_T) void rb_fwd2_kernel(RBArgs a) {
  extern __shared__ double rb_smem[];
  RBRegs<R> y;
  rb_fwd2_body<R>(a, rb_smem, y);
}

// fwd2 of ResBlock 1 and fwd1 of ResBlock 2 (its input = ResBlock 1's output) in one launch
template <class R>
__global__ __launch_bounds__(RB_T) void rb_fwd21_kernel(RBArgs a1, RBArgs a2) {
  extern __shared__ double rb_smem[];
  RBRegs<R> y;
  rb_fwd2_body<R>(a1, rb_smem, y);
  __syncthreads();  // LDS reused
  rb_fwd1_body<R, true>(a2, rb_smem, y);
}

template <class R>
__global__ __launch_bounds__(RB_T) void rb_eval_kernel(RBArgs a) {
  extern __shared__ double rb_smem[];
  float* S1 = reinterpret_cast<float*>(rb_smem);
  float* S2 = S1 + R::PLANE;
  float* A = S2 + R::PLANE;  // conv1's panel, then conv2's (conv2's weights wait in registers)
  float* Pc = A + R::PANEL;
  const int b = blockIdx.x;
  const int64_t img0 = (int64_t)b * R::C * R::P;
  const RBElems<R> el;
  float v[R::CPW][R::PPL], pv1[R::UP], pv2[R::UP];
  float a1[R::CPW], b1[R::CPW], a2[R::CPW], b2[R::CPW], sc[R::CPW], sh[R::CPW];
  rb_load<R>(a.x, img0, el, v);
  rb_load_panel<R, false>(a.w1, pv1);
  rb_load_panel<R, false>(a.w2, pv2);
  rb_param<R>(a.a1, el, a1);
  rb_param<R>(a.b1, el, b1);
  rb_param<R>(a.a2, el, a2);
  rb_param<R>(a.b2, el, b2);
#pragma unroll
  for (int u = 0; u < R::CPW; ++u) {  // bn_eval_prep_kernel's affine form
    const int c = el.c[u] < R::C ? el.c[u] : 0;
    const float inv = 1.0f / sqrtf(a.rvar[c] + a.eps);
    sc[u] = (a.bn_w ? a.bn_w[c] : 1.f) * inv;
    sh[u] = (a.bn_b ? a.bn_b[c] : 0.f) - a.rmean[c] * sc[u];
  }
  rb_border<R>(S1);
  rb_border<R>(S2);
  rb_put_panel<R>(A, pv1);
#pragma unroll
  for (int u = 0; u < R::CPW; ++u)
#pragma unroll
    for (int q = 0; q < R::PPL; ++q)
      if (el.ok(u, q)) S1[el.cell(u, q)] = snake_f(v[u][q], a1[u], 1.0f / a1[u]);
  __syncthreads();
  rb_conv_items<R, false>(A, S1, Pc);
  __syncthreads();
#pragma unroll
  for (int u = 0; u < R::CPW; ++u)
#pragma unroll
    for (int q = 0; q < R::PPL; ++q)
      if (el.ok(u, q)) {
        const float hv = fmaf(rb_conv_at<R>(Pc, el, u, q) + b1[u], sc[u], sh[u]);
        S2[el.cell(u, q)] = snake_f(hv, a2[u], 1.0f / a2[u]);
      }
  rb_put_panel<R>(A, pv2);  // every wave is past conv1 (the barrier above)
  __syncthreads();          // S2, conv2's panel complete; conv1's partials consumed
  rb_conv_items<R, false>(A, S2, Pc);
  __syncthreads();
#pragma unroll
  for (int u = 0; u < R::CPW; ++u)
#pragma unroll
    for (int q = 0; q < R::PPL; ++q)
      if (el.ok(u, q)) a.y[el.gi(img0, u, q)] = v[u][q] + (rb_conv_at<R>(Pc, el, u, q) + b2[u]);
}

template <class R, bool DYREG>
__device__ __forceinline__ void rb_bwd2_body(const RBArgs& a, double* rb_smem,
                                             const RBRegs<R>& dyin) {
  float* G = reinterpret_cast<float*>(rb_smem);  // g2 planes
  float* S = G + R::PLANE;                         // s2 planes
  float* A = S + R::PLANE;                         // transposed w2
  float* Pc = A + R::PANEL;
  float* Pw = Pc;  // summed before the conv items write Pc
  float* K1 = reinterpret_cast<float*>(rb_smem) + R::K1OFF;  // ones | zeros planes
  const int b = blockIdx.x;
  const int64_t img0 = (int64_t)b * R::C * R::P;
  RB_MARK(0);
  const RBElems<R> el;
  float vg[R::CPW][R::PPL], vh[R::CPW][R::PPL], pv[R::UP];
  float a2[R::CPW], sc[R::CPW], sh[R::CPW], mu[R::CPW], is[R::CPW];
  rb_load_panel<R, true>(a.w2, pv);
  if constexpr (DYREG) {
#pragma unroll
    for (int u = 0; u < R::CPW; ++u)
#pragma unroll
      for (int q = 0; q < R::PPL; ++q) vg[u][q] = dyin[u][q];
  } else {
    rb_load<R>(a.dy, img0, el, vg);
  }
  rb_load<R>(a.h, img0, el, vh);
  rb_param<R>(a.a2, el, a2);
  rb_param<R>(a.save + 2 * R::C, el, sc);
  rb_param<R>(a.save + 3 * R::C, el, sh);
  rb_param<R>(a.save, el, mu);
  rb_param<R>(a.save + R::C, el, is);
  rb_border<R>(G);
  rb_border<R>(S);
  rb_const_planes<R>(K1);
  rb_put_panel<R, true>(A, pv);
  RB_MARK(1);
  const uint64_t seed = a.drop_p > 0.f ? mix_seed(a.seed_ptr, a.offset) : 0ull;
#pragma unroll
  for (int u = 0; u < R::CPW; ++u)
#pragma unroll
    for (int q = 0; q < R::PPL; ++q) {
      if (!el.ok(u, q)) continue;
      float d = vg[u][q];
      if (a.drop_p > 0.f)
        d = uniform01(seed, (uint64_t)el.gi(img0, u, q)) >= a.drop_p ? d * a.drop_scale : 0.f;
      const float sv = snake_f(fmaf(vh[u][q], sc[u], sh[u]), a2[u], 1.0f / a2[u]);
      G[el.cell(u, q)] = d;
      S[el.cell(u, q)] = sv;
      if constexpr (R::WEXT) {
        if (a.wext) {
          const int64_t gi = el.gi(img0, u, q);
          a.gp2[gi] = d;
          a.sp2[gi] = sv;
        }
      }
    }
  __syncthreads();
  RB_MARK(2);
  if (!(R::WEXT && a.wext)) {
    float* slab_row = a.slab2 + (int64_t)b * R::C * R::KC;
    rb_wgrad_items<R>(G, S, K1, Pw, slab_row);
    if (R::WPS > 1) {  // the partials, then the region is the conv items'
      __syncthreads();
      rb_wgrad_sum<R>(Pw, slab_row);
      __syncthreads();
    }
  }
  RB_MARK(3);
  rb_conv_items<R, true>(A, G, Pc);
  __syncthreads();
  RB_MARK(4);
  double s[3][R::CPW][R::PPL];
#pragma unroll
  for (int u = 0; u < R::CPW; ++u)
#pragma unroll
    for (int q = 0; q < R::PPL; ++q) {
      s[0][u][q] = s[1][u][q] = s[2][u][q] = 0.0;
      if (!el.ok(u, q)) continue;
      const float av = a2[u], inv_a = 1.0f / av;
      const float hv = vh[u][q];
      const float gs = rb_conv_at<R>(Pc, el, u, q);  // d loss / d s2
      const float uu = fmaf(hv, sc[u], sh[u]);
      float sn, cs;
      sincosf(av * uu, &sn, &cs);
      const float t = 2.0f * sn * cs;
      const float d = gs + gs * inv_a * t * av;  // d loss / d u (bn_bwd_partial_kernel)
      const float xhat = (hv - mu[u]) * is[u];
      s[0][u][q] = d;
      s[1][u][q] = (double)d * xhat;
      s[2][u][q] = (double)(gs * inv_a * t * uu) - (double)(gs * (sn * sn) * inv_a * inv_a);
      a.du[el.gi(img0, u, q)] = d;
    }
  RB_MARK(5);
  rb_channel_sums<R, 2>(s, el, a.B, b, a.part);
  rb_slab_row_sums<R>(s, 2, el, b, a.slabda2);
  RB_MARK(6);
}

template <class R>
__global__ __launch_bounds__(RB_T) void rb_bwd2_kernel(RBArgs a) {
  extern __shared__ double rb_smem[];
  RBRegs<R> none;
  rb_bwd2_body<R, false>(a, rb_smem, none);
}

// dxout: this lane's dx elements (the previous block's output gradient in a fused pair)
template <class R>
__device__ __forceinline__ void rb_bwd1_body(const RBArgs& a, double* rb_smem, RBRegs<R>& dxout) {
  float* G = reinterpret_cast<float*>(rb_smem);  // dh planes
  float* S = G + R::PLANE;                         // s1 planes
  float* A = S + R::PLANE;                         // transposed w1
  float* Pc = A + R::PANEL;
  float* Pw = Pc;  // summed before the conv items write Pc
  float* K1 = reinterpret_cast<float*>(rb_smem) + R::K1OFF;  // ones | zeros planes
  const int b = blockIdx.x, l = threadIdx.x & 63;
  const int64_t img0 = (int64_t)b * R::C * R::P;
  RB_MARK(0);
  const RBElems<R> el;
  float vd[R::CPW][R::PPL], vh[R::CPW][R::PPL], vx[R::CPW][R::PPL], vy[R::CPW][R::PPL];
  float pv[R::UP], a1[R::CPW], mu[R::CPW], is[R::CPW], bw[R::CPW], md[R::CPW], mx[R::CPW];
  rb_load_panel<R, true>(a.w1, pv);
  rb_load<R>(a.du, img0, el, vd);
  rb_load<R>(a.h, img0, el, vh);
  rb_load<R>(a.x, img0, el, vx);
  rb_load<R>(a.dy, img0, el, vy);
  rb_param<R>(a.a1, el, a1);
  rb_param<R>(a.save, el, mu);
  rb_param<R>(a.save + R::C, el, is);
  rb_param<R>(a.bn_w, el, bw, 1.f);
  // BN backward coefficients (sum du, sum du*xhat) from rb_bwd2's per-image partials;
  // block 0 writes the BN weight / bias gradients
  double bv[R::CPW][RB_UB][2], bs[R::CPW][2];
  rb_batch_issue<R, 2>(a.part, a.B, el, bv);
  rb_border<R>(G);
  rb_border<R>(S);
  rb_const_planes<R>(K1);
  rb_put_panel<R, true>(A, pv);
  rb_batch_sums<R, 2>(a.part, a.B, el, bv, bs);
#pragma unroll
  for (int u = 0; u < R::CPW; ++u) {
    const int c = el.c[u] < R::C ? el.c[u] : 0;
    md[u] = (float)bs[u][0] * a.invN;
    mx[u] = (float)bs[u][1] * a.invN;
    if (b == 0 && l == 0 && el.c[u] < R::C)
      bn_bwd_params_from_sums(bs[u][0], bs[u][1], 0.0, c, a.bfin);
  }
  RB_MARK(1);
  // dh = w*invstd*(du - mean(du) - xhat*mean(du*xhat))  (bn_bwd_apply_kernel)
#pragma unroll
  for (int u = 0; u < R::CPW; ++u)
#pragma unroll
    for (int q = 0; q < R::PPL; ++q) {
      if (!el.ok(u, q)) continue;
      const float xhat = (vh[u][q] - mu[u]) * is[u];
      const float gv = bw[u] * is[u] * (vd[u][q] - md[u] - xhat * mx[u]);
      const float sv = snake_f(vx[u][q], a1[u], 1.0f / a1[u]);
      G[el.cell(u, q)] = gv;
      S[el.cell(u, q)] = sv;
      if constexpr (R::WEXT) {
        if (a.wext) {
          const int64_t gi = el.gi(img0, u, q);
          a.gp1[gi] = gv;
          a.sp1[gi] = sv;
        }
      }
    }
  __syncthreads();
  RB_MARK(2);
  if (!(R::WEXT && a.wext)) {
    float* slab_row = a.slab1 + (int64_t)b * R::C * R::KC;
    rb_wgrad_items<R>(G, S, K1, Pw, slab_row);
    if (R::WPS > 1) {  // the partials, then the region is the conv items'
      __syncthreads();
      rb_wgrad_sum<R>(Pw, slab_row);
      __syncthreads();
    }
  }
  RB_MARK(3);
  rb_conv_items<R, true>(A, G, Pc);
  __syncthreads();
  RB_MARK(4);
  double s[1][R::CPW][R::PPL];
#pragma unroll
  for (int u = 0; u < R::CPW; ++u)
#pragma unroll
    for (int q = 0; q < R::PPL; ++q) {
      s[0][u][q] = 0.0;
      dxout[u][q] = 0.f;
      if (!el.ok(u, q)) continue;
      const float av = a1[u], inv_a = 1.0f / av;
      const float xv = vx[u][q];
      const float gs = rb_conv_at<R>(Pc, el, u, q);  // d loss / d s1
      float sn, cs;
      sincosf(av * xv, &sn, &cs);
      const float t = 2.0f * sn * cs;
      // snake_bwd_kernel, plus the identity skip's gradient
      dxout[u][q] = (gs + gs * inv_a * t * av) + vy[u][q];
      a.dx[el.gi(img0, u, q)] = dxout[u][q];
      s[0][u][q] = (double)(gs * inv_a * t * xv) - (double)(gs * (sn * sn) * inv_a * inv_a);
    }
  RB_MARK(5);
  // this image's da1 term per channel -> its row of the da1 slab
  rb_slab_row_sums<R>(s, 0, el, b, a.slabda);
  RB_MARK(6);
}

template <class R>
__global__ __launch_bounds__(RB_T) void rb_bwd1_kernel(RBArgs a) {
  extern __shared__ double rb_smem[];
  RBRegs<R> dx;
  rb_bwd1_body<R>(a, rb_smem, dx);
}

// bwd1 of ResBlock 2 and bwd2 of ResBlock 1 (its output gradient = ResBlock 2's input
// gradient) in one launch
template <class R>
__global__ __launch_bounds__(RB_T) void rb_bwd12_kernel(RBArgs a2, RBArgs a1) {
  extern __shared__ double rb_smem[];
  RBRegs<R> d;
  rb_bwd1_body<R>(a2, rb_smem, d);
  __syncthreads();  // LDS reused
  rb_bwd2_body<R, true>(a1, rb_smem, d);
}

// ---------------------------------------------------------------- host side
template <class R>
static size_t rb_lds(int kind) {
  const size_t PL = R::PLANE, PA = R::PANEL, PC = R::PARTC;
  switch (kind) {
    case 0: return 4 * (PL + PA + PC);               // fwd1
    case 1: return 4 * (PL + PA + PC);               // fwd2
    case 2: return 4 * (2 * PL + PA + PC);           // eval
    default: return 4 * (2 * PL + PA + R::PARTCW + R::CONSTP);  // bwd2, bwd1
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
  static const char* const names[5] = {"rb_fwd1", "rb_fwd2", "rb_eval", "rb_bwd2", "rb_bwd1"};
  TVQ_PLAN("%s C%d W%d B%d", names[kind < 4 ? kind : 4], R::C, R::W, a.B);
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

// a fused pair of consecutive ResBlocks' kernels: kind 0 = rb_fwd21 (first = block 1,
// second = block 2), kind 1 = rb_bwd12 (first = block 2, second = block 1)
template <class R>
static void rb_launch_pair(int kind, const RBArgs& first, const RBArgs& second, hipStream_t st) {
  const size_t lf = rb_lds<R>(0) > rb_lds<R>(1) ? rb_lds<R>(0) : rb_lds<R>(1);
  const size_t lb = rb_lds<R>(3) > rb_lds<R>(4) ? rb_lds<R>(3) : rb_lds<R>(4);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&rb_fwd21_kernel<R>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lf);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&rb_bwd12_kernel<R>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lb);
    attr = true;
  }
  const dim3 grid(first.B), block(RB_T);
  TVQ_PLAN("%s C%d W%d B%d", kind == 0 ? "rb_fwd21" : "rb_bwd12", R::C, R::W, first.B);
  if (kind == 0)
    hipLaunchKernelGGL(rb_fwd21_kernel<R>, grid, block, lf, st, first, second);
  else
    hipLaunchKernelGGL(rb_bwd12_kernel<R>, grid, block, lb, st, first, second);
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

static bool rb_dispatch_pair(int C, int W, int kind, const RBArgs& first,
                             const RBArgs& second, hipStream_t st) {
#define RB_CASE(CC, WW)                                    \
  if (C == CC && W == WW) {                                \
    rb_launch_pair<RB<CC, WW>>(kind, first, second, st);   \
    return true;                                           \
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
  size_t part, slabda, slabda2, slab2, slab1, du, total;
};
static RBWs rb_ws(int64_t B, int64_t C, int64_t W) {
  RBWs w;
  const int64_t kc = 9 * C + 1;
  const size_t slab = (size_t)(B * C * kc + reduce_rows_scratch(B, C * kc));
  w.part = 0;
  const size_t slabd = (size_t)(B * C + reduce_rows_scratch(B, C)) * 4;
  w.slabda = w.part + rb_align((size_t)B * C * 2 * 8);
  w.slabda2 = w.slabda + rb_align(slabd);
  w.slab2 = w.slabda2 + rb_align(slabd);
  w.slab1 = w.slab2 + rb_align(slab * 4);
  w.du = w.slab1 + rb_align(slab * 4);
  w.total = w.du + rb_align((size_t)B * C * 3 * W * 4);
  return w;
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// the external-weight-gradient form (RB::WEXT) for this shape and batch
static bool rb_wext(int64_t B, int64_t C, int64_t W) {
  if (!(C == 32 && W == 16) || !conv_wgrad_w16_fits(B, C, C)) return false;
  // the g / s planes and the small slab fit in the per-image slab region they replace
  const int64_t pl = B * C * 3 * W;
  return 2 * pl + conv_wgrad_w16_slab_floats(B, C, C) <= B * C * (9 * C + 1);
}

// the LF band's 64-channel ResBlock on (B, 64, 3, 8) (tvq_resblock_w8.hip)
bool w8_supported(int64_t B, int64_t C, int64_t H, int64_t W);
int64_t w8_workspace(int64_t B);
int64_t w8_saved_floats(int64_t B);
int w8_train_fwd(const float* x, int64_t B, const float* a1, const float* w1, const float* b1,
                 const float* bn_w, const float* bn_b, float* running_mean, float* running_var,
                 int64_t* nbt, float momentum, float eps, const float* a2, const float* w2,
                 const float* b2, float drop_p, const int64_t* seed_ptr, uint64_t offset,
                 float* saved, float* y, float* save, void* workspace, hipStream_t st);
int w8_eval_fwd(const float* x, int64_t B, const float* a1, const float* w1, const float* b1,
                const float* bn_w, const float* bn_b, const float* running_mean,
                const float* running_var, float eps, const float* a2, const float* w2,
                const float* b2, float* y, hipStream_t st);
int w8_bwd(const float* dy, const float* x, const float* saved, int64_t B, const float* a1,
           const float* w1, const float* bn_w, const float* save, const float* a2,
           const float* w2, float drop_p, const int64_t* seed_ptr, uint64_t offset, float* dx,
           float* da1, float* dw1, float* db1, float* dbn_w, float* dbn_b, float* da2, float* dw2,
           float* db2, int64_t accumulate, void* workspace, hipStream_t st);
int w8_pair_train_fwd(const float* x, int64_t B, const float* const* p1, const float* const* p2,
                      float* const* rs1, float* const* rs2, int64_t* nbt1, int64_t* nbt2,
                      float momentum, float eps, float drop_p, const int64_t* seed_ptr,
                      uint64_t off1, uint64_t off2, float* saved1, float* y1, float* save1,
                      float* saved2, float* y2, float* save2, void* ws1, void* ws2,
                      hipStream_t st);
int w8_pair_bwd(const float* dy, const float* x, int64_t B, const float* const* q1,
                const float* const* q2, const float* saved1, const float* y1,
                const float* saved2, float drop_p, const int64_t* seed_ptr, uint64_t off1,
                uint64_t off2, float* dx, float* dy1, float* const* g1, float* const* g2,
                int64_t accumulate, void* ws1, void* ws2, hipStream_t st);

static RBArgs rb_fwd_args(const float* x, int64_t B, int64_t C, int64_t W, const float* a1,
                          const float* w1, const float* b1, const float* bn_w, const float* bn_b,
                          float* running_mean, float* running_var, int64_t* nbt, float momentum,
                          float eps, const float* a2, const float* w2, const float* b2,
                          float drop_p, const int64_t* seed_ptr, uint64_t offset, float* h,
                          float* y, float* save, void* workspace) {
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
           nbt, save, save + C, save + 2 * C, save + 3 * C};
  return a;
}

static RBArgs rb_bwd_args(const float* dy, const float* x, const float* h, int64_t B, int64_t C,
                          int64_t W, const float* a1, const float* w1, const float* bn_w,
                          const float* save, const float* a2, const float* w2, float drop_p,
                          const int64_t* seed_ptr, uint64_t offset, float* dx, float* dbn_w,
                          float* dbn_b, int64_t accumulate, void* workspace) {
  const RBWs w = rb_ws(B, C, W);
  char* ws = (char*)workspace;
  RBArgs a = {};
  a.x = x; a.h = h; a.dy = dy; a.a1 = a1; a.w1 = w1; a.a2 = a2; a.w2 = w2; a.bn_w = bn_w;
  a.save = save;
  a.slabda2 = (float*)(ws + w.slabda2);
  a.du = (float*)(ws + w.du); a.dx = dx;
  a.slab1 = (float*)(ws + w.slab1); a.slab2 = (float*)(ws + w.slab2);
  a.slabda = (float*)(ws + w.slabda);
  a.part = (double*)(ws + w.part);
  if (rb_wext(B, C, W)) {  // the planes and small slabs in the big slabs' regions
    const int64_t pl = B * C * 3 * W;
    a.wext = 1;
    a.gp2 = a.slab2; a.sp2 = a.slab2 + pl; a.wsl2 = a.slab2 + 2 * pl;
    a.gp1 = a.slab1; a.sp1 = a.slab1 + pl; a.wsl1 = a.slab1 + 2 * pl;
  }
  a.B = (int)B; a.accumulate = (int)accumulate;
  a.drop_p = drop_p;
  a.drop_scale = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
  a.seed_ptr = seed_ptr; a.offset = offset;
  a.invN = 1.0f / (float)(B * 3 * W);
  a.bfin = {(int)C, (int)B, nullptr, dbn_w, dbn_b, nullptr, (int)accumulate};
  return a;
}

// the weight gradients out of the backward kernels' per-image slabs (deferred in a
// wgrad_deferred region)
static void rb_bwd_finish(const RBArgs& a, int64_t C, float* da1, float* dw1, float* db1,
                          float* da2, float* dw2, float* db2, hipStream_t st) {
  const int64_t kc = 9 * C + 1;
  if (a.wext) {  // both convs' weight gradients from the planes, one launch
    const float* x[2] = {a.sp2, a.sp1};
    const float* dy[2] = {a.gp2, a.gp1};
    float* ws[2] = {a.wsl2, a.wsl1};
    float* dw[2] = {dw2, dw1};
    float* db[2] = {db2, db1};
    conv_wgrad_w16_multi(2, x, dy, ws, dw, db, a.B, C, C, a.accumulate, st);
  } else {
    conv_wgrad_finish(a.slab2, a.B, C, kc, dw2, db2, a.accumulate, st);
    conv_wgrad_finish(a.slab1, a.B, C, kc, dw1, db1, a.accumulate, st);
  }
  conv_wgrad_finish(a.slabda, a.B, C, 1, da1, nullptr, a.accumulate, st);
  conv_wgrad_finish(a.slabda2, a.B, C, 1, da2, nullptr, a.accumulate, st);
}

// a pair's four weight gradients in one launch when both blocks take the planes
static void rb_bwd_finish_pair(const RBArgs& b2, const RBArgs& b1, int64_t C, float* const* g2,
                               float* const* g1, hipStream_t st) {
  // g = {da1, dw1, db1, dbn_w, dbn_b, da2, dw2, db2}
  if (!(b2.wext && b1.wext)) {
    rb_bwd_finish(b2, C, g2[0], g2[1], g2[2], g2[5], g2[6], g2[7], st);
    rb_bwd_finish(b1, C, g1[0], g1[1], g1[2], g1[5], g1[6], g1[7], st);
    return;
  }
  const float* x[4] = {b2.sp2, b2.sp1, b1.sp2, b1.sp1};
  const float* dy[4] = {b2.gp2, b2.gp1, b1.gp2, b1.gp1};
  float* ws[4] = {b2.wsl2, b2.wsl1, b1.wsl2, b1.wsl1};
  float* dw[4] = {g2[6], g2[1], g1[6], g1[1]};
  float* db[4] = {g2[7], g2[2], g1[7], g1[2]};
  conv_wgrad_w16_multi(4, x, dy, ws, dw, db, b2.B, C, C, b2.accumulate, st);
  conv_wgrad_finish(b2.slabda, b2.B, C, 1, g2[0], nullptr, b2.accumulate, st);
  conv_wgrad_finish(b2.slabda2, b2.B, C, 1, g2[5], nullptr, b2.accumulate, st);
  conv_wgrad_finish(b1.slabda, b1.B, C, 1, g1[0], nullptr, b1.accumulate, st);
  conv_wgrad_finish(b1.slabda2, b1.B, C, 1, g1[5], nullptr, b1.accumulate, st);
}

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
  if (w8_supported(B, C, H, W)) return w8_workspace(B);
  if (!rb_supported(B, C, H, W)) return -1;
  return (int64_t)rb_ws(B, C, W).total;
}

extern "C" int64_t tvq_resblock_saved_floats(int64_t B, int64_t C, int64_t H, int64_t W) {
  if (w8_supported(B, C, H, W)) return w8_saved_floats(B);
  if (!rb_supported(B, C, H, W)) return -1;
  return B * C * H * W;
}

extern "C" int tvq_resblock_train_fwd(const float* x, int64_t B, int64_t C, int64_t H, int64_t W,
                                      const float* a1, const float* w1, const float* b1,
                                      const float* bn_w, const float* bn_b, float* running_mean,
                                      float* running_var, int64_t* num_batches_tracked,
                                      float momentum, float eps, const float* a2, const float* w2,
                                      const float* b2, float drop_p, const int64_t* seed_ptr,
                                      uint64_t offset, float* h, float* y, float* save,
                                      void* workspace, tvq_stream_t stream) {
  const bool w8 = w8_supported(B, C, H, W);
  TVQ_CHECK_ARG(w8 || rb_supported(B, C, H, W), "tvq_resblock_train_fwd: unsupported shape");
  TVQ_CHECK_ARG(x && a1 && w1 && a2 && w2 && h && y && save && workspace && running_mean &&
                    running_var && aligned16(x) && aligned16(h),
                "tvq_resblock_train_fwd: bad arguments");
  TVQ_CHECK_ARG(drop_p >= 0.f && drop_p < 1.f && (drop_p == 0.f || seed_ptr),
                "tvq_resblock_train_fwd: bad dropout");
  hipStream_t st = (hipStream_t)stream;
  if (w8)
    return w8_train_fwd(x, B, a1, w1, b1, bn_w, bn_b, running_mean, running_var,
                        num_batches_tracked, momentum, eps, a2, w2, b2, drop_p, seed_ptr, offset, h,
                        y, save, workspace, st);
  const RBArgs a = rb_fwd_args(x, B, C, W, a1, w1, b1, bn_w, bn_b, running_mean, running_var,
                               num_batches_tracked, momentum, eps, a2, w2, b2, drop_p, seed_ptr,
                               offset, h, y, save, workspace);
  rb_dispatch((int)C, (int)W, 0, &a, st, nullptr);
  rb_dispatch((int)C, (int)W, 1, &a, st, nullptr);
  return launch_status("tvq_resblock_train_fwd");
}

extern "C" int tvq_resblock_eval_fwd(const float* x, int64_t B, int64_t C, int64_t H, int64_t W,
                                     const float* a1, const float* w1, const float* b1,
                                     const float* bn_w, const float* bn_b,
                                     const float* running_mean, const float* running_var,
                                     float eps, const float* a2, const float* w2, const float* b2,
                                     float* y, tvq_stream_t stream) {
  const bool w8 = w8_supported(B, C, H, W);
  TVQ_CHECK_ARG(w8 || rb_supported(B, C, H, W), "tvq_resblock_eval_fwd: unsupported shape");
  TVQ_CHECK_ARG(x && a1 && w1 && a2 && w2 && y && running_mean && running_var && aligned16(x),
                "tvq_resblock_eval_fwd: bad arguments");
  if (w8)
    return w8_eval_fwd(x, B, a1, w1, b1, bn_w, bn_b, running_mean, running_var, eps, a2, w2, b2,
                       y, (hipStream_t)stream);
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
  const bool w8 = w8_supported(B, C, H, W);
  TVQ_CHECK_ARG(w8 || rb_supported(B, C, H, W), "tvq_resblock_bwd: unsupported shape");
  TVQ_CHECK_ARG(dy && x && h && a1 && w1 && save && a2 && w2 && dx && da1 && dw1 && db1 && da2 &&
                    dw2 && db2 && workspace && aligned16(dy) && aligned16(x) && aligned16(h),
                "tvq_resblock_bwd: bad arguments");
  TVQ_CHECK_ARG(drop_p >= 0.f && drop_p < 1.f && (drop_p == 0.f || seed_ptr),
                "tvq_resblock_bwd: bad dropout");
  hipStream_t st = (hipStream_t)stream;
  if (w8)
    return w8_bwd(dy, x, h, B, a1, w1, bn_w, save, a2, w2, drop_p, seed_ptr, offset, dx, da1, dw1,
                  db1, dbn_w, dbn_b, da2, dw2, db2, accumulate, workspace, st);
  const RBArgs a = rb_bwd_args(dy, x, h, B, C, W, a1, w1, bn_w, save, a2, w2, drop_p, seed_ptr,
                               offset, dx, dbn_w, dbn_b, accumulate, workspace);
  rb_dispatch((int)C, (int)W, 3, &a, st, nullptr);
  rb_dispatch((int)C, (int)W, 4, &a, st, nullptr);
  rb_bwd_finish(a, C, da1, dw1, db1, da2, dw2, db2, st);
  return launch_status("tvq_resblock_bwd");
}

extern "C" int tvq_resblock_pair_supported(int64_t B, int64_t C, int64_t H, int64_t W) {
  return w8_supported(B, C, H, W) || rb_supported(B, C, H, W);
}

extern "C" int tvq_resblock_pair_train_fwd(const float* x, int64_t B, int64_t C, int64_t H,
                                           int64_t W, const float* const* p1,
                                           const float* const* p2, float* const* rs1,
                                           float* const* rs2, int64_t* nbt1, int64_t* nbt2,
                                           float momentum, float eps, float drop_p,
                                           const int64_t* seed_ptr, uint64_t offset1,
                                           uint64_t offset2, float* h1, float* y1, float* save1,
                                           float* h2, float* y2, float* save2, void* ws1,
                                           void* ws2, tvq_stream_t stream) {
  TVQ_CHECK_ARG(tvq_resblock_pair_supported(B, C, H, W),
                "tvq_resblock_pair_train_fwd: unsupported shape");
  TVQ_CHECK_ARG(x && p1 && p2 && rs1 && rs2 && h1 && y1 && save1 && h2 && y2 && save2 && ws1 &&
                    ws2 && aligned16(x) && aligned16(h1) && aligned16(h2) && aligned16(y1),
                "tvq_resblock_pair_train_fwd: bad arguments");
  for (int i = 0; i < 8; ++i)
    TVQ_CHECK_ARG((p1[i] && p2[i]) || i == 2 || i == 3 || i == 4 || i == 7,
                  "tvq_resblock_pair_train_fwd: missing parameter");
  TVQ_CHECK_ARG(rs1[0] && rs1[1] && rs2[0] && rs2[1],
                "tvq_resblock_pair_train_fwd: missing running statistics");
  TVQ_CHECK_ARG(drop_p >= 0.f && drop_p < 1.f && (drop_p == 0.f || seed_ptr),
                "tvq_resblock_pair_train_fwd: bad dropout");
  hipStream_t st = (hipStream_t)stream;
  if (w8_supported(B, C, H, W))
    return w8_pair_train_fwd(x, B, p1, p2, rs1, rs2, nbt1, nbt2, momentum, eps, drop_p, seed_ptr,
                             offset1, offset2, h1, y1, save1, h2, y2, save2, ws1, ws2, st);
  // p = {a1, w1, b1, bn_w, bn_b, a2, w2, b2}, rs = {running_mean, running_var}
  const RBArgs a1 = rb_fwd_args(x, B, C, W, p1[0], p1[1], p1[2], p1[3], p1[4], rs1[0], rs1[1],
                                nbt1, momentum, eps, p1[5], p1[6], p1[7], drop_p, seed_ptr,
                                offset1, h1, y1, save1, ws1);
  const RBArgs a2 = rb_fwd_args(y1, B, C, W, p2[0], p2[1], p2[2], p2[3], p2[4], rs2[0], rs2[1],
                                nbt2, momentum, eps, p2[5], p2[6], p2[7], drop_p, seed_ptr,
                                offset2, h2, y2, save2, ws2);
  rb_dispatch((int)C, (int)W, 0, &a1, st, nullptr);
  rb_dispatch_pair((int)C, (int)W, 0, a1, a2, st);
  rb_dispatch((int)C, (int)W, 1, &a2, st, nullptr);
  return launch_status("tvq_resblock_pair_train_fwd");
}

extern "C" int tvq_resblock_pair_bwd(const float* dy, const float* x, int64_t B, int64_t C,
                                     int64_t H, int64_t W, const float* const* q1,
                                     const float* const* q2, const float* h1, const float* y1,
                                     const float* h2, float drop_p, const int64_t* seed_ptr,
                                     uint64_t offset1, uint64_t offset2, float* dx, float* dy1,
                                     float* const* g1, float* const* g2, int64_t accumulate,
                                     void* ws1, void* ws2, tvq_stream_t stream) {
  TVQ_CHECK_ARG(tvq_resblock_pair_supported(B, C, H, W), "tvq_resblock_pair_bwd: unsupported shape");
  TVQ_CHECK_ARG(dy && x && q1 && q2 && h1 && y1 && h2 && dx && dy1 && g1 && g2 && ws1 && ws2 &&
                    aligned16(dy) && aligned16(x) && aligned16(h1) && aligned16(h2) &&
                    aligned16(y1) && aligned16(dy1),
                "tvq_resblock_pair_bwd: bad arguments");
  for (int i = 0; i < 6; ++i)
    TVQ_CHECK_ARG((q1[i] && q2[i]) || i == 2, "tvq_resblock_pair_bwd: missing parameter");
  for (int i = 0; i < 8; ++i)
    TVQ_CHECK_ARG((g1[i] && g2[i]) || i == 3 || i == 4, "tvq_resblock_pair_bwd: missing gradient");
  TVQ_CHECK_ARG(drop_p >= 0.f && drop_p < 1.f && (drop_p == 0.f || seed_ptr),
                "tvq_resblock_pair_bwd: bad dropout");
  hipStream_t st = (hipStream_t)stream;
  if (w8_supported(B, C, H, W))
    return w8_pair_bwd(dy, x, B, q1, q2, h1, y1, h2, drop_p, seed_ptr, offset1, offset2, dx, dy1,
                       g1, g2, accumulate, ws1, ws2, st);
  // q = {a1, w1, bn_w, save, a2, w2}, g = {da1, dw1, db1, dbn_w, dbn_b, da2, dw2, db2}
  const RBArgs b2 = rb_bwd_args(dy, y1, h2, B, C, W, q2[0], q2[1], q2[2], q2[3], q2[4], q2[5],
                                drop_p, seed_ptr, offset2, dy1, g2[3], g2[4], accumulate, ws2);
  const RBArgs b1 = rb_bwd_args(dy1, x, h1, B, C, W, q1[0], q1[1], q1[2], q1[3], q1[4], q1[5],
                                drop_p, seed_ptr, offset1, dx, g1[3], g1[4], accumulate, ws1);
  rb_dispatch((int)C, (int)W, 3, &b2, st, nullptr);
  rb_dispatch_pair((int)C, (int)W, 1, b2, b1, st);
  rb_dispatch((int)C, (int)W, 4, &b1, st, nullptr);
  rb_bwd_finish_pair(b2, b1, C, g2, g1, st);
  return launch_status("tvq_resblock_pair_bwd");
}

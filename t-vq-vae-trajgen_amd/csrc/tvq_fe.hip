// FidelityEnhancer (models/fidelity_enhancer.py) eval forward on gfx950: the Unet1D's
// 1-D convs (weight-standardised or plain, zero/replicate padding, nearest-x2 input),
// GroupNorm+Snake, channel LayerNorm, linear and full attention, and the
// interpolate+concat skips.  (B, C, L) fp32 row-major throughout; every kernel reads its
// input once from HBM/L2 and writes its output once.  No atomics: results are
// deterministic and independent of the launch order.
#include "tvq_common.h"

namespace tvq {
namespace {

constexpr int FE_TILE = 64;  // output positions per conv block (one per lane)
constexpr int FE_COB = 16;   // output channels per conv block (4 per wave)

// WeightStandardizedConv2d.forward (fidelity_enhancer.py:102-106): per output channel o,
// (w - mean_o) * rsqrt(var_o + eps), var biased.  One block per o; n = Ci * K.
__global__ __launch_bounds__(256) void ws_kernel(const float* __restrict__ w, int n, float eps,
                                                 float* __restrict__ out) {
  __shared__ float red[4];
  const float* row = w + (int64_t)blockIdx.x * n;
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += row[i];
  const float mean = block_sum(s, red) / (float)n;
  float q = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float d = row[i] - mean;
    q += d * d;
  }
  const float rstd = rsqrtf(block_sum(q, red) / (float)n + eps);
  for (int i = threadIdx.x; i < n; i += blockDim.x)
    out[(int64_t)blockIdx.x * n + i] = (row[i] - mean) * rstd;
}

// y[b, o, l] = bias[o] + sum_{c,k} w[o, c, k] * xin[b, c, l*S + k - P] (+ residual)
// xin = x, or x nearest-upsampled by 2 (up2); out-of-range taps read 0 or the clamped
// edge sample (replicate).  Block: one batch item, FE_COB output channels, FE_TILE
// positions; the input span for the tile is staged once in LDS (all Ci rows) and each
// wave walks 4 output channels whose weights are wave-uniform (scalar loads).
__global__ __launch_bounds__(256) void conv1d_kernel(const float* __restrict__ x, int Ci, int Lin,
                                                     const float* __restrict__ w,
                                                     const float* __restrict__ bias, int Co,
                                                     int K, int S, int P, int up2, int replicate,
                                                     const float* __restrict__ res,
                                                     float* __restrict__ y, int Lout, int span) {
  extern __shared__ float tile[];  // Ci x span
  const int b = blockIdx.z, o0 = blockIdx.y * FE_COB, l0 = blockIdx.x * FE_TILE;
  const int Leff = up2 ? 2 * Lin : Lin;
  const float* xb = x + (int64_t)b * Ci * Lin;
  const int start = l0 * S - P;
  for (int i = threadIdx.x; i < Ci * span; i += blockDim.x) {
    const int c = i / span, j = i - c * span;
    int p = start + j;
    float v = 0.f;
    if (replicate) p = min(max(p, 0), Leff - 1);
    if (p >= 0 && p < Leff) v = xb[(int64_t)c * Lin + (up2 ? (p >> 1) : p)];
    tile[i] = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l = l0 + lane;
  float acc[FE_COB / 4];
  int oc[FE_COB / 4];
#pragma unroll
  for (int j = 0; j < FE_COB / 4; ++j) {
    oc[j] = min(o0 + wv + 4 * j, Co - 1);
    acc[j] = bias ? bias[oc[j]] : 0.f;
  }
  const float* tl = tile + lane * S;
  for (int c = 0; c < Ci; ++c) {
    const float* tc = tl + c * span;
    for (int k = 0; k < K; ++k) {
      const float v = tc[k];
#pragma unroll
      for (int j = 0; j < FE_COB / 4; ++j) acc[j] = fmaf(w[((int64_t)oc[j] * Ci + c) * K + k], v, acc[j]);
    }
  }
  if (l >= Lout) return;
#pragma unroll
  for (int j = 0; j < FE_COB / 4; ++j) {
    const int o = o0 + wv + 4 * j;
    if (o >= Co) continue;
    const int64_t at = ((int64_t)b * Co + o) * Lout + l;
    y[at] = acc[j] + (res ? res[at] : 0.f);
  }
}

// Register-blocked conv1d (the FidelityEnhancer's shapes: Ci <= 96, K <= 7, S <= 2).
// Block tile TC = 4 TCY output channels x TP = RP TPX positions; each thread owns 4
// channels x RP positions (positions tx + i TPX, so LDS reads of the input are consecutive
// across lanes).  Input channels are streamed in chunks of 16: the chunk's input span and
// its weights (as [c][k][co], read as float4) are staged in LDS, then every (c, k) does
// 16 FMAs for 4 + 1 LDS reads.  Sum order per output: c ascending, then k (as
// conv1d_kernel).
template <int TPX, int TCY, int RP, int KT>
__global__ __launch_bounds__(256) void conv1d_rb_kernel(const float* __restrict__ x, int Ci, int Lin,
                                                        const float* __restrict__ w,
                                                        const float* __restrict__ bias, int Co,
                                                        int K_, int S, int P, int up2, int replicate,
                                                        const float* __restrict__ res,
                                                        float* __restrict__ y, int Lout, int span) {
  constexpr int RC = 4, CC = 16, TP = TPX * RP, TC = TCY * RC;
  const int K = KT > 0 ? KT : K_;  // KT: taps known at compile time (k loop unrolled)
  extern __shared__ float sm[];
  float* xs = sm;                // CC x span
  float* wsm = sm + CC * span;   // CC x K x TC
  const int b = blockIdx.z, o0 = blockIdx.y * TC, l0 = blockIdx.x * TP;
  const int tx = threadIdx.x % TPX, ty = threadIdx.x / TPX;
  const int Leff = up2 ? 2 * Lin : Lin;
  const float* xb = x + (int64_t)b * Ci * Lin;
  const int start = l0 * S - P;
  float acc[RC][RP];
#pragma unroll
  for (int r = 0; r < RC; ++r) {
    const int co = o0 + ty * RC + r;
    const float bv = (bias && co < Co) ? bias[co] : 0.f;
#pragma unroll
    for (int i = 0; i < RP; ++i) acc[r][i] = bv;
  }
  for (int c0 = 0; c0 < Ci; c0 += CC) {
    const int cc = min(CC, Ci - c0);
    __syncthreads();
    {  // x span rows of the chunk; (c, j) advanced incrementally (one division per thread)
      int c = threadIdx.x / span, j = threadIdx.x - (threadIdx.x / span) * span;
      for (int i = threadIdx.x; i < cc * span; i += 256) {
        int p = start + j;
        if (replicate) p = min(max(p, 0), Leff - 1);
        xs[i] = (p >= 0 && p < Leff) ? xb[(int64_t)(c0 + c) * Lin + (up2 ? (p >> 1) : p)] : 0.f;
        j += 256;
        while (j >= span) j -= span, ++c;
      }
    }
    {  // weights as [c k][o]: row ck of output channel o is w[o][c0 K + ck]
      const int o = threadIdx.x % TC;
      const bool ok = o0 + o < Co;
      const float* wo = w + ((int64_t)(o0 + o) * Ci + c0) * K;
      for (int ck = threadIdx.x / TC; ck < cc * K; ck += 256 / TC) wsm[ck * TC + o] = ok ? wo[ck] : 0.f;
    }
    __syncthreads();
    for (int c = 0; c < cc; ++c) {
      const float* xr = xs + c * span + tx * S;
      const float* wr = wsm + c * K * TC + ty * RC;
#pragma unroll
      for (int k = 0; k < (KT > 0 ? KT : K); ++k) {
        const floatx4 wv = *reinterpret_cast<const floatx4*>(wr + k * TC);
        float xv[RP];
#pragma unroll
        for (int i = 0; i < RP; ++i) xv[i] = xr[i * TPX * S + k];
#pragma unroll
        for (int r = 0; r < RC; ++r)
#pragma unroll
          for (int i = 0; i < RP; ++i) acc[r][i] = fmaf(wv[r], xv[i], acc[r][i]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < RC; ++r) {
    const int co = o0 + ty * RC + r;
    if (co >= Co) continue;
#pragma unroll
    for (int i = 0; i < RP; ++i) {
      const int l = l0 + tx + i * TPX;
      if (l >= Lout) continue;
      const int64_t at = ((int64_t)b * Co + co) * Lout + l;
      y[at] = acc[r][i] + (res ? res[at] : 0.f);
    }
  }
}

// nn.GroupNorm(G, C) (eps) then SnakeActivation (train_utils.py:446-448), + residual:
// Block.forward + ResnetBlock's `h + res_conv(x)` (fidelity_enhancer.py:193-231).  One
// block per (b, g); the group's (C/G) x L values are contiguous.
template <int PT>  // PT > 0: the group (<= 256 PT values) is held in registers, one HBM read
__global__ __launch_bounds__(256) void gn_snake_kernel(const float* __restrict__ x, int C, int L,
                                                       int G, const float* __restrict__ gamma,
                                                       const float* __restrict__ beta,
                                                       const float* __restrict__ a, float eps,
                                                       const float* __restrict__ res,
                                                       float* __restrict__ y) {
  __shared__ float red[4];
  const int cg = C / G, n = cg * L;
  const int64_t base = (int64_t)blockIdx.x * n;  // blockIdx.x = b * G + g
  const int c0 = (blockIdx.x % G) * cg;
  float v[PT > 0 ? PT : 1];
  float s = 0.f;
  if (PT > 0) {
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int e = threadIdx.x + i * 256;
      v[i] = e < n ? x[base + e] : 0.f;
      s += v[i];
    }
  } else {
    for (int i = threadIdx.x; i < n; i += blockDim.x) s += x[base + i];
  }
  const float mean = block_sum(s, red) / (float)n;
  float q = 0.f;
  if (PT > 0) {
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const float d = v[i] - mean;
      q += threadIdx.x + i * 256 < n ? d * d : 0.f;
    }
  } else {
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const float d = x[base + i] - mean;
      q += d * d;
    }
  }
  const float rstd = rsqrtf(block_sum(q, red) / (float)n + eps);
  auto out = [&](int i, float xv) {
    const int c = c0 + i / L;
    const float sc = rstd * gamma[c];
    float t = (xv - mean) * sc + beta[c];
    const float ac = a[c];
    t = snake_f(t, ac, 1.0f / ac);
    y[base + i] = t + (res ? res[base + i] : 0.f);
  };
  if (PT > 0) {
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int e = threadIdx.x + i * 256;
      if (e < n) out(e, v[i]);
    }
  } else {
    for (int i = threadIdx.x; i < n; i += blockDim.x) out(i, x[base + i]);
  }
}

// LayerNorm over channels, gamma only (fidelity_enhancer.py:119-127), + residual.
// One thread per (b, l); the channel loop is coalesced across l.
template <int CT>  // CT > 0: C == CT, the column held in registers (one HBM read)
__global__ __launch_bounds__(256) void chan_ln_kernel(const float* __restrict__ x, int B, int C,
                                                      int L, const float* __restrict__ g,
                                                      float eps, const float* __restrict__ res,
                                                      float* __restrict__ y) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * L) return;
  const int b = t / L, l = t - b * L;
  const float* xb = x + (int64_t)b * C * L + l;
  float v[CT > 0 ? CT : 1];
  float s = 0.f;
  if (CT > 0) {
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      v[c] = xb[(int64_t)c * L];
      s += v[c];
    }
  } else {
    for (int c = 0; c < C; ++c) s += xb[(int64_t)c * L];
  }
  const float mean = s / (float)C;
  float q = 0.f;
  if (CT > 0) {
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      const float d = v[c] - mean;
      q += d * d;
    }
  } else {
    for (int c = 0; c < C; ++c) {
      const float d = xb[(int64_t)c * L] - mean;
      q += d * d;
    }
  }
  const float rstd = rsqrtf(q / (float)C + eps);
  const int64_t at0 = (int64_t)b * C * L + l;
  if (CT > 0) {
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      const int64_t at = at0 + (int64_t)c * L;
      y[at] = (v[c] - mean) * rstd * g[c] + (res ? res[at] : 0.f);
    }
  } else {
    for (int c = 0; c < C; ++c) {
      const int64_t at = at0 + (int64_t)c * L;
      y[at] = (x[at] - mean) * rstd * g[c] + (res ? res[at] : 0.f);
    }
  }
}

// LinearAttention core (fidelity_enhancer.py:245-260) for one (b, h), dh = 32:
//   k <- softmax over n, q <- softmax over d * dh^-1/2,
//   ctx[d, e] = sum_n k[d, n] v[e, n],  out[e, n] = sum_d ctx[d, e] q[d, n].
// qkv (B, 3 H dh, n) as to_qkv writes it (chunk order q, k, v; head-major channels).
constexpr int FE_DH = 32;
constexpr int CTX_LD = FE_DH + 4;
// dst[r][j] (row stride ld) = sum_c wl[c][row0 + r] * xs[c][j], r < NR, j < n, c ascending
// from 0 (the order conv1d_rb_kernel sums a bias-free 1x1 conv in: bitwise equal).  Each
// thread owns 4 rows x 4 columns: per c one float4 weight read + 4 input reads for 16 FMAs.
template <int NR>
__device__ __forceinline__ void la_rows_matmul(const float* __restrict__ wl, int row0,
                                               const float* __restrict__ xs, int C, int n,
                                               float* __restrict__ dst, int ld) {
  constexpr int TCOL = 256 / (NR / 4);  // threads along columns
  const int tr = threadIdx.x / TCOL, tc = threadIdx.x % TCOL;
  for (int jb = 0; jb < n; jb += 4 * TCOL) {
    float acc[4][4] = {};
    for (int c = 0; c < C; ++c) {
      const floatx4 w4 = *reinterpret_cast<const floatx4*>(wl + c * 96 + row0 + tr * 4);
      float xv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = jb + tc + i * TCOL;
        xv[i] = j < n ? xs[c * n + j] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[r][i] = fmaf(w4[r], xv[i], acc[r][i]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = jb + tc + i * TCOL;
        if (j < n) dst[(tr * 4 + r) * ld + j] = acc[r][i];
      }
  }
}

// FUSED: `qkv` is the block input x (B, C, n) and wqkv the to_qkv weight (3 H dh, C): the
// block computes its head's 96 q/k/v rows from x and the weights staged in LDS, so the
// (B, 3 H dh, n) qkv tensor never goes through HBM.
template <bool FUSED>
__global__ __launch_bounds__(256) void linear_attn_kernel(const float* __restrict__ qkv,
                                                          const float* __restrict__ wqkv, int C,
                                                          int H, int n, float scale,
                                                          float* __restrict__ out) {
  extern __shared__ float sm[];
  const int ld = n + 1;  // padded row stride: the context loop reads v[e][*] across lanes
  float* ks = sm;
  float* vs = sm + FE_DH * ld;
  // the j-quarter partials of ctx overlay k/v once both are consumed
  const int kv = max(2 * FE_DH * ld, 4 * FE_DH * CTX_LD);
  float* part = sm;
  float* ctx = sm + kv;  // FE_DH x CTX_LD (float4-aligned rows)
  const int b = blockIdx.x / H, h = blockIdx.x - b * H;
  const int HD = H * FE_DH;
  const float* q = qkv + ((int64_t)b * 3 * HD + h * FE_DH) * n;
  float* xs = ctx + FE_DH * CTX_LD;  // FUSED: x[b] (C x n), then wl (C x 96)
  float* wl = xs + C * n;
  if (FUSED) {
    const float* xb = qkv + (int64_t)b * C * n;
    for (int i = threadIdx.x; i < C * n; i += blockDim.x) xs[i] = xb[i];
    for (int i = threadIdx.x; i < 96 * C; i += blockDim.x) {
      const int r = i / C, c = i - r * C;  // r: q 0..31, k 32..63, v 64..95
      wl[c * 96 + r] = wqkv[((int64_t)(r >> 5) * HD + h * FE_DH + (r & 31)) * C + c];
    }
    __syncthreads();
    la_rows_matmul<2 * FE_DH>(wl, FE_DH, xs, C, n, ks, ld);  // k rows then v rows (vs = ks + 32 ld)
  } else {
    const float* k = q + (int64_t)HD * n;
    const float* v = k + (int64_t)HD * n;
    if ((n & 3) == 0) {  // 16-byte loads (rows of k / v are n floats, 16-byte aligned)
      const int n4 = n >> 2;
      for (int i = threadIdx.x; i < FE_DH * n4; i += blockDim.x) {
        const int d = i / n4, j = (i - d * n4) * 4;
        const floatx4 kv4 = *reinterpret_cast<const floatx4*>(k + (int64_t)d * n + j);
        const floatx4 vv4 = *reinterpret_cast<const floatx4*>(v + (int64_t)d * n + j);
  #pragma unroll
        for (int t = 0; t < 4; ++t) {
          ks[d * ld + j + t] = kv4[t];
          vs[d * ld + j + t] = vv4[t];
        }
      }
    } else {
      for (int i = threadIdx.x; i < FE_DH * n; i += blockDim.x) {
        const int d = i / n, j = i - d * n;
        ks[d * ld + j] = k[i];
        vs[d * ld + j] = v[i];
      }
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int d = wv; d < FE_DH; d += 4) {  // softmax of each k row over n
    float* row = ks + d * ld;
    float m = -INFINITY;
    for (int j = lane; j < n; j += 64) m = fmaxf(m, row[j]);
    m = wave_max(m);
    float s = 0.f;
    for (int j = lane; j < n; j += 64) {
      const float e = expf(row[j] - m);
      row[j] = e;
      s += e;
    }
    s = wave_sum(s);
    for (int j = lane; j < n; j += 64) row[j] = row[j] / s;
  }
  __syncthreads();
  {
    // ctx partials: 4 quarters of n x (8 d-groups x 8 e-groups), 4 d x 4 e per thread
    // (16 FMAs per 8 LDS reads); quarters summed in order 0..3 below
    const int qt = threadIdx.x >> 6, dg = (threadIdx.x >> 3) & 7, eg = threadIdx.x & 7;
    const int per = (n + 3) / 4, j0 = qt * per, j1 = min(n, j0 + per);
    float acc[4][4] = {};
#pragma unroll 2
    for (int j = j0; j < j1; ++j) {
      float kd[4], ve[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        kd[r] = ks[(dg * 4 + r) * ld + j];
        ve[r] = vs[(eg * 4 + r) * ld + j];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r][c] = fmaf(kd[r], ve[c], acc[r][c]);
    }
    __syncthreads();  // k and v consumed: the partials overlay them
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        part[(qt * FE_DH + dg * 4 + r) * CTX_LD + eg * 4 + c] = acc[r][c];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < FE_DH * FE_DH; i += blockDim.x) {
    const int d = i >> 5, e = i & 31;
    float s = part[d * CTX_LD + e];
#pragma unroll
    for (int t = 1; t < 4; ++t) s += part[(t * FE_DH + d) * CTX_LD + e];
    ctx[d * CTX_LD + e] = s;
  }
  __syncthreads();
  // q softmax over d (x scale) per column, into the k rows (k is consumed)
  if (FUSED) {
    la_rows_matmul<FE_DH>(wl, 0, xs, C, n, ks, ld);
    __syncthreads();
  }
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    float qd[FE_DH];
    float m = -INFINITY;
#pragma unroll
    for (int d = 0; d < FE_DH; ++d) {
      qd[d] = FUSED ? ks[d * ld + j] : q[(int64_t)d * n + j];
      m = fmaxf(m, qd[d]);
    }
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < FE_DH; ++d) {
      qd[d] = expf(qd[d] - m);
      s += qd[d];
    }
#pragma unroll
    for (int d = 0; d < FE_DH; ++d) ks[d * ld + j] = qd[d] / s * scale;
  }
  __syncthreads();
  // out[e, j] = sum_d ctx[d, e] q[d, j]: each thread 4 e x 4 j (16 FMAs per 5 LDS reads)
  float* ob = out + ((int64_t)b * HD + h * FE_DH) * n;
  const int te = threadIdx.x & 7, tj = threadIdx.x >> 3;
  for (int jb = 0; jb < n; jb += 128) {
    float acc[4][4] = {};
#pragma unroll 2
    for (int d = 0; d < FE_DH; ++d) {
      const floatx4 cv = *reinterpret_cast<const floatx4*>(ctx + d * CTX_LD + te * 4);
      float qv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = jb + tj + 32 * i;
        qv[i] = j < n ? ks[d * ld + j] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[r][i] = fmaf(cv[r], qv[i], acc[r][i]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = jb + tj + 32 * i;
        if (j < n) ob[(int64_t)(te * 4 + r) * n + j] = acc[r][i];
      }
  }
}

// Attention core (fidelity_enhancer.py:273-283) for one (b, h), dh = 32:
// out[b, h dh + d, i] = sum_j softmax_j(q_i . k_j * scale) v[d, j].  One thread per query
// i, exact two-pass softmax over the keys staged in LDS.
__global__ __launch_bounds__(256) void attn_kernel(const float* __restrict__ qkv, int H, int n,
                                                   float scale, float* __restrict__ out) {
  extern __shared__ float sm[];
  float* ks = sm;                 // n x FE_DH (key-major: broadcast reads)
  float* vs = sm + n * FE_DH;     // n x FE_DH
  const int b = blockIdx.x / H, h = blockIdx.x - b * H;
  const int HD = H * FE_DH;
  const float* q = qkv + ((int64_t)b * 3 * HD + h * FE_DH) * n;
  const float* k = q + (int64_t)HD * n;
  const float* v = k + (int64_t)HD * n;
  for (int i = threadIdx.x; i < FE_DH * n; i += blockDim.x) {
    const int d = i / n, j = i - d * n;
    ks[j * FE_DH + d] = k[i];
    vs[j * FE_DH + d] = v[i];
  }
  __syncthreads();
  float* ob = out + ((int64_t)b * HD + h * FE_DH) * n;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    float qi[FE_DH];
#pragma unroll
    for (int d = 0; d < FE_DH; ++d) qi[d] = q[(int64_t)d * n + i] * scale;
    float m = -INFINITY;
    for (int j = 0; j < n; ++j) {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < FE_DH; ++d) s = fmaf(qi[d], ks[j * FE_DH + d], s);
      m = fmaxf(m, s);
    }
    float o[FE_DH];
#pragma unroll
    for (int d = 0; d < FE_DH; ++d) o[d] = 0.f;
    float den = 0.f;
    for (int j = 0; j < n; ++j) {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < FE_DH; ++d) s = fmaf(qi[d], ks[j * FE_DH + d], s);
      const float p = expf(s - m);
      den += p;
#pragma unroll
      for (int d = 0; d < FE_DH; ++d) o[d] = fmaf(p, vs[j * FE_DH + d], o[d]);
    }
    const float inv = 1.0f / den;
#pragma unroll
    for (int d = 0; d < FE_DH; ++d) ob[(int64_t)d * n + i] = o[d] * inv;
  }
}

// out (B, Ca + Cb, L) = cat(interp(a -> L), interp(b -> L)) along channels, linear
// interpolation with align_corners=False (torch area_pixel_compute_source_index; equal
// lengths copy exactly).  Unet1D skips and final concat (fidelity_enhancer.py:434-452).
__device__ __forceinline__ float lerp_at(const float* __restrict__ row, int Lin, float ratio,
                                         int i) {
  float src = ratio * ((float)i + 0.5f) - 0.5f;
  if (src < 0.f) src = 0.f;
  const int i0 = (int)src;
  const int i1 = i0 + (i0 < Lin - 1 ? 1 : 0);
  const float l1 = fminf(fmaxf(src - (float)i0, 0.f), 1.f);
  return (1.f - l1) * row[i0] + l1 * row[i1];
}
__global__ __launch_bounds__(256) void cat_interp_kernel(const float* __restrict__ a, int Ca,
                                                         int La, const float* __restrict__ bb,
                                                         int Cb, int Lb, int B, int L,
                                                         float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int C = Ca + Cb;
  if (t >= (int64_t)B * C * L) return;
  const int i = (int)(t % L);
  const int64_t bc = t / L;
  const int c = (int)(bc % C), b = (int)(bc / C);
  float v;
  if (c < Ca)
    v = La == L ? a[((int64_t)b * Ca + c) * La + i]
                : lerp_at(a + ((int64_t)b * Ca + c) * La, La, (float)La / (float)L, i);
  else
    v = Lb == L ? bb[((int64_t)b * Cb + (c - Ca)) * Lb + i]
                : lerp_at(bb + ((int64_t)b * Cb + (c - Ca)) * Lb, Lb, (float)Lb / (float)L, i);
  out[t] = v;
}

// allow the dynamic-LDS kernels the whole 160 KB of a gfx950 CU (default cap is 64 KB)
void fe_lds_attr() {
  static bool done = false;
  if (done) return;
  done = true;
  const int cap = 160 * 1024;
  (void)hipFuncSetAttribute((const void*)conv1d_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, cap);
  (void)hipFuncSetAttribute((const void*)linear_attn_kernel<false>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, cap);
  (void)hipFuncSetAttribute((const void*)linear_attn_kernel<true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, cap);
  (void)hipFuncSetAttribute((const void*)attn_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, cap);
}

}  // namespace
}  // namespace tvq

using namespace tvq;

extern "C" {

int64_t tvq_fe_conv1d_out_len(int64_t Lin, int64_t K, int64_t S, int64_t P, int64_t up2) {
  const int64_t Leff = up2 ? 2 * Lin : Lin;
  return (Leff + 2 * P - K) / S + 1;
}

int tvq_fe_ws_weight(const float* w, int64_t Co, int64_t n, float eps, float* out,
                     tvq_stream_t stream) {
  TVQ_CHECK_ARG(w && out && Co > 0 && n > 0, "tvq_fe_ws_weight: bad arguments");
  hipLaunchKernelGGL(ws_kernel, dim3((unsigned)Co), dim3(256), 0, (hipStream_t)stream, w, (int)n,
                     eps, out);
  return launch_status("tvq_fe_ws_weight");
}

int tvq_fe_conv1d(const float* x, int64_t B, int64_t Ci, int64_t Lin, const float* w,
                  const float* bias, int64_t Co, int64_t K, int64_t S, int64_t P, int64_t up2,
                  int64_t replicate, const float* residual, float* y, int64_t Lout,
                  tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && w && y && B > 0 && Ci > 0 && Lin > 0 && Co > 0 && K > 0 && S > 0 && P >= 0,
                "tvq_fe_conv1d: bad arguments");
  TVQ_CHECK_ARG(Lout == tvq_fe_conv1d_out_len(Lin, K, S, P, up2) && Lout > 0,
                "tvq_fe_conv1d: Lout %lld does not match the conv geometry", (long long)Lout);
  if (S <= 2 && K <= 7) {
    // register-blocked path: pick the tile (TP positions x TC channels) that pads least
    struct V { int tp, tc; };
    const V vs[4] = {{256, 16}, {128, 32}, {64, 64}, {32, 64}};
    int best = 0;
    int64_t best_area = -1;
    for (int v = 0; v < 4; ++v) {
      const int64_t area = ((Lout + vs[v].tp - 1) / vs[v].tp) * vs[v].tp *
                           ((Co + vs[v].tc - 1) / vs[v].tc) * vs[v].tc;
      // ties go to the later (wider-channel) tile, except the 2-position one (v = 3)
      if (best_area < 0 || area < best_area || (area == best_area && v < 3)) best = v, best_area = area;
    }
    const int64_t span = (vs[best].tp - 1) * S + K;
    const size_t lds = (size_t)(16 * span + 16 * K * vs[best].tc) * sizeof(float);
    TVQ_CHECK_ARG(B <= 65535 && (Co + vs[best].tc - 1) / vs[best].tc <= 65535,
                  "tvq_fe_conv1d: grid too large");
    dim3 grid((unsigned)((Lout + vs[best].tp - 1) / vs[best].tp),
              (unsigned)((Co + vs[best].tc - 1) / vs[best].tc), (unsigned)B);
#define FE_RB_LAUNCH_K(TPX, TCY, RP, KT)                                                      \
  hipLaunchKernelGGL((conv1d_rb_kernel<TPX, TCY, RP, KT>), grid, dim3(256), lds, (hipStream_t)stream, x, \
                     (int)Ci, (int)Lin, w, bias, (int)Co, (int)K, (int)S, (int)P, (int)up2,      \
                     (int)replicate, residual, y, (int)Lout, (int)span)
#define FE_RB_LAUNCH(TPX, TCY, RP)             \
  do {                                          \
    if (K == 1) FE_RB_LAUNCH_K(TPX, TCY, RP, 1); \
    else if (K == 3) FE_RB_LAUNCH_K(TPX, TCY, RP, 3); \
    else FE_RB_LAUNCH_K(TPX, TCY, RP, 0);       \
  } while (0)
    if (best == 0) FE_RB_LAUNCH(64, 4, 4);
    else if (best == 1) FE_RB_LAUNCH(32, 8, 4);
    else if (best == 2) FE_RB_LAUNCH(16, 16, 4);
    else FE_RB_LAUNCH(16, 16, 2);
#undef FE_RB_LAUNCH
#undef FE_RB_LAUNCH_K
    return launch_status("tvq_fe_conv1d");
  }
  const int64_t span = (FE_TILE - 1) * S + K;
  const int64_t lds = Ci * span * (int64_t)sizeof(float);
  TVQ_CHECK_ARG(lds <= 160 * 1024, "tvq_fe_conv1d: Ci %lld x span %lld exceeds LDS",
                (long long)Ci, (long long)span);
  TVQ_CHECK_ARG(B <= 65535 && (Co + FE_COB - 1) / FE_COB <= 65535, "tvq_fe_conv1d: grid too large");
  fe_lds_attr();
  dim3 grid((unsigned)((Lout + FE_TILE - 1) / FE_TILE), (unsigned)((Co + FE_COB - 1) / FE_COB),
            (unsigned)B);
  hipLaunchKernelGGL(conv1d_kernel, grid, dim3(256), (size_t)lds, (hipStream_t)stream, x, (int)Ci,
                     (int)Lin, w, bias, (int)Co, (int)K, (int)S, (int)P, (int)up2, (int)replicate,
                     residual, y, (int)Lout, (int)span);
  return launch_status("tvq_fe_conv1d");
}

int tvq_fe_group_norm_snake(const float* x, int64_t B, int64_t C, int64_t L, int64_t G,
                            const float* gamma, const float* beta, const float* a, float eps,
                            const float* residual, float* y, tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && y && gamma && beta && a && B > 0 && C > 0 && L > 0 && G > 0 && C % G == 0,
                "tvq_fe_group_norm_snake: bad arguments");
  const int64_t n = C / G * L;
  const dim3 grid((unsigned)(B * G));
  const hipStream_t st = (hipStream_t)stream;
  if (n <= 256 * 2)
    hipLaunchKernelGGL(gn_snake_kernel<2>, grid, dim3(256), 0, st, x, (int)C, (int)L, (int)G, gamma,
                       beta, a, eps, residual, y);
  else if (n <= 256 * 8)
    hipLaunchKernelGGL(gn_snake_kernel<8>, grid, dim3(256), 0, st, x, (int)C, (int)L, (int)G, gamma,
                       beta, a, eps, residual, y);
  else
    hipLaunchKernelGGL(gn_snake_kernel<0>, grid, dim3(256), 0, st, x, (int)C, (int)L, (int)G, gamma,
                       beta, a, eps, residual, y);
  return launch_status("tvq_fe_group_norm_snake");
}

int tvq_fe_channel_layernorm(const float* x, int64_t B, int64_t C, int64_t L, const float* g,
                             float eps, const float* residual, float* y, tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && y && g && B > 0 && C > 0 && L > 0, "tvq_fe_channel_layernorm: bad arguments");
  const int64_t n = B * L;
  const dim3 grid((unsigned)((n + 255) / 256));
  const hipStream_t st = (hipStream_t)stream;
#define FE_LN(CT) \
  hipLaunchKernelGGL(chan_ln_kernel<CT>, grid, dim3(256), 0, st, x, (int)B, (int)C, (int)L, g, eps, residual, y)
  if (C == 8) FE_LN(8);
  else if (C == 16) FE_LN(16);
  else if (C == 32) FE_LN(32);
  else if (C == 64) FE_LN(64);
  else FE_LN(0);
#undef FE_LN
  return launch_status("tvq_fe_channel_layernorm");
}

int tvq_fe_linear_attention(const float* qkv, int64_t B, int64_t H, int64_t dh, int64_t n,
                            float* out, tvq_stream_t stream) {
  TVQ_CHECK_ARG(qkv && out && B > 0 && H > 0 && n > 0 && dh == FE_DH,
                "tvq_fe_linear_attention: bad arguments (dim_head must be %d)", FE_DH);
  const int64_t kv = 2 * FE_DH * (n + 1) > 4 * FE_DH * CTX_LD ? 2 * FE_DH * (n + 1) : 4 * FE_DH * CTX_LD;
  const int64_t lds = (kv + FE_DH * CTX_LD) * (int64_t)sizeof(float);
  TVQ_CHECK_ARG(lds <= 160 * 1024, "tvq_fe_linear_attention: n %lld exceeds LDS", (long long)n);
  fe_lds_attr();
  hipLaunchKernelGGL(linear_attn_kernel<false>, dim3((unsigned)(B * H)), dim3(256), (size_t)lds,
                     (hipStream_t)stream, qkv, nullptr, 0, (int)H, (int)n,
                     1.0f / sqrtf((float)dh), out);
  return launch_status("tvq_fe_linear_attention");
}

int tvq_fe_linear_attention_fused(const float* x, int64_t B, int64_t C, int64_t n,
                                  const float* wqkv, int64_t H, int64_t dh, float* out,
                                  tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && wqkv && out && B > 0 && C > 0 && H > 0 && n > 0 && dh == FE_DH,
                "tvq_fe_linear_attention_fused: bad arguments (dim_head must be %d)", FE_DH);
  const int64_t kv = 2 * FE_DH * (n + 1) > 4 * FE_DH * CTX_LD ? 2 * FE_DH * (n + 1) : 4 * FE_DH * CTX_LD;
  const int64_t lds = (kv + FE_DH * CTX_LD + C * n + 96 * C) * (int64_t)sizeof(float);
  TVQ_CHECK_ARG(lds <= 160 * 1024, "tvq_fe_linear_attention_fused: C %lld x n %lld exceeds LDS",
                (long long)C, (long long)n);
  fe_lds_attr();
  hipLaunchKernelGGL(linear_attn_kernel<true>, dim3((unsigned)(B * H)), dim3(256), (size_t)lds,
                     (hipStream_t)stream, x, wqkv, (int)C, (int)H, (int)n,
                     1.0f / sqrtf((float)dh), out);
  return launch_status("tvq_fe_linear_attention_fused");
}

int tvq_fe_attention(const float* qkv, int64_t B, int64_t H, int64_t dh, int64_t n, float* out,
                     tvq_stream_t stream) {
  TVQ_CHECK_ARG(qkv && out && B > 0 && H > 0 && n > 0 && dh == FE_DH,
                "tvq_fe_attention: bad arguments (dim_head must be %d)", FE_DH);
  const int64_t lds = 2 * n * FE_DH * (int64_t)sizeof(float);
  TVQ_CHECK_ARG(lds <= 160 * 1024, "tvq_fe_attention: n %lld exceeds LDS", (long long)n);
  fe_lds_attr();
  hipLaunchKernelGGL(attn_kernel, dim3((unsigned)(B * H)), dim3(256), (size_t)lds,
                     (hipStream_t)stream, qkv, (int)H, (int)n, 1.0f / sqrtf((float)dh), out);
  return launch_status("tvq_fe_attention");
}

int tvq_fe_cat_interp(const float* a, int64_t Ca, int64_t La, const float* b, int64_t Cb,
                      int64_t Lb, int64_t B, int64_t L, float* out, tvq_stream_t stream) {
  TVQ_CHECK_ARG(a && out && B > 0 && Ca > 0 && La > 0 && L > 0 && Cb >= 0 && (Cb == 0 || (b && Lb > 0)),
                "tvq_fe_cat_interp: bad arguments");
  const int64_t n = B * (Ca + Cb) * L;
  hipLaunchKernelGGL(cat_interp_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, a, (int)Ca, (int)La, b, (int)Cb, (int)Lb, (int)B, (int)L,
                     out);
  return launch_status("tvq_fe_cat_interp");
}

}  // extern "C"

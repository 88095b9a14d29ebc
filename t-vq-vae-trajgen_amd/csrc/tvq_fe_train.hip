// FidelityEnhancer training (Stage3, reference trainers/stage3.py:197-231 over
// models/fidelity_enhancer.py:96-455) on gfx950: the training-mode forward pieces that
// differ from the eval kernels of tvq_fe.hip (GroupNorm+Snake with the Block's dropout
// and saved statistics) and the backward of every Unet1D op that is not a convolution
// (the convs run on the conv engine, tvq_conv.hip, as H = 1 images):
//
//   fe_ws_bwd               WeightStandardizedConv2d weight: dw = r (g - mean g - w^ mean(g w^))
//   fe_gn_snake_train_fwd   GroupNorm -> Snake -> Dropout (+ ResnetBlock skip), per (b, g)
//   fe_gn_snake_bwd         Dropout' -> Snake' -> GroupNorm' per (b, g); the per-element
//                           terms of dgamma / dbeta / da for a deterministic channel sum
//   fe_chan_ln_bwd          channel LayerNorm (gamma only) backward per (b, l)
//   fe_linattn_bwd          LinearAttention core backward per (b, h): softmax over d (q) and
//                           over n (k), context k v^T, out ctx^T q
//   fe_attn_bwd             Attention core backward per (b, h): P and dS staged in LDS
//   fe_cat_interp_bwd       the skips' interpolate+concat backward (gather form, no atomics)
//
// (B, C, L) fp32 row-major; every reduction has a fixed order (no atomics), so gradients
// are run-to-run identical.  Formulas follow the reference ops' autograd arithmetic.
#include "tvq_common.h"

namespace tvq {
namespace {

constexpr int DH = 32;  // dim_head of both FidelityEnhancer attentions

// ---------------------------------------------------------------- weight standardisation
__global__ __launch_bounds__(256) void fe_ws_bwd_kernel(const float* __restrict__ w, int n,
                                                        float eps, const float* __restrict__ g,
                                                        float* __restrict__ dw, int accumulate) {
  __shared__ float red[4];
  const int64_t o = (int64_t)blockIdx.x * n;
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += w[o + i];
  const float mean = block_sum(s, red) / (float)n;
  float q = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float d = w[o + i] - mean;
    q += d * d;
  }
  const float rstd = rsqrtf(block_sum(q, red) / (float)n + eps);
  float sg = 0.f, sgw = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float wh = (w[o + i] - mean) * rstd;
    sg += g[o + i];
    sgw += g[o + i] * wh;
  }
  const float mg = block_sum(sg, red) / (float)n;
  const float mgw = block_sum(sgw, red) / (float)n;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float wh = (w[o + i] - mean) * rstd;
    const float v = rstd * (g[o + i] - mg - wh * mgw);
    dw[o + i] = accumulate ? dw[o + i] + v : v;
  }
}

// ---------------------------------------------------------------- GroupNorm + Snake
// y = Dropout_p(Snake_a(GroupNorm(x))) (+ res); mean / rstd of each (b, g) saved.
__global__ __launch_bounds__(256) void fe_gn_snake_train_kernel(
    const float* __restrict__ x, int C, int L, int G, const float* __restrict__ gamma,
    const float* __restrict__ beta, const float* __restrict__ a, float eps, float drop_p,
    float drop_scale, const int64_t* __restrict__ seed_ptr, uint64_t offset,
    const float* __restrict__ res, float* __restrict__ y, float* __restrict__ mean_out,
    float* __restrict__ rstd_out) {
  __shared__ float red[4];
  const int cg = C / G, n = cg * L;
  const int64_t base = (int64_t)blockIdx.x * n;  // blockIdx.x = b * G + g
  const int c0 = (blockIdx.x % G) * cg;
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += x[base + i];
  const float mean = block_sum(s, red) / (float)n;
  float q = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float d = x[base + i] - mean;
    q += d * d;
  }
  const float rstd = rsqrtf(block_sum(q, red) / (float)n + eps);
  if (threadIdx.x == 0) {
    mean_out[blockIdx.x] = mean;
    rstd_out[blockIdx.x] = rstd;
  }
  const uint64_t seed = drop_p > 0.f ? mix_seed(seed_ptr, offset) : 0ull;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int c = c0 + i / L;
    float t = (x[base + i] - mean) * (rstd * gamma[c]) + beta[c];
    const float ac = a[c];
    t = snake_f(t, ac, 1.0f / ac);
    if (drop_p > 0.f) t = uniform01(seed, (uint64_t)(base + i)) >= drop_p ? t * drop_scale : 0.f;
    y[base + i] = t + (res ? res[base + i] : 0.f);
  }
}

// dx; and per element tgam = du * xhat, tbet = du, tda = the Snake a-gradient term (each
// (B, C, L)), summed over (b, l) per channel by tvq_channel_sum afterwards.
__global__ __launch_bounds__(256) void fe_gn_snake_bwd_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, int C, int L, int G,
    const float* __restrict__ gamma, const float* __restrict__ beta, const float* __restrict__ a,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in, float drop_p,
    float drop_scale, const int64_t* __restrict__ seed_ptr, uint64_t offset,
    float* __restrict__ dx, float* __restrict__ tgam, float* __restrict__ tbet,
    float* __restrict__ tda) {
  __shared__ float red[4];
  const int cg = C / G, n = cg * L;
  const int64_t base = (int64_t)blockIdx.x * n;
  const int c0 = (blockIdx.x % G) * cg;
  const float mean = mean_in[blockIdx.x], rstd = rstd_in[blockIdx.x];
  const uint64_t seed = drop_p > 0.f ? mix_seed(seed_ptr, offset) : 0ull;
  float s1 = 0.f, s2 = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int c = c0 + i / L;
    const float xh = (x[base + i] - mean) * rstd;
    const float u = xh * gamma[c] + beta[c];
    float gs = dy[base + i];
    if (drop_p > 0.f) gs = uniform01(seed, (uint64_t)(base + i)) >= drop_p ? gs * drop_scale : 0.f;
    const float av = a[c], inv_a = 1.0f / av;
    float sn, cs;
    sincosf(av * u, &sn, &cs);
    const float t = 2.0f * sn * cs;
    const float du = gs + gs * inv_a * t * av;
    tgam[base + i] = du * xh;
    tbet[base + i] = du;
    tda[base + i] = gs * inv_a * t * u - gs * (sn * sn) * inv_a * inv_a;
    const float dxh = du * gamma[c];
    s1 += dxh;
    s2 += dxh * xh;
  }
  const float m1 = block_sum(s1, red) / (float)n;
  const float m2 = block_sum(s2, red) / (float)n;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int c = c0 + i / L;
    const float xh = (x[base + i] - mean) * rstd;
    const float dxh = tbet[base + i] * gamma[c];
    dx[base + i] = rstd * (dxh - m1 - xh * m2);
  }
}

// ---------------------------------------------------------------- channel LayerNorm
// y = (x - mean_c) rsqrt(var_c + eps) g  per (b, l) over C; dx and tg = dy * xhat
__global__ __launch_bounds__(256) void fe_chan_ln_bwd_kernel(const float* __restrict__ dy,
                                                             const float* __restrict__ x, int B,
                                                             int C, int L,
                                                             const float* __restrict__ g,
                                                             float eps, float* __restrict__ dx,
                                                             float* __restrict__ tg) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * L) return;
  const int b = t / L, l = t - b * L;
  const int64_t at0 = (int64_t)b * C * L + l;
  float s = 0.f;
  for (int c = 0; c < C; ++c) s += x[at0 + (int64_t)c * L];
  const float mean = s / (float)C;
  float q = 0.f;
  for (int c = 0; c < C; ++c) {
    const float d = x[at0 + (int64_t)c * L] - mean;
    q += d * d;
  }
  const float rstd = rsqrtf(q / (float)C + eps);
  float s1 = 0.f, s2 = 0.f;
  for (int c = 0; c < C; ++c) {
    const int64_t at = at0 + (int64_t)c * L;
    const float xh = (x[at] - mean) * rstd;
    const float dxh = dy[at] * g[c];
    tg[at] = dy[at] * xh;
    s1 += dxh;
    s2 += dxh * xh;
  }
  const float m1 = s1 / (float)C, m2 = s2 / (float)C;
  for (int c = 0; c < C; ++c) {
    const int64_t at = at0 + (int64_t)c * L;
    const float xh = (x[at] - mean) * rstd;
    dx[at] = rstd * (dy[at] * g[c] - m1 - xh * m2);
  }
}

// ---------------------------------------------------------------- linear attention core
// One block per (b, h).  LDS: qsm (softmax over d, unscaled), ks (softmax over n), v, each
// DH x n (row stride n+1); ctx, dctx DH x DH.  dout / outputs through global memory.
__global__ __launch_bounds__(256) void fe_linattn_bwd_kernel(const float* __restrict__ qkv,
                                                             const float* __restrict__ dout,
                                                             int H, int n, float scale,
                                                             float* __restrict__ dqkv) {
  extern __shared__ float sm[];
  const int ld = n + 1;
  float* qs = sm;                    // qsm, later dks
  float* ks = qs + DH * ld;
  float* vs = ks + DH * ld;
  float* ctx = vs + DH * ld;         // [d][e], stride DH + 1
  float* dctx = ctx + DH * (DH + 1);
  const int b = blockIdx.x / H, h = blockIdx.x - b * H;
  const int HD = H * DH;
  const float* q = qkv + ((int64_t)b * 3 * HD + h * DH) * n;
  const float* k = q + (int64_t)HD * n;
  const float* v = k + (int64_t)HD * n;
  const float* go = dout + ((int64_t)b * HD + h * DH) * n;
  float* dq = dqkv + ((int64_t)b * 3 * HD + h * DH) * n;
  float* dk = dq + (int64_t)HD * n;
  float* dv = dk + (int64_t)HD * n;
  for (int i = threadIdx.x; i < DH * n; i += blockDim.x) {
    const int d = i / n, j = i - d * n;
    qs[d * ld + j] = q[i];
    ks[d * ld + j] = k[i];
    vs[d * ld + j] = v[i];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int d = wv; d < DH; d += 4) {  // k: softmax over n per row (as the forward)
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
  for (int j = threadIdx.x; j < n; j += blockDim.x) {  // q: softmax over d per column
    float m = -INFINITY;
    for (int d = 0; d < DH; ++d) m = fmaxf(m, qs[d * ld + j]);
    float s = 0.f;
    for (int d = 0; d < DH; ++d) {
      const float e = expf(qs[d * ld + j] - m);
      qs[d * ld + j] = e;
      s += e;
    }
    for (int d = 0; d < DH; ++d) qs[d * ld + j] = qs[d * ld + j] / s;
  }
  __syncthreads();
  // ctx[d][e] = sum_n ks[d][n] v[e][n];  dctx[d][e] = sum_n scale qsm[d][n] dout[e][n]
  for (int i = threadIdx.x; i < DH * DH; i += blockDim.x) {
    const int d = i >> 5, e = i & 31;
    float c = 0.f, dc = 0.f;
    for (int j = 0; j < n; ++j) {
      c = fmaf(ks[d * ld + j], vs[e * ld + j], c);
      dc = fmaf(qs[d * ld + j] * scale, go[(int64_t)e * n + j], dc);
    }
    ctx[d * (DH + 1) + e] = c;
    dctx[d * (DH + 1) + e] = dc;
  }
  __syncthreads();
  // dq: per column, g = scale * sum_e ctx[d][e] dout[e][n]; dq = qsm (g - sum_d qsm g)
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    float gq[DH];
    float dot = 0.f;
#pragma unroll
    for (int d = 0; d < DH; ++d) {
      float acc = 0.f;
      for (int e = 0; e < DH; ++e) acc = fmaf(ctx[d * (DH + 1) + e], go[(int64_t)e * n + j], acc);
      gq[d] = acc * scale;
      dot += qs[d * ld + j] * gq[d];
    }
#pragma unroll
    for (int d = 0; d < DH; ++d) dq[(int64_t)d * n + j] = qs[d * ld + j] * (gq[d] - dot);
  }
  __syncthreads();  // qs no longer needed: it holds dks below
  // dv[e][n] = sum_d dctx[d][e] ks[d][n];  dks[d][n] = sum_e dctx[d][e] v[e][n]
  for (int i = threadIdx.x; i < DH * n; i += blockDim.x) {
    const int r = i / n, j = i - r * n;
    float a1 = 0.f, a2 = 0.f;
    for (int t = 0; t < DH; ++t) {
      a1 = fmaf(dctx[t * (DH + 1) + r], ks[t * ld + j], a1);
      a2 = fmaf(dctx[r * (DH + 1) + t], vs[t * ld + j], a2);
    }
    dv[(int64_t)r * n + j] = a1;
    qs[r * ld + j] = a2;
  }
  __syncthreads();
  for (int d = wv; d < DH; d += 4) {  // dk = ks (dks - sum_n ks dks) per row
    const float* kr = ks + d * ld;
    const float* gr = qs + d * ld;
    float dot = 0.f;
    for (int j = lane; j < n; j += 64) dot += kr[j] * gr[j];
    dot = wave_sum(dot);
    for (int j = lane; j < n; j += 64) dk[(int64_t)d * n + j] = kr[j] * (gr[j] - dot);
  }
}

// ---------------------------------------------------------------- full attention core
// One block per (b, h); n <= 128 keys.  LDS: q*scale, k, v, do (n x DH each), P and dS
// (n x (n+1)).
__global__ __launch_bounds__(256) void fe_attn_bwd_kernel(const float* __restrict__ qkv,
                                                          const float* __restrict__ dout, int H,
                                                          int n, float scale,
                                                          float* __restrict__ dqkv) {
  extern __shared__ float sm[];
  const int pl = n + 1;
  float* qs = sm;              // [i][d] q * scale
  float* ks = qs + n * DH;     // [j][d]
  float* vs = ks + n * DH;     // [j][d]
  float* gs = vs + n * DH;     // [i][d] dout
  float* P = gs + n * DH;      // [i][j]
  float* dS = P + n * pl;      // [i][j]
  const int b = blockIdx.x / H, h = blockIdx.x - b * H;
  const int HD = H * DH;
  const float* q = qkv + ((int64_t)b * 3 * HD + h * DH) * n;
  const float* k = q + (int64_t)HD * n;
  const float* v = k + (int64_t)HD * n;
  const float* go = dout + ((int64_t)b * HD + h * DH) * n;
  float* dq = dqkv + ((int64_t)b * 3 * HD + h * DH) * n;
  float* dk = dq + (int64_t)HD * n;
  float* dv = dk + (int64_t)HD * n;
  for (int i = threadIdx.x; i < DH * n; i += blockDim.x) {
    const int d = i / n, j = i - d * n;
    qs[j * DH + d] = q[i] * scale;
    ks[j * DH + d] = k[i];
    vs[j * DH + d] = v[i];
    gs[j * DH + d] = go[i];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {  // row i: P, dP, dS
    float m = -INFINITY;
    for (int j = 0; j < n; ++j) {
      float s = 0.f;
      for (int d = 0; d < DH; ++d) s = fmaf(qs[i * DH + d], ks[j * DH + d], s);
      P[i * pl + j] = s;
      m = fmaxf(m, s);
    }
    float den = 0.f;
    for (int j = 0; j < n; ++j) {
      const float p = expf(P[i * pl + j] - m);
      P[i * pl + j] = p;
      den += p;
    }
    const float inv = 1.0f / den;
    float rs = 0.f;
    for (int j = 0; j < n; ++j) {
      const float p = P[i * pl + j] * inv;
      P[i * pl + j] = p;
      float dp = 0.f;
      for (int d = 0; d < DH; ++d) dp = fmaf(gs[i * DH + d], vs[j * DH + d], dp);
      dS[i * pl + j] = dp;
      rs += p * dp;
    }
    for (int j = 0; j < n; ++j) dS[i * pl + j] = P[i * pl + j] * (dS[i * pl + j] - rs);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < n * DH; t += blockDim.x) {
    const int r = t / DH, d = t - r * DH;
    float aq = 0.f, ak = 0.f, av = 0.f;
    for (int j = 0; j < n; ++j) {
      aq = fmaf(dS[r * pl + j], ks[j * DH + d], aq);   // dq_r = scale sum_j dS[r][j] k_j
      ak = fmaf(dS[j * pl + r], qs[j * DH + d], ak);   // dk_r = sum_i dS[i][r] (q_i scale)
      av = fmaf(P[j * pl + r], gs[j * DH + d], av);    // dv_r = sum_i P[i][r] do_i
    }
    dq[(int64_t)d * n + r] = aq * scale;
    dk[(int64_t)d * n + r] = ak;
    dv[(int64_t)d * n + r] = av;
  }
}

// ---------------------------------------------------------------- interpolate + concat
// Backward of out[:, :Ca] = interp(a -> L), out[:, Ca:] = interp(b -> L) (linear,
// align_corners=False, source index clamped at 0, as cat_interp_kernel).  Each input
// sample gathers the output samples whose two taps reference it.
__device__ __forceinline__ float lerp_bwd_at(const float* __restrict__ grow, int Lin, int L,
                                             int j) {
  if (Lin == L) return grow[j];
  const float ratio = (float)Lin / (float)L;
  // outputs i with i0(i) or i1(i) == j lie within (j - 1, j + 1] / ratio; scan a margin
  int lo = (int)floorf(((float)j - 1.5f) / ratio) - 2;
  int hi = (int)ceilf(((float)j + 1.5f) / ratio) + 2;
  lo = lo < 0 ? 0 : lo;
  hi = hi > L - 1 ? L - 1 : hi;
  float s = 0.f;
  for (int i = lo; i <= hi; ++i) {
    float src = ratio * ((float)i + 0.5f) - 0.5f;
    if (src < 0.f) src = 0.f;
    const int i0 = (int)src;
    const int i1 = i0 + (i0 < Lin - 1 ? 1 : 0);
    const float l1 = fminf(fmaxf(src - (float)i0, 0.f), 1.f);
    if (i0 == j) s += (1.f - l1) * grow[i];
    if (i1 == j) s += l1 * grow[i];
  }
  return s;
}

__global__ __launch_bounds__(256) void fe_cat_interp_bwd_kernel(const float* __restrict__ gout,
                                                                int Ca, int La, int Cb, int Lb,
                                                                int B, int L,
                                                                float* __restrict__ da,
                                                                float* __restrict__ db) {
  const int64_t na = (int64_t)B * Ca * La, nb = (int64_t)B * Cb * Lb;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int C = Ca + Cb;
  if (t < na) {
    const int j = (int)(t % La);
    const int64_t bc = t / La;
    const int c = (int)(bc % Ca), b = (int)(bc / Ca);
    da[t] = lerp_bwd_at(gout + ((int64_t)b * C + c) * L, La, L, j);
  } else if (t < na + nb) {
    const int64_t u = t - na;
    const int j = (int)(u % Lb);
    const int64_t bc = u / Lb;
    const int c = (int)(bc % Cb), b = (int)(bc / Cb);
    db[u] = lerp_bwd_at(gout + ((int64_t)b * C + Ca + c) * L, Lb, L, j);
  }
}

void fe_train_lds_attr() {
  static bool done = false;
  if (done) return;
  done = true;
  const int cap = 160 * 1024;
  (void)hipFuncSetAttribute((const void*)fe_linattn_bwd_kernel,
                            hipFuncAttributeMaxDynamicSharedMemorySize, cap);
  (void)hipFuncSetAttribute((const void*)fe_attn_bwd_kernel,
                            hipFuncAttributeMaxDynamicSharedMemorySize, cap);
}

}  // namespace
}  // namespace tvq

using namespace tvq;

extern "C" int tvq_fe_ws_weight_bwd(const float* w, int64_t O, int64_t n, float eps,
                                    const float* g, float* dw, int64_t accumulate,
                                    tvq_stream_t stream) {
  TVQ_CHECK_ARG(w && g && dw && O > 0 && n > 1, "tvq_fe_ws_weight_bwd: bad arguments");
  hipLaunchKernelGGL(fe_ws_bwd_kernel, dim3((unsigned)O), dim3(256), 0, (hipStream_t)stream, w,
                     (int)n, eps, g, dw, (int)accumulate);
  return launch_status("tvq_fe_ws_weight_bwd");
}

extern "C" int tvq_fe_gn_snake_train_fwd(const float* x, int64_t B, int64_t C, int64_t L,
                                         int64_t G, const float* gamma, const float* beta,
                                         const float* a, float eps, float drop_p,
                                         const int64_t* seed_ptr, uint64_t offset,
                                         const float* residual, float* y, float* mean,
                                         float* rstd, tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && gamma && beta && a && y && mean && rstd && B > 0 && G > 0 && C % G == 0,
                "tvq_fe_gn_snake_train_fwd: bad arguments");
  TVQ_CHECK_ARG(drop_p >= 0.f && drop_p < 1.f && (drop_p == 0.f || seed_ptr),
                "tvq_fe_gn_snake_train_fwd: bad dropout");
  hipLaunchKernelGGL(fe_gn_snake_train_kernel, dim3((unsigned)(B * G)), dim3(256), 0,
                     (hipStream_t)stream, x, (int)C, (int)L, (int)G, gamma, beta, a, eps, drop_p,
                     drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.f, seed_ptr, offset, residual, y,
                     mean, rstd);
  return launch_status("tvq_fe_gn_snake_train_fwd");
}

extern "C" int tvq_fe_gn_snake_bwd(const float* dy, const float* x, int64_t B, int64_t C,
                                   int64_t L, int64_t G, const float* gamma, const float* beta,
                                   const float* a, const float* mean, const float* rstd,
                                   float drop_p, const int64_t* seed_ptr, uint64_t offset,
                                   float* dx, float* tgam, float* tbet, float* tda,
                                   tvq_stream_t stream) {
  TVQ_CHECK_ARG(dy && x && gamma && beta && a && mean && rstd && dx && tgam && tbet && tda &&
                    B > 0 && G > 0 && C % G == 0,
                "tvq_fe_gn_snake_bwd: bad arguments");
  hipLaunchKernelGGL(fe_gn_snake_bwd_kernel, dim3((unsigned)(B * G)), dim3(256), 0,
                     (hipStream_t)stream, dy, x, (int)C, (int)L, (int)G, gamma, beta, a, mean,
                     rstd, drop_p, drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.f, seed_ptr, offset,
                     dx, tgam, tbet, tda);
  return launch_status("tvq_fe_gn_snake_bwd");
}

extern "C" int tvq_fe_channel_layernorm_bwd(const float* dy, const float* x, int64_t B,
                                            int64_t C, int64_t L, const float* g, float eps,
                                            float* dx, float* tg, tvq_stream_t stream) {
  TVQ_CHECK_ARG(dy && x && g && dx && tg && B > 0 && C > 0 && L > 0,
                "tvq_fe_channel_layernorm_bwd: bad arguments");
  const int64_t n = B * L;
  hipLaunchKernelGGL(fe_chan_ln_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, dy, x, (int)B, (int)C, (int)L, g, eps, dx, tg);
  return launch_status("tvq_fe_channel_layernorm_bwd");
}

extern "C" int tvq_fe_linear_attention_bwd(const float* qkv, const float* dout, int64_t B,
                                           int64_t H, int64_t dh, int64_t n, float* dqkv,
                                           tvq_stream_t stream) {
  TVQ_CHECK_ARG(qkv && dout && dqkv && dh == DH && B > 0 && H > 0 && n > 0,
                "tvq_fe_linear_attention_bwd: bad arguments");
  const size_t lds = ((size_t)3 * DH * (n + 1) + 2 * DH * (DH + 1)) * 4;
  TVQ_CHECK_ARG(lds <= 160 * 1024, "tvq_fe_linear_attention_bwd: n too large");
  fe_train_lds_attr();
  hipLaunchKernelGGL(fe_linattn_bwd_kernel, dim3((unsigned)(B * H)), dim3(256), lds,
                     (hipStream_t)stream, qkv, dout, (int)H, (int)n, 1.0f / sqrtf((float)DH),
                     dqkv);
  return launch_status("tvq_fe_linear_attention_bwd");
}

extern "C" int tvq_fe_attention_bwd(const float* qkv, const float* dout, int64_t B, int64_t H,
                                    int64_t dh, int64_t n, float* dqkv, tvq_stream_t stream) {
  TVQ_CHECK_ARG(qkv && dout && dqkv && dh == DH && B > 0 && H > 0 && n > 0,
                "tvq_fe_attention_bwd: bad arguments");
  const size_t lds = ((size_t)4 * n * DH + 2 * n * (n + 1)) * 4;
  TVQ_CHECK_ARG(lds <= 160 * 1024, "tvq_fe_attention_bwd: n too large");
  fe_train_lds_attr();
  hipLaunchKernelGGL(fe_attn_bwd_kernel, dim3((unsigned)(B * H)), dim3(256), lds,
                     (hipStream_t)stream, qkv, dout, (int)H, (int)n, 1.0f / sqrtf((float)DH),
                     dqkv);
  return launch_status("tvq_fe_attention_bwd");
}

extern "C" int tvq_fe_cat_interp_bwd(const float* gout, int64_t Ca, int64_t La, int64_t Cb,
                                     int64_t Lb, int64_t B, int64_t L, float* da, float* db,
                                     tvq_stream_t stream) {
  TVQ_CHECK_ARG(gout && da && (Cb == 0 || db) && B > 0 && L > 0 && La > 0,
                "tvq_fe_cat_interp_bwd: bad arguments");
  const int64_t n = B * Ca * La + B * Cb * Lb;
  hipLaunchKernelGGL(fe_cat_interp_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, gout, (int)Ca, (int)La, (int)Cb, (int)Lb, (int)B,
                     (int)L, da, db);
  return launch_status("tvq_fe_cat_interp_bwd");
}

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

// nn.GroupNorm(G, C) (eps) then SnakeActivation (train_utils.py:446-448), + residual:
// Block.forward + ResnetBlock's `h + res_conv(x)` (fidelity_enhancer.py:193-231).  One
// block per (b, g); the group's (C/G) x L values are contiguous.
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
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += x[base + i];
  const float mean = block_sum(s, red) / (float)n;
  float q = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float d = x[base + i] - mean;
    q += d * d;
  }
  const float rstd = rsqrtf(block_sum(q, red) / (float)n + eps);
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int c = c0 + i / L;
    const float sc = rstd * gamma[c];
    float v = (x[base + i] - mean) * sc + beta[c];
    const float ac = a[c];
    v = snake_f(v, ac, 1.0f / ac);
    y[base + i] = v + (res ? res[base + i] : 0.f);
  }
}

// LayerNorm over channels, gamma only (fidelity_enhancer.py:119-127), + residual.
// One thread per (b, l); the channel loop is coalesced across l.
__global__ __launch_bounds__(256) void chan_ln_kernel(const float* __restrict__ x, int B, int C,
                                                      int L, const float* __restrict__ g,
                                                      float eps, const float* __restrict__ res,
                                                      float* __restrict__ y) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * L) return;
  const int b = t / L, l = t - b * L;
  const float* xb = x + (int64_t)b * C * L + l;
  float s = 0.f;
  for (int c = 0; c < C; ++c) s += xb[(int64_t)c * L];
  const float mean = s / (float)C;
  float q = 0.f;
  for (int c = 0; c < C; ++c) {
    const float d = xb[(int64_t)c * L] - mean;
    q += d * d;
  }
  const float rstd = rsqrtf(q / (float)C + eps);
  for (int c = 0; c < C; ++c) {
    const int64_t at = (int64_t)b * C * L + (int64_t)c * L + l;
    y[at] = (x[at] - mean) * rstd * g[c] + (res ? res[at] : 0.f);
  }
}

// LinearAttention core (fidelity_enhancer.py:245-260) for one (b, h), dh = 32:
//   k <- softmax over n, q <- softmax over d * dh^-1/2,
//   ctx[d, e] = sum_n k[d, n] v[e, n],  out[e, n] = sum_d ctx[d, e] q[d, n].
// qkv (B, 3 H dh, n) as to_qkv writes it (chunk order q, k, v; head-major channels).
constexpr int FE_DH = 32;
__global__ __launch_bounds__(256) void linear_attn_kernel(const float* __restrict__ qkv, int H,
                                                          int n, float scale,
                                                          float* __restrict__ out) {
  extern __shared__ float sm[];
  const int ld = n + 1;  // padded row stride: the context loop reads v[e][*] across lanes
  float* ks = sm;
  float* vs = sm + FE_DH * ld;
  float* ctx = vs + FE_DH * ld;  // FE_DH x (FE_DH + 1)
  const int b = blockIdx.x / H, h = blockIdx.x - b * H;
  const int HD = H * FE_DH;
  const float* q = qkv + ((int64_t)b * 3 * HD + h * FE_DH) * n;
  const float* k = q + (int64_t)HD * n;
  const float* v = k + (int64_t)HD * n;
  for (int i = threadIdx.x; i < FE_DH * n; i += blockDim.x) {
    const int d = i / n, j = i - d * n;
    ks[d * ld + j] = k[i];
    vs[d * ld + j] = v[i];
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
    const int e = threadIdx.x & 31, d0 = threadIdx.x >> 5;  // 8 x 32 threads, 4 d each
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < n; ++j) {
      const float vv = vs[e * ld + j];
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] = fmaf(ks[(d0 + 8 * r) * ld + j], vv, acc[r]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) ctx[(d0 + 8 * r) * (FE_DH + 1) + e] = acc[r];
  }
  __syncthreads();
  float* ob = out + ((int64_t)b * HD + h * FE_DH) * n;
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    float qd[FE_DH];
    float m = -INFINITY;
#pragma unroll
    for (int d = 0; d < FE_DH; ++d) {
      qd[d] = q[(int64_t)d * n + j];
      m = fmaxf(m, qd[d]);
    }
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < FE_DH; ++d) {
      qd[d] = expf(qd[d] - m);
      s += qd[d];
    }
#pragma unroll
    for (int d = 0; d < FE_DH; ++d) qd[d] = qd[d] / s * scale;
#pragma unroll 4
    for (int e = 0; e < FE_DH; ++e) {
      float o = 0.f;
#pragma unroll
      for (int d = 0; d < FE_DH; ++d) o = fmaf(ctx[d * (FE_DH + 1) + e], qd[d], o);
      ob[(int64_t)e * n + j] = o;
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
  (void)hipFuncSetAttribute((const void*)linear_attn_kernel,
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
  hipLaunchKernelGGL(gn_snake_kernel, dim3((unsigned)(B * G)), dim3(256), 0, (hipStream_t)stream,
                     x, (int)C, (int)L, (int)G, gamma, beta, a, eps, residual, y);
  return launch_status("tvq_fe_group_norm_snake");
}

int tvq_fe_channel_layernorm(const float* x, int64_t B, int64_t C, int64_t L, const float* g,
                             float eps, const float* residual, float* y, tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && y && g && B > 0 && C > 0 && L > 0, "tvq_fe_channel_layernorm: bad arguments");
  const int64_t n = B * L;
  hipLaunchKernelGGL(chan_ln_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, x, (int)B, (int)C, (int)L, g, eps, residual, y);
  return launch_status("tvq_fe_channel_layernorm");
}

int tvq_fe_linear_attention(const float* qkv, int64_t B, int64_t H, int64_t dh, int64_t n,
                            float* out, tvq_stream_t stream) {
  TVQ_CHECK_ARG(qkv && out && B > 0 && H > 0 && n > 0 && dh == FE_DH,
                "tvq_fe_linear_attention: bad arguments (dim_head must be %d)", FE_DH);
  const int64_t lds = (2 * FE_DH * (n + 1) + FE_DH * (FE_DH + 1)) * (int64_t)sizeof(float);
  TVQ_CHECK_ARG(lds <= 160 * 1024, "tvq_fe_linear_attention: n %lld exceeds LDS", (long long)n);
  fe_lds_attr();
  hipLaunchKernelGGL(linear_attn_kernel, dim3((unsigned)(B * H)), dim3(256), (size_t)lds,
                     (hipStream_t)stream, qkv, (int)H, (int)n, 1.0f / sqrtf((float)dh), out);
  return launch_status("tvq_fe_linear_attention");
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

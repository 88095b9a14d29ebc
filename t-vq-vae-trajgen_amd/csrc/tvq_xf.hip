// MaskGIT bidirectional-transformer kernels (K11-K16 in SURVEY.md §2.2).
//
//  rmsnorm     x-transformers RMSNorm: F.normalize(x) * sqrt(D) * g
//  layernorm   LayerNorm over the last dim (gamma [+ beta]), eps given
//  (attention: tvq_attn.hip)
//  embedding   table gather (+ dropout on non-mask tokens) and a deterministic
//              per-row scatter-add backward (no float atomics)
//  masked CE   cross_entropy over the masked positions (maskgit.py:183-191)
//  mask tokens _randomly_mask_tokens (maskgit.py:194-216) fully on device
//  upsample    F.interpolate(mode='nearest') along the last dim and its backward
//  gelu        elementwise GELU(erf) fwd/bwd
#include <float.h>
#include <math.h>

#include "tvq_common.h"
#include "tvq_conv_internal.h"
#include "tvq_reduce.h"

namespace tvq {

__device__ __forceinline__ float gelu_f(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f));
}
__device__ __forceinline__ float gelu_grad(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752440f));
  const float pdf = 0.39894228040143267794f * expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// ------------------------------------------------------------------ RMSNorm
// one wave per row
__global__ void rmsnorm_fwd_kernel(const float* __restrict__ x, int64_t M, int D,
                                   const float* __restrict__ g, float scale, float* __restrict__ y,
                                   float* __restrict__ inv_norm) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= M) return;
  const float* xr = x + row * D;
  float s = 0.f;
  for (int d = lane; d < D; d += 64) s += xr[d] * xr[d];
  s = wave_sum(s);
  const float inv = 1.0f / fmaxf(sqrtf(s), 1e-12f);
  for (int d = lane; d < D; d += 64) y[row * D + d] = xr[d] * inv * scale * g[d];
  if (lane == 0) inv_norm[row] = inv;
}

// Narrow rows (D = 4L, L in {8, 16, 32, 64} lanes): one float4 per lane, 64 / L rows per
// wave, the row sum over its L lanes by xor shuffles.  The one-wave-per-row form above
// left half to 7/8 of the lanes idle on the HF prior's D = 32 rows and issued one 4-B load
// per element (42 us for 1024 x 97 rows while sampling, ~0.3 TB/s).
template <int L>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = L / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int L>
__global__ __launch_bounds__(256) void rmsnorm_fwd_vec_kernel(const float4* __restrict__ x,
                                                              int64_t M,
                                                              const float4* __restrict__ g,
                                                              float scale, float4* __restrict__ y,
                                                              float* __restrict__ inv_norm) {
  const int lane = threadIdx.x & 63, sub = lane % L;
  const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 / L) + lane / L;
  const bool ok = row < M;
  const float4 v = ok ? x[row * L + sub] : make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 gv = g[sub];
  float s = v.x * v.x;
  s = fmaf(v.y, v.y, s);
  s = fmaf(v.z, v.z, s);
  s = fmaf(v.w, v.w, s);
  s = group_sum<L>(s);
  const float inv = 1.0f / fmaxf(sqrtf(s), 1e-12f);
  if (!ok) return;
  y[row * L + sub] = make_float4(v.x * inv * scale * gv.x, v.y * inv * scale * gv.y,
                                 v.z * inv * scale * gv.z, v.w * inv * scale * gv.w);
  if (sub == 0) inv_norm[row] = inv;
}

template <int L>
__global__ __launch_bounds__(256) void layernorm_fwd_vec_kernel(
    const float4* __restrict__ x, int64_t M, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float4* __restrict__ y, float* __restrict__ mean_out,
    float* __restrict__ rstd_out) {
  constexpr int D = 4 * L;
  const int lane = threadIdx.x & 63, sub = lane % L;
  const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 / L) + lane / L;
  const bool ok = row < M;
  const float4 v = ok ? x[row * L + sub] : make_float4(0.f, 0.f, 0.f, 0.f);
  const float mean = group_sum<L>((v.x + v.y) + (v.z + v.w)) / (float)D;
  const float t0 = v.x - mean, t1 = v.y - mean, t2 = v.z - mean, t3 = v.w - mean;
  float q = t0 * t0;
  q = fmaf(t1, t1, q);
  q = fmaf(t2, t2, q);
  q = fmaf(t3, t3, q);
  const float var = group_sum<L>(q) / (float)D;
  const float rstd = 1.0f / sqrtf(var + eps);
  if (!ok) return;
  const int d = 4 * sub;
  const float4 gm = gamma ? *reinterpret_cast<const float4*>(gamma + d) : make_float4(1.f, 1.f, 1.f, 1.f);
  float4 o = make_float4(t0 * rstd * gm.x, t1 * rstd * gm.y, t2 * rstd * gm.z, t3 * rstd * gm.w);
  if (beta) {
    const float4 bt = *reinterpret_cast<const float4*>(beta + d);
    o.x += bt.x; o.y += bt.y; o.z += bt.z; o.w += bt.w;
  }
  y[row * L + sub] = o;
  if (sub == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

static bool a16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// dx; and per-block partial dg (deterministic, reduced by colsum_kernel)
__global__ void rmsnorm_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                   int64_t M, int D, const float* __restrict__ g, float scale,
                                   const float* __restrict__ inv_norm,
                                   const float* __restrict__ dres, float* __restrict__ dx,
                                   float* __restrict__ dg_part, int rows_per_block) {
  extern __shared__ float sh[];  // [waves][D] partial dg
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int d = threadIdx.x; d < nw * D; d += blockDim.x) sh[d] = 0.f;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  for (int64_t row = r0 + wid; row < min(M, r0 + rows_per_block); row += nw) {
    const float* xr = x + row * D;
    const float* gr = dy + row * D;
    const float inv = inv_norm[row];
    // y = x * inv * scale * g ; norm = 1/inv (assumes ||x|| > 1e-12)
    float dot = 0.f;
    for (int d = lane; d < D; d += 64) dot += gr[d] * g[d] * xr[d];
    dot = wave_sum(dot);
    const float c = dot * scale * inv * inv * inv;
    for (int d = lane; d < D; d += 64) {
      const float v = gr[d] * g[d] * scale * inv - xr[d] * c;
      dx[row * D + d] = dres ? v + dres[row * D + d] : v;  // + the residual path's gradient
      sh[wid * D + d] += gr[d] * xr[d] * inv * scale;
    }
  }
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float s = 0.f;
    for (int w = 0; w < nw; ++w) s += sh[w * D + d];
    dg_part[(int64_t)blockIdx.x * D + d] = s;
  }
}

// The same backward with each row held in registers (D <= 64 ND): a wave loads its next
// row while it reduces and stores the current one (the loop above pays two dependent
// load round trips per row).  Every sum has the loop above's order: bitwise equal.
template <int ND>
__global__ __launch_bounds__(256) void rmsnorm_bwd_reg_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, int64_t M, int D,
    const float* __restrict__ g, float scale, const float* __restrict__ inv_norm,
    const float* __restrict__ dres, float* __restrict__ dx, float* __restrict__ dg_part,
    int rows_per_block) {
  extern __shared__ float sh[];  // [waves][D] partial dg
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int d = threadIdx.x; d < nw * D; d += blockDim.x) sh[d] = 0.f;
  float gv[ND];
#pragma unroll
  for (int j = 0; j < ND; ++j) gv[j] = lane + 64 * j < D ? g[lane + 64 * j] : 0.f;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  float cx[ND], cg[ND], cr[ND], nx[ND], ng[ND], nr[ND];
  float cinv = 0.f, ninv = 0.f;
  auto load = [&](int64_t row, float(&xv)[ND], float(&gvv)[ND], float(&rv)[ND], float& inv) {
    const int64_t rr = row < r1 ? row : r0;  // past the block's rows: a valid row, unused
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const int d = lane + 64 * j;
      const int64_t o = rr * D + (d < D ? d : 0);
      xv[j] = x[o];
      gvv[j] = dy[o];
      rv[j] = dres ? dres[o] : 0.f;
    }
    inv = inv_norm[rr];
  };
  int64_t row = r0 + wid;
  if (row < r1) load(row, cx, cg, cr, cinv);
  for (; row < r1; row += nw) {
    load(row + nw, nx, ng, nr, ninv);
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < ND; ++j)
      if (lane + 64 * j < D) dot += cg[j] * gv[j] * cx[j];
    dot = wave_sum(dot);
    const float c = dot * scale * cinv * cinv * cinv;
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const int d = lane + 64 * j;
      if (d < D) {
        const float v = cg[j] * gv[j] * scale * cinv - cx[j] * c;
        dx[row * D + d] = dres ? v + cr[j] : v;
        sh[wid * D + d] += cg[j] * cx[j] * cinv * scale;
      }
    }
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      cx[j] = nx[j];
      cg[j] = ng[j];
      cr[j] = nr[j];
    }
    cinv = ninv;
  }
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float s = 0.f;
    for (int w = 0; w < nw; ++w) s += sh[w * D + d];
    dg_part[(int64_t)blockIdx.x * D + d] = s;
  }
}

// D <= 32 (the HF prior): each half-wave takes a row, so a wave runs two rows at a time
// (the one-row form left half of every wave idle); per-half dg partials in LDS.
__global__ __launch_bounds__(256) void rmsnorm_bwd_half_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, int64_t M, int D,
    const float* __restrict__ g, float scale, const float* __restrict__ inv_norm,
    const float* __restrict__ dres, float* __restrict__ dx, float* __restrict__ dg_part,
    int rows_per_block) {
  extern __shared__ float sh[];  // [2 * waves][D] partial dg
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int hl = lane >> 5, d = lane & 31;
  const int slot = 2 * wid + hl, nslot = 2 * nw;
  for (int i = threadIdx.x; i < nslot * D; i += blockDim.x) sh[i] = 0.f;
  const float gv = d < D ? g[d] : 0.f;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  float cx, cg, cr, cinv, nx, ng, nr, ninv;
  auto load = [&](int64_t row, float& xv, float& gg, float& rv, float& inv) {
    const int64_t rr = row < r1 ? row : r0;
    const int64_t o = rr * D + (d < D ? d : 0);
    xv = x[o];
    gg = dy[o];
    rv = dres ? dres[o] : 0.f;
    inv = inv_norm[rr];
  };
  int64_t row = r0 + slot;
  load(row, cx, cg, cr, cinv);
  for (; row - hl < r1; row += nslot) {  // both halves iterate together (wave-uniform trip)
    load(row + nslot, nx, ng, nr, ninv);
    const bool live = row < r1 && d < D;
    float dot = live ? cg * gv * cx : 0.f;
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) dot += __shfl_xor(dot, o, 64);
    const float c = dot * scale * cinv * cinv * cinv;
    if (live) {
      const float v = cg * gv * scale * cinv - cx * c;
      dx[row * D + d] = dres ? v + cr : v;
      sh[slot * D + d] += cg * cx * cinv * scale;
    }
    cx = nx;
    cg = ng;
    cr = nr;
    cinv = ninv;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < D; i += blockDim.x) {
    float t = 0.f;
    for (int w = 0; w < nslot; ++w) t += sh[w * D + i];
    dg_part[(int64_t)blockIdx.x * D + i] = t;
  }
}

// out[d] (+)= sum_p part[p][d]
__global__ void colsum_kernel(const float* __restrict__ part, int P, int D, float* __restrict__ out,
                              int accumulate) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= D) return;
  float s = 0.f;
  for (int p = 0; p < P; ++p) s += part[(int64_t)p * D + d];
  out[d] = accumulate ? out[d] + s : s;
}

// ---------------------------------------------------------------- LayerNorm
__global__ void layernorm_fwd_kernel(const float* __restrict__ x, int64_t M, int D,
                                     const float* __restrict__ gamma,
                                     const float* __restrict__ beta, float eps,
                                     float* __restrict__ y, float* __restrict__ mean_out,
                                     float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= M) return;
  const float* xr = x + row * D;
  float s = 0.f;
  for (int d = lane; d < D; d += 64) s += xr[d];
  const float mean = wave_sum(s) / (float)D;
  float v = 0.f;
  for (int d = lane; d < D; d += 64) {
    const float t = xr[d] - mean;
    v += t * t;
  }
  const float var = wave_sum(v) / (float)D;
  const float rstd = 1.0f / sqrtf(var + eps);
  for (int d = lane; d < D; d += 64) {
    float t = (xr[d] - mean) * rstd * (gamma ? gamma[d] : 1.f);
    if (beta) t += beta[d];
    y[row * D + d] = t;
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

__global__ void layernorm_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                     int64_t M, int D, const float* __restrict__ gamma,
                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                     float* __restrict__ dx, float* __restrict__ part,
                                     int rows_per_block) {
  extern __shared__ float sh[];  // [waves][2][D]: dgamma, dbeta partials
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int d = threadIdx.x; d < nw * 2 * D; d += blockDim.x) sh[d] = 0.f;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  for (int64_t row = r0 + wid; row < min(M, r0 + rows_per_block); row += nw) {
    const float* xr = x + row * D;
    const float* gr = dy + row * D;
    const float mu = mean[row], rs = rstd[row];
    float s1 = 0.f, s2 = 0.f;
    for (int d = lane; d < D; d += 64) {
      const float xh = (xr[d] - mu) * rs;
      const float gg = gr[d] * (gamma ? gamma[d] : 1.f);
      s1 += gg;
      s2 += gg * xh;
      sh[(wid * 2) * D + d] += gr[d] * xh;
      sh[(wid * 2 + 1) * D + d] += gr[d];
    }
    s1 = wave_sum(s1) / (float)D;
    s2 = wave_sum(s2) / (float)D;
    for (int d = lane; d < D; d += 64) {
      const float xh = (xr[d] - mu) * rs;
      const float gg = gr[d] * (gamma ? gamma[d] : 1.f);
      dx[row * D + d] = rs * (gg - s1 - xh * s2);
    }
  }
  __syncthreads();
  for (int d = threadIdx.x; d < 2 * D; d += blockDim.x) {
    const int k = d / D, dd = d - k * D;
    float s = 0.f;
    for (int w = 0; w < nw; ++w) s += sh[(w * 2 + k) * D + dd];
    part[((int64_t)k * gridDim.x + blockIdx.x) * D + dd] = s;  // [gamma | beta][block][D]
  }
}

// The same backward with each row in registers (D <= 64 ND) and the next row loading
// while the current one reduces; the sums keep the loop above's order (bitwise equal).
template <int ND>
__global__ __launch_bounds__(256) void layernorm_bwd_reg_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, int64_t M, int D,
    const float* __restrict__ gamma, const float* __restrict__ mean,
    const float* __restrict__ rstd, float* __restrict__ dx, float* __restrict__ part,
    int rows_per_block) {
  extern __shared__ float sh[];  // [waves][2][D]: dgamma, dbeta partials
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int d = threadIdx.x; d < nw * 2 * D; d += blockDim.x) sh[d] = 0.f;
  float gm[ND];
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    const int d = lane + 64 * j;
    gm[j] = gamma && d < D ? gamma[d] : 1.f;
  }
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  float cx[ND], cg[ND], nx[ND], ng[ND];
  float cmu = 0.f, crs = 0.f, nmu = 0.f, nrs = 0.f;
  auto load = [&](int64_t row, float(&xv)[ND], float(&gv)[ND], float& mu, float& rs) {
    const int64_t rr = row < r1 ? row : r0;  // past the block's rows: a valid row, unused
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const int d = lane + 64 * j;
      const int64_t o = rr * D + (d < D ? d : 0);
      xv[j] = x[o];
      gv[j] = dy[o];
    }
    mu = mean[rr];
    rs = rstd[rr];
  };
  int64_t row = r0 + wid;
  if (row < r1) load(row, cx, cg, cmu, crs);
  for (; row < r1; row += nw) {
    load(row + nw, nx, ng, nmu, nrs);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const int d = lane + 64 * j;
      if (d < D) {
        const float xh = (cx[j] - cmu) * crs;
        const float gg = cg[j] * gm[j];
        s1 += gg;
        s2 += gg * xh;
        sh[(wid * 2) * D + d] += cg[j] * xh;
        sh[(wid * 2 + 1) * D + d] += cg[j];
      }
    }
    s1 = wave_sum(s1) / (float)D;
    s2 = wave_sum(s2) / (float)D;
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const int d = lane + 64 * j;
      if (d < D) {
        const float xh = (cx[j] - cmu) * crs;
        const float gg = cg[j] * gm[j];
        dx[row * D + d] = crs * (gg - s1 - xh * s2);
      }
    }
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      cx[j] = nx[j];
      cg[j] = ng[j];
    }
    cmu = nmu;
    crs = nrs;
  }
  __syncthreads();
  for (int d = threadIdx.x; d < 2 * D; d += blockDim.x) {
    const int k = d / D, dd = d - k * D;
    float s = 0.f;
    for (int w = 0; w < nw; ++w) s += sh[(w * 2 + k) * D + dd];
    part[((int64_t)k * gridDim.x + blockIdx.x) * D + dd] = s;  // [gamma | beta][block][D]
  }
}

// dgamma[d] (+)= sum_p ws[p][0][d], dbeta[d] (+)= sum_p ws[p][1][d]
__global__ void ln_colsum2_kernel(const float* __restrict__ ws, int P, int D,
                                  float* __restrict__ dgamma, float* __restrict__ dbeta,
                                  int accumulate) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= 2 * D) return;
  const int k = e / D, d = e - k * D;
  float* dst = k == 0 ? dgamma : dbeta;
  if (!dst) return;
  float s = 0.f;
  for (int p = 0; p < P; ++p) s += ws[((int64_t)p * 2 + k) * D + d];
  dst[d] = accumulate ? dst[d] + s : s;
}

// ---------------------------------------------------------------- embedding
// out[m, :] = table[idx[m], :]  (* dropout where idx[m] != keep_id) ; out row stride ldo
__global__ void embedding_fwd_kernel(const int64_t* __restrict__ idx, int64_t M, int D,
                                     const float* __restrict__ table, float* __restrict__ out,
                                     int64_t ldo, int64_t mask_id, float drop_p,
                                     const int64_t* seed_ptr, uint64_t offset) {
  const uint64_t seed = drop_p > 0.f ? mix_seed(seed_ptr, offset) : 0ull;
  const float sc = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
  const int64_t tot = M * D;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < tot;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = e / D;
    const int d = (int)(e - m * D);
    const int64_t t = idx[m];
    float v = table[t * D + d];
    if (drop_p > 0.f && t != mask_id) v = uniform01(seed, (uint64_t)e) >= drop_p ? v * sc : 0.f;
    out[m * ldo + d] = v;
  }
}

// ---------------------------------------------------------------- masked CE
// per row (one wave): if !keep[m]: loss_m = lse(logits[m,:K]) - logits[m, t]; part sums
__global__ __launch_bounds__(256) void masked_ce_fwd_kernel(const float* __restrict__ logits,
                                                            int64_t ldl, int64_t M, int K,
                                                            const int64_t* __restrict__ target,
                                                            const bool* __restrict__ keep,
                                                            float* __restrict__ lse_out,
                                                            float* __restrict__ part) {
  __shared__ float red[2][4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float ls = 0.f, cnt = 0.f;
  for (int64_t m = (int64_t)blockIdx.x * 4 + wid; m < M; m += (int64_t)gridDim.x * 4) {
    if (keep[m]) continue;  // only masked positions contribute
    const float* lr = logits + m * ldl;
    float mx = -INFINITY;
    for (int k = lane; k < K; k += 64) mx = fmaxf(mx, lr[k]);
    mx = wave_max(mx);
    float s = 0.f;
    for (int k = lane; k < K; k += 64) s += expf(lr[k] - mx);
    s = wave_sum(s);
    const float lse = mx + logf(s);
    if (lane == 0) {
      lse_out[m] = lse;
      ls += lse - lr[target[m]];
      cnt += 1.f;
    }
  }
  if (lane == 0) { red[0][wid] = ls; red[1][wid] = cnt; }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    part[2 * blockIdx.x + 1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  }
}

__global__ __launch_bounds__(256) void masked_ce_final_kernel(const float* __restrict__ part, int P,
                                                              float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f, c = 0.f;
  for (int i = threadIdx.x; i < P; i += 256) { s += part[2 * i]; c += part[2 * i + 1]; }
  s = block_sum(s, red);
  c = block_sum(c, red);
  if (threadIdx.x == 0) { out[0] = s / c; out[1] = c; }
}

void masked_ce_final(const float* part, int P, float* out, hipStream_t st) {
  hipLaunchKernelGGL(masked_ce_final_kernel, dim3(1), dim3(256), 0, st, part, P, out);
}

// dlogits[m,k] = keep[m] ? 0 : g/cnt * (softmax - onehot)
__global__ void masked_ce_bwd_kernel(const float* __restrict__ logits, int64_t ldl, int64_t M, int K,
                                     const int64_t* __restrict__ target,
                                     const bool* __restrict__ keep, const float* __restrict__ lse,
                                     const float* __restrict__ stats, const float* __restrict__ gout,
                                     float* __restrict__ dlogits, int64_t ldd) {
  const float gc = gout[0] / stats[1];
  const int64_t tot = M * K;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < tot;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = e / K;
    const int k = (int)(e - m * K);
    float v = 0.f;
    if (!keep[m]) {
      v = expf(logits[m * ldl + k] - lse[m]);
      if (k == target[m]) v -= 1.0f;
      v *= gc;
    }
    dlogits[m * ldd + k] = v;
  }
}

// ---------------------------------------------------------------- masking
// maskgit.py:194-216 on device.  Per row: ratio ~ U[0,1); n_unmask =
// clip(floor(cos(ratio*pi/2) * n), 0, n-1); keep the n_unmask positions with the
// largest U[0,1) scores (ties -> lower index, like torch.topk).  s_M = keep ? s : mask_id.
__global__ void mask_tokens_kernel(const int64_t* __restrict__ s, int B, int n, int64_t mask_id,
                                   const int64_t* seed_ptr, uint64_t offset,
                                   const double* __restrict__ ratio_in,
                                   const float* __restrict__ rand_in, int64_t* __restrict__ s_M,
                                   bool* __restrict__ keep) {
  extern __shared__ float sc[];  // [n]
  const int b = blockIdx.x;
  const uint64_t seed = mix_seed(seed_ptr, offset);
  for (int j = threadIdx.x; j < n; j += blockDim.x)
    sc[j] = rand_in ? rand_in[(int64_t)b * n + j] : uniform01(seed, (uint64_t)b * (n + 1) + 1 + j);
  __syncthreads();
  const double ratio = ratio_in ? ratio_in[b] : (double)uniform01(seed, (uint64_t)b * (n + 1));
  // numpy float64 in the reference: floor(cos(r*pi/2) * n), clip to [0, n-1]
  double nu = floor(cos(ratio * 3.14159265358979323846 / 2.0) * (double)n);
  nu = fmin(fmax(nu, 0.0), (double)(n - 1));
  const int n_unmask = (int)nu;
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    const float v = sc[j];
    int rank = 0;
    for (int k = 0; k < n; ++k) rank += (sc[k] > v) || (sc[k] == v && k < j);
    const bool kp = rank < n_unmask;
    keep[(int64_t)b * n + j] = kp;
    s_M[(int64_t)b * n + j] = kp ? s[(int64_t)b * n + j] : mask_id;
  }
}

// ---------------------------------------------------------------- misc
// nearest interpolation along the last dim: out[r, j] = in[r, floor(j * scale)]
__global__ void upsample_nearest_kernel(const float* __restrict__ x, int64_t R, int Lin, int Lout,
                                        float scale, float* __restrict__ y) {
  const int64_t tot = R * Lout;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < tot;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / Lout;
    const int j = (int)(e - r * Lout);
    int src = (int)floorf((float)j * scale);
    if (src > Lin - 1) src = Lin - 1;
    y[e] = x[r * Lin + src];
  }
}

__global__ void upsample_nearest_bwd_kernel(const float* __restrict__ dy, int64_t R, int Lin,
                                            int Lout, float scale, float* __restrict__ dx) {
  const int64_t tot = R * Lin;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < tot;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / Lin;
    const int i = (int)(e - r * Lin);
    float s = 0.f;
    // outputs j with floor(j*scale) == i
    int j0 = (int)floorf((float)i / scale) - 2;
    if (j0 < 0) j0 = 0;
    for (int j = j0; j < Lout; ++j) {
      int src = (int)floorf((float)j * scale);
      if (src > Lin - 1) src = Lin - 1;
      if (src > i) break;
      if (src == i) s += dy[r * Lout + j];
    }
    dx[e] = s;
  }
}

__global__ void gelu_fwd_kernel(const float* __restrict__ x, int64_t n, float* __restrict__ y) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] = gelu_f(x[i]);
}
__global__ void gelu_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x, int64_t n,
                                float* __restrict__ dx) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dx[i] = dy[i] * gelu_grad(x[i]);
}

static int grid_for(int64_t n, int cap = 8192) {
  int64_t b = (n + 255) / 256;
  if (b < 1) b = 1;
  return (int)(b < cap ? b : cap);
}

static int norm_rows_per_block(int64_t M) {
  // ~256 blocks of rows for the deterministic partial-sum backward
  int64_t r = (M + 255) / 256;
  return (int)(r < 4 ? 4 : r);
}


// ------------------------------------------------------- embedding assembly
// bidirectional_transformer.py:185,229-231: embed = cat(cls_emb, tok + pos_emb[:n], dim=1)
// with tok = [t1 | t2] along features (HF: Upscale(LF emb) | HF emb; LF: t1 only).
// Token inputs are read through strides (the Upscale output is a (b, m, d) view of a
// (b, d, m) tensor); the backward writes their gradients with the same strides.
struct AsmTok {
  const float* p;
  float* g;
  int64_t sb, sn, sd;
  int D;
};

__global__ void embed_assemble_kernel(const float* __restrict__ cls, AsmTok t1, AsmTok t2,
                                      const float* __restrict__ pos, int B, int n,
                                      float* __restrict__ out) {
  const int Dt = t1.D + t2.D;
  const int64_t tot = (int64_t)B * (n + 1) * Dt;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < tot;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int d = (int)(e % Dt);
    const int64_t r = e / Dt;
    const int i = (int)(r % (n + 1));
    const int b = (int)(r / (n + 1));
    float v;
    if (i == 0) {
      v = cls[(int64_t)b * Dt + d];
    } else {
      const int j = i - 1;
      const float tv = d < t1.D ? t1.p[b * t1.sb + j * t1.sn + d * t1.sd]
                                : t2.p[b * t2.sb + j * t2.sn + (d - t1.D) * t2.sd];
      v = tv + pos[(int64_t)j * Dt + d];
    }
    out[e] = v;
  }
}

// dcls[b, d] = dout[b, 0, d]; dt[b, j, d] = dout[b, 1 + j, d] (through the tokens' strides)
__global__ void embed_assemble_split_kernel(const float* __restrict__ dout, int B, int n,
                                            float* __restrict__ dcls, AsmTok t1, AsmTok t2) {
  const int Dt = t1.D + t2.D;
  const int64_t tot = (int64_t)B * (n + 1) * Dt;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < tot;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int d = (int)(e % Dt);
    const int64_t r = e / Dt;
    const int i = (int)(r % (n + 1));
    const int b = (int)(r / (n + 1));
    const float v = dout[e];
    if (i == 0) {
      if (dcls) dcls[(int64_t)b * Dt + d] = v;
    } else if (d < t1.D) {
      if (t1.g) t1.g[b * t1.sb + (i - 1) * t1.sn + d * t1.sd] = v;
    } else if (t2.g) {
      t2.g[b * t2.sb + (i - 1) * t2.sn + (d - t1.D) * t2.sd] = v;
    }
  }
}

// bidirectional_transformer.py:124-150 class conditioning in training: idx[b] = y[b] where
// u_b > p_unconditional, else the null class; u_b injected (tests) or drawn from the
// device counter RNG
__global__ void class_index_kernel(const int64_t* __restrict__ y, int B, float p, int64_t null_id,
                                   const int64_t* __restrict__ seed_ptr, uint64_t offset,
                                   const float* __restrict__ rnd, int64_t* __restrict__ idx) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float u = rnd ? rnd[b] : uniform01(mix_seed(seed_ptr, offset), (uint64_t)b);
  idx[b] = u > p ? y[b] : null_id;
}

// Upscale's transpose + nearest upsample in one pass: x (B, Lin, D) (the token layout)
// -> y (B, D, Lout); backward dy (B, D, Lout) -> dx (B, Lin, D)
__global__ void upsample_nearest_t_kernel(const float* __restrict__ x, int B, int Lin, int D,
                                          int Lout, float scale, float* __restrict__ y) {
  const int64_t tot = (int64_t)B * D * Lout;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < tot;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(e % Lout);
    const int64_t r = e / Lout;
    const int d = (int)(r % D);
    const int b = (int)(r / D);
    int src = (int)floorf((float)j * scale);
    if (src > Lin - 1) src = Lin - 1;
    y[e] = x[((int64_t)b * Lin + src) * D + d];
  }
}

__global__ void upsample_nearest_t_bwd_kernel(const float* __restrict__ dy, int B, int Lin, int D,
                                              int Lout, float scale, float* __restrict__ dx) {
  const int64_t tot = (int64_t)B * Lin * D;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < tot;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int d = (int)(e % D);
    const int64_t r = e / D;
    const int i = (int)(r % Lin);
    const int b = (int)(r / Lin);
    const float* row = dy + ((int64_t)b * D + d) * Lout;
    float s = 0.f;
    int j0 = (int)floorf((float)i / scale) - 2;  // outputs j with floor(j*scale) == i
    if (j0 < 0) j0 = 0;
    for (int j = j0; j < Lout; ++j) {
      int src = (int)floorf((float)j * scale);
      if (src > Lin - 1) src = Lin - 1;
      if (src > i) break;
      if (src == i) s += row[j];
    }
    dx[e] = s;
  }
}

// Same gradient, one block per (b, 64-channel tile): lanes walk consecutive i (so the dY
// rows are read along j, coalesced) with the per-element loop above, the tile goes through
// LDS and is written token-major with lanes along d.  Lin <= 128.
constexpr int UPT_D = 64;
__global__ __launch_bounds__(256) void upsample_nearest_t_bwd_tile_kernel(
    const float* __restrict__ dy, int Lin, int D, int Lout, float scale, float* __restrict__ dx) {
  __shared__ float T[128 * (UPT_D + 1)];
  const int dtiles = (D + UPT_D - 1) / UPT_D;
  const int b = blockIdx.x / dtiles, d0 = (blockIdx.x - b * dtiles) * UPT_D;
  for (int e = threadIdx.x; e < UPT_D * Lin; e += 256) {
    const int dd = e / Lin, i = e - dd * Lin, d = d0 + dd;
    float s = 0.f;
    if (d < D) {
      const float* row = dy + ((int64_t)b * D + d) * Lout;
      int j0 = (int)floorf((float)i / scale) - 2;
      if (j0 < 0) j0 = 0;
      for (int j = j0; j < Lout; ++j) {
        int src = (int)floorf((float)j * scale);
        if (src > Lin - 1) src = Lin - 1;
        if (src > i) break;
        if (src == i) s += row[j];
      }
    }
    T[i * (UPT_D + 1) + dd] = s;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < UPT_D * Lin; e += 256) {
    const int i = e / UPT_D, dd = e - i * UPT_D;
    if (d0 + dd < D) dx[((int64_t)b * Lin + i) * D + d0 + dd] = T[i * (UPT_D + 1) + dd];
  }
}

// out[j*ldo + d] (+)= sum_b in[b*sb + j*sj + d]: batch sums of position tables (the
// tied-logits bias (n, K+1), the position embedding).  Block = 32 columns x 8 batch parts:
// part q sums its images in order, then the 8 partials are added in part order (a fixed
// order, bitwise reproducible); one thread per column summing all B serially left the
// launch at 50-200 blocks and 15 us.
constexpr int BCS_COLS = 32, BCS_PARTS = 8;
__global__ __launch_bounds__(256) void batch_colsum8_kernel(const float* __restrict__ in, int B,
                                                            int64_t sb, int n, int64_t sj, int D,
                                                            float* __restrict__ out, int64_t ldo,
                                                            int accumulate) {
  __shared__ float part[BCS_PARTS][BCS_COLS];
  const int c = threadIdx.x % BCS_COLS, q = threadIdx.x / BCS_COLS;
  const int64_t e = (int64_t)blockIdx.x * BCS_COLS + c;
  const bool ok = e < (int64_t)n * D;
  const int j = ok ? (int)(e / D) : 0, d = ok ? (int)(e - (int64_t)j * D) : 0;
  const int per = (B + BCS_PARTS - 1) / BCS_PARTS;
  const int b0 = q * per, b1 = min(B, b0 + per);
  const float* p = in + j * sj + d;
  float s = 0.f;
#pragma unroll 8
  for (int b = b0; b < b1; ++b) s += p[b * sb];
  part[q][c] = s;
  __syncthreads();
  if (q != 0 || !ok) return;
  float t = part[0][c];
#pragma unroll
  for (int k = 1; k < BCS_PARTS; ++k) t += part[k][c];
  float* o = out + j * ldo + d;
  *o = accumulate ? *o + t : t;
}


__global__ void scale_by_kernel(const float4* __restrict__ x, int64_t n4, const float* __restrict__ s,
                                float4* __restrict__ y) {
  const float f = *s;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = x[i];
    y[i] = make_float4(v.x * f, v.y * f, v.z * f, v.w * f);
  }
}

}  // namespace tvq

using namespace tvq;

extern "C" int tvq_embed_assemble(const float* cls, const float* t1, int64_t s1b, int64_t s1n,
                                  int64_t s1d, int64_t D1, const float* t2, int64_t s2b,
                                  int64_t s2n, int64_t s2d, int64_t D2, const float* pos,
                                  int64_t B, int64_t n, float* out, tvq_stream_t stream) {
  TVQ_CHECK_ARG(cls && t1 && pos && out && B > 0 && n > 0 && D1 > 0 && D2 >= 0 &&
                    (D2 == 0 || t2),
                "tvq_embed_assemble: bad arguments");
  const AsmTok a1 = {t1, nullptr, s1b, s1n, s1d, (int)D1};
  const AsmTok a2 = {t2, nullptr, s2b, s2n, s2d, (int)D2};
  hipLaunchKernelGGL(embed_assemble_kernel, dim3(grid_for(B * (n + 1) * (D1 + D2))), dim3(256), 0,
                     (hipStream_t)stream, cls, a1, a2, pos, (int)B, (int)n, out);
  return launch_status("tvq_embed_assemble");
}

extern "C" int tvq_embed_assemble_bwd(const float* dout, int64_t B, int64_t n, int64_t D1,
                                      int64_t D2, float* dcls, float* dt1, int64_t s1b, int64_t s1n,
                                      int64_t s1d, float* dt2, int64_t s2b, int64_t s2n,
                                      int64_t s2d, float* dpos, int64_t accumulate,
                                      tvq_stream_t stream) {
  TVQ_CHECK_ARG(dout && B > 0 && n > 0 && D1 > 0 && D2 >= 0, "tvq_embed_assemble_bwd: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  const AsmTok a1 = {nullptr, dt1, s1b, s1n, s1d, (int)D1};
  const AsmTok a2 = {nullptr, dt2, s2b, s2n, s2d, (int)D2};
  if (dcls || dt1 || dt2)
    hipLaunchKernelGGL(embed_assemble_split_kernel, dim3(grid_for(B * (n + 1) * (D1 + D2))),
                       dim3(256), 0, st, dout, (int)B, (int)n, dcls, a1, a2);
  if (dpos) {
    const int64_t Dt = D1 + D2;
    hipLaunchKernelGGL(batch_colsum8_kernel, dim3((unsigned)((n * Dt + BCS_COLS - 1) / BCS_COLS)), dim3(256), 0, st,
                       dout + Dt, (int)B, (n + 1) * Dt, (int)n, Dt, (int)Dt, dpos, Dt,
                       (int)accumulate);
  }
  return launch_status("tvq_embed_assemble_bwd");
}

extern "C" int tvq_class_index(const int64_t* y, int64_t B, float p, int64_t null_id,
                               const int64_t* seed_ptr, uint64_t offset, const float* rnd,
                               int64_t* idx, tvq_stream_t stream) {
  TVQ_CHECK_ARG(y && idx && B > 0 && (rnd || seed_ptr), "tvq_class_index: bad arguments");
  hipLaunchKernelGGL(class_index_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, y, (int)B, p, null_id, seed_ptr, offset, rnd, idx);
  return launch_status("tvq_class_index");
}

extern "C" int tvq_upsample_nearest_t(const float* x, int64_t B, int64_t Lin, int64_t D,
                                      int64_t Lout, float* y, tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && y && B > 0 && Lin > 0 && D > 0 && Lout > 0, "tvq_upsample_nearest_t: bad args");
  hipLaunchKernelGGL(upsample_nearest_t_kernel, dim3(grid_for(B * D * Lout)), dim3(256), 0,
                     (hipStream_t)stream, x, (int)B, (int)Lin, (int)D, (int)Lout,
                     (float)Lin / (float)Lout, y);
  return launch_status("tvq_upsample_nearest_t");
}

extern "C" int tvq_upsample_nearest_t_bwd(const float* dy, int64_t B, int64_t Lin, int64_t D,
                                          int64_t Lout, float* dx, tvq_stream_t stream) {
  TVQ_CHECK_ARG(dy && dx && B > 0 && Lin > 0 && D > 0 && Lout > 0,
                "tvq_upsample_nearest_t_bwd: bad args");
  if (Lin <= 128) {
    const int64_t blocks = B * ((D + UPT_D - 1) / UPT_D);
    hipLaunchKernelGGL(upsample_nearest_t_bwd_tile_kernel, dim3((unsigned)blocks), dim3(256), 0,
                       (hipStream_t)stream, dy, (int)Lin, (int)D, (int)Lout,
                       (float)Lin / (float)Lout, dx);
    return launch_status("tvq_upsample_nearest_t_bwd");
  }
  hipLaunchKernelGGL(upsample_nearest_t_bwd_kernel, dim3(grid_for(B * Lin * D)), dim3(256), 0,
                     (hipStream_t)stream, dy, (int)B, (int)Lin, (int)D, (int)Lout,
                     (float)Lin / (float)Lout, dx);
  return launch_status("tvq_upsample_nearest_t_bwd");
}

extern "C" int tvq_batch_colsum(const float* in, int64_t B, int64_t sb, int64_t n, int64_t sj,
                                int64_t D, float* out, int64_t ldo, int64_t accumulate,
                                tvq_stream_t stream) {
  TVQ_CHECK_ARG(in && out && B > 0 && n > 0 && D > 0, "tvq_batch_colsum: bad arguments");
  hipLaunchKernelGGL(batch_colsum8_kernel, dim3((unsigned)((n * D + BCS_COLS - 1) / BCS_COLS)),
                     dim3(256), 0, (hipStream_t)stream, in, (int)B, sb, (int)n, sj, (int)D, out, ldo,
                     (int)accumulate);
  return launch_status("tvq_batch_colsum");
}

extern "C" int tvq_scale_by(const float* x, int64_t n, const float* s, float* y,
                            tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && s && y && n > 0 && n % 4 == 0 && ((uintptr_t)x & 15) == 0 &&
                    ((uintptr_t)y & 15) == 0,
                "tvq_scale_by: bad arguments");
  const int64_t n4 = n / 4;
  const int blocks = (int)((n4 + 255) / 256 < 2048 ? (n4 + 255) / 256 : 2048);
  hipLaunchKernelGGL(scale_by_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                     (const float4*)x, n4, s, (float4*)y);
  return launch_status("tvq_scale_by");
}

extern "C" int tvq_rmsnorm_fwd(const float* x, int64_t M, int64_t D, const float* g, float scale,
                               float* y, float* inv_norm, tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && g && y && inv_norm && M > 0 && D > 0, "tvq_rmsnorm_fwd: bad arguments");
  if ((D == 32 || D == 64 || D == 128 || D == 256) && a16(x) && a16(g) && a16(y)) {
    const int L = (int)(D / 4), rows = 4 * (64 / L);
    const dim3 grid((unsigned)((M + rows - 1) / rows));
    hipStream_t st = (hipStream_t)stream;
    TVQ_PLAN("rmsnorm_fwd_vec D%lld", (long long)D);
#define RN_(LV)                                                                               \
  hipLaunchKernelGGL(rmsnorm_fwd_vec_kernel<LV>, grid, dim3(256), 0, st, (const float4*)x, M, \
                     (const float4*)g, scale, (float4*)y, inv_norm)
    if (L == 8) RN_(8); else if (L == 16) RN_(16); else if (L == 32) RN_(32); else RN_(64);
#undef RN_
    return launch_status("tvq_rmsnorm_fwd");
  }
  hipLaunchKernelGGL(rmsnorm_fwd_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, x, M, (int)D, g, scale, y, inv_norm);
  return launch_status("tvq_rmsnorm_fwd");
}

extern "C" int64_t tvq_norm_bwd_workspace(int64_t M, int64_t D) {
  const int rpb = norm_rows_per_block(M);
  const int64_t nb = (M + rpb - 1) / rpb;
  return nb * 2 * D + 2 * reduce_rows_scratch(nb, D);
}

extern "C" int tvq_rmsnorm_bwd(const float* dy, const float* x, int64_t M, int64_t D,
                               const float* g, float scale, const float* inv_norm,
                               const float* dres, float* dx, float* dg, int64_t accumulate,
                               float* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(dy && x && g && inv_norm && dx && dg && workspace, "tvq_rmsnorm_bwd: bad args");
  const int rpb = norm_rows_per_block(M);
  const int nb = (int)((M + rpb - 1) / rpb);
  hipStream_t st = (hipStream_t)stream;
  const size_t lds = 4 * D * sizeof(float);
  if (D <= 32)
    hipLaunchKernelGGL(rmsnorm_bwd_half_kernel, dim3(nb), dim3(256), 2 * lds, st, dy, x, M, (int)D,
                       g, scale, inv_norm, dres, dx, workspace, rpb);
  else if (D <= 64)
    hipLaunchKernelGGL(rmsnorm_bwd_reg_kernel<1>, dim3(nb), dim3(256), lds, st, dy, x, M, (int)D, g,
                       scale, inv_norm, dres, dx, workspace, rpb);
  else if (D <= 128)
    hipLaunchKernelGGL(rmsnorm_bwd_reg_kernel<2>, dim3(nb), dim3(256), lds, st, dy, x, M, (int)D, g,
                       scale, inv_norm, dres, dx, workspace, rpb);
  else if (D <= 256)
    hipLaunchKernelGGL(rmsnorm_bwd_reg_kernel<4>, dim3(nb), dim3(256), lds, st, dy, x, M, (int)D, g,
                       scale, inv_norm, dres, dx, workspace, rpb);
  else
    hipLaunchKernelGGL(rmsnorm_bwd_kernel, dim3(nb), dim3(256), lds, st, dy, x, M, (int)D, g, scale,
                       inv_norm, dres, dx, workspace, rpb);
  // the gain gradient: into the flat gradient (accumulate) it joins an open deferral scope
  if (accumulate)
    param_rows_finish(workspace, nb, D, dg, 1, workspace + (int64_t)nb * 2 * D, st);
  else
    reduce_rows(workspace, nb, D, D, dg, nullptr, 0, 0, workspace + (int64_t)nb * 2 * D, st);
  return launch_status("tvq_rmsnorm_bwd");
}

extern "C" int tvq_layernorm_fwd(const float* x, int64_t M, int64_t D, const float* gamma,
                                 const float* beta, float eps, float* y, float* mean, float* rstd,
                                 tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && y && mean && rstd && M > 0 && D > 0, "tvq_layernorm_fwd: bad arguments");
  if ((D == 32 || D == 64 || D == 128 || D == 256) && a16(x) && a16(y) && a16(gamma) &&
      a16(beta)) {
    const int L = (int)(D / 4), rows = 4 * (64 / L);
    const dim3 grid((unsigned)((M + rows - 1) / rows));
    hipStream_t st = (hipStream_t)stream;
    TVQ_PLAN("layernorm_fwd_vec D%lld", (long long)D);
#define LN_(LV)                                                                                   \
  hipLaunchKernelGGL(layernorm_fwd_vec_kernel<LV>, grid, dim3(256), 0, st, (const float4*)x, M, \
                     gamma, beta, eps, (float4*)y, mean, rstd)
    if (L == 8) LN_(8); else if (L == 16) LN_(16); else if (L == 32) LN_(32); else LN_(64);
#undef LN_
    return launch_status("tvq_layernorm_fwd");
  }
  hipLaunchKernelGGL(layernorm_fwd_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, x, M, (int)D, gamma, beta, eps, y, mean, rstd);
  return launch_status("tvq_layernorm_fwd");
}

extern "C" int tvq_layernorm_bwd(const float* dy, const float* x, int64_t M, int64_t D,
                                 const float* gamma, const float* mean, const float* rstd,
                                 float* dx, float* dgamma, float* dbeta, int64_t accumulate,
                                 float* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(dy && x && mean && rstd && dx && workspace, "tvq_layernorm_bwd: bad args");
  const int rpb = norm_rows_per_block(M);
  const int nb = (int)((M + rpb - 1) / rpb);
  hipStream_t st = (hipStream_t)stream;
  const size_t lds = 8 * D * sizeof(float);
  if (D <= 64)
    hipLaunchKernelGGL(layernorm_bwd_reg_kernel<1>, dim3(nb), dim3(256), lds, st, dy, x, M, (int)D,
                       gamma, mean, rstd, dx, workspace, rpb);
  else if (D <= 128)
    hipLaunchKernelGGL(layernorm_bwd_reg_kernel<2>, dim3(nb), dim3(256), lds, st, dy, x, M, (int)D,
                       gamma, mean, rstd, dx, workspace, rpb);
  else if (D <= 256)
    hipLaunchKernelGGL(layernorm_bwd_reg_kernel<4>, dim3(nb), dim3(256), lds, st, dy, x, M, (int)D,
                       gamma, mean, rstd, dx, workspace, rpb);
  else
    hipLaunchKernelGGL(layernorm_bwd_kernel, dim3(nb), dim3(256), lds, st, dy, x, M, (int)D, gamma,
                       mean, rstd, dx, workspace, rpb);
  // workspace [gamma | beta][nb][D]: two slabs of contiguous rows; into the flat gradient
  // (accumulate) they join an open deferral scope
  float* rs = workspace + (int64_t)nb * 2 * D;
  float* rs2 = rs + reduce_rows_scratch(nb, D);
  if (accumulate) {
    if (dgamma) param_rows_finish(workspace, nb, D, dgamma, 1, rs, st);
    if (dbeta) param_rows_finish(workspace + (int64_t)nb * D, nb, D, dbeta, 1, rs2, st);
  } else {
    if (dgamma) reduce_rows(workspace, nb, D, D, dgamma, nullptr, 0, 0, rs, st);
    if (dbeta) reduce_rows(workspace + (int64_t)nb * D, nb, D, D, dbeta, nullptr, 0, 0, rs2, st);
  }
  return launch_status("tvq_layernorm_bwd");
}

extern "C" int tvq_embedding_fwd(const int64_t* idx, int64_t M, int64_t D, const float* table,
                                 float* out, int64_t ldo, int64_t mask_id, float drop_p,
                                 const int64_t* seed_ptr, uint64_t offset, tvq_stream_t stream) {
  TVQ_CHECK_ARG(idx && table && out && M > 0 && D > 0, "tvq_embedding_fwd: bad arguments");
  hipLaunchKernelGGL(embedding_fwd_kernel, dim3(grid_for(M * D)), dim3(256), 0, (hipStream_t)stream,
                     idx, M, (int)D, table, out, ldo, mask_id, drop_p, seed_ptr, offset);
  return launch_status("tvq_embedding_fwd");
}

extern "C" int64_t tvq_embedding_bwd_workspace(int64_t M, int64_t V) {
  // 4-byte words: offsets | perm | group-by scratch | (aligned) float chunk partials (D <= 512)
  const int64_t ints = (V + 1) + M + group_by_scratch_ints(M, V);
  return ((ints + 3) / 4) * 4 + seg_rowsum_scratch_floats(M, V, 512);
}

// table_grad[r, :] (+)= sum_{m: idx[m] == r} g[m, :] * dropout-mask, rows summed in position
// order via a stable group-by (deterministic, no float atomics)
extern "C" int tvq_embedding_bwd(const int64_t* idx, int64_t M, int64_t D, const float* g,
                                 int64_t ldg, int64_t V, float* tgrad, int64_t accumulate,
                                 int64_t mask_id, float drop_p, const int64_t* seed_ptr,
                                 uint64_t offset, int32_t* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(idx && g && tgrad && workspace && M > 0 && D > 0 && D <= 512 && V > 0,
                "tvq_embedding_bwd: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  int* offsets = workspace;
  int* perm = offsets + (V + 1);
  int* scratch = perm + M;
  const int64_t ints = (V + 1) + M + group_by_scratch_ints(M, V);
  float* part = (float*)(workspace + ((ints + 3) / 4) * 4);
  group_by_i64(idx, M, V, offsets, perm, scratch, st);
  SegRows r;
  r.src = g; r.N = M; r.sB = 0; r.sN = ldg; r.sD = 1; r.D = (int)D;
  r.drop_p = drop_p; r.seed_ptr = seed_ptr; r.offset = offset; r.mask_id = mask_id;
  seg_rowsum(r, offsets, perm, group_by_seg_start(scratch, M, V), M, V, tgrad, (int)accumulate,
             part, st);
  return launch_status("tvq_embedding_bwd");
}

extern "C" int64_t tvq_masked_ce_workspace(int64_t M) {
  int64_t nb = (M + 3) / 4;
  if (nb > 1024) nb = 1024;
  return 2 * nb;
}

// out: device float[2] = {loss, count}; lse: [M] scratch kept for the backward
extern "C" int tvq_masked_ce_fwd(const float* logits, int64_t ldl, int64_t M, int64_t K,
                                 const int64_t* target, const bool* keep, float* lse, float* out,
                                 float* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(logits && target && keep && lse && out && workspace && M > 0 && K > 0,
                "tvq_masked_ce_fwd: bad arguments");
  const int nb = (int)(tvq_masked_ce_workspace(M) / 2);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(masked_ce_fwd_kernel, dim3(nb), dim3(256), 0, st, logits, ldl, M, (int)K,
                     target, keep, lse, workspace);
  hipLaunchKernelGGL(masked_ce_final_kernel, dim3(1), dim3(256), 0, st, workspace, nb, out);
  return launch_status("tvq_masked_ce_fwd");
}

extern "C" int tvq_masked_ce_bwd(const float* logits, int64_t ldl, int64_t M, int64_t K,
                                 const int64_t* target, const bool* keep, const float* lse,
                                 const float* stats, const float* gout, float* dlogits,
                                 int64_t ldd, tvq_stream_t stream) {
  TVQ_CHECK_ARG(logits && target && keep && lse && stats && gout && dlogits,
                "tvq_masked_ce_bwd: bad arguments");
  hipLaunchKernelGGL(masked_ce_bwd_kernel, dim3(grid_for(M * K)), dim3(256), 0, (hipStream_t)stream,
                     logits, ldl, M, (int)K, target, keep, lse, stats, gout, dlogits, ldd);
  return launch_status("tvq_masked_ce_bwd");
}

extern "C" int tvq_mask_tokens(const int64_t* s, int64_t B, int64_t n, int64_t mask_id,
                               const int64_t* seed_ptr, uint64_t offset, const double* ratio,
                               const float* rand, int64_t* s_M, bool* keep, tvq_stream_t stream) {
  TVQ_CHECK_ARG(s && s_M && keep && B > 0 && n > 0 && n <= 4096, "tvq_mask_tokens: bad arguments");
  hipLaunchKernelGGL(mask_tokens_kernel, dim3((unsigned)B), dim3(128), n * sizeof(float),
                     (hipStream_t)stream, s, (int)B, (int)n, mask_id, seed_ptr, offset, ratio, rand,
                     s_M, keep);
  return launch_status("tvq_mask_tokens");
}

extern "C" int tvq_upsample_nearest(const float* x, int64_t R, int64_t Lin, int64_t Lout, float* y,
                                    tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && y && R > 0 && Lin > 0 && Lout > 0, "tvq_upsample_nearest: bad arguments");
  const float scale = (float)Lin / (float)Lout;
  hipLaunchKernelGGL(upsample_nearest_kernel, dim3(grid_for(R * Lout)), dim3(256), 0,
                     (hipStream_t)stream, x, R, (int)Lin, (int)Lout, scale, y);
  return launch_status("tvq_upsample_nearest");
}

extern "C" int tvq_upsample_nearest_bwd(const float* dy, int64_t R, int64_t Lin, int64_t Lout,
                                        float* dx, tvq_stream_t stream) {
  TVQ_CHECK_ARG(dy && dx && R > 0 && Lin > 0 && Lout > 0, "tvq_upsample_nearest_bwd: bad args");
  const float scale = (float)Lin / (float)Lout;
  hipLaunchKernelGGL(upsample_nearest_bwd_kernel, dim3(grid_for(R * Lin)), dim3(256), 0,
                     (hipStream_t)stream, dy, R, (int)Lin, (int)Lout, scale, dx);
  return launch_status("tvq_upsample_nearest_bwd");
}

extern "C" int tvq_gelu_fwd(const float* x, int64_t n, float* y, tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && y && n >= 0, "tvq_gelu_fwd: bad arguments");
  if (n == 0) return TVQ_OK;
  hipLaunchKernelGGL(gelu_fwd_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, n, y);
  return launch_status("tvq_gelu_fwd");
}

extern "C" int tvq_gelu_bwd(const float* dy, const float* x, int64_t n, float* dx,
                            tvq_stream_t stream) {
  TVQ_CHECK_ARG(dy && x && dx && n >= 0, "tvq_gelu_bwd: bad arguments");
  if (n == 0) return TVQ_OK;
  hipLaunchKernelGGL(gelu_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, dy, x, n,
                     dx);
  return launch_status("tvq_gelu_bwd");
}

// ---------------------------------------------------------------- drop the class token
// y[b, i, :] = x[b, i + 1, :] (embed[:, 1:, :].contiguous(), bidirectional_transformer.py:
// 188, 233) and its adjoint dx[b, 0, :] = 0, dx[b, i + 1, :] = dy[b, i, :]: float4 lanes
namespace tvq {
__global__ __launch_bounds__(256) void drop_first_kernel(const float4* __restrict__ src,
                                                         float4* __restrict__ dst, int64_t B,
                                                         int n, int D4, int backward) {
  const int64_t tot = backward ? B * (n + 1) * D4 : B * n * D4;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < tot; e += (int64_t)gridDim.x * 256) {
    const int d = (int)(e % D4);
    const int64_t r = e / D4;
    if (backward) {  // dst row r = (b, j) of (B, n + 1)
      const int64_t b = r / (n + 1);
      const int j = (int)(r - b * (n + 1));
      dst[e] = j == 0 ? make_float4(0.f, 0.f, 0.f, 0.f) : src[(b * n + j - 1) * D4 + d];
    } else {  // dst row r = (b, i) of (B, n)
      const int64_t b = r / n;
      const int i = (int)(r - b * n);
      dst[e] = src[(b * (n + 1) + i + 1) * D4 + d];
    }
  }
}
}  // namespace tvq

extern "C" int tvq_drop_first_token(const float* x, int64_t B, int64_t n, int64_t D, float* y,
                                    int64_t backward, tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && y && B > 0 && n > 0 && D > 0 && D % 4 == 0 && ((uintptr_t)x & 15) == 0 &&
                    ((uintptr_t)y & 15) == 0, "tvq_drop_first_token: bad arguments");
  const int64_t tot = (backward ? B * (n + 1) : B * n) * (D / 4);
  hipLaunchKernelGGL(drop_first_kernel, dim3(grid_for(tot)), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const float4*>(x), reinterpret_cast<float4*>(y), B, (int)n,
                     (int)(D / 4), (int)backward);
  return launch_status("tvq_drop_first_token");
}

// The attention branch of the LF prior's pre-norm layers in training, one launch forward and
// one backward (bidirectional_transformer.py:92-110: x-transformers Encoder with
// pre_norm=True, RMSNorm, Attention(dim 128, 2 heads x 64), attention dropout, layer dropout):
//
//   forward:  xn = RMSNorm(x) = x / max(|x|, 1e-12) * sqrt(128) * g
//             q, k, v = xn Wq^T, xn Wk^T, xn Wv^T;  per head P = dropout(softmax(q k^T / 8))
//             o = P v;  y = x + gate * (o Wo^T)
//   backward: from gy: dO = (gate gy) Wo; the attention backward (dV = P~^T dO, dS = P (dP -
//             rowsum(dO o)), dQ = dS K / 8, dK = dS^T Q / 8); dxn = dQ Wq + dK Wk + dV Wv;
//             dx = gy + RMSNorm'(dxn); the gain gradient as a per-sequence slab row
//
// The per-op path ran these as 4 launches forward (RMSNorm, the QKV GEMM, attention, the
// gated out-projection) and 5 backward (out-projection and QKV data gradients, attention,
// RMSNorm, its gain reduction), each a latency-bound grid over the 6,400 token rows.  Here a
// 4-wave block owns one sequence (S <= 32 tokens: the LF prior's 25, padded to one 32-token
// MFMA tile) and every operand stays in registers or LDS:
//   * token on the lane: a 32-feature tile of a token-row operand lives in the accumulator
//     layout of a v_mfma_f32_32x32x2_f32 whose columns are tokens (tvq_ff.h), so the RMSNorm
//     output, Q, K, V, O and their gradients are produced and consumed without data movement;
//   * wave w owns feature tile w of every 128-wide operand: the Q / K / V / O tiles of head
//     w >> 1's dims 32 (w & 1) ..; a head's scores are the sum of its two waves' partial
//     Q K^T tiles, exchanged through LDS once (both waves then hold the same scores);
//   * the three operands that need the other register order (V for P V, dO / Q / K for the
//     dV / dK / dQ products, dS for dQ) go through one 32 x 33 LDS transpose each;
//   * the out-projection and the dxn products need whole 128-feature rows: the 4 waves'
//     tiles are exchanged into the B-row layout (ff_exchange) as in the fused feed-forward.
// The weight gradients (dWqkv = dqkv^T xn, dWo = (gate gy)^T o) stay with the grouped
// deferred launch of the backward (timevqvae.hip.wgrad); so the forward also writes xn, the
// q|k|v rows, o and the per-query log-sum-exp, and the backward writes dqkv and gate * gy.
// Arithmetic follows the per-op kernels (tvq_rmsnorm_*, tvq_attention_*, the gated Linear
// epilogue, the attention-dropout hash at ((b*H + head)*S + query)*S + key) up to fp32
// summation order.
#include <math.h>

#include "tvq_common.h"
#include "tvq_conv_internal.h"
#include "tvq_ff.h"
#include "tvq_reduce.h"

namespace tvq {

namespace xa {

constexpr int D = 128, H = 2, T = 256, TP = 33;  // width, heads, threads, transpose pitch

struct Args {
  const float *x, *g, *Wqkv, *Wo, *gate, *gy;
  const float *inv_in, *qkv_in, *o_in, *lse_in;
  float *y, *xn, *inv, *qkv, *o, *lse;
  float *dx, *dqkv, *gyg, *dg_slab;
  const int64_t* seed_ptr;
  uint64_t offset;
  float nscale, scale, p, dscale;
  int B, S;
};

__device__ __forceinline__ int wid() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

__device__ __forceinline__ bool keep(uint64_t seed, int64_t bh, int S, int i, int j, float p) {
  return uniform01(seed, ((uint64_t)bh * S + i) * S + j) >= p;  // tvq_attn.hip attn_keep
}

// feature-major tile (features f0 + ff_crow(r, h)) of a token row: 4 float4 loads / stores
__device__ __forceinline__ floatx16 load_fm(const float* __restrict__ row, int f0, int h) {
  floatx16 t;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float4 v = *reinterpret_cast<const float4*>(row + f0 + 8 * g + 4 * h);
    t[4 * g] = v.x; t[4 * g + 1] = v.y; t[4 * g + 2] = v.z; t[4 * g + 3] = v.w;
  }
  return t;
}
__device__ __forceinline__ void store_fm(float* __restrict__ row, int f0, int h, const floatx16& t) {
#pragma unroll
  for (int g = 0; g < 4; ++g)
    *reinterpret_cast<float4*>(row + f0 + 8 * g + 4 * h) =
        make_float4(t[4 * g], t[4 * g + 1], t[4 * g + 2], t[4 * g + 3]);
}
// the tile of B-row registers v for feature tile w (wave-uniform w, no dynamic register index)
__device__ __forceinline__ floatx16 slice(const float (&v)[64], int w) {
  floatx16 t;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (q == w)
#pragma unroll
      for (int r = 0; r < 16; ++r) t[r] = v[16 * q + r];
  return t;
}
__device__ __forceinline__ void to_arr(const floatx16& t, float (&a)[16]) {
#pragma unroll
  for (int r = 0; r < 16; ++r) a[r] = t[r];
}
// transpose through LDS: put (token l & 31, feature crow(r, h)) = t[r]; get tr[s] = the
// element (token crow(s, h), feature l & 31)
__device__ __forceinline__ void tr_put(float* __restrict__ T32, const floatx16& t, int j, int h) {
#pragma unroll
  for (int r = 0; r < 16; ++r) T32[j * TP + ff_crow(r, h)] = t[r];
}
__device__ __forceinline__ void tr_get(const float* __restrict__ T32, float (&tr)[16], int j, int h) {
#pragma unroll
  for (int s = 0; s < 16; ++s) tr[s] = T32[ff_crow(s, h) * TP + j];
}

// ---------------------------------------------------------------- forward
__global__ __launch_bounds__(T) void xattn_fwd_kernel(Args a) {
  __shared__ float ex[4][16][64];      // partial score tiles; then the ff_exchange buffer
  __shared__ float tt[4][32 * TP];     // per-wave V transpose
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5, w = wid();
  const int b = blockIdx.x, S = a.S;
  const bool valid = j < S;
  const int64_t row = (int64_t)b * S + (valid ? j : S - 1);
  float xb[64], wa[64], wb[64];
  ff_load_row(a.x + row * D, h, xb);
  ff_wload<false>(a.Wqkv, 32 * w, lane, wa);  // Wq's rows: in flight during the RMSNorm
  __builtin_amdgcn_sched_barrier(0);
  // RMSNorm (tvq_rmsnorm_fwd's arithmetic)
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 64; ++i) ss += xb[i] * xb[i];
  ss += __shfl_xor(ss, 32, 64);
  const float inv = 1.0f / fmaxf(sqrtf(ss), 1e-12f);
  float xn[64];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 gv = ff_vec4(a.g, q, g, h);
      const float gg[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) xn[16 * q + 4 * g + e] = xb[16 * q + 4 * g + e] * inv * a.nscale * gg[e];
    }
  if (valid) {
    store_fm(a.xn + row * D, 32 * w, h, slice(xn, w));
    if (w == 0 && h == 0) a.inv[row] = inv;
  }
  // Q / K / V tiles w (token on the lane); each tile's weights requested before the previous
  // tile's MFMAs
  ff_wload<false>(a.Wqkv + D * D, 32 * w, lane, wb);
  __builtin_amdgcn_sched_barrier(0);
  const floatx16 qt = ff_mma(wa, xn, ff_zero());
  ff_wload<false>(a.Wqkv + 2 * D * D, 32 * w, lane, wa);
  __builtin_amdgcn_sched_barrier(0);
  const floatx16 kt = ff_mma(wb, xn, ff_zero());
  ff_wload<false>(a.Wo, 32 * w, lane, wb);  // the out-projection's, kept for the end
  __builtin_amdgcn_sched_barrier(0);
  const floatx16 vt = ff_mma(wa, xn, ff_zero());
  if (valid) {
    float* qr = a.qkv + row * 3 * D;
    store_fm(qr, 32 * w, h, qt);
    store_fm(qr + D, 32 * w, h, kt);
    store_fm(qr + 2 * D, 32 * w, h, vt);
  }
  // this wave's partial S^T (key crow(r, h), query j) over its 32 dims of the head
  floatx16 st;
#pragma unroll
  for (int r = 0; r < 16; ++r) st[r] = 0.f;
#pragma unroll
  for (int t = 0; t < 16; ++t) st = __builtin_amdgcn_mfma_f32_32x32x2f32(kt[t], qt[t], st, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 16; ++r) ex[w][r][lane] = st[r];
  tr_put(tt[w], vt, j, h);
  __syncthreads();
  const int hd = w >> 1, w0 = 2 * hd;
  float s[16], vtr[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) s[r] = ex[w0][r][lane] + ex[w0 + 1][r][lane];
  tr_get(tt[w], vtr, j, h);  // vtr[t] = V[token crow(t, h)][dim 32 w + j]
  // softmax over the keys (registers and the partner half), tvq_attention_fwd's arithmetic
  float mx = -INFINITY;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int key = ff_crow(r, h);
    s[r] = key < S ? s[r] * a.scale : -INFINITY;
    mx = fmaxf(mx, s[r]);
  }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    s[r] = expf(s[r] - mx);
    sum += s[r];
  }
  sum += __shfl_xor(sum, 32, 64);
  const float isum = 1.0f / sum;
  const int64_t bh = (int64_t)b * H + hd;
  if (h == 0 && valid && (w & 1) == 0) a.lse[bh * S + j] = mx + logf(sum);
  const uint64_t seed = a.p > 0.f ? mix_seed(a.seed_ptr, a.offset) : 0ull;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float pv = s[r] * isum;
    if (a.p > 0.f) {
      const int key = ff_crow(r, h);
      pv = (valid && key < S && keep(seed, bh, S, j, key, a.p)) ? pv * a.dscale : 0.f;
    }
    s[r] = pv;
  }
  // O tile w (query j, dims 32 w + crow(r, h)) = sum over keys of V^T P^T
  floatx16 ot;
#pragma unroll
  for (int r = 0; r < 16; ++r) ot[r] = 0.f;
#pragma unroll
  for (int t = 0; t < 16; ++t) ot = __builtin_amdgcn_mfma_f32_32x32x2f32(vtr[t], s[t], ot, 0, 0, 0);
  if (valid) store_fm(a.o + row * D, 32 * w, h, ot);
  __syncthreads();  // ex free again
  float oa[16], ob[64];
  to_arr(ot, oa);
  ff_exchange(reinterpret_cast<float4(*)[4][64]>(&ex[0][0][0]), w, oa, ob, lane);
  const floatx16 yt = ff_mma(wb, ob, ff_zero());
  const float gt = a.gate ? *a.gate : 1.0f;
  const floatx16 xr = slice(xb, w);
  floatx16 yv;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float v = yt[r];
    if (a.gate) v *= gt;
    yv[r] = v + xr[r];
  }
  if (valid) store_fm(a.y + row * D, 32 * w, h, yv);
}

// ---------------------------------------------------------------- backward
// dynamic LDS (floats): EX 8192 (the S and dP partial tiles; then the dS transposes; then the
// ff_exchange buffer) | TT 4 x 3 x 32*TP (dO, Q, K transposes) | DD 4 x 64 | LS 2 x 32 | DT 4 x 64
constexpr int B_EX = 0, B_TT = 8192, B_DD = B_TT + 12 * 32 * TP, B_LS = B_DD + 256,
              B_DT = B_LS + 64, B_TOT = B_DT + 256;

__global__ __launch_bounds__(T) void xattn_bwd_kernel(Args a) {
  extern __shared__ float sm[];
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5, w = wid();
  const int b = blockIdx.x, S = a.S;
  const bool valid = j < S;
  const int64_t row = (int64_t)b * S + (valid ? j : S - 1);
  const float gt = a.gate ? *a.gate : 1.0f;
  floatx16 dot;  // dO tile w: (gate gy) Wo
  float wa[64];
  {
    float gb[64];
    ff_load_row(a.gy + row * D, h, gb);
    ff_wload<true>(a.Wo, 32 * w, lane, wa);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 64; ++i) gb[i] *= gt;
    if (a.gyg && valid) store_fm(a.gyg + row * D, 32 * w, h, slice(gb, w));
    dot = ff_mma(wa, gb, ff_zero());
  }
  ff_wload<true>(a.Wqkv, 32 * w, lane, wa);  // the dxn product's first weights, early
  __builtin_amdgcn_sched_barrier(0);
  const float* qr = a.qkv_in + row * 3 * D;
  const floatx16 qt = load_fm(qr, 32 * w, h);
  const floatx16 kt = load_fm(qr + D, 32 * w, h);
  const floatx16 vt = load_fm(qr + 2 * D, 32 * w, h);
  const floatx16 ot = load_fm(a.o_in + row * D, 32 * w, h);
  const int hd = w >> 1, w0 = 2 * hd;
  // rowsum(dO o) of query j over this wave's dims; S and dP partials (query crow(r, h), key j)
  float dpart = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) dpart = fmaf(dot[r], ot[r], dpart);
  dpart += __shfl_xor(dpart, 32, 64);
  floatx16 sp, pp;
#pragma unroll
  for (int r = 0; r < 16; ++r) sp[r] = pp[r] = 0.f;
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    sp = __builtin_amdgcn_mfma_f32_32x32x2f32(qt[t], kt[t], sp, 0, 0, 0);
    pp = __builtin_amdgcn_mfma_f32_32x32x2f32(dot[t], vt[t], pp, 0, 0, 0);
  }
  float* exS = sm + B_EX;
  float* exP = sm + B_EX + 4096;
  float* ttw = sm + B_TT + w * 3 * 32 * TP;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    exS[(w * 16 + r) * 64 + lane] = sp[r];
    exP[(w * 16 + r) * 64 + lane] = pp[r];
  }
  tr_put(ttw, dot, j, h);
  tr_put(ttw + 32 * TP, qt, j, h);
  tr_put(ttw + 64 * TP, kt, j, h);
  if (h == 0) sm[B_DD + w * 64 + j] = dpart;
  if (w < 2 && h == 0) sm[B_LS + w * 32 + j] = valid ? a.lse_in[((int64_t)b * H + w) * S + j] : 0.f;
  __syncthreads();
  const int64_t bh = (int64_t)b * H + hd;
  const uint64_t seed = a.p > 0.f ? mix_seed(a.seed_ptr, a.offset) : 0ull;
  float pd[16], ds[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int ql = ff_crow(r, h);
    const float sv = exS[(w0 * 16 + r) * 64 + lane] + exS[((w0 + 1) * 16 + r) * 64 + lane];
    float dv = exP[(w0 * 16 + r) * 64 + lane] + exP[((w0 + 1) * 16 + r) * 64 + lane];
    float p = 0.f, g = 0.f;
    if (ql < S && valid) {  // valid: the key j
      p = expf(sv * a.scale - sm[B_LS + hd * 32 + ql]);
      float pq = p;
      if (a.p > 0.f) {
        const bool kp = keep(seed, bh, S, ql, j, a.p);
        pq = kp ? p * a.dscale : 0.f;
        dv = kp ? dv * a.dscale : 0.f;
      }
      const float Dq = sm[B_DD + w0 * 64 + ql] + sm[B_DD + (w0 + 1) * 64 + ql];
      g = p * (dv - Dq);
      p = pq;
    }
    pd[r] = p;
    ds[r] = g;
  }
  float dotr[16], qtr[16], ktr[16], dst[16];
  tr_get(ttw, dotr, j, h);  // dO[query crow(t, h)][dim 32 w + j]
  tr_get(ttw + 32 * TP, qtr, j, h);
  tr_get(ttw + 64 * TP, ktr, j, h);
  __syncthreads();  // the partial tiles are read: EX holds the dS transposes now
  float* tds = sm + B_EX + w * 32 * TP;
#pragma unroll
  for (int r = 0; r < 16; ++r) tds[ff_crow(r, h) * TP + j] = ds[r];  // (query, key)
  __syncthreads();
#pragma unroll
  for (int s = 0; s < 16; ++s) dst[s] = tds[j * TP + ff_crow(s, h)];  // query j, key crow(s, h)
  // dV, dK, dQ tiles w (token on the lane, dims 32 w + crow(r, h))
  floatx16 dvt, dkt, dqt;
#pragma unroll
  for (int r = 0; r < 16; ++r) dvt[r] = dkt[r] = dqt[r] = 0.f;
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    dvt = __builtin_amdgcn_mfma_f32_32x32x2f32(dotr[t], pd[t], dvt, 0, 0, 0);
    dkt = __builtin_amdgcn_mfma_f32_32x32x2f32(qtr[t], ds[t], dkt, 0, 0, 0);
    dqt = __builtin_amdgcn_mfma_f32_32x32x2f32(ktr[t], dst[t], dqt, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    dkt[r] *= a.scale;
    dqt[r] *= a.scale;
  }
  if (valid) {
    float* dr = a.dqkv + row * 3 * D;
    store_fm(dr, 32 * w, h, dqt);
    store_fm(dr + D, 32 * w, h, dkt);
    store_fm(dr + 2 * D, 32 * w, h, dvt);
  }
  // dxn tile w = dQ Wq + dK Wk + dV Wv (whole rows through the exchange buffer)
  __syncthreads();  // the dS transposes are read
  auto* buf = reinterpret_cast<float4(*)[4][64]>(sm + B_EX);
  float ta[16], bx[64], wb[64];
  to_arr(dqt, ta);
  ff_exchange(buf, w, ta, bx, lane);
  ff_wload<true>(a.Wqkv + D * D, 32 * w, lane, wb);
  __builtin_amdgcn_sched_barrier(0);
  floatx16 dn = ff_mma(wa, bx, ff_zero());
  __syncthreads();
  to_arr(dkt, ta);
  ff_exchange(buf, w, ta, bx, lane);
  ff_wload<true>(a.Wqkv + 2 * D * D, 32 * w, lane, wa);
  __builtin_amdgcn_sched_barrier(0);
  dn = ff_mma(wb, bx, dn);
  __syncthreads();
  to_arr(dvt, ta);
  ff_exchange(buf, w, ta, bx, lane);
  dn = ff_mma(wa, bx, dn);
  // RMSNorm backward (tvq_rmsnorm_bwd's arithmetic) + the residual path's gradient
  const floatx16 xt = load_fm(a.x + row * D, 32 * w, h);
  const floatx16 gyt = load_fm(a.gy + row * D, 32 * w, h);
  const floatx16 gw = load_fm(a.g, 32 * w, h);
  const float inv = a.inv_in[row];
  float dp = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) dp += dn[r] * gw[r] * xt[r];
  dp += __shfl_xor(dp, 32, 64);
  if (h == 0) sm[B_DT + w * 64 + j] = dp;
  __syncthreads();
  const float dsum = sm[B_DT + j] + sm[B_DT + 64 + j] + sm[B_DT + 128 + j] + sm[B_DT + 192 + j];
  const float c = dsum * a.nscale * inv * inv * inv;
  floatx16 dxt;
#pragma unroll
  for (int r = 0; r < 16; ++r) dxt[r] = (dn[r] * gw[r] * a.nscale * inv - xt[r] * c) + gyt[r];
  if (valid) store_fm(a.dx + row * D, 32 * w, h, dxt);
  // the gain gradient of this sequence: sum over its tokens of dxn * x * inv * scale
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float v = valid ? dn[r] * xt[r] * inv * a.nscale : 0.f;
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) v += __shfl_xor(v, o, 64);
    if (j == 0) a.dg_slab[(int64_t)b * D + 32 * w + ff_crow(r, h)] = v;
  }
}

static bool aligned(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace xa
}  // namespace tvq

using namespace tvq;

extern "C" int64_t tvq_attn_branch_workspace(int64_t B, int64_t D) {
  // floats: the per-sequence gain-gradient slab and its reduction scratch
  return B * D + reduce_rows_scratch(B, D);
}

extern "C" int tvq_attn_branch_fwd(const float* x, int64_t B, int64_t S, int64_t D, int64_t heads,
                                   const float* g, float nscale, const float* Wqkv,
                                   const float* Wo, const float* gate, float drop_p,
                                   const int64_t* seed_ptr, uint64_t offset, float* y, float* xn,
                                   float* inv, float* qkv, float* o, float* lse,
                                   tvq_stream_t stream) {
  using namespace xa;
  TVQ_CHECK_ARG(x && g && Wqkv && Wo && y && xn && inv && qkv && o && lse && B > 0,
                "tvq_attn_branch_fwd: bad arguments");
  TVQ_CHECK_ARG(D == xa::D && heads == xa::H && S >= 1 && S <= 32,
                "tvq_attn_branch_fwd: needs D = 128, 2 heads of 64, S <= 32");
  TVQ_CHECK_ARG(drop_p >= 0.f && drop_p < 1.f && (drop_p == 0.f || seed_ptr),
                "tvq_attn_branch_fwd: bad dropout");
  TVQ_CHECK_ARG(aligned(x) && aligned(g) && aligned(Wqkv) && aligned(Wo) && aligned(y) &&
                    aligned(xn) && aligned(qkv) && aligned(o),
                "tvq_attn_branch_fwd: pointers must be 16-byte aligned");
  Args a = {};
  a.x = x; a.g = g; a.Wqkv = Wqkv; a.Wo = Wo; a.gate = gate;
  a.y = y; a.xn = xn; a.inv = inv; a.qkv = qkv; a.o = o; a.lse = lse;
  a.seed_ptr = seed_ptr; a.offset = offset;
  a.nscale = nscale; a.scale = 0.125f; a.p = drop_p;
  a.dscale = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
  a.B = (int)B; a.S = (int)S;
  hipLaunchKernelGGL(xattn_fwd_kernel, dim3((unsigned)B), dim3(T), 0, (hipStream_t)stream, a);
  TVQ_PLAN("attn_branch_fwd B%lld S%lld", (long long)B, (long long)S);
  return launch_status("tvq_attn_branch_fwd");
}

extern "C" int tvq_attn_branch_bwd(const float* gy, const float* x, int64_t B, int64_t S,
                                   int64_t D, int64_t heads, const float* g, float nscale,
                                   const float* inv, const float* Wqkv, const float* Wo,
                                   const float* gate, float drop_p, const int64_t* seed_ptr,
                                   uint64_t offset, const float* qkv, const float* o,
                                   const float* lse, float* dx, float* dqkv, float* gy_gated,
                                   float* dg, int64_t accumulate, float* workspace,
                                   tvq_stream_t stream) {
  using namespace xa;
  TVQ_CHECK_ARG(gy && x && g && inv && Wqkv && Wo && qkv && o && lse && dx && dqkv && dg &&
                    workspace && B > 0,
                "tvq_attn_branch_bwd: bad arguments");
  TVQ_CHECK_ARG(D == xa::D && heads == xa::H && S >= 1 && S <= 32,
                "tvq_attn_branch_bwd: needs D = 128, 2 heads of 64, S <= 32");
  TVQ_CHECK_ARG(drop_p >= 0.f && drop_p < 1.f && (drop_p == 0.f || seed_ptr),
                "tvq_attn_branch_bwd: bad dropout");
  TVQ_CHECK_ARG(aligned(gy) && aligned(x) && aligned(g) && aligned(Wqkv) && aligned(Wo) &&
                    aligned(qkv) && aligned(o) && aligned(dx) && aligned(dqkv) &&
                    aligned(gy_gated),
                "tvq_attn_branch_bwd: pointers must be 16-byte aligned");
  hipStream_t st = (hipStream_t)stream;
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)xattn_bwd_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, B_TOT * 4);
    return true;
  }();
  (void)attr;
  Args a = {};
  a.x = x; a.g = g; a.Wqkv = Wqkv; a.Wo = Wo; a.gate = gate; a.gy = gy;
  a.inv_in = inv; a.qkv_in = qkv; a.o_in = o; a.lse_in = lse;
  a.dx = dx; a.dqkv = dqkv; a.gyg = gate ? gy_gated : nullptr; a.dg_slab = workspace;
  a.seed_ptr = seed_ptr; a.offset = offset;
  a.nscale = nscale; a.scale = 0.125f; a.p = drop_p;
  a.dscale = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
  a.B = (int)B; a.S = (int)S;
  hipLaunchKernelGGL(xattn_bwd_kernel, dim3((unsigned)B), dim3(T), B_TOT * 4, st, a);
  TVQ_PLAN("attn_branch_bwd B%lld S%lld", (long long)B, (long long)S);
  int rc = launch_status("tvq_attn_branch_bwd");
  if (rc) return rc;
  // the gain gradient: into the flat gradient it joins an open deferral scope
  if (accumulate)
    param_rows_finish(workspace, B, D, dg, 1, workspace + B * D, st);
  else
    reduce_rows(workspace, B, D, D, dg, nullptr, 0, 0, workspace + B * D, st);
  return launch_status("tvq_attn_branch_bwd");
}

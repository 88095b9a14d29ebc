// The x-transformers feed-forward branch of the LF prior in training, forward and data
// backward, one launch each (bidirectional_transformer.py:92-110; x-transformers
// FeedForward = Linear -> GELU -> Dropout -> Linear, here with the pre-norm residual and the
// layer-dropout gate of the Encoder):
//
//   forward:  pre = xn W1^T + b1;  hd = dropout(GELU(pre));  y = (hd W2^T + b2) * gate + r
//   backward: d_hd = gate * (gy W2);  d_pre = dropout'(d_hd) * GELU'(pre);  dxn = d_pre W1
//
// The per-op path ran these as 3 launches forward (Linear+GELU, dropout, Linear+residual)
// and 5 backward (gate scale, Linear data gradient, dropout, GELU', Linear data gradient),
// each a latency-bound grid over 6,400 x 128.  Here a block owns 32 token rows: its 4 waves
// each compute one 32-feature tile of the first Linear (token on the lane: the weight rows
// are the MFMA A operand, the token rows the B operand), the tiles meet in LDS in exactly
// the register layout the second Linear's B operand needs, and each wave computes one tile
// of the second Linear.  The weight gradients stay with the grouped launch of the backward
// (timevqvae.hip.wgrad): the forward writes pre and hd, the backward writes d_pre.
//
// Arithmetic follows the per-op kernels (bias before gate before residual, erf GELU, the
// dropout mask of tvq_dropout_bwd at element m * 128 + n); sums over K run in MFMA order.
#include <math.h>

#include "tvq_common.h"
#include "tvq_ff.h"

namespace tvq {

__device__ __forceinline__ float ff_gelu(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f));
}
__device__ __forceinline__ float ff_gelu_grad(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752440f));
  const float pdf = 0.39894228040143267794f * expf(-0.5f * x * x);
  return cdf + x * pdf;
}

struct FfArgs {
  const float *xn, *r, *W1, *b1, *W2, *b2, *gate, *gy, *pre_in;
  float *y, *pre, *hd, *d_pre, *dxn, *gy_gated;
  const int64_t* seed_ptr;
  uint64_t offset;
  float p, scale;
  int M;
};

__global__ __launch_bounds__(256) void ffn_fwd_kernel(FfArgs a) {
  __shared__ float4 buf[4][4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, j = lane & 31, h = lane >> 5;
  const int m0 = blockIdx.x * 32;
  const bool ok = m0 + j < a.M;
  const int64_t m = ok ? m0 + j : a.M - 1;
  const uint64_t seed = a.p > 0.f ? mix_seed(a.seed_ptr, a.offset) : 0ull;
  float hd[16], wa[64], wb[64];
  {
    float xb[64];
    ff_load_row(a.xn + m * FF_D, h, xb);
    ff_wload<false>(a.W1, 32 * w, lane, wa);
    ff_wload<false>(a.W2, 32 * w, lane, wb);  // the second Linear's, in flight meanwhile
    __builtin_amdgcn_sched_barrier(0);
    const floatx16 acc = ff_mma(wa, xb, ff_zero());
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 bb = ff_vec4(a.b1, w, g, h);
      const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
      float pv[4], hv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = 32 * w + 8 * g + 4 * h + e;
        pv[e] = acc[4 * g + e] + bv[e];
        float v = ff_gelu(pv[e]);
        if (a.p > 0.f) v = uniform01(seed, (uint64_t)(m * FF_D + n)) >= a.p ? v * a.scale : 0.f;
        hv[e] = v;
        hd[4 * g + e] = v;
      }
      if (ok) {
        const int64_t o = m * FF_D + 32 * w + 8 * g + 4 * h;
        *reinterpret_cast<float4*>(a.pre + o) = make_float4(pv[0], pv[1], pv[2], pv[3]);
        *reinterpret_cast<float4*>(a.hd + o) = make_float4(hv[0], hv[1], hv[2], hv[3]);
      }
    }
  }
  float hb[64];
  ff_exchange(buf, w, hd, hb, lane);
  const floatx16 acc = ff_mma(wb, hb, ff_zero());
  const float gt = a.gate ? *a.gate : 1.0f;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float4 bb = ff_vec4(a.b2, w, g, h);
    const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
    const int64_t o = m * FF_D + 32 * w + 8 * g + 4 * h;
    const float4 rr = *reinterpret_cast<const float4*>(a.r + o);
    const float rv[4] = {rr.x, rr.y, rr.z, rr.w};
    float yv[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = acc[4 * g + e] + bv[e];
      if (a.gate) v *= gt;
      yv[e] = v + rv[e];
    }
    if (ok) *reinterpret_cast<float4*>(a.y + o) = make_float4(yv[0], yv[1], yv[2], yv[3]);
  }
}

__global__ __launch_bounds__(256) void ffn_bwd_kernel(FfArgs a) {
  __shared__ float4 buf[4][4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, j = lane & 31, h = lane >> 5;
  const int m0 = blockIdx.x * 32;
  const bool ok = m0 + j < a.M;
  const int64_t m = ok ? m0 + j : a.M - 1;
  const uint64_t seed = a.p > 0.f ? mix_seed(a.seed_ptr, a.offset) : 0ull;
  const float gt = a.gate ? *a.gate : 1.0f;
  float dp[16], wa[64], wb[64];
  {
    float gb[64];
    ff_load_row(a.gy + m * FF_D, h, gb);
    ff_wload<true>(a.W2, 32 * w, lane, wa);
    __builtin_amdgcn_sched_barrier(0);
    // gate * gy for the W2 / b2 gradients (a dropped branch's weights get a zero gradient):
    // wave w stores the row's 32-feature slice w, already in registers
    if (a.gy_gated && ok) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (q == w)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<float4*>(a.gy_gated + m * FF_D + 32 * q + 8 * g + 4 * h) =
                make_float4(gt * gb[16 * q + 4 * g], gt * gb[16 * q + 4 * g + 1],
                            gt * gb[16 * q + 4 * g + 2], gt * gb[16 * q + 4 * g + 3]);
    }
    // d_hd (inner features 32 w ..) = gy W2: A(i, k) = W2[k][32 w + i]
    ff_wload<true>(a.W1, 32 * w, lane, wb);  // the second product's, in flight meanwhile
    __builtin_amdgcn_sched_barrier(0);
    const floatx16 acc = ff_mma(wa, gb, ff_zero());
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int64_t o = m * FF_D + 32 * w + 8 * g + 4 * h;
      const float4 pp = *reinterpret_cast<const float4*>(a.pre_in + o);
      const float pv[4] = {pp.x, pp.y, pp.z, pp.w};
      float dv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = a.gate ? acc[4 * g + e] * gt : acc[4 * g + e];
        if (a.p > 0.f)
          v = uniform01(seed, (uint64_t)(o + e)) >= a.p ? v * a.scale : 0.f;
        dv[e] = v * ff_gelu_grad(pv[e]);
        dp[4 * g + e] = dv[e];
      }
      if (ok) *reinterpret_cast<float4*>(a.d_pre + o) = make_float4(dv[0], dv[1], dv[2], dv[3]);
    }
  }
  float db[64];
  ff_exchange(buf, w, dp, db, lane);
  // dxn (features 32 w ..) = d_pre W1: A(i, k) = W1[k][32 w + i]
  const floatx16 acc = ff_mma(wb, db, ff_zero());
#pragma unroll
  for (int g = 0; g < 4; ++g)
    if (ok)
      *reinterpret_cast<float4*>(a.dxn + m * FF_D + 32 * w + 8 * g + 4 * h) =
          make_float4(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]);
}

static bool ff_aligned(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace tvq

using namespace tvq;

extern "C" int tvq_ffn_fwd(const float* xn, const float* r, int64_t M, int64_t D,
                           const float* W1, const float* b1, const float* W2, const float* b2,
                           const float* gate, float p, const int64_t* seed_ptr, uint64_t offset,
                           float* y, float* pre, float* hd, tvq_stream_t stream) {
  TVQ_CHECK_ARG(xn && r && W1 && b1 && W2 && b2 && y && pre && hd && M > 0 && D == FF_D &&
                    p >= 0.f && p < 1.f && (p == 0.f || seed_ptr),
                "tvq_ffn_fwd: bad arguments (D must be 128)");
  TVQ_CHECK_ARG(ff_aligned(xn) && ff_aligned(r) && ff_aligned(W1) && ff_aligned(b1) && ff_aligned(W2) &&
                    ff_aligned(b2) && ff_aligned(y) && ff_aligned(pre) && ff_aligned(hd),
                "tvq_ffn_fwd: pointers must be 16-byte aligned");
  FfArgs a = {};
  a.xn = xn; a.r = r; a.W1 = W1; a.b1 = b1; a.W2 = W2; a.b2 = b2; a.gate = gate;
  a.y = y; a.pre = pre; a.hd = hd; a.seed_ptr = seed_ptr; a.offset = offset;
  a.p = p; a.scale = p > 0.f ? 1.0f / (1.0f - p) : 1.0f; a.M = (int)M;
  hipLaunchKernelGGL(ffn_fwd_kernel, dim3((unsigned)((M + 31) / 32)), dim3(256), 0,
                     (hipStream_t)stream, a);
  TVQ_PLAN("ffn_fwd M=%lld", (long long)M);
  return launch_status("tvq_ffn_fwd");
}

extern "C" int tvq_ffn_bwd(const float* gy, const float* pre, int64_t M, int64_t D,
                           const float* W1, const float* W2, const float* gate, float p,
                           const int64_t* seed_ptr, uint64_t offset, float* d_pre, float* dxn,
                           float* gy_gated, tvq_stream_t stream) {
  TVQ_CHECK_ARG(gy && pre && W1 && W2 && d_pre && dxn && M > 0 && D == FF_D && p >= 0.f &&
                    p < 1.f && (p == 0.f || seed_ptr),
                "tvq_ffn_bwd: bad arguments (D must be 128)");
  TVQ_CHECK_ARG(ff_aligned(gy) && ff_aligned(pre) && ff_aligned(d_pre) && ff_aligned(dxn) &&
                    ff_aligned(gy_gated),
                "tvq_ffn_bwd: pointers must be 16-byte aligned");
  FfArgs a = {};
  a.gy = gy; a.pre_in = pre; a.W1 = W1; a.W2 = W2; a.gate = gate;
  a.d_pre = d_pre; a.dxn = dxn; a.gy_gated = gate ? gy_gated : nullptr; a.seed_ptr = seed_ptr; a.offset = offset;
  a.p = p; a.scale = p > 0.f ? 1.0f / (1.0f - p) : 1.0f; a.M = (int)M;
  hipLaunchKernelGGL(ffn_bwd_kernel, dim3((unsigned)((M + 31) / 32)), dim3(256), 0,
                     (hipStream_t)stream, a);
  TVQ_PLAN("ffn_bwd M=%lld", (long long)M);
  return launch_status("tvq_ffn_bwd");
}

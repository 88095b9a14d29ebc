// Register-tile helpers of the priors' fused training kernels (tvq_ffn.hip: the feed-forward
// branch; tvq_xattn.hip: the attention branch), D = 128 token rows on the
// v_mfma_f32_32x32x2_f32 matrix cores.  A 32 x 32 tile in the "feature-major" layout holds
// X[token l & 31][f0 + ff_crow(r, l >> 5)] in register r of lane l: the MFMA accumulator layout
// of a tile whose columns are tokens.  A whole row in the "B-row" layout (ff_load_row) is 64
// registers v[16 q + r] = row[32 q + ff_crow(r, h)]: the concatenation of its four 32-feature
// tiles in that layout.
#pragma once
#include "tvq_common.h"

namespace tvq {

constexpr int FF_D = 128;  // model width == inner width (ff_mult 1)

__device__ __forceinline__ int ff_crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// B operand of a token row in the register layout: v[16 q + 4 g + e] = row[32 q + 8 g + 4 h + e]
__device__ __forceinline__ void ff_load_row(const float* __restrict__ row, int h, float (&v)[64]) {
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 x = *reinterpret_cast<const float4*>(row + 32 * q + 8 * g + 4 * h);
      v[16 * q + 4 * g] = x.x;
      v[16 * q + 4 * g + 1] = x.y;
      v[16 * q + 4 * g + 2] = x.z;
      v[16 * q + 4 * g + 3] = x.w;
    }
}

// acc[r] (row i = crow(r, h) of the wave's 32-row tile, column = the lane's token) +=
// sum_t A(i, k_t) B(k_t, token), k_t = 32 (t >> 4) + crow(t & 15, h): A from the weight row
// W[row0 + (l & 31)][k] (row-major, ld 128: 16-B loads) or, TRANS, W[k][col0 + (l & 31)]
// (the transposed access of a data gradient: one 4-B load per step, 128 B per half-wave).
// ff_wload issues all 64 A values of a tile at once (one L2 round trip per tile; a kernel can
// request the next tile's while it multiplies this one), ff_mma runs the 64 MFMA steps.
template <bool TRANS>
__device__ __forceinline__ void ff_wload(const float* __restrict__ W, int rc0, int lane,
                                         float (&wa)[64]) {
  const int i = lane & 31, h = lane >> 5;
  if (!TRANS) {
    const float* wr = W + (int64_t)(rc0 + i) * FF_D;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 v = *reinterpret_cast<const float4*>(wr + 32 * q + 8 * g + 4 * h);
        wa[16 * q + 4 * g] = v.x;
        wa[16 * q + 4 * g + 1] = v.y;
        wa[16 * q + 4 * g + 2] = v.z;
        wa[16 * q + 4 * g + 3] = v.w;
      }
  } else {
    const float* wc = W + rc0 + i;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) wa[16 * q + r] = wc[(int64_t)(32 * q + ff_crow(r, h)) * FF_D];
  }
}
__device__ __forceinline__ floatx16 ff_mma(const float (&wa)[64], const float (&b)[64], floatx16 acc) {
#pragma unroll
  for (int t = 0; t < 64; ++t) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[t], b[t], acc, 0, 0, 0);
  return acc;
}
__device__ __forceinline__ floatx16 ff_zero() {
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  return acc;
}
template <bool TRANS>
__device__ __forceinline__ floatx16 ff_tile_acc(const float* __restrict__ W, int rc0,
                                                const float (&b)[64], int lane, floatx16 acc) {
  float wa[64];
  ff_wload<TRANS>(W, rc0, lane, wa);
  return ff_mma(wa, b, acc);
}
template <bool TRANS>
__device__ __forceinline__ floatx16 ff_tile(const float* __restrict__ W, int rc0, const float (&b)[64],
                                            int lane) {
  return ff_tile_acc<TRANS>(W, rc0, b, lane, ff_zero());
}

// 4 values of a per-feature vector for register group g of tile w: p[32 w + 8 g + 4 h ..]
__device__ __forceinline__ float4 ff_vec4(const float* __restrict__ p, int w, int g, int h) {
  return *reinterpret_cast<const float4*>(p + 32 * w + 8 * g + 4 * h);
}

// the 4 waves' tiles -> every wave's B operand (the LDS holds them in register order)
__device__ __forceinline__ void ff_exchange(float4 (*buf)[4][64], int w, const float (&mine)[16],
                                            float (&b)[64], int lane) {
#pragma unroll
  for (int g = 0; g < 4; ++g)
    buf[w][g][lane] = make_float4(mine[4 * g], mine[4 * g + 1], mine[4 * g + 2], mine[4 * g + 3]);
  __syncthreads();
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 v = buf[t][g][lane];
      b[16 * t + 4 * g] = v.x;
      b[16 * t + 4 * g + 1] = v.y;
      b[16 * t + 4 * g + 2] = v.z;
      b[16 * t + 4 * g + 3] = v.w;
    }
}

}  // namespace tvq

// BatchNorm training-statistics finalization shared by tvq_norm.hip (the standalone BN
// kernels) and tvq_resblock.hip (the fused small-channel ResBlock): per-channel partial
// sums in fp64 -> mean / invstd / affine scale+shift / running stats (forward) and the
// backward coefficients + parameter gradients, in a fixed combine order.
#pragma once
#include "tvq_common.h"

namespace tvq {

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double block_sum_d(double v, double* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
  return t;
}

// s[k] = sum over i < chunks of part[(c*chunks + i)*NS + k]: per lane in increasing i (the
// lane's write-through loads all issued before the adds), then a fixed xor tree
template <int NS>
__device__ __forceinline__ void wave_chunk_sums(const double* part, int c, int chunks, int lane,
                                                double (&s)[NS]) {
#pragma unroll
  for (int k = 0; k < NS; ++k) s[k] = 0.0;
  for (int i0 = lane; i0 < chunks; i0 += 64 * 8) {
    double v[8][NS];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + 64 * u;
#pragma unroll
      for (int k = 0; k < NS; ++k)
        v[u][k] = i < chunks ? ld_wt(part + ((int64_t)c * chunks + i) * NS + k) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int k = 0; k < NS; ++k) s[k] += v[u][k];
  }
#pragma unroll
  for (int k = 0; k < NS; ++k) s[k] = wave_sum_d(s[k]);
}

struct BNFinal {  // per-channel finalize of the training statistics
  int C, chunks;
  int64_t N;
  float eps, momentum;
  const float *w, *b;
  float *rmean, *rvar;
  int64_t* nbt;
  float *save_mean, *save_invstd, *scale, *shift;
};

// one wave (lane 0..63) finalizes channel c: lanes stride the chunk partials, fixed
// xor-tree combine; running stats with momentum, unbiased running var
// channel c's affine scale / shift from its sums (s1 = sum x, s2 = sum x^2); `write`: also
// store save_mean / save_invstd / scale / shift and update the running statistics
__device__ __forceinline__ void bn_final_from_sums(double s1, double s2, int c, const BNFinal& f,
                                                   bool write, float& sc, float& sh) {
  const double mean = s1 / (double)f.N;
  double var = s2 / (double)f.N - mean * mean;
  if (var < 0.0) var = 0.0;
  const double invstd = 1.0 / sqrt(var + (double)f.eps);
  sc = (float)((double)(f.w ? f.w[c] : 1.f) * invstd);
  sh = (f.b ? f.b[c] : 0.f) - (float)mean * sc;
  if (!write) return;
  if (f.rmean) {
    const double unb = f.N > 1 ? var * (double)f.N / (double)(f.N - 1) : var;
    f.rmean[c] = (float)((1.0 - f.momentum) * f.rmean[c] + f.momentum * mean);
    f.rvar[c] = (float)((1.0 - f.momentum) * f.rvar[c] + f.momentum * unb);
  }
  f.save_mean[c] = (float)mean;
  f.save_invstd[c] = (float)invstd;
  f.scale[c] = sc;
  f.shift[c] = sh;
}

__device__ __forceinline__ void bn_final_channel(const double* part, int c, int lane,
                                                 const BNFinal& f) {
  if (c == 0 && lane == 0 && f.nbt) f.nbt[0] += 1;
  double s[2];
  wave_chunk_sums<2>(part, c, f.chunks, lane, s);
  if (lane != 0) return;
  float sc, sh;
  bn_final_from_sums(s[0], s[1], c, f, true, sc, sh);
}

struct BNBwdFinal {
  int C, chunks;
  float *coef, *dw, *db, *da;
  int accumulate;
};

// coef[c] = (sum ds, sum ds*xhat) and the parameter grads of channel c (one wave)
// the parameter gradients of channel c from its sums (s0 = sum ds, s1 = sum ds*xhat,
// s2 = the Snake a term)
__device__ __forceinline__ void bn_bwd_params_from_sums(double s0, double s1, double s2, int c,
                                                        const BNBwdFinal& f) {
  if (f.dw) f.dw[c] = f.accumulate ? f.dw[c] + (float)s1 : (float)s1;
  if (f.db) f.db[c] = f.accumulate ? f.db[c] + (float)s0 : (float)s0;
  if (f.da) f.da[c] = f.accumulate ? f.da[c] + (float)s2 : (float)s2;
}

__device__ __forceinline__ void bn_bwd_final_channel(const double* part, int c, int lane,
                                                     const BNBwdFinal& f) {
  double s[3];
  wave_chunk_sums<3>(part, c, f.chunks, lane, s);
  if (lane != 0) return;
  f.coef[2 * c] = (float)s[0];
  f.coef[2 * c + 1] = (float)s[1];
  bn_bwd_params_from_sums(s[0], s[1], s[2], c, f);
}

__device__ __forceinline__ void snake_bwd_final_channel(const double* part, int C, int chunks,
                                                        int c, float* da, int accumulate) {
  double s[1];
  wave_chunk_sums<1>(part, c, chunks, threadIdx.x & 63, s);
  if (threadIdx.x == 0) da[c] = accumulate ? da[c] + (float)s[0] : (float)s[0];
}

// separate finishing launches (no counter pool registered)
void bn_stats_final_launch(const double* part, const BNFinal& f, hipStream_t st);
void bn_bwd_final_launch(const double* part, const BNBwdFinal& f, hipStream_t st);
void snake_da_final_launch(const double* part, int C, int chunks, float* da, int accumulate,
                           hipStream_t st);

}  // namespace tvq

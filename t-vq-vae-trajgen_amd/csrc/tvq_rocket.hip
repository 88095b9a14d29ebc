// ROCKET random-convolution features for gfx950.
//
// Reference: timevqvae/evaluation/rocket_functions.py:60-126 (apply_kernel /
// apply_kernels, numba on the CPU).  For every (series, kernel): the dilated, optionally
// padded 1-D correlation s_i = bias + sum_t w_t x[i + t d] over i in [-p, L + p - (len-1) d),
// and two features, ppv = #(s_i > 0) / output_length and max_i s_i.
//
// One block per (series, 64 kernels): the series is staged once in LDS (float64), each
// wave takes a kernel at a time with its weights in scalar registers and its 64 lanes on
// consecutive output positions (conflict-free ds_read_b64), and reduces ppv / max across
// the wave with shuffles.  Arithmetic is float64 with separate multiply and add in t
// order (no contraction), so results equal the reference's interpreted float64 loop
// bit for bit.  HBM traffic is tiny (the series once per block); the bound is the
// LDS/FP64 issue rate.
#include <float.h>

#include "tvq_common.h"

namespace tvq {

constexpr int ROCKET_KPB = 64;  // kernels per block
constexpr int ROCKET_MAXLEN = 16;

__global__ __launch_bounds__(256) void rocket_kernel(
    const double* __restrict__ X, int L, int64_t ldx, const double* __restrict__ w,
    const int32_t* __restrict__ woff, const int32_t* __restrict__ lengths,
    const double* __restrict__ biases, const int32_t* __restrict__ dilations,
    const int32_t* __restrict__ paddings, int nk, double* __restrict__ out) {
  extern __shared__ double xs[];
  const int e = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const double* x = X + (int64_t)e * ldx;
  for (int i = threadIdx.x; i < L; i += blockDim.x) xs[i] = x[i];
  __syncthreads();
  const int k0 = blockIdx.y * ROCKET_KPB;
  const int k1 = min(nk, k0 + ROCKET_KPB);
  for (int k = k0 + wid; k < k1; k += 4) {
    const int len = lengths[k];
    const int d = dilations[k], p = paddings[k];
    if (len < 1 || len > ROCKET_MAXLEN || d < 1) {  // outside the ABI contract: loud NaNs
      if (lane == 0) {
        double* o = out + (int64_t)e * 2 * nk + 2 * k;
        o[0] = o[1] = __longlong_as_double(0x7ff8000000000000ll);
      }
      continue;
    }
    const double b = biases[k];
    double wk[ROCKET_MAXLEN];
#pragma unroll
    for (int t = 0; t < ROCKET_MAXLEN; ++t) wk[t] = t < len ? w[woff[k] + t] : 0.0;
    const int end = (L + p) - (len - 1) * d;
    const int olen = (L + 2 * p) - (len - 1) * d;
    int ppv = 0;
    double mx = -INFINITY;
    for (int i = -p + lane; i < end; i += 64) {
#pragma clang fp contract(off)
      double s = b;
      int idx = i;
#pragma unroll
      for (int t = 0; t < ROCKET_MAXLEN; ++t) {
        if (t < len) {
          const bool ok = idx > -1 && idx < L;
          const double xv = xs[ok ? idx : 0];
          if (ok) s = s + wk[t] * xv;  // unfused (contract off): the reference's rounding
        }
        idx += d;
      }
      if (s > mx) mx = s;
      ppv += s > 0.0 ? 1 : 0;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      ppv += __shfl_xor(ppv, o, 64);
      const double om = __shfl_xor(mx, o, 64);
      mx = om > mx ? om : mx;
    }
    if (lane == 0) {
      double* o = out + (int64_t)e * 2 * nk + 2 * k;
      o[0] = (double)ppv / (double)olen;
      o[1] = mx;
    }
  }
}

}  // namespace tvq

using namespace tvq;

extern "C" int tvq_rocket_apply(const double* X, int64_t n, int64_t L, int64_t ldx,
                                const double* weights, const int32_t* woff,
                                const int32_t* lengths, const double* biases,
                                const int32_t* dilations, const int32_t* paddings, int64_t nk,
                                double* out, tvq_stream_t stream) {
  TVQ_CHECK_ARG(X && weights && woff && lengths && biases && dilations && paddings && out &&
                    n > 0 && nk > 0 && L > 0 && ldx >= L,
                "tvq_rocket_apply: bad arguments");
  TVQ_CHECK_ARG(L * 8 <= 64 * 1024, "tvq_rocket_apply: series length %lld exceeds 8192",
                (long long)L);
  TVQ_CHECK_ARG(n < (1ll << 31) && (nk + ROCKET_KPB - 1) / ROCKET_KPB < 65536,
                "tvq_rocket_apply: too many series or kernels");
  dim3 grid((unsigned)n, (unsigned)((nk + ROCKET_KPB - 1) / ROCKET_KPB));
  hipLaunchKernelGGL(rocket_kernel, grid, dim3(256), (size_t)L * 8, (hipStream_t)stream, X,
                     (int)L, ldx, weights, woff, lengths, biases, dilations, paddings, (int)nk,
                     out);
  return launch_status("tvq_rocket_apply");
}

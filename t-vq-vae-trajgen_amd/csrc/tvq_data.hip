// Trajectory data format on gfx950 (reference utils/data_utils.py:84-110 get_data and
// scripts/generate.py:14-20 post_processed_generated_trajectories):
//   rows = flights, columns = L timesteps x F features interleaved ([t0 f0, t0 f1, ...]),
//   sklearn MinMaxScaler(feature_range=(lo, hi)) fitted per column, then viewed as
//   (N, L, F) and transposed to the model's (N, F, L) layout.
// The fit is a column min/max (exact in any order: deterministic); the transform fuses the
// scale with the (L, F) -> (F, L) transpose and the float64 -> float32 cast, in sklearn's
// float64 arithmetic, so the result equals sklearn's bit for bit.  The inverse reproduces
// numpy's in-place float32 `X -= min_; X /= scale_` (each op in float64, rounded to
// float32) fused with the (F, L) -> (L, F) transpose.
#include "tvq_common.h"

namespace tvq {
namespace {

constexpr int MM_CHUNKS = 64;  // row chunks of the column min/max partial pass

__global__ __launch_bounds__(256) void colminmax_partial(const double* __restrict__ X, int64_t N,
                                                         int64_t Fc, double* __restrict__ part) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= Fc) return;
  const int64_t per = (N + gridDim.y - 1) / gridDim.y;
  const int64_t r0 = blockIdx.y * per, r1 = min(N, r0 + per);
  double mn = NAN, mx = NAN;  // fmin / fmax skip NaN (np.nanmin / np.nanmax)
  for (int64_t r = r0; r < r1; ++r) {
    const double v = X[r * Fc + c];
    mn = fmin(mn, v);
    mx = fmax(mx, v);
  }
  part[(int64_t)blockIdx.y * 2 * Fc + c] = mn;
  part[(int64_t)blockIdx.y * 2 * Fc + Fc + c] = mx;
}

// MinMaxScaler._partial_fit / fit (sklearn): data_range = max - min, zero ranges -> 1
// (_handle_zeros_in_scale), scale_ = (hi - lo) / range, min_ = lo - data_min * scale_.
__global__ __launch_bounds__(256) void colminmax_finish(const double* __restrict__ part, int chunks,
                                                        int64_t Fc, double lo, double hi,
                                                        double* __restrict__ data_min,
                                                        double* __restrict__ data_max,
                                                        double* __restrict__ scale,
                                                        double* __restrict__ min_) {
#pragma clang fp contract(off)
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= Fc) return;
  double mn = NAN, mx = NAN;
  for (int k = 0; k < chunks; ++k) {
    mn = fmin(mn, part[(int64_t)k * 2 * Fc + c]);
    mx = fmax(mx, part[(int64_t)k * 2 * Fc + Fc + c]);
  }
  double range = mx - mn;
  if (range < 10.0 * 2.220446049250313e-16) range = 1.0;  // _handle_zeros_in_scale
  const double s = (hi - lo) / range;
  data_min[c] = mn;
  data_max[c] = mx;
  scale[c] = s;
  min_[c] = lo - mn * s;  // contract(off): numpy's two roundings, no FMA
}

// out[n, f, l] = (float)(X[n, l F + f] * scale[l F + f] + min_[l F + f]); one thread per
// output element, the write coalesced along l.
__global__ __launch_bounds__(256) void minmax_transform(const double* __restrict__ X, int64_t N,
                                                        int L, int F,
                                                        const double* __restrict__ scale,
                                                        const double* __restrict__ min_,
                                                        float* __restrict__ out) {
#pragma clang fp contract(off)
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t per = (int64_t)L * F;
  if (t >= N * per) return;
  const int64_t n = t / per;
  const int r = (int)(t - n * per);
  const int f = r / L, l = r - f * L;
  const int c = l * F + f;
  double v = X[n * per + c];
  v = v * scale[c] + min_[c];  // X *= scale_; X += min_ (contract(off): two roundings)
  out[t] = (float)v;
}

// out[n, l F + f] = fl(fl(x[n, f, l] - min_) / scale) (numpy float32 in-place ops with
// float64 operands), one thread per output element, the write coalesced.
__global__ __launch_bounds__(256) void minmax_inverse(const float* __restrict__ x, int64_t N, int L,
                                                      int F, const double* __restrict__ scale,
                                                      const double* __restrict__ min_,
                                                      float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t per = (int64_t)L * F;
  if (t >= N * per) return;
  const int64_t n = t / per;
  const int c = (int)(t - n * per);
  const int l = c / F, f = c - l * F;
  const float v1 = (float)((double)x[n * per + (int64_t)f * L + l] - min_[c]);
  out[t] = (float)((double)v1 / scale[c]);
}

}  // namespace
}  // namespace tvq

using namespace tvq;

extern "C" {

int64_t tvq_minmax_fit_workspace(int64_t Fc) { return (int64_t)MM_CHUNKS * 2 * Fc; }

int tvq_minmax_fit(const double* X, int64_t N, int64_t Fc, double lo, double hi, double* data_min,
                   double* data_max, double* scale, double* min_, double* workspace,
                   tvq_stream_t stream) {
  TVQ_CHECK_ARG(X && data_min && data_max && scale && min_ && workspace && N > 0 && Fc > 0 && hi > lo,
                "tvq_minmax_fit: bad arguments");
  const unsigned gx = (unsigned)((Fc + 255) / 256);
  const int chunks = (int)(N < MM_CHUNKS ? N : MM_CHUNKS);
  hipLaunchKernelGGL(colminmax_partial, dim3(gx, (unsigned)chunks), dim3(256), 0,
                     (hipStream_t)stream, X, N, Fc, workspace);
  hipLaunchKernelGGL(colminmax_finish, dim3(gx), dim3(256), 0, (hipStream_t)stream, workspace,
                     chunks, Fc, lo, hi, data_min, data_max, scale, min_);
  return launch_status("tvq_minmax_fit");
}

int tvq_minmax_transform(const double* X, int64_t N, int64_t L, int64_t F, const double* scale,
                         const double* min_, float* out, tvq_stream_t stream) {
  TVQ_CHECK_ARG(X && scale && min_ && out && N > 0 && L > 0 && F > 0,
                "tvq_minmax_transform: bad arguments");
  const int64_t n = N * L * F;
  hipLaunchKernelGGL(minmax_transform, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, X, N, (int)L, (int)F, scale, min_, out);
  return launch_status("tvq_minmax_transform");
}

int tvq_minmax_inverse(const float* x, int64_t N, int64_t L, int64_t F, const double* scale,
                       const double* min_, float* out, tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && scale && min_ && out && N > 0 && L > 0 && F > 0,
                "tvq_minmax_inverse: bad arguments");
  const int64_t n = N * L * F;
  hipLaunchKernelGGL(minmax_inverse, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, x, N, (int)L, (int)F, scale, min_, out);
  return launch_status("tvq_minmax_inverse");
}

}  // extern "C"

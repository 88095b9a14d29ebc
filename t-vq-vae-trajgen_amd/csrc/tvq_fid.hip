// FID feature statistics for gfx950.
//
// Reference: timevqvae/evaluation/eval_utils.py:56-81 calculate_fid: mu = z.mean(0),
// sigma = np.cov(z, rowvar=False) (float64, divisor N-1), then on the host
// ssdiff + trace(s1 + s2 - 2 sqrtm(s1 s2)).  Here the two O(N D^2) moments run on the
// device in float64; the D x D matrix square root stays on the host in float64
// (scipy.linalg.sqrtm, as the reference), see timevqvae/evaluation/eval_utils.py.
//
//   fid_mean_kernel   mu[d] = (sum_n z[n, d]) / N, one thread per column, rows in order
//   fid_cov_kernel    one block per upper-triangular 64 x 64 tile (ti <= tj): the centred
//                     rows of both column panels are staged through LDS 32 at a time,
//                     each thread accumulates a 4 x 4 fp64 sub-tile in row order, the
//                     tile is written to (ti, tj) and mirrored to (tj, ti).
// Every sum has a fixed order, so results are run-to-run identical.  The bound is the
// fp64 FMA rate (2 N D^2 flop; the N x D input is read D/64 times from L2).
#include "tvq_common.h"

namespace tvq {

constexpr int FID_T = 64;   // output tile edge
constexpr int FID_R = 32;   // rows staged per step

__global__ __launch_bounds__(256) void fid_mean_kernel(const double* __restrict__ z, int64_t N,
                                                       int64_t D, double* __restrict__ mu) {
  const int64_t d = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (d >= D) return;
  double s = 0.0;
  for (int64_t n = 0; n < N; ++n) s += z[n * D + d];
  mu[d] = s / (double)N;
}

__global__ __launch_bounds__(256) void fid_cov_kernel(const double* __restrict__ z, int64_t N,
                                                      int64_t D, const double* __restrict__ mu,
                                                      double* __restrict__ cov, int nt) {
  __shared__ double As[FID_R][FID_T + 1];
  __shared__ double Bs[FID_R][FID_T + 1];
  // blockIdx.x -> (ti, tj), ti <= tj, row-major over the upper triangle
  int t = blockIdx.x, ti = 0;
  while (t >= nt - ti) {
    t -= nt - ti;
    ++ti;
  }
  const int tj = ti + t;
  const int64_t i0 = (int64_t)ti * FID_T, j0 = (int64_t)tj * FID_T;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;  // 16 x 16 threads, 4 x 4 each
  double acc[4][4] = {};
  for (int64_t n0 = 0; n0 < N; n0 += FID_R) {
    for (int e = threadIdx.x; e < FID_R * FID_T; e += 256) {
      const int r = e / FID_T, c = e - r * FID_T;
      const int64_t n = n0 + r;
      const int64_t ci = i0 + c, cj = j0 + c;
      As[r][c] = (n < N && ci < D) ? z[n * D + ci] - mu[ci] : 0.0;
      Bs[r][c] = (n < N && cj < D) ? z[n * D + cj] - mu[cj] : 0.0;
    }
    __syncthreads();
#pragma unroll 4
    for (int r = 0; r < FID_R; ++r) {
      double a[4], b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] = As[r][ty + 16 * u];
        b[u] = Bs[r][tx + 16 * u];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[u][v] = fma(a[u], b[v], acc[u][v]);
    }
    __syncthreads();
  }
  const double inv = 1.0 / (double)(N - 1);
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int64_t i = i0 + ty + 16 * u, j = j0 + tx + 16 * v;
      if (i < D && j < D) {
        const double c = acc[u][v] * inv;
        cov[i * D + j] = c;
        if (ti != tj) cov[j * D + i] = c;
      }
    }
}

}  // namespace tvq

using namespace tvq;

// mu (D) and the sample covariance (D x D, divisor N-1) of the rows of z (N x D, float64,
// row-major), as numpy's z.mean(0) / np.cov(z, rowvar=False).
extern "C" int tvq_fid_moments(const double* z, int64_t N, int64_t D, double* mu, double* cov,
                               tvq_stream_t stream) {
  TVQ_CHECK_ARG(z && mu && cov && N >= 2 && D >= 1, "tvq_fid_moments: bad arguments");
  TVQ_CHECK_ARG(D <= (1 << 20), "tvq_fid_moments: D too large");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(fid_mean_kernel, dim3((unsigned)((D + 255) / 256)), dim3(256), 0, st, z, N,
                     D, mu);
  const int nt = (int)((D + FID_T - 1) / FID_T);
  const int64_t tiles = (int64_t)nt * (nt + 1) / 2;
  hipLaunchKernelGGL(fid_cov_kernel, dim3((unsigned)tiles), dim3(256), 0, st, z, N, D, mu, cov,
                     nt);
  return launch_status("tvq_fid_moments");
}

// BatchNorm2d/1d (+ fused SnakeActivation), standalone Snake, dropout backward.
//
// BN training statistics accumulate in fp64 (torch's CPU accumulator type for
// fp32): per-(channel, chunk) partial sums -> per-channel finalize (done by the last
// block of the channel when a counter pool is registered, else a second launch)
// (mean, biased var for normalisation, unbiased var for running_var, momentum
// 0.1, num_batches_tracked += 1) producing the affine form y = x*scale + shift
// (scale = w*invstd, shift = b - mean*scale), then one streaming apply kernel
// that also applies Snake:  x + (1/a) sin(a x)^2  (train_utils.py:421-448).
// Backward recomputes the BN output from x and (mean, invstd); reductions are
// fixed-order (deterministic).
#include "tvq_common.h"
#include "tvq_bn.h"

namespace tvq {

// per-channel reductions: chunks of ~2048 elements (8 per thread) so each thread has
// all its loads in flight at once and C*chunks blocks fill the chip
static constexpr int NU = 8;
static int bn_chunks(int64_t B, int64_t HW) {
  int64_t c = (B * HW + 256 * NU - 1) / (256 * NU);
  if (c > 512) c = 512;
  if (c < 1) c = 1;
  return (int)c;
}

// element i of channel c's (b, p) sequence -> flat NCHW offset; i*HW < 2^32 checked on host
__device__ __forceinline__ int64_t chan_off(int i, int C, int c, int HW, const Div16& dhw) {
  const int b = div16(i, dhw);
  return ((int64_t)b * C + c) * HW + (i - b * HW);
}

// partial [c][chunk][2] = (sum x, sum x^2); with `cnt`, the last block of channel c
// finalizes it (bn_final_channel) instead of a separate launch
__global__ __launch_bounds__(256) void bn_stats_partial_kernel(const float* __restrict__ x, int B,
                                                               int C, int HW, Div16 dhw,
                                                               int chunks,
                                                               double* __restrict__ part,
                                                               int* __restrict__ cnt, BNFinal f) {
  __shared__ double red[4];
  const int c = blockIdx.x, ch = blockIdx.y;
  const int tot = B * HW;
  const int per = (tot + chunks - 1) / chunks;
  const int lo = ch * per, hi = min(tot, lo + per);
  double s1 = 0.0, s2 = 0.0;
  for (int i0 = lo + threadIdx.x; i0 < hi; i0 += 256 * NU) {
    float v[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int i = i0 + u * 256;
      v[u] = x[chan_off(i < hi ? i : lo, C, c, HW, dhw)];
    }
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      if (i0 + u * 256 < hi) {
        s1 += (double)v[u];
        s2 += (double)v[u] * (double)v[u];
      }
    }
  }
  s1 = block_sum_d(s1, red);
  s2 = block_sum_d(s2, red);
  if (threadIdx.x == 0) {
    st_wt(part + ((int64_t)c * chunks + ch) * 2 + 0, s1);
    st_wt(part + ((int64_t)c * chunks + ch) * 2 + 1, s2);
  }
  if (cnt && last_block(cnt + c, chunks) && threadIdx.x < 64)
    bn_final_channel(part, c, threadIdx.x, f);
}

__global__ __launch_bounds__(64) void bn_stats_final_kernel(const double* __restrict__ part,
                                                            BNFinal f) {
  bn_final_channel(part, blockIdx.x, threadIdx.x, f);
}

__global__ void bn_eval_prep_kernel(const float* __restrict__ w, const float* __restrict__ b,
                                    const float* __restrict__ rm, const float* __restrict__ rv,
                                    float eps, int C, float* __restrict__ scale,
                                    float* __restrict__ shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float inv = 1.0f / sqrtf(rv[c] + eps);
  const float sc = (w ? w[c] : 1.f) * inv;
  scale[c] = sc;
  shift[c] = (b ? b[c] : 0.f) - rm[c] * sc;
}

__device__ __forceinline__ float snake_fwd(float s, float a) {
  const float inv = 1.0f / a;
  const float sn = sinf(a * s);
  return s + inv * (sn * sn);
}

// y = snake?(x*scale[c] + shift[c]) over the flat NCHW tensor; channel = (i / HW) % C
__global__ __launch_bounds__(256) void affine_snake_kernel(const float* __restrict__ x, int n,
                                                           int C, int HW, Div16 dhw,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift,
                                                           const float* __restrict__ a,
                                                           float* __restrict__ y) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int c = div16(i, dhw) % C;
    const float sc = scale ? scale[c] : 1.f, sh = shift ? shift[c] : 0.f;
    float s = fmaf(x[i], sc, sh);
    if (a) s = snake_fwd(s, a[c]);
    y[i] = s;
  }
}

// Training BatchNorm (+ Snake) from the per-block statistics the producing conv wrote in its
// epilogue (tvq_conv2d_fwd_bnstats, the stride-2 EncBlock / DecBlock convs): block (c, ch)
// sums channel c's nblk partial pairs in one fixed order -- the same in every block of the
// channel, so all agree bit for bit -- finalizes them (bn_final_channel's arithmetic; block
// (c, 0) writes save / running statistics, block (0, 0) num_batches_tracked) and applies
// affine + Snake (affine_snake_kernel's arithmetic) to chunk ch of the channel.  One launch
// instead of bn_stats_partial (a full read of x) + affine_snake.
__global__ __launch_bounds__(256) void bn_apply_part_kernel(const float* __restrict__ x, int B,
                                                            int C, int HW, Div16 dhw, int chunks,
                                                            const double* __restrict__ part,
                                                            int nblk, BNFinal f,
                                                            const float* __restrict__ a,
                                                            float* __restrict__ y) {
  __shared__ double red[4];
  const int c = blockIdx.x, ch = blockIdx.y;
  const double* pc = part + (int64_t)c * nblk * 2;
  double s1 = 0.0, s2 = 0.0;
  for (int i0 = threadIdx.x; i0 < nblk; i0 += 256 * 4) {
    double v[4][2];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + 256 * u;
      v[u][0] = i < nblk ? pc[2 * i] : 0.0;
      v[u][1] = i < nblk ? pc[2 * i + 1] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      s1 += v[u][0];
      s2 += v[u][1];
    }
  }
  s1 = block_sum_d(s1, red);
  s2 = block_sum_d(s2, red);
  if (c == 0 && ch == 0 && threadIdx.x == 0 && f.nbt) f.nbt[0] += 1;
  float sc, sh;
  bn_final_from_sums(s1, s2, c, f, ch == 0 && threadIdx.x == 0, sc, sh);
  const float av = a ? a[c] : 1.f;
  const int tot = B * HW;
  const int per = (tot + chunks - 1) / chunks;
  const int lo = ch * per, hi = min(tot, lo + per);
  for (int i0 = lo + threadIdx.x; i0 < hi; i0 += 256 * NU) {
    float v[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int i = i0 + u * 256;
      v[u] = x[chan_off(i < hi ? i : lo, C, c, HW, dhw)];
    }
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int i = i0 + u * 256;
      if (i >= hi) continue;
      float t = fmaf(v[u], sc, sh);
      if (a) t = snake_fwd(t, av);
      y[chan_off(i, C, c, HW, dhw)] = t;
    }
  }
}

// backward partials: [c][chunk][3] = (sum ds, sum ds*xhat, sum da-term); with `cnt`
// the last block of channel c finalizes it
__global__ __launch_bounds__(256) void bn_bwd_partial_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, int B, int C, int HW, Div16 dhw,
    int chunks, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ a,
    double* __restrict__ part, int* __restrict__ cnt, BNBwdFinal f) {
  __shared__ double red[4];
  const int c = blockIdx.x, ch = blockIdx.y;
  const int tot = B * HW;
  const int per = (tot + chunks - 1) / chunks;
  const int lo = ch * per, hi = min(tot, lo + per);
  const float mu = mean[c], is = invstd[c], sc = scale[c], sh = shift[c];
  const float av = a ? a[c] : 1.f, inv_a = 1.0f / av;
  double s_ds = 0.0, s_dsx = 0.0, s_da = 0.0;
  for (int i0 = lo + threadIdx.x; i0 < hi; i0 += 256 * NU) {
    float xv[NU], g[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int i = i0 + u * 256;
      const int64_t o = chan_off(i < hi ? i : lo, C, c, HW, dhw);
      xv[u] = x[o];
      g[u] = dy[o];
    }
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      if (i0 + u * 256 >= hi) continue;
      float ds = g[u];
      if (a) {
        const float s = fmaf(xv[u], sc, sh);
        float sn, cs;
        sincosf(av * s, &sn, &cs);
        const float t = 2.0f * sn * cs;
        ds = g[u] + g[u] * inv_a * t * av;
        s_da += (double)(g[u] * inv_a * t * s) - (double)(g[u] * (sn * sn) * inv_a * inv_a);
      }
      const float xhat = (xv[u] - mu) * is;
      s_ds += ds;
      s_dsx += (double)ds * xhat;
    }
  }
  s_ds = block_sum_d(s_ds, red);
  s_dsx = block_sum_d(s_dsx, red);
  s_da = block_sum_d(s_da, red);
  if (threadIdx.x == 0) {
    double* pp = part + ((int64_t)c * chunks + ch) * 3;
    st_wt(pp + 0, s_ds);
    st_wt(pp + 1, s_dsx);
    st_wt(pp + 2, s_da);
  }
  if (cnt && last_block(cnt + c, chunks) && threadIdx.x < 64)
    bn_bwd_final_channel(part, c, threadIdx.x, f);
}

__global__ __launch_bounds__(64) void bn_bwd_final_kernel(const double* __restrict__ part,
                                                          BNBwdFinal f) {
  bn_bwd_final_channel(part, blockIdx.x, threadIdx.x, f);
}

// dx = w*invstd/N * (N*ds - sum ds - xhat * sum ds*xhat), flat over NCHW
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, int n, int C, int HW, Div16 dhw,
    int64_t N, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ w, const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ a, const float* __restrict__ coef, float* __restrict__ dx) {
  const float invN = 1.0f / (float)N;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int c = div16(i, dhw) % C;
    const float mu = mean[c], is = invstd[c], sc = scale[c], sh = shift[c];
    const float wc = w ? w[c] : 1.f;
    const float mds = coef[2 * c] * invN, mdsx = coef[2 * c + 1] * invN;
    const float xv = x[i], g = dy[i];
    float ds = g;
    if (a) {
      const float av = a[c], inv_a = 1.0f / av;
      const float s = fmaf(xv, sc, sh);
      float sn, cs;
      sincosf(av * s, &sn, &cs);
      ds = g + g * inv_a * (2.0f * sn * cs) * av;
    }
    const float xhat = (xv - mu) * is;
    dx[i] = wc * is * (ds - mds - xhat * mdsx);
  }
}

__global__ __launch_bounds__(256) void snake_fwd_kernel(const float* __restrict__ x, int n, int C,
                                                        int HW, Div16 dhw,
                                                        const float* __restrict__ a,
                                                        float* __restrict__ y) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
    y[i] = snake_fwd(x[i], a[div16(i, dhw) % C]);
}

// dx (elementwise) and per-(channel, chunk) partials of da; with `cnt` the last block
// of channel c sums them into da[c]
__global__ __launch_bounds__(256) void snake_bwd_kernel(const float* __restrict__ dy,
                                                        const float* __restrict__ x, int B, int C,
                                                        int HW, Div16 dhw, int chunks,
                                                        const float* __restrict__ a,
                                                        const float* __restrict__ dx_add,
                                                        float* __restrict__ dx,
                                                        double* __restrict__ part,
                                                        int* __restrict__ cnt,
                                                        float* __restrict__ da, int accumulate) {
  __shared__ double red[4];
  const int c = blockIdx.x, ch = blockIdx.y;
  const int tot = B * HW;
  const int per = (tot + chunks - 1) / chunks;
  const int lo = ch * per, hi = min(tot, lo + per);
  const float av = a[c], inv_a = 1.0f / av;
  double s_da = 0.0;
  for (int i0 = lo + threadIdx.x; i0 < hi; i0 += 256 * NU) {
    float xv[NU], g[NU];
    int64_t o[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int i = i0 + u * 256;
      o[u] = chan_off(i < hi ? i : lo, C, c, HW, dhw);
      xv[u] = x[o[u]];
      g[u] = dy[o[u]];
    }
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      if (i0 + u * 256 >= hi) continue;
      float sn, cs;
      sincosf(av * xv[u], &sn, &cs);
      const float t = 2.0f * sn * cs;
      const float d = g[u] + g[u] * inv_a * t * av;
      dx[o[u]] = dx_add ? d + dx_add[o[u]] : d;
      s_da += (double)(g[u] * inv_a * t * xv[u]) - (double)(g[u] * (sn * sn) * inv_a * inv_a);
    }
  }
  s_da = block_sum_d(s_da, red);
  if (threadIdx.x == 0) st_wt(part + (int64_t)c * chunks + ch, s_da);
  if (cnt && last_block(cnt + c, chunks) && threadIdx.x < 64)
    snake_bwd_final_channel(part, C, chunks, c, da, accumulate);
}

__global__ __launch_bounds__(64) void snake_bwd_final_kernel(const double* __restrict__ part,
                                                             int C, int chunks,
                                                             float* __restrict__ da,
                                                             int accumulate) {
  snake_bwd_final_channel(part, C, chunks, blockIdx.x, da, accumulate);
}

__global__ void dropout_bwd_kernel(const float* __restrict__ dy, int64_t n, float p, float scale,
                                   const int64_t* __restrict__ seed_ptr, uint64_t offset,
                                   float* __restrict__ dx) {
  const uint64_t seed = mix_seed(seed_ptr, offset);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dx[i] = (uniform01(seed, (uint64_t)i) >= p) ? dy[i] * scale : 0.f;
}

// ---- whole-channel forms: one block owns a channel (B*HW <= BNC_T * PT elements, held
// in registers), so the statistics and the apply are one launch with no cross-block
// hand-off.  Per-thread sums in element order, then block_sum_d's fixed tree.
constexpr int BNC_T = 512;

// training forward: sums -> bn_final_channel's arithmetic (thread 0 publishes save /
// running statistics / scale / shift) -> y = snake?(x*scale + shift)
template <int PT>
__global__ __launch_bounds__(BNC_T) void bn_train_chan_kernel(const float* __restrict__ x, int B,
                                                             int C, int HW, Div16 dhw,
                                                             const float* __restrict__ a,
                                                             float* __restrict__ y, BNFinal f) {
  __shared__ double red[BNC_T / 64];
  const int c = blockIdx.x, tid = threadIdx.x, tot = B * HW;
  float v[PT];
  int64_t o[PT];
#pragma unroll
  for (int u = 0; u < PT; ++u) {
    const int i = tid + BNC_T * u;
    o[u] = chan_off(i < tot ? i : 0, C, c, HW, dhw);
    v[u] = x[o[u]];
  }
  double s1 = 0.0, s2 = 0.0;
#pragma unroll
  for (int u = 0; u < PT; ++u)
    if (tid + BNC_T * u < tot) {
      s1 += (double)v[u];
      s2 += (double)v[u] * (double)v[u];
    }
  s1 = block_sum_d(s1, red);
  s2 = block_sum_d(s2, red);
  if (c == 0 && tid == 0 && f.nbt) f.nbt[0] += 1;
  float sc, sh;
  bn_final_from_sums(s1, s2, c, f, tid == 0, sc, sh);
  const float av = a ? a[c] : 1.f;
#pragma unroll
  for (int u = 0; u < PT; ++u) {
    if (tid + BNC_T * u >= tot) continue;
    float t = fmaf(v[u], sc, sh);
    if (a) t = snake_fwd(t, av);
    y[o[u]] = t;
  }
}

// backward: ds = dy * Snake'(x*scale + shift) (Snake a term), the three channel sums, the
// parameter gradients (thread 0), then dx = w*invstd*(ds - mean(ds) - xhat*mean(ds*xhat))
// -- bn_bwd_partial_kernel + bn_bwd_final_channel + bn_bwd_apply_kernel's arithmetic
template <int PT>
__global__ __launch_bounds__(BNC_T) void bn_bwd_chan_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, int B, int C, int HW, Div16 dhw,
    const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ w, const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ a, float* __restrict__ dx, BNBwdFinal f) {
  __shared__ double red[BNC_T / 64];
  const int c = blockIdx.x, tid = threadIdx.x, tot = B * HW;
  float xv[PT], g[PT];
  int64_t o[PT];
#pragma unroll
  for (int u = 0; u < PT; ++u) {
    const int i = tid + BNC_T * u;
    o[u] = chan_off(i < tot ? i : 0, C, c, HW, dhw);
    xv[u] = x[o[u]];
    g[u] = dy[o[u]];
  }
  const float mu = mean[c], is = invstd[c], sc = scale[c], sh = shift[c];
  const float av = a ? a[c] : 1.f, inv_a = 1.0f / av;
  double s_ds = 0.0, s_dsx = 0.0, s_da = 0.0;
#pragma unroll
  for (int u = 0; u < PT; ++u) {
    if (tid + BNC_T * u >= tot) continue;
    float ds = g[u];
    if (a) {
      const float s = fmaf(xv[u], sc, sh);
      float sn, cs;
      sincosf(av * s, &sn, &cs);
      const float t = 2.0f * sn * cs;
      ds = g[u] + g[u] * inv_a * t * av;
      s_da += (double)(g[u] * inv_a * t * s) - (double)(g[u] * (sn * sn) * inv_a * inv_a);
    }
    g[u] = ds;
    const float xhat = (xv[u] - mu) * is;
    s_ds += ds;
    s_dsx += (double)ds * xhat;
  }
  s_ds = block_sum_d(s_ds, red);
  s_dsx = block_sum_d(s_dsx, red);
  s_da = block_sum_d(s_da, red);
  if (tid == 0) bn_bwd_params_from_sums(s_ds, s_dsx, s_da, c, f);
  const float invN = 1.0f / (float)tot;
  const float wc = w ? w[c] : 1.f;
  const float mds = (float)s_ds * invN, mdsx = (float)s_dsx * invN;
#pragma unroll
  for (int u = 0; u < PT; ++u) {
    if (tid + BNC_T * u >= tot) continue;
    const float xhat = (xv[u] - mu) * is;
    dx[o[u]] = wc * is * (g[u] - mds - xhat * mdsx);
  }
}

// eval: y = snake?(x*scale + shift) with scale / shift from the running statistics
// (bn_eval_prep_kernel's arithmetic per element: no separate prep launch)
__global__ __launch_bounds__(256) void bn_eval_snake_kernel(
    const float* __restrict__ x, int n, int C, Div16 dhw, const float* __restrict__ w,
    const float* __restrict__ b, const float* __restrict__ rm, const float* __restrict__ rv,
    float eps, const float* __restrict__ a, float* __restrict__ y) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int c = div16(i, dhw) % C;
    const float inv = 1.0f / sqrtf(rv[c] + eps);
    const float sc = (w ? w[c] : 1.f) * inv;
    const float sh = (b ? b[c] : 0.f) - rm[c] * sc;
    float s = fmaf(x[i], sc, sh);
    if (a) s = snake_fwd(s, a[c]);
    y[i] = s;
  }
}

// whole-channel form for C >= 32 channels of <= BNC_T*48 elements (smaller C: 16-32
// blocks leave the chip idle, measured slower); returns the per-thread element count PT
// (0: the chunked form)
static int bn_chan_pt(int64_t B, int64_t C, int64_t HW) {
  constexpr int cmin = 32;
  const int64_t n = B * HW;
  if (C < cmin || n > (int64_t)BNC_T * 48) return 0;
  const int64_t pt = (n + BNC_T - 1) / BNC_T;
  return pt <= 8 ? 8 : pt <= 16 ? 16 : pt <= 24 ? 24 : pt <= 32 ? 32 : 48;
}

#define BNC_CASES(X) X(8) X(16) X(24) X(32) X(48)

void bn_stats_final_launch(const double* part, const BNFinal& f, hipStream_t st) {
  hipLaunchKernelGGL(bn_stats_final_kernel, dim3(f.C), dim3(64), 0, st, part, f);
}
void bn_bwd_final_launch(const double* part, const BNBwdFinal& f, hipStream_t st) {
  hipLaunchKernelGGL(bn_bwd_final_kernel, dim3(f.C), dim3(64), 0, st, part, f);
}
void snake_da_final_launch(const double* part, int C, int chunks, float* da, int accumulate,
                           hipStream_t st) {
  hipLaunchKernelGGL(snake_bwd_final_kernel, dim3(C), dim3(64), 0, st, part, C, chunks, da,
                     accumulate);
}

static dim3 ew_grid(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g > 16384) g = 16384;
  return dim3((unsigned)(g < 1 ? 1 : g));
}

// the flat index n = B*C*HW times HW must stay below 2^32 for div16
static bool norm_dims_ok(int64_t B, int64_t C, int64_t HW) {
  const int64_t n = B * C * HW;
  return n < (1ll << 31) && n * HW < (1ll << 32);
}

}  // namespace tvq

using namespace tvq;

extern "C" int64_t tvq_bn_workspace(int64_t B, int64_t C, int64_t HW) {
  // bytes: partials (C*chunks*3 doubles) + 6*C floats
  return (int64_t)C * bn_chunks(B, HW) * 3 * 8 + 6 * C * 4 + 64;
}

// Training-mode BatchNorm (+Snake).  save (3*C floats): mean | invstd | (scratch)
// The workspace must hold tvq_bn_workspace() bytes; it keeps scale/shift for bwd.
extern "C" int tvq_bn_train_fwd(const float* x, int64_t B, int64_t C, int64_t HW, const float* w,
                                const float* b, float* running_mean, float* running_var,
                                int64_t* num_batches_tracked, float momentum, float eps,
                                const float* snake_a, float* y, float* save_mean,
                                float* save_invstd, float* scale_shift, void* workspace,
                                tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && y && save_mean && save_invstd && scale_shift && workspace && B > 0 && C > 0,
                "tvq_bn_train_fwd: bad arguments");
  TVQ_CHECK_ARG(norm_dims_ok(B, C, HW), "tvq_bn_train_fwd: tensor too large");
  hipStream_t st = (hipStream_t)stream;
  const int chunks = bn_chunks(B, HW);
  const Div16 dhw = make_div16(HW);
  double* part = (double*)workspace;
  const BNFinal f = {(int)C, chunks, B * HW, eps, momentum, w, b, running_mean, running_var,
                     num_batches_tracked, save_mean, save_invstd, scale_shift, scale_shift + C};
  if (const int pt = bn_chan_pt(B, C, HW)) {
#define M_(PT)                                                                                \
  if (pt == PT)                                                                               \
    hipLaunchKernelGGL(bn_train_chan_kernel<PT>, dim3((int)C), dim3(BNC_T), 0, st, x, (int)B, \
                       (int)C, (int)HW, dhw, snake_a, y, f);
    BNC_CASES(M_)
#undef M_
    return launch_status("tvq_bn_train_fwd");
  }
  int* cnt = counters(C, FIN_NORM);
  hipLaunchKernelGGL(bn_stats_partial_kernel, dim3((int)C, chunks), dim3(256), 0, st, x, (int)B,
                     (int)C, (int)HW, dhw, chunks, part, cnt, f);
  if (!cnt)
    hipLaunchKernelGGL(bn_stats_final_kernel, dim3((int)C), dim3(64), 0, st, part, f);
  hipLaunchKernelGGL(affine_snake_kernel, ew_grid(B * C * HW), dim3(256), 0, st, x,
                     (int)(B * C * HW), (int)C, (int)HW, dhw, scale_shift, scale_shift + C, snake_a,
                     y);
  return launch_status("tvq_bn_train_fwd");
}

// Training BatchNorm (+Snake) forward from the producing conv's per-block statistics (part:
// C x nblk x 2 doubles, tvq_conv2d_fwd_bnstats); same outputs as tvq_bn_train_fwd.
extern "C" int tvq_bn_train_apply_part(const float* x, int64_t B, int64_t C, int64_t HW,
                                       const double* part, int64_t nblk, const float* w,
                                       const float* b, float* running_mean, float* running_var,
                                       int64_t* num_batches_tracked, float momentum, float eps,
                                       const float* snake_a, float* y, float* save_mean,
                                       float* save_invstd, float* scale_shift,
                                       tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && y && part && nblk > 0 && save_mean && save_invstd && scale_shift && B > 0 &&
                    C > 0,
                "tvq_bn_train_apply_part: bad arguments");
  TVQ_CHECK_ARG(norm_dims_ok(B, C, HW), "tvq_bn_train_apply_part: tensor too large");
  const int chunks = bn_chunks(B, HW);
  const BNFinal f = {(int)C, chunks, B * HW, eps, momentum, w, b, running_mean, running_var,
                     num_batches_tracked, save_mean, save_invstd, scale_shift, scale_shift + C};
  TVQ_PLAN("bn_apply_part C%lld nblk%lld", (long long)C, (long long)nblk);
  hipLaunchKernelGGL(bn_apply_part_kernel, dim3((unsigned)C, (unsigned)chunks), dim3(256), 0,
                     (hipStream_t)stream, x, (int)B, (int)C, (int)HW, make_div16(HW), chunks, part,
                     (int)nblk, f, snake_a, y);
  return launch_status("tvq_bn_train_apply_part");
}

// Eval-mode BatchNorm (+Snake) from running statistics. scale_shift: 2*C floats scratch.
extern "C" int tvq_bn_eval_fwd(const float* x, int64_t B, int64_t C, int64_t HW, const float* w,
                               const float* b, const float* running_mean,
                               const float* running_var, float eps, const float* snake_a, float* y,
                               float* scale_shift, tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && y && running_mean && running_var && scale_shift, "tvq_bn_eval_fwd: bad args");
  TVQ_CHECK_ARG(norm_dims_ok(B, C, HW), "tvq_bn_eval_fwd: tensor too large");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(bn_eval_snake_kernel, ew_grid(B * C * HW), dim3(256), 0, st, x,
                     (int)(B * C * HW), (int)C, make_div16(HW), w, b, running_mean, running_var,
                     eps, snake_a, y);
  return launch_status("tvq_bn_eval_fwd");
}

extern "C" int tvq_bn_bwd(const float* dy, const float* x, int64_t B, int64_t C, int64_t HW,
                          const float* w, const float* snake_a, const float* save_mean,
                          const float* save_invstd, const float* scale_shift, float* dx,
                          float* dw, float* db, float* da, int64_t accumulate, void* workspace,
                          tvq_stream_t stream) {
  TVQ_CHECK_ARG(dy && x && dx && save_mean && save_invstd && scale_shift && workspace,
                "tvq_bn_bwd: bad arguments");
  TVQ_CHECK_ARG(norm_dims_ok(B, C, HW), "tvq_bn_bwd: tensor too large");
  hipStream_t st = (hipStream_t)stream;
  const int chunks = bn_chunks(B, HW);
  const Div16 dhw = make_div16(HW);
  double* part = (double*)workspace;
  float* coef = (float*)(part + (int64_t)C * chunks * 3);
  const BNBwdFinal f = {(int)C, chunks, coef, dw, db, snake_a ? da : nullptr, (int)accumulate};
  if (const int pt = bn_chan_pt(B, C, HW)) {
#define M_(PT)                                                                                 \
  if (pt == PT)                                                                                \
    hipLaunchKernelGGL(bn_bwd_chan_kernel<PT>, dim3((int)C), dim3(BNC_T), 0, st, dy, x, (int)B,  \
                       (int)C, (int)HW, dhw, save_mean, save_invstd, w, scale_shift,             \
                       scale_shift + C, snake_a, dx, f);
    BNC_CASES(M_)
#undef M_
    return launch_status("tvq_bn_bwd");
  }
  int* cnt = counters(C, FIN_NORM);
  hipLaunchKernelGGL(bn_bwd_partial_kernel, dim3((int)C, chunks), dim3(256), 0, st, dy, x, (int)B,
                     (int)C, (int)HW, dhw, chunks, save_mean, save_invstd, scale_shift,
                     scale_shift + C, snake_a, part, cnt, f);
  if (!cnt) hipLaunchKernelGGL(bn_bwd_final_kernel, dim3((int)C), dim3(64), 0, st, part, f);
  hipLaunchKernelGGL(bn_bwd_apply_kernel, ew_grid(B * C * HW), dim3(256), 0, st, dy, x,
                     (int)(B * C * HW), (int)C, (int)HW, dhw, B * HW, save_mean, save_invstd, w,
                     scale_shift, scale_shift + C, snake_a, coef, dx);
  return launch_status("tvq_bn_bwd");
}

extern "C" int tvq_snake_fwd(const float* x, int64_t B, int64_t C, int64_t HW, const float* a,
                             float* y, tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && a && y && B > 0 && C > 0 && HW > 0, "tvq_snake_fwd: bad arguments");
  TVQ_CHECK_ARG(norm_dims_ok(B, C, HW), "tvq_snake_fwd: tensor too large");
  hipLaunchKernelGGL(snake_fwd_kernel, ew_grid(B * C * HW), dim3(256), 0, (hipStream_t)stream, x,
                     (int)(B * C * HW), (int)C, (int)HW, make_div16(HW), a, y);
  return launch_status("tvq_snake_fwd");
}

extern "C" int64_t tvq_snake_workspace(int64_t B, int64_t C, int64_t HW) {
  return (int64_t)C * bn_chunks(B, HW) * 8;
}

extern "C" int tvq_snake_bwd(const float* dy, const float* x, int64_t B, int64_t C, int64_t HW,
                             const float* a, const float* dx_add, float* dx, float* da,
                             int64_t accumulate, void* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(dy && x && a && dx && da && workspace, "tvq_snake_bwd: bad arguments");
  TVQ_CHECK_ARG(norm_dims_ok(B, C, HW), "tvq_snake_bwd: tensor too large");
  hipStream_t st = (hipStream_t)stream;
  const int chunks = bn_chunks(B, HW);
  int* cnt = counters(C, FIN_NORM);
  hipLaunchKernelGGL(snake_bwd_kernel, dim3((int)C, chunks), dim3(256), 0, st, dy, x, (int)B,
                     (int)C, (int)HW, make_div16(HW), chunks, a, dx_add, dx, (double*)workspace,
                     cnt, da,
                     (int)accumulate);
  if (!cnt)
    hipLaunchKernelGGL(snake_bwd_final_kernel, dim3((int)C), dim3(64), 0, st,
                       (const double*)workspace, (int)C, chunks, da, (int)accumulate);
  return launch_status("tvq_snake_bwd");
}

extern "C" int tvq_dropout_bwd(const float* dy, int64_t n, float p, const int64_t* seed_ptr,
                               uint64_t offset, float* dx, tvq_stream_t stream) {
  TVQ_CHECK_ARG(dy && dx && n >= 0 && p >= 0.f && p < 1.f, "tvq_dropout_bwd: bad arguments");
  if (n == 0) return TVQ_OK;
  const int blocks = (int)((n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192);
  hipLaunchKernelGGL(dropout_bwd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, dy, n, p,
                     1.0f / (1.0f - p), seed_ptr, offset, dx);
  return launch_status("tvq_dropout_bwd");
}

// n_fft = 4 STFT / iSTFT kernels (K1/K6 in SURVEY.md §2.2), HBM-bound.
//
// STFT (time_to_timefreq, train_utils.py:293-307): hop 1, periodic Hann
// w = [0, .5, 1, .5], reflect-pad 2, normalized (x 1/2), one-sided (3 bins):
//   re0 = .5(.5 x1 + x2 + .5 x3), re1 = -.5 x2, im1 = .5(-.5 x1 + .5 x3),
//   re2 = .5(-.5 x1 + x2 - .5 x3), im0 = im2 = 0,  xk = xpad[t+k].
// Channel layout: 2c + {0 real, 1 imag}; H = bin; W = frame (T+1 frames).
// iSTFT (timefreq_to_time, train_utils.py:310-321) of a (B,2C,3,W) image:
//   X = 2*xf; y_t[1] = (X0 - X2 - 2 X1i)/4, y_t[2] = (X0 + X2 - 2 X1r)/4,
//   y_t[3] = (X0 - X2 + 2 X1i)/4  (imag of DC/Nyquist ignored);
//   out[i] = (.5 y_{i+1}[1] + y_i[2] + .5 y_{i-1}[3]) / env[i], env = 1.25 (i=0) else 1.5,
//   i in [0, W-1).
// band: 0 = LF (zero_pad_high_freq: keep bin 0), 1 = HF (zero_pad_low_freq: bins 1,2),
// 2 = all bins (plain timefreq_to_time).
#include "tvq_common.h"

namespace tvq {

__device__ __forceinline__ float xpad(const float* __restrict__ xr, int T, int j) {
  // reflect pad of 2 (torch.stft center=True, pad_mode='reflect')
  j -= 2;
  if (j < 0) j = -j;
  if (j >= T) j = 2 * (T - 1) - j;
  return xr[j];
}

struct Bins {
  float re0, re1, im1, re2;
};
__device__ __forceinline__ Bins stft_frame(const float* __restrict__ xr, int T, int t) {
  const float x1 = xpad(xr, T, t + 1), x2 = xpad(xr, T, t + 2), x3 = xpad(xr, T, t + 3);
  Bins b;
  b.re0 = 0.5f * (0.5f * x1 + x2 + 0.5f * x3);
  b.re1 = 0.5f * (-x2);
  b.im1 = 0.5f * (-0.5f * x1 + 0.5f * x3);
  b.re2 = 0.5f * (-0.5f * x1 + x2 - 0.5f * x3);
  return b;
}

// iSTFT sample i from the (masked) bins of frames i-1, i, i+1
__device__ __forceinline__ float istft_sample(Bins fm1, Bins f0, Bins fp1, int i, int band) {
  auto y = [&](const Bins& f, int n) {
    float X0 = 2.f * f.re0, X1r = 2.f * f.re1, X1i = 2.f * f.im1, X2 = 2.f * f.re2;
    if (band == 0) { X1r = X1i = X2 = 0.f; } else if (band == 1) { X0 = 0.f; }
    if (n == 1) return (X0 - X2 - 2.f * X1i) / 4.f;
    if (n == 2) return (X0 + X2 - 2.f * X1r) / 4.f;
    return (X0 - X2 + 2.f * X1i) / 4.f;
  };
  float s = 0.5f * y(fp1, 1) + y(f0, 2);
  float env = 1.25f;
  if (i > 0) { s += 0.5f * y(fm1, 3); env = 1.5f; }
  return s / env;
}

// One thread per (b, c, t), t in [0, T]: writes the LF/HF encoder inputs (copy bands)
// for frame t and, for t < T, the LF/HF reconstruction targets at sample t.
__global__ void stft_encode_kernel(const float* __restrict__ x, int B, int C, int T,
                                   float* __restrict__ raw, float* __restrict__ enc_l, float* __restrict__ enc_h,
                                   float* __restrict__ tgt_l, float* __restrict__ tgt_h) {
  const int64_t tot = (int64_t)B * C * (T + 1);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < tot;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(i % (T + 1));
    const int64_t bc = i / (T + 1);
    const int c = (int)(bc % C);
    const int64_t b = bc / C;
    const float* xr = x + bc * T;
    const Bins f = stft_frame(xr, T, t);
    const int W = T + 1;
    // image layout (B, 2C, 3, W): channel 2c real, 2c+1 imag
    const int64_t re = ((b * 2 * C + 2 * c) * 3) * W + t;
    const int64_t im = ((b * 2 * C + 2 * c + 1) * 3) * W + t;
    if (raw) {
      raw[re] = f.re0; raw[re + W] = f.re1; raw[re + 2 * W] = f.re2;
      raw[im] = 0.f;   raw[im + W] = f.im1; raw[im + 2 * W] = 0.f;
    }
    if (enc_l) {
      enc_l[re] = f.re0; enc_l[re + W] = f.re0; enc_l[re + 2 * W] = f.re0;
      enc_l[im] = 0.f;   enc_l[im + W] = 0.f;   enc_l[im + 2 * W] = 0.f;
    }
    if (enc_h) {
      enc_h[re] = f.re1; enc_h[re + W] = f.re1; enc_h[re + 2 * W] = f.re2;
      enc_h[im] = f.im1; enc_h[im + W] = f.im1; enc_h[im + 2 * W] = 0.f;
    }
    if (t < T && (tgt_l || tgt_h)) {
      const Bins fm1 = t > 0 ? stft_frame(xr, T, t - 1) : f;
      const Bins fp1 = stft_frame(xr, T, t + 1);
      if (tgt_l) tgt_l[bc * T + t] = istft_sample(fm1, f, fp1, t, 0);
      if (tgt_h) tgt_h[bc * T + t] = istft_sample(fm1, f, fp1, t, 1);
    }
  }
}

// ---- decoder tail: band-mask -> iSTFT -> linear interpolation (L = W-1 -> Tout)
struct Interp {
  float ratio;  // (float)L / (float)Tout  (area_pixel_compute_scale)
  int L;
};
__device__ __forceinline__ void interp_src(const Interp& ip, int i, int& i0, int& i1, float& l0,
                                           float& l1) {
  float src = ip.ratio * ((float)i + 0.5f) - 0.5f;
  if (src < 0.f) src = 0.f;
  i0 = (int)src;
  i1 = i0 + (i0 < ip.L - 1 ? 1 : 0);
  l1 = fminf(fmaxf(src - (float)i0, 0.f), 1.f);
  l0 = 1.f - l1;
}

__device__ __forceinline__ Bins load_bins(const float* __restrict__ img, int W, int t) {
  // img points at (b, 2c, 0, 0); imag channel is +3W
  Bins f;
  f.re0 = img[t];
  f.re1 = img[W + t];
  f.re2 = img[2 * W + t];
  f.im1 = img[3 * W + W + t];
  return f;
}

__device__ __forceinline__ float istft_at(const float* __restrict__ img, int W, int s, int band) {
  const Bins f0 = load_bins(img, W, s);
  const Bins fp1 = load_bins(img, W, s + 1);
  const Bins fm1 = s > 0 ? load_bins(img, W, s - 1) : f0;
  return istft_sample(fm1, f0, fp1, s, band);
}

__global__ void istft_decode_kernel(const float* __restrict__ h, int B, int C, int W, int band,
                                    Interp ip, int Tout, float* __restrict__ y) {
  const int64_t tot = (int64_t)B * C * Tout;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < tot;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(i % Tout);
    const int64_t bc = i / Tout;
    const int64_t b = bc / C, c = bc % C;
    const float* img = h + ((b * 2 * C + 2 * c) * 3) * W;
    int i0, i1;
    float l0, l1;
    interp_src(ip, t, i0, i1, l0, l1);
    const float v0 = istft_at(img, W, i0, band);
    const float v1 = istft_at(img, W, i1, band);
    y[i] = l0 * v0 + l1 * v1;
  }
}

// d(istft output)[s] = sum over interp outputs that read sample s (gather, deterministic)
__device__ __forceinline__ float dsample(const float* __restrict__ dyr, const Interp& ip, int Tout,
                                         int s) {
  // outputs i with src in [s-1, s+1): i ~ (s + 0.5)/ratio - 0.5
  const float inv = 1.0f / ip.ratio;
  int lo = (int)floorf(((float)s - 1.0f + 0.5f) * inv - 0.5f) - 2;
  int hi = (int)ceilf(((float)s + 1.0f + 0.5f) * inv - 0.5f) + 2;
  lo = lo < 0 ? 0 : lo;
  hi = hi > Tout - 1 ? Tout - 1 : hi;
  float acc = 0.f;
  for (int i = lo; i <= hi; ++i) {
    int i0, i1;
    float l0, l1;
    interp_src(ip, i, i0, i1, l0, l1);
    if (i0 == s) acc += l0 * dyr[i];
    if (i1 == s) acc += l1 * dyr[i];
  }
  return acc;
}

// one thread per image element (b, 2c+z, f, t): gradient of the masked iSTFT + interp
__global__ void istft_decode_bwd_kernel(const float* __restrict__ dy, int B, int C, int W, int band,
                                        Interp ip, int Tout, float* __restrict__ dh) {
  const int64_t tot = (int64_t)B * 2 * C * 3 * W;
  const int L = W - 1;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < tot;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(e % W);
    int64_t r = e / W;
    const int f = (int)(r % 3);
    r /= 3;
    const int ch = (int)(r % (2 * C));
    const int64_t b = r / (2 * C);
    const int c = ch >> 1, z = ch & 1;
    float g = 0.f;
    // which synthesis terms read this bin (after the band mask and DC/Nyquist imag drop)
    const bool live = (band == 0)   ? (f == 0 && z == 0)
                      : (band == 1) ? (f >= 1 && !(f == 2 && z == 1))
                                    : !(z == 1 && f != 1);
    if (live) {
      const float* dyr = dy + (b * C + c) * Tout;
      // dy_t[n]/d bin (the X = 2 xf scaling folded in): coefficients per n = 1,2,3
      float k1, k2, k3;
      if (f == 0) { k1 = 0.5f; k2 = 0.5f; k3 = 0.5f; }
      else if (f == 2) { k1 = -0.5f; k2 = 0.5f; k3 = -0.5f; }
      else if (z == 0) { k1 = 0.f; k2 = -1.0f; k3 = 0.f; }
      else { k1 = -1.0f; k2 = 0.f; k3 = 1.0f; }
      // frame t feeds samples s = t-1 (n=1, w .5), s = t (n=2, w 1), s = t+1 (n=3, w .5)
      if (k1 != 0.f && t - 1 >= 0 && t - 1 < L) {
        const int s = t - 1;
        g += dsample(dyr, ip, Tout, s) * 0.5f * k1 / (s == 0 ? 1.25f : 1.5f);
      }
      if (k2 != 0.f && t < L) {
        const int s = t;
        g += dsample(dyr, ip, Tout, s) * 1.0f * k2 / (s == 0 ? 1.25f : 1.5f);
      }
      if (k3 != 0.f && t + 1 < L) {
        const int s = t + 1;
        g += dsample(dyr, ip, Tout, s) * 0.5f * k3 / 1.5f;
      }
    }
    dh[e] = g;
  }
}

// Same gradient, one block per (b, c) row: the interpolation's adjoint d(sample)[s] is
// computed once per sample into LDS (the per-element kernel above recomputes it for each of
// the up to 3 frames and 6 image planes that read it: ~18x the gather work), then every
// image element of the row reads its <= 3 samples with the same per-term arithmetic.
__global__ void istft_decode_bwd_row_kernel(const float* __restrict__ dy, int C, int W, int band,
                                            Interp ip, int Tout, float* __restrict__ dh) {
  extern __shared__ float ds[];
  const int L = W - 1;
  const int64_t bc = blockIdx.x;
  const int64_t b = bc / C;
  const int c = (int)(bc - b * C);
  const float* dyr = dy + bc * Tout;
  for (int s = threadIdx.x; s < L; s += blockDim.x) ds[s] = dsample(dyr, ip, Tout, s);
  __syncthreads();
  const int n = 2 * 3 * W;
  float* out = dh + ((b * 2 * C + 2 * c) * 3) * (int64_t)W;  // (b, 2c + z, f, t), z-major
  for (int e = threadIdx.x; e < n; e += blockDim.x) {
    const int z = e / (3 * W), rem = e - z * 3 * W, f = rem / W, t = rem - f * W;
    float g = 0.f;
    const bool live = (band == 0)   ? (f == 0 && z == 0)
                      : (band == 1) ? (f >= 1 && !(f == 2 && z == 1))
                                    : !(z == 1 && f != 1);
    if (live) {
      float k1, k2, k3;
      if (f == 0) { k1 = 0.5f; k2 = 0.5f; k3 = 0.5f; }
      else if (f == 2) { k1 = -0.5f; k2 = 0.5f; k3 = -0.5f; }
      else if (z == 0) { k1 = 0.f; k2 = -1.0f; k3 = 0.f; }
      else { k1 = -1.0f; k2 = 0.f; k3 = 1.0f; }
      if (k1 != 0.f && t - 1 >= 0 && t - 1 < L) {
        const int s = t - 1;
        g += ds[s] * 0.5f * k1 / (s == 0 ? 1.25f : 1.5f);
      }
      if (k2 != 0.f && t < L) {
        const int s = t;
        g += ds[s] * 1.0f * k2 / (s == 0 ? 1.25f : 1.5f);
      }
      if (k3 != 0.f && t + 1 < L) {
        const int s = t + 1;
        g += ds[s] * 0.5f * k3 / 1.5f;
      }
    }
    out[e] = g;
  }
}

static int ew_blocks(int64_t n) {
  int64_t b = (n + 255) / 256;
  return (int)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

}  // namespace tvq

using namespace tvq;

extern "C" int tvq_stft_encode(const float* x, int64_t B, int64_t C, int64_t T, float* raw,
                               float* enc_l, float* enc_h, float* tgt_l, float* tgt_h,
                               tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && B > 0 && C > 0 && T >= 3, "tvq_stft_encode: bad arguments");
  const int64_t n = B * C * (T + 1);
  hipLaunchKernelGGL(stft_encode_kernel, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream, x,
                     (int)B, (int)C, (int)T, raw, enc_l, enc_h, tgt_l, tgt_h);
  return launch_status("tvq_stft_encode");
}

extern "C" int tvq_istft_decode(const float* h, int64_t B, int64_t C, int64_t W, int64_t band,
                                int64_t Tout, float* y, tvq_stream_t stream) {
  TVQ_CHECK_ARG(h && y && B > 0 && C > 0 && W >= 3 && Tout > 0 && band >= 0 && band <= 2,
                "tvq_istft_decode: bad arguments");
  Interp ip;
  ip.L = (int)W - 1;
  ip.ratio = (float)ip.L / (float)Tout;
  const int64_t n = B * C * Tout;
  hipLaunchKernelGGL(istft_decode_kernel, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream, h,
                     (int)B, (int)C, (int)W, (int)band, ip, (int)Tout, y);
  return launch_status("tvq_istft_decode");
}

extern "C" int tvq_istft_decode_bwd(const float* dy, int64_t B, int64_t C, int64_t W, int64_t band,
                                    int64_t Tout, float* dh, tvq_stream_t stream) {
  TVQ_CHECK_ARG(dy && dh && B > 0 && C > 0 && W >= 3 && Tout > 0, "tvq_istft_decode_bwd: bad args");
  Interp ip;
  ip.L = (int)W - 1;
  ip.ratio = (float)ip.L / (float)Tout;
  if (W - 1 <= 16384 && B * C < (1ll << 31)) {  // the row's samples fit the LDS
    hipLaunchKernelGGL(istft_decode_bwd_row_kernel, dim3((unsigned)(B * C)), dim3(256),
                       (size_t)(W - 1) * sizeof(float), (hipStream_t)stream, dy, (int)C, (int)W,
                       (int)band, ip, (int)Tout, dh);
    return launch_status("tvq_istft_decode_bwd");
  }
  const int64_t n = B * 2 * C * 3 * W;
  hipLaunchKernelGGL(istft_decode_bwd_kernel, dim3(ew_blocks(n)), dim3(256), 0,
                     (hipStream_t)stream, dy, (int)B, (int)C, (int)W, (int)band, ip, (int)Tout, dh);
  return launch_status("tvq_istft_decode_bwd");
}

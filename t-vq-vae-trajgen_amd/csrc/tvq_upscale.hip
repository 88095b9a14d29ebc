// The HF prior's Upscale first conv on the nearest-upsampled LF token embeddings
// (reference bidirectional_transformer.py:12-30: x (b n d) -> interpolate(size m, nearest)
// -> Conv1d(d, H, k=3, pad 1) -> GELU -> ...), computed on the n-token grid instead of the
// m = f n upsampled one.
//
// With x_up[i] = x[i / f] (f = m / n >= 2, integer) and the taps W_0, W_1, W_2, the output
// at i = f j + r is W_0 x_up[i-1] + W_1 x_up[i] + W_2 x_up[i+1] + b, and every x_up term
// is x[j] except x_up[f j - 1] = x[j - 1] (r = 0, tap 0) and x_up[f j + f] = x[j + 1]
// (r = f - 1, tap 2).  So with Z = x [W_0; W_1; W_2]^T (per token: A_j | B_j | C_j, one
// GEMM over the n tokens, K = d):
//   out[f j]         = b + A_{j-1} + B_j + C_j
//   out[f j + r]     = b + A_j     + B_j + C_j        (0 < r < f - 1)
//   out[f j + f - 1] = b + A_j     + B_j + C_{j+1}
// (A_{-1} = C_n = 0: the zero padding).  The backward is the transpose: with
// S_t[j] = sum of dY over the outputs that read x[j] through tap t,
//   S_0[j] = dY[f j + 1 .. f j + f],  S_1[j] = dY[f j .. f j + f - 1],
//   S_2[j] = dY[f j - 1 .. f j + f - 2]   (out-of-range dY = 0),
// dx_j = sum_t W_t^T S_t[j] (one GEMM, K = 3 H) and dW_t = S_t^T x (one GEMM over the n
// tokens), db = sum dY.  Every GEMM runs over n rows instead of m = f n: f x fewer FLOPs
// (4x for the HF prior, 96 = 4 x 24), and the (b, d, m) upsampled tensor is never formed.
// Same function as upsample -> conv up to fp32 reassociation.
//
// Kernels here: the tap-major weight pack W (H, d, 3) -> Wcat (3 H, d); the combine
// (+ bias, + GELU, or + GELU + eval BatchNorm for sampling) from Z to the (b, H, m) output;
// the window sums S (+ the GELU derivative, + per-image bias partials) from dY; the
// scatter of dWcat back to the conv weight layout.  The GEMMs are the library's
// (tvq_gemm: gemm_skinny forward, gemm_dk / gemm_kt backward).
#include "tvq_common.h"

namespace tvq {

constexpr int UPS_CT = 64;  // channels per combine / sums block
constexpr int UPS_T = 256;

// the training GELU of tvq_xf.hip (gelu_f / gelu_grad: library erff), so GELU(conv) here is
// bit for bit what tvq_gelu_fwd / tvq_gelu_bwd give on the same conv output
__device__ __forceinline__ float ups_gelu(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f));
}
__device__ __forceinline__ float ups_gelu_grad(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752440f));
  const float pdf = 0.39894228040143267794f * expf(-0.5f * x * x);
  return cdf + x * pdf;
}

__global__ __launch_bounds__(256) void ups_pack_kernel(const float* __restrict__ w, int H, int D,
                                                       float* __restrict__ wcat) {
  const int n = 3 * H * D;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) {
    const int row = e / D, d = e - row * D;  // row = t*H + c
    const int t = row / H, c = row - t * H;
    wcat[e] = w[((int64_t)c * D + d) * 3 + t];
  }
}

__global__ __launch_bounds__(256) void ups_wscatter_kernel(const float* __restrict__ dwcat, int H,
                                                           int D, float* __restrict__ dw,
                                                           int accumulate) {
  const int n = 3 * H * D;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) {
    const int t = e % 3, cd = e / 3, c = cd / D, d = cd - c * D;
    const float v = dwcat[((int64_t)t * H + c) * D + d];
    dw[e] = accumulate ? dw[e] + v : v;
  }
}

// mode 0: out = GELU(v), pre = v (training; pre is the GELU backward's input)
// mode 1: out = v
// mode 2: out = BN_eval(GELU_as(v)) (sampling: the conv -> GELU -> BatchNorm1d epilogue of
//         tvq_conv2d_fwd_bn_eval, same arithmetic)
struct UpsBN {
  const float *w, *b, *rm, *rv;
  float eps;
};

__global__ __launch_bounds__(UPS_T) void ups_combine_kernel(const float* __restrict__ z, int n,
                                                            int f, int H,
                                                            const float* __restrict__ bias,
                                                            int mode, UpsBN bn,
                                                            float* __restrict__ out,
                                                            float* __restrict__ pre) {
  extern __shared__ float zs[];  // [3][n][UPS_CT + 1]
  __shared__ float cbias[UPS_CT], csc[UPS_CT], csh[UPS_CT];
  constexpr int RS = UPS_CT + 1;
  const int b = blockIdx.x, c0 = blockIdx.y * UPS_CT;
  const int nc = min(UPS_CT, H - c0);
  const int m = f * n, ld = 3 * H;
  for (int e = threadIdx.x; e < 3 * n * UPS_CT; e += UPS_T) {
    const int cc = e % UPS_CT, tj = e / UPS_CT, t = tj / n, j = tj - t * n;
    zs[tj * RS + cc] = cc < nc ? z[((int64_t)b * n + j) * ld + t * H + c0 + cc] : 0.f;
  }
  if (threadIdx.x < nc) {  // per-channel terms once per block
    const int c = c0 + threadIdx.x;
    cbias[threadIdx.x] = bias ? bias[c] : 0.f;
    if (mode == 2) {
      const float inv = 1.0f / sqrtf(bn.rv[c] + bn.eps);
      const float sc = (bn.w ? bn.w[c] : 1.f) * inv;
      csc[threadIdx.x] = sc;
      csh[threadIdx.x] = (bn.b ? bn.b[c] : 0.f) - bn.rm[c] * sc;
    }
  }
  __syncthreads();
  const float* A = zs;
  const float* Bm = zs + n * RS;
  const float* Cm = zs + 2 * n * RS;
  // output i = f j + r: b + A_{j-1 or j} + B_j + C_{j or j+1}
  auto value = [&](int cc, int j, int r) {
    const float a = r == 0 ? (j > 0 ? A[(j - 1) * RS + cc] : 0.f) : A[j * RS + cc];
    const float cv = r == f - 1 ? (j + 1 < n ? Cm[(j + 1) * RS + cc] : 0.f) : Cm[j * RS + cc];
    return cbias[cc] + (a + (Bm[j * RS + cc] + cv));
  };
  auto post = [&](int cc, float v) {
    return mode == 2 ? fmaf(gelu_as(v), csc[cc], csh[cc]) : (mode == 0 ? ups_gelu(v) : v);
  };
  if ((f & 3) == 0) {  // 4 consecutive outputs of one token per thread: 16-B stores
    const int mq = m >> 2;
    for (int e = threadIdx.x; e < nc * mq; e += UPS_T) {
      const int cc = e / mq, i0 = 4 * (e - cc * mq);
      const int j = i0 / f, r0 = i0 - j * f;
      float v[4], y[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[k] = value(cc, j, r0 + k);
        y[k] = post(cc, v[k]);
      }
      const int64_t o = ((int64_t)b * H + c0 + cc) * m + i0;
      if (mode == 0) *reinterpret_cast<float4*>(pre + o) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(out + o) = make_float4(y[0], y[1], y[2], y[3]);
    }
    return;
  }
  for (int e = threadIdx.x; e < nc * m; e += UPS_T) {
    const int cc = e / m, i = e - cc * m;
    const int j = i / f, r = i - j * f;
    const float v = value(cc, j, r);
    const int64_t o = ((int64_t)b * H + c0 + cc) * m + i;
    if (mode == 0) pre[o] = v;
    out[o] = post(cc, v);
  }
}

// S (b n, 3 H) [S_0 | S_1 | S_2] from dY (b, H, m) (times GELU'(pre) when pre is given);
// part[b][c] = sum_i dY1[b][c][i] in order (the bias gradient's per-image partials)
__global__ __launch_bounds__(UPS_T) void ups_sums_kernel(const float* __restrict__ dy,
                                                         const float* __restrict__ pre, int n,
                                                         int f, int H, float* __restrict__ s,
                                                         float* __restrict__ part) {
  extern __shared__ float gs[];  // [UPS_CT][m + 1]
  const int b = blockIdx.x, c0 = blockIdx.y * UPS_CT;
  const int nc = min(UPS_CT, H - c0);
  const int m = f * n, RS = m + 1, ld = 3 * H;
  if ((m & 3) == 0) {  // 16-B loads
    const int mq = m >> 2;
    for (int e = threadIdx.x; e < nc * mq; e += UPS_T) {
      const int cc = e / mq, i0 = 4 * (e - cc * mq);
      const int64_t o = ((int64_t)b * H + c0 + cc) * m + i0;
      const float4 g4 = *reinterpret_cast<const float4*>(dy + o);
      float g[4] = {g4.x, g4.y, g4.z, g4.w};
      if (pre) {
        const float4 p4 = *reinterpret_cast<const float4*>(pre + o);
        g[0] *= ups_gelu_grad(p4.x);
        g[1] *= ups_gelu_grad(p4.y);
        g[2] *= ups_gelu_grad(p4.z);
        g[3] *= ups_gelu_grad(p4.w);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) gs[cc * RS + i0 + k] = g[k];
    }
  } else {
    for (int e = threadIdx.x; e < nc * m; e += UPS_T) {
      const int cc = e / m, i = e - cc * m;
      const int64_t o = ((int64_t)b * H + c0 + cc) * m + i;
      float g = dy[o];
      if (pre) g = g * ups_gelu_grad(pre[o]);
      gs[cc * RS + i] = g;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < n * UPS_CT; e += UPS_T) {
    const int cc = e % UPS_CT, j = e / UPS_CT;
    if (cc >= nc) continue;
    const float* g = gs + cc * RS;
    const int i0 = f * j;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
    for (int r = 0; r < f; ++r) {
      s1 += g[i0 + r];
      if (i0 + r + 1 < m) s0 += g[i0 + r + 1];
      if (i0 + r - 1 >= 0) s2 += g[i0 + r - 1];
    }
    float* row = s + ((int64_t)b * n + j) * ld + c0 + cc;
    row[0] = s0;
    row[H] = s1;
    row[2 * H] = s2;
  }
  if (part && threadIdx.x < nc) {
    const float* g = gs + threadIdx.x * RS;
    float t = 0.f;
    for (int i = 0; i < m; ++i) t += g[i];
    part[(int64_t)b * H + c0 + threadIdx.x] = t;
  }
}

// ---- the HF prior's project_in with Upscale's second conv folded in (training).
// z = project_in(cat(cls, cat(Upscale(tl), th) + pos)) is assembled from the folded pieces
// (hip/upscale.py hf_embed_folded): v = conv(u, W_l W2) + W_l b2 (B, d, m), R = th W_h^T
// (B m, d), P = pos[:m] W_in^T (m, d), Cp = cls W_in^T (B, d):
//   z[b, 0] = Cp[b],   z[b, 1 + i] = (v[b, :, i] + R[b m + i]) + P[i]
// One block per image: v[b] staged through LDS (coalesced both ways).  The backward splits
// dz back: dCp[b] = dz[b, 0], dR = dz[:, 1:] (contiguous), dv[b] = dz[b, 1:]^T.
constexpr int HFE_T = 256;
__global__ __launch_bounds__(HFE_T) void hfe_assemble_kernel(const float* __restrict__ v,
                                                             const float* __restrict__ R,
                                                             const float* __restrict__ P,
                                                             const float* __restrict__ Cp, int m,
                                                             int d, float* __restrict__ z) {
  extern __shared__ float vs[];  // [d][m + 1]
  const int b = blockIdx.x, RS = m + 1;
  for (int e = threadIdx.x; e < d * m; e += HFE_T) {
    const int f = e / m, i = e - f * m;
    vs[f * RS + i] = v[((int64_t)b * d + f) * m + i];
  }
  __syncthreads();
  float* zb = z + (int64_t)b * (m + 1) * d;
  for (int e = threadIdx.x; e < (m + 1) * d; e += HFE_T) {
    const int row = e / d, f = e - row * d;
    if (row == 0) {
      zb[e] = Cp[(int64_t)b * d + f];
    } else {
      const int i = row - 1;
      zb[e] = (vs[f * RS + i] + R[((int64_t)b * m + i) * d + f]) + P[(int64_t)i * d + f];
    }
  }
}

__global__ __launch_bounds__(HFE_T) void hfe_assemble_bwd_kernel(const float* __restrict__ dz,
                                                                 int m, int d,
                                                                 float* __restrict__ dv,
                                                                 float* __restrict__ dR,
                                                                 float* __restrict__ dCp) {
  extern __shared__ float gs[];  // [d][m + 1]
  const int b = blockIdx.x, RS = m + 1;
  const float* zb = dz + (int64_t)b * (m + 1) * d;
  for (int e = threadIdx.x; e < (m + 1) * d; e += HFE_T) {
    const int row = e / d, f = e - row * d;
    const float g = zb[e];
    if (row == 0) {
      dCp[(int64_t)b * d + f] = g;
    } else {
      dR[((int64_t)b * m + row - 1) * d + f] = g;
      gs[f * RS + row - 1] = g;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < d * m; e += HFE_T) {
    const int f = e / m, i = e - f * m;
    dv[((int64_t)b * d + f) * m + i] = gs[f * RS + i];
  }
}

static bool ups_dims_ok(int64_t B, int64_t n, int64_t f, int64_t H) {
  // LDS: the combine holds 3 n (UPS_CT + 1) floats, the sums UPS_CT (f n + 1): <= 64 KB
  return B > 0 && n > 0 && f >= 2 && H > 0 && f * n <= 240 && n <= 64 &&
         B * H * f * n < (1ll << 31) && B * n * 3 * H < (1ll << 31);
}

}  // namespace tvq

using namespace tvq;

extern "C" int tvq_ups_pack(const float* w, int64_t H, int64_t D, float* wcat,
                            tvq_stream_t stream) {
  TVQ_CHECK_ARG(w && wcat && H > 0 && D > 0 && 3 * H * D < (1ll << 31), "tvq_ups_pack: bad arguments");
  const int64_t n = 3 * H * D;
  const int blocks = (int)((n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048);
  hipLaunchKernelGGL(ups_pack_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w, (int)H,
                     (int)D, wcat);
  return launch_status("tvq_ups_pack");
}

extern "C" int tvq_ups_wscatter(const float* dwcat, int64_t H, int64_t D, float* dw,
                                int64_t accumulate, tvq_stream_t stream) {
  TVQ_CHECK_ARG(dwcat && dw && H > 0 && D > 0 && 3 * H * D < (1ll << 31),
                "tvq_ups_wscatter: bad arguments");
  const int64_t n = 3 * H * D;
  const int blocks = (int)((n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048);
  hipLaunchKernelGGL(ups_wscatter_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, dwcat,
                     (int)H, (int)D, dw, (int)accumulate);
  return launch_status("tvq_ups_wscatter");
}

extern "C" int tvq_ups_combine(const float* z, int64_t B, int64_t n, int64_t f, int64_t H,
                               const float* bias, int64_t mode, const float* bn_w,
                               const float* bn_b, const float* bn_rm, const float* bn_rv,
                               float bn_eps, float* out, float* pre, tvq_stream_t stream) {
  TVQ_CHECK_ARG(z && out && ups_dims_ok(B, n, f, H) && mode >= 0 && mode <= 2 &&
                    ((uintptr_t)out & 15) == 0 && ((uintptr_t)pre & 15) == 0,
                "tvq_ups_combine: bad arguments (out / pre 16-byte aligned)");
  TVQ_CHECK_ARG(mode != 0 || pre, "tvq_ups_combine: mode 0 needs pre");
  TVQ_CHECK_ARG(mode != 2 || (bn_rm && bn_rv), "tvq_ups_combine: mode 2 needs running statistics");
  const UpsBN bn = {bn_w, bn_b, bn_rm, bn_rv, bn_eps};
  const size_t lds = (size_t)3 * n * (UPS_CT + 1) * sizeof(float);
  TVQ_PLAN("ups_combine B%lld n%lld f%lld H%lld mode%lld", (long long)B, (long long)n,
           (long long)f, (long long)H, (long long)mode);
  hipLaunchKernelGGL(ups_combine_kernel, dim3((unsigned)B, (unsigned)((H + UPS_CT - 1) / UPS_CT)),
                     dim3(UPS_T), lds, (hipStream_t)stream, z, (int)n, (int)f, (int)H, bias,
                     (int)mode, bn, out, pre);
  return launch_status("tvq_ups_combine");
}

extern "C" int tvq_ups_sums(const float* dy, const float* pre, int64_t B, int64_t n, int64_t f,
                            int64_t H, float* s, float* part, tvq_stream_t stream) {
  TVQ_CHECK_ARG(dy && s && ups_dims_ok(B, n, f, H) && ((uintptr_t)dy & 15) == 0 &&
                    ((uintptr_t)pre & 15) == 0,
                "tvq_ups_sums: bad arguments (dy / pre 16-byte aligned)");
  const size_t lds = (size_t)UPS_CT * (f * n + 1) * sizeof(float);
  TVQ_PLAN("ups_sums B%lld n%lld f%lld H%lld", (long long)B, (long long)n, (long long)f,
           (long long)H);
  hipLaunchKernelGGL(ups_sums_kernel, dim3((unsigned)B, (unsigned)((H + UPS_CT - 1) / UPS_CT)),
                     dim3(UPS_T), lds, (hipStream_t)stream, dy, pre, (int)n, (int)f, (int)H, s,
                     part);
  return launch_status("tvq_ups_sums");
}

extern "C" int tvq_hfe_assemble(const float* v, const float* R, const float* P, const float* Cp,
                                int64_t B, int64_t m, int64_t d, float* z, tvq_stream_t stream) {
  TVQ_CHECK_ARG(v && R && P && Cp && z && B > 0 && m > 0 && d > 0 && d * (m + 1) * 4 <= 64 * 1024,
                "tvq_hfe_assemble: bad arguments");
  hipLaunchKernelGGL(hfe_assemble_kernel, dim3((unsigned)B), dim3(HFE_T),
                     (size_t)d * (m + 1) * sizeof(float), (hipStream_t)stream, v, R, P, Cp, (int)m,
                     (int)d, z);
  return launch_status("tvq_hfe_assemble");
}

extern "C" int tvq_hfe_assemble_bwd(const float* dz, int64_t B, int64_t m, int64_t d, float* dv,
                                    float* dR, float* dCp, tvq_stream_t stream) {
  TVQ_CHECK_ARG(dz && dv && dR && dCp && B > 0 && m > 0 && d > 0 && d * (m + 1) * 4 <= 64 * 1024,
                "tvq_hfe_assemble_bwd: bad arguments");
  hipLaunchKernelGGL(hfe_assemble_bwd_kernel, dim3((unsigned)B), dim3(HFE_T),
                     (size_t)d * (m + 1) * sizeof(float), (hipStream_t)stream, dz, (int)m, (int)d,
                     dv, dR, dCp);
  return launch_status("tvq_hfe_assemble_bwd");
}

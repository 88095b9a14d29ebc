// MaskGIT iterative-decoding step (maskgit.py:294-411 first_pass / second_pass,
// mask_by_random_topk maskgit.py:238-267) on device, one block per sequence:
//
//   sample:  for every still-masked token, draw s ~ Categorical(logits) by exponential race
//            (torch.multinomial's n_sample = 1 algorithm, which Categorical.sample runs:
//            argmax_k l_k + Gumbel_k, tvq_common.h race_gumbel), keep known tokens, and
//            record p(s) (fp32 softmax, double sum; +inf for known tokens, maskgit.py:320-326)
//   remask:  confidence = log(p + 1e-5) + tau * Gumbel(u'), re-mask the k lowest per row
//            (topk(largest=False) keeps exactly k, maskgit.py:259-266)
//
// The reference loops over rows in Python and calls .item() per step; here each step is
// two launches with no host synchronisation.  Noise comes from the device seed (counter
// hash of (seed, offset, element)) or is injected (tests pin against the oracle).
#include "tvq_common.h"
#include "tvq_race.h"

namespace tvq {

__device__ __forceinline__ double wave_sum_dd(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// (value, index) argmax over the wave, ties to the lowest index (torch.argmax)
__device__ __forceinline__ void wave_argmax(float& v, int& k) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int ok = __shfl_xor(k, o, 64);
    if (ov > v || (ov == v && ok < k)) {
      v = ov;
      k = ok;
    }
  }
}

__global__ __launch_bounds__(256) void maskgit_sample_kernel(
    const float* __restrict__ logits, int64_t sb, int64_t sn, int n, int K,
    const int64_t* __restrict__ s_in, int64_t mask_id, const float* __restrict__ gumbel,
    const int64_t* __restrict__ seed_ptr, uint64_t offset, int64_t* __restrict__ sampled,
    float* __restrict__ selp, int nb) {
  // one wave per token: token t = blockIdx.x * 4 + wave (all B*n tokens in flight at once)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t t = (int64_t)blockIdx.x * 4 + wid;
  if (t >= (int64_t)nb * n) return;
  const int64_t b = t / n, i = t - b * n;
  const int64_t s0 = s_in[t];
  if (s0 != mask_id) {  // known token: kept, confidence +inf
    if (lane == 0) {
      sampled[t] = s0;
      selp[t] = INFINITY;
    }
    return;
  }
  const float* l = logits + b * sb + i * sn;
  const float* g = gumbel ? gumbel + t * K : nullptr;
  const uint32_t key = gumbel ? 0u : race_key(mix_seed(seed_ptr, offset));
  const uint32_t ctr0 = (uint32_t)t * (uint32_t)K;
  // the race argmax_k l_k + g_k and the row max, in one pass over the row
  float m = -INFINITY, best = -INFINITY;
  int bk = K;
  for (int j = lane; j < K; j += 64) {
    const float v = l[j];
    m = fmaxf(m, v);
    const float r = v + (g ? g[j] : race_gumbel(key, ctr0 + (uint32_t)j));
    if (r > best) {  // j increases along the lane: the first of equal keys is kept
      best = r;
      bk = j;
    }
  }
  m = wave_max(m);
  wave_argmax(best, bk);
  // p(sampled) of the fp32 softmax (maskgit.py:320-326): exp terms summed in double
  double part = 0.0;
  for (int j = lane; j < K; j += 64) part += (double)__expf(l[j] - m);
  const double tot = wave_sum_dd(part);
  if (lane == 0) {
    sampled[t] = bk;
    selp[t] = (float)((double)__expf(l[bk] - m) / tot);
  }
}

// masking[b, i] = rank of conf_i among row b (ascending, ties by index) < k
__global__ __launch_bounds__(256) void maskgit_remask_kernel(
    const float* __restrict__ selp, int n, int k, float temperature,
    const float* __restrict__ u_gumbel, const int64_t* __restrict__ seed_ptr, uint64_t offset,
    const int64_t* __restrict__ sampled, int64_t mask_id, int64_t* __restrict__ s_out,
    uint8_t* __restrict__ masking) {
  extern __shared__ float conf[];
  const int b = blockIdx.x;
  const uint64_t seed = u_gumbel ? 0ull : mix_seed(seed_ptr, offset);
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int64_t t = (int64_t)b * n + i;
    const float u = u_gumbel ? u_gumbel[t] : uniform01(seed, (uint64_t)t);
    const float g = -logf(fmaxf(-logf(fmaxf(u, 1e-20f)), 1e-20f));
    conf[i] = logf(selp[t] + 1e-5f) + temperature * g;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float c = conf[i];
    int rank = 0;
    for (int j = 0; j < n; ++j) {
      const float cj = conf[j];
      rank += (cj < c) || (cj == c && j < i);
    }
    const int64_t t = (int64_t)b * n + i;
    const bool msk = rank < k;
    if (masking) masking[t] = msk ? 1 : 0;
    if (s_out) s_out[t] = msk ? mask_id : sampled[t];
  }
}

// out[b, d, p] = E[idx[b, p], d]: codebook lookup written straight into the decoder's
// NCHW input (maskgit.py:461-469 embedding + 'b n c -> b c (h w)').  A block takes CG_PT
// positions of one image: their codebook rows are read whole (coalesced, d contiguous) into
// an LDS tile [d][p] and written out along p (coalesced), instead of one 4-byte gather per
// output element with a row stride of D floats between neighbouring lanes.
constexpr int CG_PT = 64;
__global__ __launch_bounds__(256) void codebook_gather_nchw_kernel(
    const int64_t* __restrict__ idx, int P, int D, const float* __restrict__ E,
    float* __restrict__ out) {
  extern __shared__ float cg_tile[];  // [D][CG_PT + 1]
  __shared__ int rows[CG_PT];
  const int ntile = (P + CG_PT - 1) / CG_PT;
  const int b = blockIdx.x / ntile, p0 = (blockIdx.x - b * ntile) * CG_PT;
  const int np = min(CG_PT, P - p0);
  if (threadIdx.x < np) rows[threadIdx.x] = (int)idx[(int64_t)b * P + p0 + threadIdx.x];
  __syncthreads();
  for (int e = threadIdx.x; e < np * D; e += 256) {
    const int j = e / D, d = e - j * D;
    cg_tile[d * (CG_PT + 1) + j] = E[(int64_t)rows[j] * D + d];
  }
  __syncthreads();
  float* ob = out + (int64_t)b * D * P + p0;
  for (int e = threadIdx.x; e < np * D; e += 256) {
    const int d = e / np, j = e - d * np;
    ob[(int64_t)d * P + j] = cg_tile[d * (CG_PT + 1) + j];
  }
}

// ---- tied logits + race sampling (the HF prior's decoding step): logits = h W[:K]^T + bias
// computed tile by tile on MFMA and consumed by the race in registers (tvq_race.h), so the
// (M, K) logits never reach HBM and no separate sampling launch reads them back.
struct TlsArgs {
  const float* h;       // (M, D) pred_head output rows
  const float4* wpk;    // packed code table: tile c, group T4, lane (tls_pack_kernel)
  const float* bpk;     // packed bias (n, Kp), Kp = 32 * Kt
  const int64_t* s_in;  // (M) current tokens
  const float* gumbel;  // (M, K) injected noise or null
  const int64_t* seed_ptr;
  uint64_t offset;
  int64_t mask_id;
  int64_t* sampled;
  float* selp;
  float* logits_out;  // (M, K) debug copy of the logits or null
  int64_t M;
  int n, K, Kt;
};

template <int D>
__global__ __launch_bounds__(256) void tls_pack_kernel(const float* __restrict__ W, int K,
                                                       const float* __restrict__ bias, int64_t ldb,
                                                       float4* __restrict__ wpk,
                                                       float* __restrict__ bpk, int Kt) {
  constexpr int G = D / 8;  // 16-B groups per lane per tile (D / 2 MFMA steps)
  const int c = blockIdx.x;
  if (c < Kt) {
    for (int e = threadIdx.x; e < G * 64; e += blockDim.x) {
      const int T4 = e >> 6, l = e & 63;
      const int row = 32 * c + (l & 31);
      const int k = 32 * (T4 >> 2) + 8 * (T4 & 3) + 4 * (l >> 5);
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row < K) v = *reinterpret_cast<const float4*>(W + (int64_t)row * D + k);
      wpk[(int64_t)c * G * 64 + e] = v;
    }
  } else {
    const int i = c - Kt, Kp = 32 * Kt;
    for (int k = threadIdx.x; k < Kp; k += blockDim.x)
      bpk[(int64_t)i * Kp + k] = k < K ? bias[(int64_t)i * ldb + k] : 0.f;
  }
}

// one wave per 32 rows (token on the lane), the code tiles streamed through registers with
// the next tile's operand groups loading while the current one multiplies
template <int D, bool INJ>
__global__ __launch_bounds__(256) void tied_logits_sample_kernel(TlsArgs a) {
  constexpr int G = D / 8;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, r32 = lane & 31, h = lane >> 5;
  const int64_t m0 = ((int64_t)blockIdx.x * 4 + wid) * 32;
  if (m0 >= a.M) return;
  const bool row_ok = m0 + r32 < a.M;
  const int64_t m = row_ok ? m0 + r32 : a.M - 1;
  // B operand of step t = 16 q + 4 g + e: h[m][32 q + 8 g + 4 h + e]
  float xb[D / 2];
#pragma unroll
  for (int q = 0; q < D / 32; ++q)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 v = *reinterpret_cast<const float4*>(a.h + m * D + 32 * q + 8 * g + 4 * h);
      xb[16 * q + 4 * g] = v.x;
      xb[16 * q + 4 * g + 1] = v.y;
      xb[16 * q + 4 * g + 2] = v.z;
      xb[16 * q + 4 * g + 3] = v.w;
    }
  const int Kp = 32 * a.Kt;
  const float* brow = a.bpk + (int64_t)(m % a.n) * Kp;
  const float* grow = a.gumbel ? a.gumbel + m * a.K : nullptr;
  const uint32_t key = a.gumbel ? 0u : race_key(mix_seed(a.seed_ptr, a.offset));
  const uint32_t ctr0 = (uint32_t)m * (uint32_t)a.K;
  RaceState st;
  race_init(st);
  // the code tiles stream as half-tiles (H groups each) through two register buffers: a
  // tile's bias loads go out first, then the second half, then the next tile's first half
  // (loads return in order: the bias and the second half never wait for the prefetch)
  constexpr int H = G / 2;
  auto load_half = [&](float4 (&w)[H], int u) {
    if (u < 2 * a.Kt) {
      const int64_t base = ((int64_t)(u >> 1) * G + (u & 1) * H) * 64 + lane;
#pragma unroll
      for (int j = 0; j < H; ++j) w[j] = a.wpk[base + j * 64];
    }
  };
  auto mfma_half = [&](const float4 (&w)[H], int t0, floatx16 acc) {
#pragma unroll
    for (int j = 0; j < H; ++j) {
      const int T4 = t0 + j;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w[j].x, xb[4 * T4], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w[j].y, xb[4 * T4 + 1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w[j].z, xb[4 * T4 + 2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w[j].w, xb[4 * T4 + 3], acc, 0, 0, 0);
    }
    return acc;
  };
  float4 wa[H], wb[H];
  load_half(wa, 0);
  for (int c = 0; c < a.Kt; ++c) {
    float4 bq[4];
#pragma unroll
    for (int g = 0; g < 4; ++g)
      bq[g] = *reinterpret_cast<const float4*>(brow + 32 * c + 8 * g + 4 * h);
    load_half(wb, 2 * c + 1);
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    acc = mfma_half(wa, 0, acc);
    load_half(wa, 2 * c + 2);
    acc = mfma_half(wb, H, acc);
    float v[16];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      v[4 * g] = acc[4 * g] + bq[g].x;
      v[4 * g + 1] = acc[4 * g + 1] + bq[g].y;
      v[4 * g + 2] = acc[4 * g + 2] + bq[g].z;
      v[4 * g + 3] = acc[4 * g + 3] + bq[g].w;
    }
    if (a.logits_out && row_ok) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int code = 32 * c + race_crow(r, h);
        if (code < a.K) a.logits_out[m * a.K + code] = v[r];
      }
    }
    race_tile<INJ>(st, v, 32 * c, h, a.K, grow, key, ctr0);
  }
  int pick;
  float p;
  race_finish(st, pick, p);
  if (h == 0 && row_ok) {
    const int64_t s0 = a.s_in[m];
    const bool known = s0 != a.mask_id;
    a.sampled[m] = known ? s0 : (int64_t)pick;
    a.selp[m] = known ? INFINITY : p;
  }
}

}  // namespace tvq

using namespace tvq;

extern "C" int tvq_maskgit_sample(const float* logits, int64_t sb, int64_t sn, int64_t B,
                                  int64_t n, int64_t K, const int64_t* s_in, int64_t mask_id,
                                  const float* gumbel, const int64_t* seed_ptr, uint64_t offset,
                                  int64_t* sampled, float* selp, tvq_stream_t stream) {
  TVQ_CHECK_ARG(logits && s_in && sampled && selp && B > 0 && n > 0 && K > 0,
                "tvq_maskgit_sample: bad arguments");
  TVQ_CHECK_ARG(gumbel || seed_ptr, "tvq_maskgit_sample: need gumbel noise or a seed");
  TVQ_CHECK_ARG(B * n * K < (int64_t)1 << 32, "tvq_maskgit_sample: B * n * K >= 2^32");
  hipLaunchKernelGGL(maskgit_sample_kernel, dim3((unsigned)((B * n + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, logits, sb, sn, (int)n, (int)K, s_in, mask_id, gumbel,
                     seed_ptr, offset, sampled, selp, (int)B);
  return launch_status("tvq_maskgit_sample");
}

extern "C" int tvq_maskgit_remask(const float* selp, int64_t B, int64_t n, int64_t k,
                                  float temperature, const float* u_gumbel,
                                  const int64_t* seed_ptr, uint64_t offset,
                                  const int64_t* sampled, int64_t mask_id, int64_t* s_out,
                                  uint8_t* masking, tvq_stream_t stream) {
  TVQ_CHECK_ARG(selp && B > 0 && n > 0 && k >= 0 && k <= n, "tvq_maskgit_remask: bad arguments");
  TVQ_CHECK_ARG(u_gumbel || seed_ptr, "tvq_maskgit_remask: need u_gumbel or a seed");
  TVQ_CHECK_ARG(!s_out || sampled, "tvq_maskgit_remask: s_out needs sampled");
  TVQ_CHECK_ARG(n * 4 <= 64 * 1024, "tvq_maskgit_remask: sequence too long");
  hipLaunchKernelGGL(maskgit_remask_kernel, dim3((unsigned)B), dim3(256), n * sizeof(float),
                     (hipStream_t)stream, selp, (int)n, (int)k, temperature, u_gumbel, seed_ptr,
                     offset, sampled, mask_id, s_out, masking);
  return launch_status("tvq_maskgit_remask");
}

extern "C" int tvq_codebook_gather_nchw(const int64_t* idx, int64_t B, int64_t P, int64_t D,
                                        const float* E, float* out, tvq_stream_t stream) {
  const int64_t blocks = B * ((P + CG_PT - 1) / CG_PT);
  TVQ_CHECK_ARG(idx && E && out && B > 0 && P > 0 && D > 0 && D <= 512 && blocks < (1ll << 31),
                "tvq_codebook_gather_nchw: bad args");
  hipLaunchKernelGGL(codebook_gather_nchw_kernel, dim3((unsigned)blocks), dim3(256),
                     (size_t)D * (CG_PT + 1) * sizeof(float), (hipStream_t)stream, idx, (int)P,
                     (int)D, E, out);
  return launch_status("tvq_codebook_gather_nchw");
}

// workspace bytes of tvq_tied_logits_sample: the packed code table and bias
extern "C" int64_t tvq_tied_logits_sample_workspace(int64_t K, int64_t D, int64_t n) {
  if (K < 1 || (D != 64 && D != 128) || n < 1) return -1;
  const int64_t Kt = (K + 31) / 32;
  return Kt * 32 * D * 4 + n * Kt * 32 * 4;
}

extern "C" int tvq_tied_logits_sample(const float* h, int64_t M, int64_t D, const float* W,
                                      int64_t K, const float* bias, int64_t n, int64_t ldb,
                                      const int64_t* s_in, int64_t mask_id, const float* gumbel,
                                      const int64_t* seed_ptr, uint64_t offset, int64_t* sampled,
                                      float* selp, float* logits_out, void* workspace,
                                      tvq_stream_t stream) {
  TVQ_CHECK_ARG(h && W && bias && s_in && sampled && selp && workspace && M > 0 && K > 0 &&
                    n > 0 && ldb >= K && (D == 64 || D == 128),
                "tvq_tied_logits_sample: bad arguments (D must be 64 or 128)");
  TVQ_CHECK_ARG(gumbel || seed_ptr, "tvq_tied_logits_sample: need gumbel noise or a seed");
  TVQ_CHECK_ARG(gumbel || M * K < (int64_t)1 << 32, "tvq_tied_logits_sample: M * K >= 2^32");
  TVQ_CHECK_ARG(((uintptr_t)h & 15) == 0 && ((uintptr_t)W & 15) == 0 &&
                    ((uintptr_t)workspace & 15) == 0,
                "tvq_tied_logits_sample: h, W and the workspace must be 16-byte aligned");
  const int Kt = (int)((K + 31) / 32);
  hipStream_t st = (hipStream_t)stream;
  TlsArgs a;
  a.h = h;
  a.wpk = reinterpret_cast<const float4*>(workspace);
  float* bpk = reinterpret_cast<float*>(workspace) + (int64_t)Kt * 32 * D;
  a.bpk = bpk;
  a.s_in = s_in; a.gumbel = gumbel; a.seed_ptr = seed_ptr; a.offset = offset;
  a.mask_id = mask_id; a.sampled = sampled; a.selp = selp; a.logits_out = logits_out;
  a.M = M; a.n = (int)n; a.K = (int)K; a.Kt = Kt;
  const unsigned blocks = (unsigned)((M + 127) / 128);
  float4* wpk = reinterpret_cast<float4*>(workspace);
  if (D == 128) {
    hipLaunchKernelGGL(tls_pack_kernel<128>, dim3((unsigned)(Kt + n)), dim3(256), 0, st, W, (int)K,
                       bias, ldb, wpk, bpk, Kt);
    if (gumbel) hipLaunchKernelGGL((tied_logits_sample_kernel<128, true>), dim3(blocks), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((tied_logits_sample_kernel<128, false>), dim3(blocks), dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL(tls_pack_kernel<64>, dim3((unsigned)(Kt + n)), dim3(256), 0, st, W, (int)K,
                       bias, ldb, wpk, bpk, Kt);
    if (gumbel) hipLaunchKernelGGL((tied_logits_sample_kernel<64, true>), dim3(blocks), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((tied_logits_sample_kernel<64, false>), dim3(blocks), dim3(256), 0, st, a);
  }
  TVQ_PLAN("tied_logits_sample D=%d K=%d M=%lld", (int)D, (int)K, (long long)M);
  return launch_status("tvq_tied_logits_sample");
}

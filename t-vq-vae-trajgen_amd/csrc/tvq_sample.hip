// MaskGIT iterative-decoding step (maskgit.py:294-411 first_pass / second_pass,
// mask_by_random_topk maskgit.py:238-267) on device, one block per sequence:
//
//   sample:  for every still-masked token, draw s ~ Categorical(softmax(logits)) by inverse
//            CDF at u (double softmax + double prefix over K), keep known tokens, and record
//            p(s) (fp32 softmax; +inf for known tokens, maskgit.py:320-326)
//   remask:  confidence = log(p + 1e-5) + tau * Gumbel(u'), re-mask the k lowest per row
//            (topk(largest=False) keeps exactly k, maskgit.py:259-266)
//
// The reference loops over rows in Python and calls .item() per step; here each step is
// two launches with no host synchronisation.  Noise comes from the device seed (counter
// hash of (seed, offset, element)) or is injected (tests pin against the oracle).
#include "tvq_common.h"

namespace tvq {

__device__ __forceinline__ double wave_sum_dd(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(256) void maskgit_sample_kernel(
    const float* __restrict__ logits, int64_t sb, int64_t sn, int n, int K,
    const int64_t* __restrict__ s_in, int64_t mask_id, const float* __restrict__ u_cat,
    const int64_t* __restrict__ seed_ptr, uint64_t offset, int64_t* __restrict__ sampled,
    float* __restrict__ selp, int nb) {
  // one wave per token: token t = blockIdx.x * 4 + wave (all B*n tokens in flight at once;
  // a block per sequence left each wave a serial loop over n / 4 tokens)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t seed = u_cat ? 0ull : mix_seed(seed_ptr, offset);
  const int per = (K + 63) / 64;  // contiguous logits per lane
  const int j0 = lane * per;
  {
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
    float m = -INFINITY;
    for (int j = lane; j < K; j += 64) m = fmaxf(m, l[j]);
    m = wave_max(m);
    // double softmax numerators over the lane's contiguous chunk
    double part = 0.0;
    for (int j = j0; j < min(K, j0 + per); ++j) part += exp((double)l[j] - (double)m);
    const double tot = wave_sum_dd(part);
    // inclusive prefix of the lane chunks (probabilities), then the first chunk whose
    // running sum exceeds v = u * total (strictly: at u = 0 a leading zero-probability
    // code must not be drawn; torch's Categorical never samples one)
    double incl = part / tot;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const double y = __shfl_up(incl, d, 64);
      if (lane >= d) incl += y;
    }
    const double cdf_last = __shfl(incl, 63, 64);
    const float u = u_cat ? u_cat[t] : uniform01(seed, (uint64_t)t);
    const double v = (double)u * cdf_last;
    const unsigned long long hit = __ballot(incl > v);
    // rounding fallback (no prefix exceeds v, u close to 1): the last chunk holding any
    // probability, never a trailing chunk of zero-probability codes
    const unsigned long long pos = __ballot(part > 0.0);
    const int src = hit ? __ffsll(hit) - 1 : (pos ? 63 - __clzll(pos) : 63);
    int pick = -1;
    if (lane == src) {
      double acc = incl - part / tot;
      int last_pos = j0;  // last code of the chunk with positive probability
      for (int j = j0; j < min(K, j0 + per); ++j) {
        const double pj = exp((double)l[j] - (double)m) / tot;
        if (pj > 0.0) last_pos = j;
        acc += pj;
        if (acc > v) {
          pick = j;
          break;
        }
      }
      if (pick < 0) pick = last_pos;  // the recomputed sum never passed v (rounding)
    }
    pick = __shfl(pick, src, 64);
    if (lane == 0) {
      sampled[t] = pick;
      // p(sampled) of the softmax (maskgit.py:320-326), rounded once from the double terms
      selp[t] = (float)(exp((double)l[pick] - (double)m) / tot);
    }
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
// NCHW input (maskgit.py:461-469 embedding + 'b n c -> b c (h w)')
__global__ __launch_bounds__(256) void codebook_gather_nchw_kernel(
    const int64_t* __restrict__ idx, int B, int P, int D, const float* __restrict__ E,
    float* __restrict__ out) {
  const int64_t tot = (int64_t)B * D * P;
  for (int64_t o = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; o < tot;
       o += (int64_t)gridDim.x * blockDim.x) {
    const int p = (int)(o % P);
    const int64_t r = o / P;
    const int d = (int)(r % D);
    const int b = (int)(r / D);
    out[o] = E[idx[(int64_t)b * P + p] * D + d];
  }
}

}  // namespace tvq

using namespace tvq;

extern "C" int tvq_maskgit_sample(const float* logits, int64_t sb, int64_t sn, int64_t B,
                                  int64_t n, int64_t K, const int64_t* s_in, int64_t mask_id,
                                  const float* u_cat, const int64_t* seed_ptr, uint64_t offset,
                                  int64_t* sampled, float* selp, tvq_stream_t stream) {
  TVQ_CHECK_ARG(logits && s_in && sampled && selp && B > 0 && n > 0 && K > 0,
                "tvq_maskgit_sample: bad arguments");
  TVQ_CHECK_ARG(u_cat || seed_ptr, "tvq_maskgit_sample: need u_cat or a seed");
  hipLaunchKernelGGL(maskgit_sample_kernel, dim3((unsigned)((B * n + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, logits, sb, sn, (int)n, (int)K, s_in, mask_id, u_cat,
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
  TVQ_CHECK_ARG(idx && E && out && B > 0 && P > 0 && D > 0, "tvq_codebook_gather_nchw: bad args");
  const int64_t tot = B * D * P;
  const int blocks = (int)((tot + 255) / 256 < 8192 ? (tot + 255) / 256 : 8192);
  hipLaunchKernelGGL(codebook_gather_nchw_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                     idx, (int)B, (int)P, (int)D, E, out);
  return launch_status("tvq_codebook_gather_nchw");
}

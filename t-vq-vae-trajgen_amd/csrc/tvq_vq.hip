// VQ codebook kernels (K7/K8/K9 in SURVEY.md §2.2) for gfx950.
//
// assign: 16 RG token rows per workgroup of 2 RG waves (RG per launch, vq_rg: 6 for the
// HF band's 24576 rows -- one workgroup per CU -- and 2 for the LF band's 6144).  Each wave
// keeps its 16 rows' x values in registers as fp32 MFMA A-fragments (D/4 VGPRs) for the
// whole launch and streams the codebook through LDS in 128-code chunks (two buffers: the
// next chunk's global loads are in flight during this chunk's MFMAs); waves 0..RG-1 own
// code columns [0,64) of every chunk, waves RG..2RG-1 columns [64,128).  x.E^T runs on
// v_mfma_f32_16x16x4_f32 (exact fp32 FMA chains); the argmin is a running
// per-lane (value, index) pair merged across the 16 code lanes by shuffles and
// across the two code halves through LDS.  The epilogue gathers q = E[idx],
// writes the straight-through value and per-block commitment partials.
#include <float.h>
#include <limits.h>

#include "tvq_common.h"
#include "tvq_reduce.h"

namespace tvq {

// a workgroup = RG row groups of 16 token rows x 2 code halves (2 RG waves); RG is chosen
// per launch (vq_rg) so that the busiest SIMD runs as few waves as possible
constexpr int VQ_RG_MAX = 6;
constexpr int VQ_CK = 128;  // codes per LDS chunk

// (v, i) "better" for argmin of t with first-index tie break.  A NaN distance beats every
// number (torch.argmax over dist = -t treats NaN as the maximum and returns the first NaN
// index, vq.py:216-222), and among NaNs the first index wins.
__device__ __forceinline__ bool better(float v, int i, float bv, int bi) {
  const bool n = v != v, bn = bv != bv;
  if (n != bn) return n;
  if (n) return i < bi;
  return v < bv || (v == bv && i < bi);
}

// ||E_k||^2 as one fmaf chain over d in order (the same value the reference's CPU sum
// rounds to here, and bitwise what the assign kernel has always used).  A block stages
// SQ_CODES codebook rows into LDS with coalesced loads, then thread k runs code k's chain
// from LDS (row stride D + 1: the threads' reads at one d hit distinct banks).  Reading
// the rows straight from HBM one element per thread step took 19 us per codebook.
constexpr int SQ_CODES = 32;
__global__ __launch_bounds__(256) void vq_sqnorm_kernel(const float* __restrict__ E, int K, int D,
                                                        float* __restrict__ ee) {
  extern __shared__ float es[];  // [SQ_CODES][D + 1]
  const int k0 = blockIdx.x * SQ_CODES;
  const int nk = min(SQ_CODES, K - k0);
  for (int e = threadIdx.x; e < nk * D; e += 256) {
    const int c = e / D, d = e - c * D;
    es[c * (D + 1) + d] = E[(int64_t)k0 * D + e];
  }
  __syncthreads();
  if ((int)threadIdx.x >= nk) return;
  const float* r = es + threadIdx.x * (D + 1);
  float s = 0.f;
  for (int d = 0; d < D; ++d) s = fmaf(r[d], r[d], s);
  ee[k0 + threadIdx.x] = s;
}

// Stochastic assignment (svq_temp > 0, vq.py:51-56 softmax_sample): idx ~
// Categorical(logits = dist / temp), drawn by Gumbel-max inside the running argmax:
// argmax(dist/temp + g) = argmin(v/temp - g) with v = -dist, g = -log(-log u).  u is a
// counter hash of (device seed, offset, m*K + k), or g is injected (M x K, tests).
struct Svq {
  float temp;
  const float* gumbel;       // nullable: injected noise, row-major (M, K)
  const int64_t* seed_ptr;   // device seed (hip/rng.py)
  uint64_t offset;
};

__device__ __forceinline__ float gumbel_at(const Svq& sv, uint64_t seed, int64_t m, int K,
                                           int code) {
  const uint64_t c = (uint64_t)m * (uint64_t)K + (uint64_t)code;
  if (sv.gumbel) return sv.gumbel[c];
  // u in (0, 1): 24-bit lattice offset by half a step, so log(u) is finite
  const float u = ((float)(hash_u32(seed * 0xD1B54A32D192ED03ull + c) >> 8) + 0.5f) *
                  (1.0f / 16777216.0f);
  return -logf(-logf(u));
}

template <int D, bool STOCH, int RG>
__global__ __launch_bounds__(128 * RG) void vq_assign_kernel(
    const float* __restrict__ x, int64_t M, int64_t N, int64_t sB, int64_t sN, int64_t sD,
    const float* __restrict__ E, const float* __restrict__ ee, int K, int training,
    float* __restrict__ quant, int64_t* __restrict__ idx, int32_t* __restrict__ idx32,
    float* __restrict__ commit_partial, Svq sv, float* __restrict__ xt) {
  constexpr int VQ_BM = 16 * RG, VQ_T = 128 * RG, NW = 2 * RG;
  constexpr int S = D + 8;  // LDS row stride (floats): conflict-free ds_read_b128 B-fragments
  constexpr int NQ = D / 16;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* es = smem;                       // [2][VQ_CK][S]
  float* xx_s = smem + 2 * VQ_CK * S;     // [VQ_BM]
  float* bv_s = xx_s + VQ_BM;             // [2][VQ_BM]
  int* bi_s = (int*)(bv_s + 2 * VQ_BM);   // [2][VQ_BM]
  float* red = (float*)(bi_s + 2 * VQ_BM);  // [NW]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int rg = wid % RG, ch = wid / RG;
  const int r16 = lane & 15, g = lane >> 4;
  const int64_t row0 = (int64_t)blockIdx.x * VQ_BM;

  // ---- A fragments: x[row0 + rg*16 + r16][16q + 4g + j] ----
  float areg[NQ * 4];
  {
    const int64_t m = row0 + rg * 16 + r16;
    const bool ok = m < M;
    const int64_t b = ok ? m / N : 0, n = ok ? m - b * N : 0;
    const float* xr = x + b * sB + n * sN;
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j) areg[q * 4 + j] = ok ? xr[(int64_t)(16 * q + 4 * g + j) * sD] : 0.f;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NQ * 4; ++i) s = fmaf(areg[i], areg[i], s);
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    if (ch == 0 && g == 0) xx_s[rg * 16 + r16] = s;
  }

  const uint64_t sseed = (STOCH && !sv.gumbel) ? mix_seed(sv.seed_ptr, sv.offset) : 0ull;
  float bestv[4];
  int besti[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { bestv[r] = INFINITY; besti[r] = INT_MAX; }

  // two chunk buffers: chunk c + 1 is loaded into registers before chunk c's MFMAs and
  // written to the other buffer after them, one barrier per chunk
  constexpr int PF = (VQ_CK * (D / 4) + VQ_T - 1) / VQ_T;
  auto stage_load = [&](int c0, float4* pf) {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int e = tid + i * VQ_T;
      const int c = e / (D / 4), d4 = e - c * (D / 4);
      pf[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < VQ_CK * (D / 4) && c0 + c < K)
        pf[i] = *reinterpret_cast<const float4*>(E + (int64_t)(c0 + c) * D + 4 * d4);
    }
  };
  auto stage_store = [&](float* buf, const float4* pf) {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int e = tid + i * VQ_T;
      const int c = e / (D / 4), d4 = e - c * (D / 4);
      if (e < VQ_CK * (D / 4)) *reinterpret_cast<float4*>(buf + c * S + 4 * d4) = pf[i];
    }
  };
  {
    float4 pf[PF];
    stage_load(0, pf);
    stage_store(es, pf);
  }
  __syncthreads();
  for (int c0 = 0, cb = 0; c0 < K; c0 += VQ_CK, cb ^= 1) {
    float4 pf[PF];
    const bool more = c0 + VQ_CK < K;
    if (more) stage_load(c0 + VQ_CK, pf);
    const float* ebuf = es + cb * (VQ_CK * S);
    floatx4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    const float* eb = ebuf + (ch * 64 + r16) * S + 4 * g;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      float4 bq[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) bq[t] = *reinterpret_cast<const float4*>(eb + t * 16 * S + 16 * q);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        acc[t] = mfma16x16x4(areg[q * 4 + 0], bq[t].x, acc[t]);
        acc[t] = mfma16x16x4(areg[q * 4 + 1], bq[t].y, acc[t]);
        acc[t] = mfma16x16x4(areg[q * 4 + 2], bq[t].z, acc[t]);
        acc[t] = mfma16x16x4(areg[q * 4 + 3], bq[t].w, acc[t]);
      }
    }
    // C layout: acc[t][r] -> row (4g + r) of the wave's 16 rows, code col r16 of tile t
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int code = c0 + ch * 64 + t * 16 + r16;
      const float e2 = code < K ? ee[code] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float xx = xx_s[rg * 16 + 4 * g + r];
        float v = (xx - 2.0f * acc[t][r]) + e2;
        if (STOCH && code < K) {
          const int64_t m = row0 + rg * 16 + 4 * g + r;
          v = v / sv.temp - gumbel_at(sv, sseed, m < M ? m : 0, K, code);
        }
        if (code >= K) v = INFINITY;
        // codes increase: strict < keeps the first; a NaN beats a number and is never beaten
        if (v < bestv[r] || (v != v && bestv[r] == bestv[r])) { bestv[r] = v; besti[r] = code; }
      }
    }
    if (more) stage_store(es + (cb ^ 1) * (VQ_CK * S), pf);
    __syncthreads();
  }
  // merge across the 16 code lanes of each row group
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      float ov = __shfl_xor(bestv[r], o, 64);
      int oi = __shfl_xor(besti[r], o, 64);
      if (better(ov, oi, bestv[r], besti[r])) { bestv[r] = ov; besti[r] = oi; }
    }
  }
  if (r16 == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bv_s[ch * VQ_BM + rg * 16 + 4 * g + r] = bestv[r];
      bi_s[ch * VQ_BM + rg * 16 + 4 * g + r] = besti[r];
    }
  }
  __syncthreads();
  if (tid < VQ_BM) {
    float v0 = bv_s[tid], v1 = bv_s[VQ_BM + tid];
    int i0 = bi_s[tid], i1 = bi_s[VQ_BM + tid];
    int bi = better(v1, i1, v0, i0) ? i1 : i0;
    if (bi < 0 || bi >= K) bi = 0;  // unreachable for K >= 1 (NaN rows pick their first NaN)
    bi_s[tid] = bi;
    const int64_t m = row0 + tid;
    if (m < M) {
      idx[m] = bi;
      idx32[m] = bi;
    }
  }
  __syncthreads();
  // epilogue: q = E[idx] (pre-update codebook); straight-through value; commit partial
  float csum = 0.f;
  const bool dfast = (sD == 1);
  for (int e = tid; e < VQ_BM * D; e += VQ_T) {
    int r, d;
    if (dfast) { r = e / D; d = e - r * D; } else { d = e / VQ_BM; r = e - d * VQ_BM; }
    const int64_t m = row0 + r;
    if (m >= M) continue;
    const int64_t b = m / N, n = m - b * N;
    const int64_t off = b * sB + n * sN + (int64_t)d * sD;
    const float qv = E[(int64_t)bi_s[r] * D + d];
    if (training) {
      const float xv = x[off];
      const float st = xv + (qv - xv);
      const float df = st - xv;
      csum = fmaf(df, df, csum);
      quant[off] = st;
      if (xt) es[r * (D + 1) + d] = xv;  // the chunk buffer is free after the last barrier
    } else {
      quant[off] = qv;
    }
  }
  if (training && xt) {
    // token-major copy of the block's rows (row m at xt + m * D): the codebook statistics
    // then sum contiguous rows instead of gathering D-strided NCHW elements
    __syncthreads();
    for (int e = tid; e < VQ_BM * D; e += VQ_T) {
      const int r = e / D, d = e - r * D;
      if (row0 + r < M) xt[(row0 + r) * D + d] = es[r * (D + 1) + d];
    }
  }
  if (training && commit_partial) {
    csum = wave_sum(csum);
    if (lane == 0) red[wid] = csum;
    __syncthreads();
    if (tid == 0) {
      float t = red[0];
#pragma unroll
      for (int w = 1; w < NW; ++w) t += red[w];
      commit_partial[blockIdx.x] = t;
    }
  }
}

// counts[k] = offsets[k+1] - offsets[k] (from the stable group-by of idx32)
__global__ void vq_ema_kernel(const float* __restrict__ cs_batch, const float* __restrict__ es_batch,
                              int D, float decay, float alpha, float* __restrict__ cluster_size,
                              float* __restrict__ embed_avg) {
  const int k = blockIdx.x;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    const int64_t o = (int64_t)k * D + d;
    embed_avg[o] = fmaf(es_batch[o], alpha, embed_avg[o] * decay);
  }
  if (threadIdx.x == 0) cluster_size[k] = fmaf(cs_batch[k], alpha, cluster_size[k] * decay);
}

__global__ __launch_bounds__(256) void vq_finalize_kernel(
    const float* __restrict__ cluster_size, const float* __restrict__ embed_avg, int K, int D,
    float eps, float* __restrict__ embed, const int32_t* __restrict__ counts, int64_t M,
    float* __restrict__ perplexity, const float* __restrict__ commit_partial, int64_t nparts,
    float* __restrict__ commit) {
  __shared__ float red[4];
  const int k = blockIdx.x, tid = threadIdx.x;
  if (embed) {
    float s = 0.f;
    for (int j = tid; j < K; j += 256) s += cluster_size[j];
    const float tot = block_sum(s, red);
    const float denom = tot + (float)K * eps;
    const float c = (cluster_size[k] + eps) / denom * tot;
    for (int d = tid; d < D; d += 256) embed[(int64_t)k * D + d] = embed_avg[(int64_t)k * D + d] / c;
  }
  if (k == 0) {
    if (perplexity) {
      float h = 0.f;
      for (int j = tid; j < K; j += 256) {
        const float p = (float)counts[j] / (float)M;
        h += p * logf(p + 1e-10f);
      }
      const float ht = block_sum(h, red);
      if (tid == 0) perplexity[0] = expf(-ht);
    }
    if (commit) {
      float s = 0.f;
      for (int64_t j = tid; j < nparts; j += 256) s += commit_partial[j];
      const float st = block_sum(s, red);
      if (tid == 0) commit[0] = st / ((float)M * (float)D);
    }
  }
}

__global__ void vq_backward_kernel(const float* __restrict__ x, const float* __restrict__ q,
                                   const float* __restrict__ dq, const float* __restrict__ gc,
                                   int64_t n, float inv_numel2, float* __restrict__ dx) {
  const float c = gc ? gc[0] * inv_numel2 : 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dx[i] = dq[i] + c * (x[i] - q[i]);
}

}  // namespace tvq

using namespace tvq;

extern "C" int tvq_vq_sqnorm(const float* E, int64_t K, int64_t D, float* ee, tvq_stream_t stream) {
  TVQ_CHECK_ARG(E && ee && K > 0 && D > 0, "tvq_vq_sqnorm: bad arguments");
  TVQ_CHECK_ARG(D <= 1024, "tvq_vq_sqnorm: D > 1024");
  hipLaunchKernelGGL(vq_sqnorm_kernel, dim3((unsigned)((K + SQ_CODES - 1) / SQ_CODES)), dim3(256),
                     (size_t)SQ_CODES * (D + 1) * sizeof(float), (hipStream_t)stream, E, (int)K,
                     (int)D, ee);
  return launch_status("tvq_vq_sqnorm");
}

// row groups per workgroup: 6 (96 rows, 12 waves) when that still fills every CU with a
// workgroup -- the HF band's 24576 rows as 256 workgroups, one per CU: 55 us, where 64-row
// workgroups (384: two on half the CUs) took 60 us and 48 / 32-row ones 66 / 85 us (each
// workgroup streams the whole codebook through LDS; single-buffered then, 53 us now); else 2
// (32 rows: the LF band's 6144 rows as 192 workgroups, 32.5 us where 96 64-row ones took 39.6,
// double-buffered both; tools/ab/r06/gpu_vqab.sh)
static int vq_rg(int64_t M) { return M >= 256 * 96 ? 6 : 2; }

extern "C" int64_t tvq_vq_assign_nblocks(int64_t M) {
  const int rg = vq_rg(M);
  return (M + 16 * rg - 1) / (16 * rg);
}

extern "C" int tvq_vq_assign(const float* x, int64_t B, int64_t N, int64_t D, int64_t sB,
                             int64_t sN, int64_t sD, const float* E, const float* ee, int64_t K,
                             int training, float* quant, int64_t* idx, int32_t* idx32,
                             float* commit_partial, tvq_stream_t stream) {
  return tvq_vq_assign_svq(x, B, N, D, sB, sN, sD, E, ee, K, training, 0.f, nullptr, nullptr, 0,
                           quant, idx, idx32, commit_partial, stream);
}

extern "C" int tvq_vq_assign_svq(const float* x, int64_t B, int64_t N, int64_t D, int64_t sB,
                                 int64_t sN, int64_t sD, const float* E, const float* ee,
                                 int64_t K, int training, float temp, const float* gumbel,
                                 const int64_t* seed_ptr, uint64_t offset, float* quant,
                                 int64_t* idx, int32_t* idx32, float* commit_partial,
                                 tvq_stream_t stream) {
  return tvq_vq_assign_rows(x, B, N, D, sB, sN, sD, E, ee, K, training, temp, gumbel, seed_ptr,
                            offset, quant, idx, idx32, commit_partial, nullptr, stream);
}

extern "C" int tvq_vq_assign_rows(const float* x, int64_t B, int64_t N, int64_t D, int64_t sB,
                                  int64_t sN, int64_t sD, const float* E, const float* ee,
                                  int64_t K, int training, float temp, const float* gumbel,
                                  const int64_t* seed_ptr, uint64_t offset, float* quant,
                                  int64_t* idx, int32_t* idx32, float* commit_partial,
                                  float* token_rows, tvq_stream_t stream) {
  float* xt = training ? token_rows : nullptr;
  TVQ_CHECK_ARG(x && E && ee && quant && idx && idx32 && B > 0 && N > 0 && K > 0,
                "tvq_vq_assign: bad arguments");
  TVQ_CHECK_ARG(temp >= 0.f && (temp == 0.f || gumbel || seed_ptr),
                "tvq_vq_assign_svq: temp > 0 needs injected noise or a device seed");
  TVQ_CHECK_ARG(!training || commit_partial, "tvq_vq_assign: training needs commit_partial");
  TVQ_CHECK_ARG(K < INT_MAX, "tvq_vq_assign: K too large");
  const int64_t M = B * N;
  const int rg = vq_rg(M);
  const int64_t nb = tvq_vq_assign_nblocks(M);
  const size_t lds_tail = (size_t)(16 * rg * 5) * 4 + 4 * 2 * VQ_RG_MAX + 32;
  hipStream_t st = (hipStream_t)stream;
  const Svq sv = {temp, gumbel, seed_ptr, offset};
  TVQ_PLAN("vq_assign D%lld rg%d nb%lld%s", (long long)D, rg, (long long)nb, temp > 0.f ? " svq" : "");
#define TVQ_ASSIGN_RG(DD, ST, RGV)                                                           \
  if (rg == RGV)                                                                             \
    hipLaunchKernelGGL((vq_assign_kernel<DD, ST, RGV>), dim3(nb), dim3(128 * RGV), lds, st, x,  \
                       M, N, sB, sN, sD, E, ee, (int)K, training, quant, idx, idx32,         \
                       commit_partial, sv, xt);
#define TVQ_ASSIGN_ST(DD, ST) \
  TVQ_ASSIGN_RG(DD, ST, 2) TVQ_ASSIGN_RG(DD, ST, 6)
#define TVQ_ASSIGN(DD)                                                                       \
  case DD: {                                                                                 \
    const size_t lds = (size_t)2 * VQ_CK * (DD + 8) * 4 + lds_tail;                              \
    if (sv.temp > 0.f) {                                                                     \
      TVQ_ASSIGN_ST(DD, true)                                                                \
    } else {                                                                                 \
      TVQ_ASSIGN_ST(DD, false)                                                               \
    }                                                                                        \
    break;                                                                                   \
  }
  switch (D) {
    TVQ_ASSIGN(32)
    TVQ_ASSIGN(64)
    TVQ_ASSIGN(128)
    default:
      set_error("tvq_vq_assign: unsupported codebook dim %lld (32/64/128)", (long long)D);
      return TVQ_ERR_ARG;
  }
#undef TVQ_ASSIGN
#undef TVQ_ASSIGN_ST
#undef TVQ_ASSIGN_RG
  return launch_status("tvq_vq_assign");
}

extern "C" int64_t tvq_vq_stats_workspace(int64_t M, int64_t K) {
  // 4-byte words: offsets | perm | group-by scratch | (aligned) float chunk partials (D <= 512)
  const int64_t ints = (K + 1) + M + group_by_scratch_ints(M, K);
  return ((ints + 3) / 4) * 4 + seg_rowsum_scratch_floats(M, K, 512);
}

extern "C" int tvq_vq_stats(const float* x, int64_t B, int64_t N, int64_t D, int64_t sB,
                            int64_t sN, int64_t sD, const int32_t* idx32, int64_t K,
                            int32_t* counts, float* cs_batch, float* es_batch, int32_t* workspace,
                            tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && idx32 && counts && cs_batch && workspace && B > 0 && N > 0 && K > 0 && D > 0 &&
                    D <= 512, "tvq_vq_stats: bad arguments");
  const int64_t M = B * N;
  hipStream_t st = (hipStream_t)stream;
  int* offsets = workspace;
  int* perm = offsets + (K + 1);
  int* scratch = perm + M;
  const int64_t ints = (K + 1) + M + group_by_scratch_ints(M, K);
  float* part = (float*)(workspace + ((ints + 3) / 4) * 4);
  // the per-code counts (and their float copy, cs_batch) come out of the group-by's scan
  group_by_i32(idx32, M, K, offsets, perm, scratch, st, counts, cs_batch);
  if (es_batch) {
    SegRows r;
    r.src = x; r.N = N; r.sB = sB; r.sN = sN; r.sD = sD; r.D = (int)D;
    r.drop_p = 0.f; r.seed_ptr = nullptr; r.offset = 0; r.mask_id = -1;
    seg_rowsum(r, offsets, perm, group_by_seg_start(scratch, M, K), M, K, es_batch, 0, part, st);
  }
  return launch_status("tvq_vq_stats");
}

extern "C" int tvq_vq_ema(const float* cs_batch, const float* es_batch, int64_t K, int64_t D,
                          float decay, float* cluster_size, float* embed_avg,
                          tvq_stream_t stream) {
  TVQ_CHECK_ARG(cs_batch && es_batch && cluster_size && embed_avg && K > 0 && D > 0,
                "tvq_vq_ema: bad arguments");
  const float alpha = (float)(1.0 - (double)decay);
  hipLaunchKernelGGL(vq_ema_kernel, dim3(K), dim3(128), 0, (hipStream_t)stream, cs_batch, es_batch,
                     (int)D, decay, alpha, cluster_size, embed_avg);
  return launch_status("tvq_vq_ema");
}

extern "C" int tvq_vq_finalize(const float* cluster_size, const float* embed_avg, int64_t K,
                               int64_t D, float eps, float* embed, const int32_t* counts,
                               int64_t M, float* perplexity, const float* commit_partial,
                               int64_t nparts, float* commit, tvq_stream_t stream) {
  TVQ_CHECK_ARG(K > 0 && D > 0, "tvq_vq_finalize: bad arguments");
  TVQ_CHECK_ARG(!embed || (cluster_size && embed_avg), "tvq_vq_finalize: embed needs buffers");
  TVQ_CHECK_ARG(!perplexity || counts, "tvq_vq_finalize: perplexity needs counts");
  TVQ_CHECK_ARG(!commit || commit_partial, "tvq_vq_finalize: commit needs partials");
  const int grid = embed ? (int)K : 1;
  hipLaunchKernelGGL(vq_finalize_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                     cluster_size, embed_avg, (int)K, (int)D, eps, embed, counts, M, perplexity,
                     commit_partial, nparts, commit);
  return launch_status("tvq_vq_finalize");
}

extern "C" int tvq_vq_backward(const float* x, const float* quant, const float* dquant,
                               const float* gcommit, int64_t n, int64_t numel, float* dx,
                               tvq_stream_t stream) {
  TVQ_CHECK_ARG(x && quant && dquant && dx && n >= 0 && numel > 0, "tvq_vq_backward: bad args");
  if (n == 0) return TVQ_OK;
  const int64_t blocks = (n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096;
  hipLaunchKernelGGL(vq_backward_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, quant,
                     dquant, gcommit, n, (float)(2.0 / (double)numel), dx);
  return launch_status("tvq_vq_backward");
}

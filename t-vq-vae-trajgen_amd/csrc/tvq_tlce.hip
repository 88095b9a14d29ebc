// The priors' training loss head in one pass per 16 tokens: tied logits, masked cross-entropy
// and its gradient with respect to the logits and to the head output
// (bidirectional_transformer.py:186-191 logits = h tok_emb[:K]^T + bias[pos]; maskgit.py:183-191
// loss = F.cross_entropy(logits[~keep], target[~keep])), for the backward pass that starts
// right at this loss (MaskGIT.forward_backward: the root gradient `gscale`, a device scalar,
// is known in the forward).  Per token m:
//   l = h_m W^T + b_{m mod n}      lse = log sum_k exp(l_k)      loss_m = lse - l_target
//   D_m = keep_m ? 0 : (softmax(l) - onehot(target)) * gscale / cnt     (cnt = #masked)
//   dh_m = D_m W
// The logits never reach memory; D (read by the tied-weight and bias gradients) and dh are
// written once.  Replaces a logits GEMM, the masked-CE forward and backward launches and the
// dh GEMM, which wrote the (M, K) logits once and read them / D three times.
//
// Layout: one wave per 16 tokens on v_mfma_f32_16x16x4_f32.  Lane l = (i = l & 15, g = l >> 4).
//   logits tile c (16 codes): rows = codes, cols = tokens; k-slot g of step s is feature
//     32 g + s, so a lane's B operands are h[token i][32 g .. 32 g + 31] (8 float4 loads) and
//     its A operands W[16 c + i][32 g + s] (float4 per 4 steps); the lane ends with codes
//     16 c + 4 g + r (r = 0..3, consecutive: one float4 of D per tile) of token i.
//   dh: rows = features (8 tiles of 16), cols = tokens; step (c, r) takes k-slot g = code
//     16 c + 4 g + r, i.e. the lane's own D register r of tile c as the B operand, and
//     A = W[that code][f]; the lane ends with features 16 ft + 4 g + r of token i (one float4
//     of dh per feature tile).
// All NT logit tiles stay in registers (NT * 4 floats per lane); the W tiles come through a
// 3-deep LDS ring of 32-code tiles shared by the block's 4 waves (two sweeps: logits, then dh).
#include <math.h>

#include "tvq_common.h"

namespace tvq {

constexpr int TLCE_D = 128;

struct TlceArgs {
  const float* h;       // (M, 128)
  const float* W;       // (>= K, 128) tied table
  const float* bias;    // (n, ldb)
  int64_t ldb;
  const int64_t* target;
  const bool* keep;
  const float* stats;   // [cnt, gscale / cnt] (tlce_count_kernel)
  float* D;             // (M, K)
  float* dh;            // (M, 128)
  float* part;          // per-wave loss sums
  int64_t M;
  int n, K;
};

// cnt = #masked tokens (integer: exact), stats = {cnt, gscale / cnt}
__global__ __launch_bounds__(1024) void tlce_count_kernel(const bool* __restrict__ keep, int64_t M,
                                                          const float* __restrict__ gscale,
                                                          float* __restrict__ stats) {
  __shared__ int red[16];
  int c = 0;
  for (int64_t m = threadIdx.x; m < M; m += 1024) c += keep[m] ? 0 : 1;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < 16; ++w) t += red[w];
    const float cnt = (float)t;
    stats[0] = cnt;
    stats[1] = gscale[0] / cnt;
  }
}

// W tiles (32 codes x 128 features) are shared by the block's 4 waves (64 tokens) through a
// 3-deep LDS ring: each tile is read from L2 once per block and sweep (the logits
// sweep, then the dh sweep), not once per wave; one barrier per 32 codes.  Row stride 132
// floats (16-B reads of 16 rows spread over the banks).
constexpr int TLCE_RS = 132, TLCE_ROWS = 32, TLCE_TILE = TLCE_ROWS * TLCE_RS;

// one 32-code tile = 1024 float4, 4 per thread (named registers: no array to index)
struct TlceStage {
  float4 r0, r1, r2, r3;
};
__device__ __forceinline__ float4 tlce_ld(const float* __restrict__ W, int j, int u) {
  const int e = threadIdx.x + 256 * u, row = e >> 5, col = (e & 31) * 4;
  return *reinterpret_cast<const float4*>(W + (int64_t)(TLCE_ROWS * j + row) * TLCE_D + col);
}
__device__ __forceinline__ void tlce_st(float* buf, int u, float4 v) {
  const int e = threadIdx.x + 256 * u, row = e >> 5, col = (e & 31) * 4;
  *reinterpret_cast<float4*>(buf + row * TLCE_RS + col) = v;
}
__device__ __forceinline__ void tlce_tile_load(const float* __restrict__ W, int j, TlceStage& r) {
  r.r0 = tlce_ld(W, j, 0);
  r.r1 = tlce_ld(W, j, 1);
  r.r2 = tlce_ld(W, j, 2);
  r.r3 = tlce_ld(W, j, 3);
}
__device__ __forceinline__ void tlce_tile_store(float* buf, const TlceStage& r) {
  tlce_st(buf, 0, r.r0);
  tlce_st(buf, 1, r.r1);
  tlce_st(buf, 2, r.r2);
  tlce_st(buf, 3, r.r3);
}

template <int NT>
__global__ __launch_bounds__(256, 2) void tlce_kernel(TlceArgs a) {
  __shared__ float wl[3 * TLCE_TILE];  // 3-deep ring: tile j + 2 loads while j computes
  constexpr int NJ = NT / 2;  // 32-code tiles
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t t0 = wave * 16;
  // every wave of the block takes part in the LDS ring (barriers); rows past M compute on a
  // clamped row and store nothing
  const bool ok = t0 + i < a.M;
  const int64_t m = ok ? t0 + i : a.M - 1;
  constexpr int K = NT * 16;
  // B operands of the logits: h[m][32 g + s]
  float xb[32];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float4 v = *reinterpret_cast<const float4*>(a.h + m * TLCE_D + 32 * g + 4 * q);
    xb[4 * q] = v.x;
    xb[4 * q + 1] = v.y;
    xb[4 * q + 2] = v.z;
    xb[4 * q + 3] = v.w;
  }
  const float* brow = a.bias + (int64_t)(m % a.n) * a.ldb + 4 * g;
  // ---- logits sweep: all NT 16-code tiles in registers
  floatx4 L[NT];
  TlceStage st;
  tlce_tile_load(a.W, 0, st);
  tlce_tile_store(wl, st);
  if (NJ > 1) tlce_tile_load(a.W, 1, st);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    // tile j + 1 (loaded during the previous iteration) into its slot, then tile j + 2 loads
    // while tile j computes
    if (j + 1 < NJ) tlce_tile_store(wl + ((j + 1) % 3) * TLCE_TILE, st);
    if (j + 2 < NJ) tlce_tile_load(a.W, j + 2, st);
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int c = 2 * j + hf;
      const float* wt = wl + (j % 3) * TLCE_TILE + (16 * hf + i) * TLCE_RS + 32 * g;
      const float b0 = brow[16 * c], b1 = brow[16 * c + 1], b2 = brow[16 * c + 2],
                  b3 = brow[16 * c + 3];  // bias rows are K + 1 long: not 16-byte aligned
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float4 w = *reinterpret_cast<const float4*>(wt + 4 * q);
        acc = mfma16x16x4(w.x, xb[4 * q], acc);
        acc = mfma16x16x4(w.y, xb[4 * q + 1], acc);
        acc = mfma16x16x4(w.z, xb[4 * q + 2], acc);
        acc = mfma16x16x4(w.w, xb[4 * q + 3], acc);
      }
      L[c][0] = acc[0] + b0;
      L[c][1] = acc[1] + b1;
      L[c][2] = acc[2] + b2;
      L[c][3] = acc[3] + b3;
    }
    __syncthreads();
  }
  // the dh sweep's first tile, loading while the softmax runs
  tlce_tile_load(a.W, 0, st);
  // ---- softmax statistics of token i over the 4 lane groups (xor 16, xor 32)
  float mx = -INFINITY;
#pragma unroll
  for (int c = 0; c < NT; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) mx = fmaxf(mx, L[c][r]);
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  const int tgt = (int)a.target[m];
  float se = 0.f, lt = 0.f;
#pragma unroll
  for (int c = 0; c < NT; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      se += expf(L[c][r] - mx);
      lt += (16 * c + 4 * g + r == tgt) ? L[c][r] : 0.f;
    }
  se += __shfl_xor(se, 16, 64);
  se += __shfl_xor(se, 32, 64);
  lt += __shfl_xor(lt, 16, 64);
  lt += __shfl_xor(lt, 32, 64);
  const float lse = mx + logf(se);
  const bool masked = ok && !a.keep[m];
  const float sc = masked ? a.stats[1] : 0.f;
  // ---- D = (softmax - onehot) * gscale / cnt (zero rows for kept tokens), one float4 per tile
  float* drow = a.D + m * K + 4 * g;
#pragma unroll
  for (int c = 0; c < NT; ++c) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float p = expf(L[c][r] - lse);
      L[c][r] = masked ? (p - ((16 * c + 4 * g + r == tgt) ? 1.0f : 0.0f)) * sc : 0.f;
    }
    if (ok) *reinterpret_cast<float4*>(drow + 16 * c) = make_float4(L[c][0], L[c][1], L[c][2], L[c][3]);
  }
  // ---- dh sweep: dh^T = W^T D^T; A = W[16 c + 4 g + r][16 ft + i] from the LDS tile, B = D
  // register r of tile c
  tlce_tile_store(wl, st);
  if (NJ > 1) tlce_tile_load(a.W, 1, st);
  __syncthreads();
  floatx4 dacc[8];
#pragma unroll
  for (int ft = 0; ft < 8; ++ft) dacc[ft] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    if (j + 1 < NJ) tlce_tile_store(wl + ((j + 1) % 3) * TLCE_TILE, st);
    if (j + 2 < NJ) tlce_tile_load(a.W, j + 2, st);
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int c = 2 * j + hf;
      const float* wt = wl + (j % 3) * TLCE_TILE + (16 * hf + 4 * g) * TLCE_RS + i;
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int ft = 0; ft < 8; ++ft)
          dacc[ft] = mfma16x16x4(wt[r * TLCE_RS + 16 * ft], L[c][r], dacc[ft]);
    }
    __syncthreads();
  }
  if (ok) {
    float* hrow = a.dh + m * TLCE_D + 4 * g;
#pragma unroll
    for (int ft = 0; ft < 8; ++ft)
      *reinterpret_cast<float4*>(hrow + 16 * ft) =
          make_float4(dacc[ft][0], dacc[ft][1], dacc[ft][2], dacc[ft][3]);
  }
  // ---- the wave's loss sum over its masked tokens (lane group 0 holds one copy per token)
  float ls = (masked && g == 0) ? lse - lt : 0.f;
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) ls += __shfl_xor(ls, o, 64);
  if (lane == 0 && t0 < a.M) a.part[wave] = ls;
}

// loss = sum of the wave partials (fixed order) / cnt; out = {loss, cnt}
__global__ __launch_bounds__(256) void tlce_final_kernel(const float* __restrict__ part, int P,
                                                         const float* __restrict__ stats,
                                                         float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < P; i += 256) s += part[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    out[0] = s / stats[0];
    out[1] = stats[0];
  }
}

}  // namespace tvq

using namespace tvq;

static bool tlce_nt_ok(int64_t K) { return K == 64 || K == 128 || K == 256 || K == 512; }

extern "C" int64_t tvq_tied_logits_ce_workspace(int64_t M, int64_t K) {
  if (M < 1 || !tlce_nt_ok(K)) return -1;
  // stats (4) | wave partials
  return 4 + (M + 15) / 16;
}

extern "C" int tvq_tied_logits_ce(const float* h, int64_t M, int64_t D, const float* W, int64_t K,
                                  const float* bias, int64_t n, int64_t ldb, const int64_t* target,
                                  const bool* keep, const float* gscale, float* dlogits,
                                  float* dh, float* out, float* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(h && W && bias && target && keep && gscale && dlogits && dh && out && workspace &&
                    M > 0 && n > 0 && ldb >= K && D == TLCE_D && tlce_nt_ok(K),
                "tvq_tied_logits_ce: bad arguments (D 128, K in {64, 128, 256, 512})");
  TVQ_CHECK_ARG(((uintptr_t)h & 15) == 0 && ((uintptr_t)W & 15) == 0 &&
                    ((uintptr_t)dlogits & 15) == 0 && ((uintptr_t)dh & 15) == 0 &&
                    ((uintptr_t)workspace & 15) == 0,
                "tvq_tied_logits_ce: pointers must be 16-byte aligned");
  hipStream_t st = (hipStream_t)stream;
  float* stats = workspace;
  float* part = workspace + 4;
  const int64_t waves = (M + 15) / 16;
  hipLaunchKernelGGL(tlce_count_kernel, dim3(1), dim3(1024), 0, st, keep, M, gscale, stats);
  TlceArgs a;
  a.h = h; a.W = W; a.bias = bias; a.ldb = ldb; a.target = target; a.keep = keep;
  a.stats = stats; a.D = dlogits; a.dh = dh; a.part = part; a.M = M; a.n = (int)n; a.K = (int)K;
  const dim3 grid((unsigned)((waves + 3) / 4));
  TVQ_PLAN("tied_logits_ce M=%lld K=%lld", (long long)M, (long long)K);
  if (K == 512) hipLaunchKernelGGL(tlce_kernel<32>, grid, dim3(256), 0, st, a);
  else if (K == 256) hipLaunchKernelGGL(tlce_kernel<16>, grid, dim3(256), 0, st, a);
  else if (K == 128) hipLaunchKernelGGL(tlce_kernel<8>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(tlce_kernel<4>, grid, dim3(256), 0, st, a);
  hipLaunchKernelGGL(tlce_final_kernel, dim3(1), dim3(256), 0, st, part, (int)waves, stats, out);
  return launch_status("tvq_tied_logits_ce");
}

__global__ void scalar_ratio_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                    float* __restrict__ out) {
  if (threadIdx.x == 0) out[0] = a[0] / b[0];
}

// out[0] = a[0] / b[0] (device scalars; _TiedLogitsCE's root-gradient rescale)
extern "C" int tvq_scalar_ratio(const float* a, const float* b, float* out, tvq_stream_t stream) {
  TVQ_CHECK_ARG(a && b && out, "tvq_scalar_ratio: null argument");
  hipLaunchKernelGGL(scalar_ratio_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, a, b, out);
  return launch_status("tvq_scalar_ratio");
}

// Tied logits + masked cross-entropy of the MaskGIT priors in training, fused so the
// (rows x K) logits never reach HBM.
//
// Reference (bidirectional_transformer.py:186-191, maskgit.py:183-191):
//   logits = embed @ tok_emb.weight[:K]^T + bias[:, :K]          (rows m, position m % n)
//   loss   = F.cross_entropy(logits[~keep], s[~keep])            (mean over masked rows)
// The unfused path wrote the logits (50 MB for the HF prior at B = 256), read them for the
// CE, wrote d logits and read them twice more (input and weight gradients): ~420 us of kernel
// time per step on two 16 TFLOP/s GEMMs and four memory passes.  Here:
//   ce_fwd_kernel   per 32-row tile, the 4 waves split the codes; each wave computes
//                   logits^T tiles (32 codes x 32 rows) on v_mfma_f32_32x32x2_f32 (a lane
//                   owns one row and 16 codes of the tile), keeps a running max / sum per
//                   row, picks the target logit; the waves' (max, sum) are merged in wave
//                   order -> lse per row (kept for the backward), per-block masked loss sum
//                   and count -> masked_ce_final_kernel (mean)
//   ce_dh_kernel    the same tiles again, dl = (softmax - onehot) * g / count on masked
//                   rows, and dh += dl W with the tile's accumulator registers as the A
//                   operand directly (the code order of the k steps is the accumulator's)
//   ce_dw_kernel    grid (32-code tile, row split): logits tiles the other way round (a lane
//                   owns one code and 16 rows), dl, dW += dl^T h from the accumulator again,
//                   and the bias gradient per (position, code) in LDS in program order;
//                   per-split slabs summed in split order (the deferred slab batch)
// Everything is fixed-order: no atomics, bitwise reproducible.  Arithmetic: fp32 MFMA
// (exact k-ordered fma chains), online log-sum-exp (max, rescaled sum) -- within 1e-6 of
// torch's two-pass CE.
#include <math.h>

#include "tvq_common.h"
#include "tvq_conv_internal.h"
#include "tvq_reduce.h"

namespace tvq {

struct CeArgs {
  const float* h;  // (M, D) row-major
  const float* W;  // (>= K, D) row-major: the tied token-embedding table
  const float* bias;  // row m % n, row stride ldb (>= K)
  const int64_t* target;
  const bool* keep;
  float* lse;        // [M]
  float* part;       // fwd: [2 * blocks] (loss sum, masked count)
  const float* stats;  // bwd: {loss, count}
  const float* gout;   // bwd: d loss
  float* dh;           // bwd: (M, D)
  float* slab_w;       // bwd: [S][K][D]
  float* slab_b;       // bwd: [S][n][ldb]
  int M, D, K, n, ldb, S;
};

__device__ __forceinline__ int ce_crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

template <int HK>
__device__ __forceinline__ void ce_load_row(const float* __restrict__ p, float (&v)[HK]) {
#pragma unroll
  for (int t = 0; t < HK; t += 4) {
    const float4 q = *reinterpret_cast<const float4*>(p + t);
    v[t] = q.x; v[t + 1] = q.y; v[t + 2] = q.z; v[t + 3] = q.w;
  }
}

// logits^T tile: C[code crow(r, h)][row l & 31] = sum_d W[code0 + ...][d] h[row][d]; the
// lane's B operand (its row's half of d, HK floats) is in registers, the A operand (code
// code0 + (l & 31), same half of d) streams from L2 in 16-float chunks
template <int HK>
__device__ __forceinline__ floatx16 ce_tile_t(const float* __restrict__ wrow, const float (&hb)[HK]) {
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  constexpr int CH = HK < 16 ? HK : 16;
#pragma unroll
  for (int c0 = 0; c0 < HK; c0 += CH) {
    float wa[CH];
#pragma unroll
    for (int t = 0; t < CH; t += 4) {
      const float4 q = *reinterpret_cast<const float4*>(wrow + c0 + t);
      wa[t] = q.x; wa[t + 1] = q.y; wa[t + 2] = q.z; wa[t + 3] = q.w;
    }
#pragma unroll
    for (int t = 0; t < CH; ++t)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[t], hb[c0 + t], acc, 0, 0, 0);
  }
  return acc;
}

template <int D>
__global__ __launch_bounds__(256) void ce_fwd_kernel(CeArgs a) {
  constexpr int HK = D / 2;
  __shared__ float red[3][4][32];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r32 = lane & 31, hh = lane >> 5;
  const int m0 = blockIdx.x * 32;
  const int row = min(m0 + r32, a.M - 1);
  float hb[HK];
  ce_load_row<HK>(a.h + (int64_t)row * D + HK * hh, hb);
  const int tgt = (int)a.target[row];
  const float* brow = a.bias + (int64_t)(row % a.n) * a.ldb;
  float mx = -INFINITY, sm = 0.f, lt = 0.f;
  for (int ct = w; ct < a.K / 32; ct += 4) {
    const int code0 = ct * 32;
    const floatx16 acc = ce_tile_t<HK>(a.W + (int64_t)(code0 + r32) * D + HK * hh, hb);
    float v[16], tm = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int code = code0 + ce_crow(r, hh);
      v[r] = acc[r] + brow[code];
      if (code == tgt) lt = v[r];
      tm = fmaxf(tm, v[r]);
    }
    const float mn = fmaxf(mx, tm);
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) s += expf(v[r] - mn);
    sm = sm * expf(mx - mn) + s;
    mx = mn;
  }
  {  // the row's other half of the codes (lane l ^ 32)
    const float m2 = __shfl_xor(mx, 32, 64), s2 = __shfl_xor(sm, 32, 64), l2 = __shfl_xor(lt, 32, 64);
    const float mn = fmaxf(mx, m2);
    const float a0 = hh == 0 ? sm * expf(mx - mn) : s2 * expf(m2 - mn);
    const float a1 = hh == 0 ? s2 * expf(m2 - mn) : sm * expf(mx - mn);
    sm = (mn == -INFINITY) ? 0.f : a0 + a1;
    mx = mn;
    lt = hh == 0 ? lt + l2 : l2 + lt;
  }
  if (hh == 0) {
    red[0][w][r32] = mx;
    red[1][w][r32] = sm;
    red[2][w][r32] = lt;
  }
  __syncthreads();
  if (w != 0) return;
  float ls = 0.f, cnt = 0.f;
  if (lane < 32) {
    float m = red[0][0][lane];
#pragma unroll
    for (int k = 1; k < 4; ++k) m = fmaxf(m, red[0][k][lane]);
    float s = 0.f, t = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (red[0][k][lane] != -INFINITY) s += red[1][k][lane] * expf(red[0][k][lane] - m);
      t += red[2][k][lane];
    }
    const float lse = m + logf(s);
    if (m0 + lane < a.M) {
      a.lse[m0 + lane] = lse;
      if (!a.keep[m0 + lane]) {
        ls = lse - t;
        cnt = 1.f;
      }
    }
  }
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) {
    ls += __shfl_xor(ls, o, 64);
    cnt += __shfl_xor(cnt, o, 64);
  }
  if (lane == 0) {
    a.part[2 * blockIdx.x] = ls;
    a.part[2 * blockIdx.x + 1] = cnt;
  }
}

// dh = dl W for a 32-row tile; the waves split the codes and their partial dh are summed in
// wave order through LDS
template <int D>
__global__ __launch_bounds__(256) void ce_dh_kernel(CeArgs a) {
  constexpr int HK = D / 2, DT = D / 32;
  extern __shared__ float pd_smem[];
  float (*pd)[32 * D] = reinterpret_cast<float (*)[32 * D]>(pd_smem);  // [4][32 D]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r32 = lane & 31, hh = lane >> 5;
  const int m0 = blockIdx.x * 32;
  const int row = min(m0 + r32, a.M - 1);
  float hb[HK];
  ce_load_row<HK>(a.h + (int64_t)row * D + HK * hh, hb);
  const int tgt = (int)a.target[row];
  const float* brow = a.bias + (int64_t)(row % a.n) * a.ldb;
  const float lse = a.lse[row];
  const float sc = (m0 + r32 < a.M && !a.keep[row]) ? a.gout[0] / a.stats[1] : 0.f;
  floatx16 dacc[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) dacc[dt][r] = 0.f;
  for (int ct = w; ct < a.K / 32; ct += 4) {
    const int code0 = ct * 32;
    floatx16 acc = ce_tile_t<HK>(a.W + (int64_t)(code0 + r32) * D + HK * hh, hb);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int code = code0 + ce_crow(r, hh);
      const float p = expf(acc[r] + brow[code] - lse);
      acc[r] = (code == tgt ? p - 1.0f : p) * sc;
    }
    // dh[row][d] += sum_code dl[row][code] W[code][d]: A = dl (lane: row r32, k half hh),
    // step t <-> codes crow(t, 0) | crow(t, 1) -- the accumulator's own order
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const float* wr = a.W + (int64_t)(code0 + ce_crow(t, hh)) * D + r32;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
        dacc[dt] = __builtin_amdgcn_mfma_f32_32x32x2f32(acc[t], wr[32 * dt], dacc[dt], 0, 0, 0);
    }
  }
  // dacc[dt][r]: row crow(r, hh), d = 32 dt + r32
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) pd[w][ce_crow(r, hh) * D + 32 * dt + r32] = dacc[dt][r];
  __syncthreads();
  for (int e = tid; e < 32 * D; e += 256) {
    const int rr = e / D;
    if (m0 + rr >= a.M) continue;
    a.dh[(int64_t)m0 * D + e] = ((pd[0][e] + pd[1][e]) + pd[2][e]) + pd[3][e];
  }
}

// dW (codes x D) and d bias (position x code) of one 32-code tile over one row split
template <int D>
__global__ __launch_bounds__(256) void ce_dw_kernel(CeArgs a, int tb_n) {
  constexpr int HK = D / 2, DT = D / 32;
  extern __shared__ float ce_smem[];
  float* pw = ce_smem;                 // [4][32 * D]: the waves' dW partials
  float* tbl = ce_smem + 4 * 32 * D;   // [4][n][32]: the waves' bias-gradient tables
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r32 = lane & 31, hh = lane >> 5;
  const int ct = blockIdx.x, s = blockIdx.y, code0 = ct * 32, code = code0 + r32;
  const int tiles = (a.M + 31) / 32;
  const int per = (tiles + a.S - 1) / a.S;
  const int t0 = s * per, t1 = min(tiles, t0 + per);
  for (int i = tid; i < 4 * a.n * 32; i += 256) tbl[i] = 0.f;
  float wb[HK];
  ce_load_row<HK>(a.W + (int64_t)code * D + HK * hh, wb);
  const float gc = a.gout[0] / a.stats[1];
  floatx16 dacc[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) dacc[dt][r] = 0.f;
  float* tw = tbl + w * a.n * 32;
  __syncthreads();
  for (int rt = t0 + w; rt < t1; rt += 4) {
    const int m0 = rt * 32;
    float ha[HK];
    ce_load_row<HK>(a.h + (int64_t)min(m0 + r32, a.M - 1) * D + HK * hh, ha);
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    // logits tile: C[row crow(r, hh)][code r32]
#pragma unroll
    for (int t = 0; t < HK; ++t) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ha[t], wb[t], acc, 0, 0, 0);
    int pos[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + ce_crow(r, hh);
      const int mc = min(m, a.M - 1);
      pos[r] = mc % a.n;
      const float p = expf(acc[r] + a.bias[(int64_t)pos[r] * a.ldb + code] - a.lse[mc]);
      const float sc = (m < a.M && !a.keep[mc]) ? gc : 0.f;
      acc[r] = ((int)a.target[mc] == code ? p - 1.0f : p) * sc;
    }
    // d bias[pos][code] in program order: the two lane halves hold different rows, whose
    // positions coincide when n < 32 -- then they take turns
    if (a.n >= 32) {
#pragma unroll
      for (int r = 0; r < 16; ++r) tw[pos[r] * 32 + r32] += acc[r];
    } else {
      for (int half = 0; half < 2; ++half) {
        if (hh == half) {
#pragma unroll
          for (int r = 0; r < 16; ++r) tw[pos[r] * 32 + r32] += acc[r];
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this half's LDS updates landed
        __builtin_amdgcn_wave_barrier();
      }
    }
    // dW[code][d] += sum_rows dl[row][code] h[row][d]: A = dl^T (lane: code r32, k half hh),
    // step t <-> rows crow(t, 0) | crow(t, 1)
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const float* hr = a.h + (int64_t)min(m0 + ce_crow(t, hh), a.M - 1) * D + r32;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
        dacc[dt] = __builtin_amdgcn_mfma_f32_32x32x2f32(acc[t], hr[32 * dt], dacc[dt], 0, 0, 0);
    }
  }
  // dacc[dt][r]: code crow(r, hh), d = 32 dt + r32
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) pw[w * 32 * D + ce_crow(r, hh) * D + 32 * dt + r32] = dacc[dt][r];
  __syncthreads();
  float* sw = a.slab_w + ((int64_t)s * a.K + code0) * D;  // 32 consecutive code rows
  for (int e = tid; e < 32 * D; e += 256)
    sw[e] = ((pw[e] + pw[32 * D + e]) + pw[64 * D + e]) + pw[96 * D + e];
  for (int e = tid; e < a.n * 32; e += 256) {
    const int p = e >> 5, c = e & 31;
    const int stride = a.n * 32;
    a.slab_b[((int64_t)s * a.n + p) * a.ldb + code0 + c] =
        ((tbl[e] + tbl[stride + e]) + tbl[2 * stride + e]) + tbl[3 * stride + e];
  }
  if (ct == a.K / 32 - 1)  // columns K .. ldb-1 (the mask token's) carry no gradient
    for (int p = tid; p < a.n; p += 256)
      for (int c = a.K; c < a.ldb; ++c) a.slab_b[((int64_t)s * a.n + p) * a.ldb + c] = 0.f;
  (void)tb_n;
}

constexpr int CE_S = 16;  // row splits of the weight / bias gradient

static int64_t ce_blocks(int64_t M) { return (M + 31) / 32; }

}  // namespace tvq

using namespace tvq;

// floats: fwd block partials | dW slab + scratch | d bias slab + scratch
extern "C" int64_t tvq_tied_ce_workspace(int64_t M, int64_t D, int64_t K, int64_t n, int64_t ldb) {
  const int64_t fw = 2 * ce_blocks(M);
  const int64_t sw = CE_S * K * D + reduce_rows_scratch(CE_S, K * D);
  const int64_t sb = CE_S * n * ldb + reduce_rows_scratch(CE_S, n * ldb);
  return ((fw + 63) / 64) * 64 + ((sw + 63) / 64) * 64 + sb;
}

static bool ce_args_ok(const float* h, int64_t M, int64_t D, const float* W, int64_t K,
                       const float* bias, int64_t n, int64_t ldb) {
  return h && W && bias && M > 0 && (D == 32 || D == 64 || D == 128) && K > 0 && K % 32 == 0 &&
         n > 0 && ldb >= K && M < (1 << 30) && ((uintptr_t)h & 15) == 0 && ((uintptr_t)W & 15) == 0;
}

extern "C" int tvq_tied_ce_fwd(const float* h, int64_t M, int64_t D, const float* W, int64_t K,
                               const float* bias, int64_t n, int64_t ldb, const int64_t* target,
                               const bool* keep, float* lse, float* out, float* workspace,
                               tvq_stream_t stream) {
  TVQ_CHECK_ARG(ce_args_ok(h, M, D, W, K, bias, n, ldb) && target && keep && lse && out && workspace,
                "tvq_tied_ce_fwd: bad arguments");
  CeArgs a = {};
  a.h = h; a.W = W; a.bias = bias; a.target = target; a.keep = keep; a.lse = lse;
  a.part = workspace; a.M = (int)M; a.D = (int)D; a.K = (int)K; a.n = (int)n; a.ldb = (int)ldb;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)ce_blocks(M));
  TVQ_PLAN("tied_ce_fwd M%lld D%lld K%lld", (long long)M, (long long)D, (long long)K);
  if (D == 32) hipLaunchKernelGGL(ce_fwd_kernel<32>, grid, dim3(256), 0, st, a);
  else if (D == 64) hipLaunchKernelGGL(ce_fwd_kernel<64>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(ce_fwd_kernel<128>, grid, dim3(256), 0, st, a);
  masked_ce_final(workspace, (int)ce_blocks(M), out, st);
  return launch_status("tvq_tied_ce_fwd");
}

extern "C" int tvq_tied_ce_bwd(const float* h, int64_t M, int64_t D, const float* W, int64_t K,
                               const float* bias, int64_t n, int64_t ldb, const int64_t* target,
                               const bool* keep, const float* lse, const float* stats,
                               const float* gout, float* dh, float* dW, float* dbias,
                               int64_t accumulate, float* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(ce_args_ok(h, M, D, W, K, bias, n, ldb) && target && keep && lse && stats && gout &&
                    workspace, "tvq_tied_ce_bwd: bad arguments");
  CeArgs a = {};
  a.h = h; a.W = W; a.bias = bias; a.target = target; a.keep = keep; a.lse = const_cast<float*>(lse);
  a.stats = stats; a.gout = gout; a.dh = dh;
  a.M = (int)M; a.D = (int)D; a.K = (int)K; a.n = (int)n; a.ldb = (int)ldb; a.S = CE_S;
  const int64_t fw = ((2 * ce_blocks(M) + 63) / 64) * 64;
  const int64_t sw = ((CE_S * K * D + reduce_rows_scratch(CE_S, K * D) + 63) / 64) * 64;
  a.slab_w = workspace + fw;
  a.slab_b = workspace + fw + sw;
  hipStream_t st = (hipStream_t)stream;
  TVQ_PLAN("tied_ce_bwd M%lld D%lld K%lld", (long long)M, (long long)D, (long long)K);
  if (dh) {
    const dim3 grid((unsigned)ce_blocks(M));
    const size_t lds = (size_t)4 * 32 * D * 4;
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&ce_dh_kernel<128>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
      attr = true;
    }
    if (D == 32) hipLaunchKernelGGL(ce_dh_kernel<32>, grid, dim3(256), lds, st, a);
    else if (D == 64) hipLaunchKernelGGL(ce_dh_kernel<64>, grid, dim3(256), lds, st, a);
    else hipLaunchKernelGGL(ce_dh_kernel<128>, grid, dim3(256), lds, st, a);
  }
  if (dW || dbias) {
    const dim3 grid((unsigned)(K / 32), CE_S);
    const size_t lds = (size_t)(4 * 32 * D + 4 * n * 32) * 4;
    TVQ_CHECK_ARG(lds <= 160 * 1024, "tvq_tied_ce_bwd: too many positions");
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&ce_dw_kernel<32>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&ce_dw_kernel<64>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&ce_dw_kernel<128>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr = true;
    }
    if (D == 32) hipLaunchKernelGGL(ce_dw_kernel<32>, grid, dim3(256), lds, st, a, (int)n);
    else if (D == 64) hipLaunchKernelGGL(ce_dw_kernel<64>, grid, dim3(256), lds, st, a, (int)n);
    else hipLaunchKernelGGL(ce_dw_kernel<128>, grid, dim3(256), lds, st, a, (int)n);
    if (dW) conv_wgrad_finish(a.slab_w, CE_S, K, D, dW, nullptr, (int)accumulate, st);
    if (dbias) conv_wgrad_finish(a.slab_b, CE_S, n, ldb, dbias, nullptr, (int)accumulate, st);
  }
  return launch_status("tvq_tied_ce_bwd");
}

// Dense fp32 GEMM on gfx950 MFMA (v_mfma_f32_16x16x4_f32) for the Linear layers
// (decoder Linear(T,T) vq_vae.py:255,263; transformer projections/FFN; pred_head).
//
//   C[m, n] = epi( sum_k A(m,k) * B(k,n) )
//   A(m,k) = A[m*sam + k*sak],  B(k,n) = B[k*sbk + n*sbn]   (any strides: X W^T,
//   dY W, dY^T X are all the same kernel)
//   epi: + bias[n], GELU (erf), + R[m*ldr + n], or accumulate into C.
// Split-K over gridDim.z writes fp32 slabs reduced in split order (deterministic), by
// the last-arriving split block of each tile (or a separate reduce launch).
// tvq_gemm first offers the call to the skinny kernels (tvq_gemm_skinny.hip: A rows
// k-contiguous, K <= 512); this generic kernel takes the rest (the weight gradients).
#include <math.h>
#include <stdlib.h>

#include "tvq_common.h"
#include "tvq_gemm.h"

namespace tvq {

__device__ __forceinline__ float apply_epi(const GemmArgs& g, int m, int n, float v) {
  v *= g.alpha;
  if (g.bias) v += g.bias[n];
  if (g.pre) g.pre[(int64_t)m * g.ldc + n] = v;
  if (g.act == 1) v = gelu_erf(v);
  if (g.gate) v *= *g.gate;
  if (g.R) v += g.R[(int64_t)(g.rmod > 0 ? m % g.rmod : m) * g.ldr + n];
  if (g.accumulate) v += g.C[(int64_t)m * g.ldc + n];
  return v;
}

template <int TM, int TN, int WM, int WN>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs g) {
  constexpr int BK = 16;
  constexpr int FM = TM / WM / 16, FN = TN / WN / 16;
  constexpr int SA = ((TM + 31) / 32) * 32 + 16;
  constexpr int SB = ((TN + 31) / 32) * 32 + 16;
  constexpr int A_PER = TM * BK / 256, B_PER = TN * BK / 256;
  static_assert(A_PER >= 1 && B_PER >= 1, "tile too small");
  __shared__ float As[BK * SA];
  __shared__ float Bs[BK * SB];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid % WM, wn = wid / WM;
  const int m0 = blockIdx.x * TM, n0 = blockIdx.y * TN;
  const int kb = blockIdx.z * g.kper;
  const int ke = min(g.K, kb + g.kper);
  const bool a_kfast = (g.sak == 1);
  const bool b_kfast = (g.sbn != 1);

  float ra[A_PER], rb[B_PER];
  int a_m[A_PER], a_k[A_PER], b_k[B_PER], b_n[B_PER];
#pragma unroll
  for (int j = 0; j < A_PER; ++j) {
    const int e = tid + j * 256;
    if (a_kfast) { a_k[j] = e % BK; a_m[j] = e / BK; } else { a_m[j] = e % TM; a_k[j] = e / TM; }
  }
#pragma unroll
  for (int j = 0; j < B_PER; ++j) {
    const int e = tid + j * 256;
    if (b_kfast) { b_k[j] = e % BK; b_n[j] = e / BK; } else { b_n[j] = e % TN; b_k[j] = e / TN; }
  }
  auto load = [&](int k0) {
#pragma unroll
    for (int j = 0; j < A_PER; ++j) {
      const int m = m0 + a_m[j], k = k0 + a_k[j];
      ra[j] = (m < g.M && k < ke) ? g.A[(int64_t)m * g.sam + (int64_t)k * g.sak] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < B_PER; ++j) {
      const int n = n0 + b_n[j], k = k0 + b_k[j];
      rb[j] = (n < g.N && k < ke) ? g.B[(int64_t)k * g.sbk + (int64_t)n * g.sbn] : 0.f;
    }
  };
  // Panels are stored [k][m] / [k][n] with m (n) XOR-swizzled by sw(k) = k & 14: the row
  // pitches are 16 mod 32 banks (ds_write banks are (a/4) mod 32), so a half-wave's stores
  // of 16 k rows x 2 columns land on 32 distinct banks, and each fragment read (rows kk,
  // kk+1 per half-wave, 16 consecutive columns each) is conflict-free too.  Layout only:
  // the MFMA k order, and so every result, is unchanged.
  auto store = [&]() {
#pragma unroll
    for (int j = 0; j < A_PER; ++j) As[a_k[j] * SA + (a_m[j] ^ ((a_k[j] & 14)))] = ra[j];
#pragma unroll
    for (int j = 0; j < B_PER; ++j) Bs[b_k[j] * SB + (b_n[j] ^ ((b_k[j] & 14)))] = rb[j];
  };
  floatx4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int r16 = lane & 15, g4 = lane >> 4;
  if (kb < ke) {
    load(kb);
    for (int k0 = kb; k0 < ke; k0 += BK) {
      __syncthreads();
      store();
      __syncthreads();
      if (k0 + BK < ke) load(k0 + BK);
#pragma unroll
      for (int kk = 0; kk < BK; kk += 4) {
        float af[FM], bf[FN];
        const int swz = r16 ^ ((kk & 12) | (g4 & 2));  // sw(kk + g4) (g4 < 4, kk % 4 == 0)
#pragma unroll
        for (int i = 0; i < FM; ++i) af[i] = As[(kk + g4) * SA + (wm * FM + i) * 16 + swz];
#pragma unroll
        for (int j = 0; j < FN; ++j) bf[j] = Bs[(kk + g4) * SB + (wn * FN + j) * 16 + swz];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = mfma16x16x4(af[i], bf[j], acc[i][j]);
      }
    }
  }
  // C layout: acc[i][j][r] -> row m0 + (wm*FM+i)*16 + 4*g4 + r, col n0 + (wn*FN+j)*16 + r16.
  // Every epilogue load is unconditional (clamped indices) so they issue together.
  int ncol[FN], ncl[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    ncol[j] = n0 + (wn * FN + j) * 16 + r16;
    ncl[j] = min(ncol[j], g.N - 1);
  }
  if (g.slab) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + (wm * FM + i) * 16 + 4 * g4 + r;
#pragma unroll
        for (int j = 0; j < FN; ++j)
          if (m < g.M && ncol[j] < g.N) {
            float* d = g.slab + ((int64_t)blockIdx.z * g.M + m) * g.N + ncol[j];
            if (g.cnt) st_wt(d, acc[i][j][r]);  // read back by the last split block
            else *d = acc[i][j][r];
          }
      }
    // the last split block of this tile sums the slabs in split order + epilogue
    // (element for element what gemm_splitk_reduce_kernel does)
    if (g.cnt && last_block(g.cnt + blockIdx.y * gridDim.x + blockIdx.x, (int)gridDim.z)) {
      const int64_t tot = (int64_t)g.M * g.N;
      for (int e = tid; e < TM * TN; e += 256) {
        const int m = m0 + e / TN, n = n0 + e % TN;
        if (m >= g.M || n >= g.N) continue;
        const int64_t i = (int64_t)m * g.N + n;
        float s = 0.f;
#pragma unroll 8
        for (int z = 0; z < (int)gridDim.z; ++z) s += ld_wt(g.slab + (int64_t)z * tot + i);
        g.C[(int64_t)m * g.ldc + n] = apply_epi(g, m, n, s);
      }
    }
    return;
  }
  float bv[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) bv[j] = g.bias ? g.bias[ncl[j]] : 0.f;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    int mrow[4], mcl[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      mrow[r] = m0 + (wm * FM + i) * 16 + 4 * g4 + r;
      mcl[r] = min(mrow[r], g.M - 1);
    }
    float v[4][FN];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < FN; ++j) v[r][j] = acc[i][j][r] * g.alpha + bv[j];
    if (g.pre) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          if (mrow[r] < g.M && ncol[j] < g.N) g.pre[(int64_t)mrow[r] * g.ldc + ncol[j]] = v[r][j];
    }
    if (g.act == 1) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < FN; ++j) v[r][j] = gelu_erf(v[r][j]);
    }
    if (g.gate) {
      const float gt = *g.gate;
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < FN; ++j) v[r][j] *= gt;
    }
    if (g.R) {
      float rv[4][FN];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t rr = (int64_t)(g.rmod > 0 ? mcl[r] % g.rmod : mcl[r]) * g.ldr;
#pragma unroll
        for (int j = 0; j < FN; ++j) rv[r][j] = g.R[rr + ncl[j]];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < FN; ++j) v[r][j] += rv[r][j];
    }
    if (g.accumulate) {
      float cv[4][FN];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < FN; ++j) cv[r][j] = g.C[(int64_t)mcl[r] * g.ldc + ncl[j]];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < FN; ++j) v[r][j] += cv[r][j];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        if (mrow[r] < g.M && ncol[j] < g.N) g.C[(int64_t)mrow[r] * g.ldc + ncol[j]] = v[r][j];
  }
}

__global__ void gemm_splitk_reduce_kernel(GemmArgs g, int splits) {
  const int64_t tot = (int64_t)g.M * g.N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < tot;
       i += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
#pragma unroll 8
    for (int z = 0; z < splits; ++z) s += g.slab[(int64_t)z * tot + i];
    const int m = (int)(i / g.N), n = (int)(i - (int64_t)m * g.N);
    g.C[(int64_t)m * g.ldc + n] = apply_epi(g, m, n, s);
  }
}

static int gemm_splits(int M, int N, int K, int tiles) {
  if (K < 1024 || tiles >= 128) return 1;
  int s = (512 + tiles - 1) / tiles;
  const int maxs = K / 256;
  if (s > maxs) s = maxs;
  if (s > 64) s = 64;
  return s < 1 ? 1 : s;
}

}  // namespace tvq

using namespace tvq;

// Largest tile that still gives >= TVQ_GEMM_MIN_BLOCKS (default 256) blocks: the GEMMs
// here have K <= 512, so filling the 256 CUs matters more than tile reuse.  (Measured:
// 1024 / 2048 minimum blocks, i.e. smaller tiles, change neither the sampler's
// M = 25600, N = 128, K = 128 projections nor the train step.)  Deep-K GEMMs that stay
// small get split-K instead.  The tile does not change the k order: results are bitwise
// the same for every tile.
static int gemm_min_blocks() { return 256; }
static void choose_tile(int64_t M, int64_t N, int* TM, int* TN) {
  static const int cand[4][2] = {{128, 64}, {64, 64}, {64, 32}, {32, 32}};
  const int64_t want = gemm_min_blocks();
  for (int i = 0; i < 4; ++i) {
    *TM = cand[i][0];
    *TN = cand[i][1];
    if (((M + *TM - 1) / *TM) * ((N + *TN - 1) / *TN) >= want) return;
  }
}

extern "C" int64_t tvq_gemm_workspace(int64_t M, int64_t N, int64_t K) {
  int TM, TN;
  choose_tile(M, N, &TM, &TN);
  const int tiles = (int)(((M + TM - 1) / TM) * ((N + TN - 1) / TN));
  int s = gemm_splits((int)M, (int)N, (int)K, tiles);
  const int sd = gemm_direct_splits(M, N, K);  // the direct weight-gradient form
  if (sd > s) s = sd;
  return s > 1 ? (int64_t)s * M * N : 0;
}

extern "C" int tvq_gemm(const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk,
                        int64_t sbn, float* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                        float alpha, const float* bias, const float* R, int64_t ldr, int64_t rmod,
                        int64_t act, float* pre, int64_t accumulate, const float* gate,
                        float* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(A && B && C && M > 0 && N > 0 && K > 0, "tvq_gemm: bad arguments");
  GemmArgs g;
  g.A = A; g.B = B; g.C = C;
  g.M = (int)M; g.N = (int)N; g.K = (int)K;
  g.sam = sam; g.sak = sak; g.sbk = sbk; g.sbn = sbn; g.ldc = ldc;
  g.bias = bias; g.R = R; g.ldr = ldr; g.rmod = rmod; g.pre = pre;
  g.act = (int)act; g.accumulate = (int)accumulate; g.gate = gate;
  g.alpha = alpha;
  g.kper = (int)K;
  g.cnt = nullptr;
  g.slab = nullptr;
  if (gemm_direct(g, workspace, (hipStream_t)stream)) return launch_status("tvq_gemm(direct)");
  if (gemm_skinny(g, (hipStream_t)stream)) return launch_status("tvq_gemm(skinny)");
  int TM, TN;
  choose_tile(M, N, &TM, &TN);
  const int tiles = (int)(((M + TM - 1) / TM) * ((N + TN - 1) / TN));
  int splits = gemm_splits((int)M, (int)N, (int)K, tiles);
  if (splits > 1 && !workspace) splits = 1;
  int kper = (int)((K + splits - 1) / splits);
  kper = (kper + 15) / 16 * 16;
  splits = (int)((K + kper - 1) / kper);
  g.kper = kper;
  g.slab = splits > 1 ? workspace : nullptr;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)((M + TM - 1) / TM), (unsigned)((N + TN - 1) / TN), (unsigned)splits);
  g.cnt = splits > 1 ? counters((int64_t)grid.x * grid.y, FIN_GEMM) : nullptr;
  if (TM == 128)
    hipLaunchKernelGGL((gemm_kernel<128, 64, 2, 2>), grid, dim3(256), 0, st, g);
  else if (TN == 64)
    hipLaunchKernelGGL((gemm_kernel<64, 64, 2, 2>), grid, dim3(256), 0, st, g);
  else if (TM == 64)
    hipLaunchKernelGGL((gemm_kernel<64, 32, 2, 2>), grid, dim3(256), 0, st, g);
  else
    hipLaunchKernelGGL((gemm_kernel<32, 32, 2, 2>), grid, dim3(256), 0, st, g);
  if (splits > 1 && !g.cnt) {
    const int64_t tot = M * N;
    const int blocks = (int)((tot + 255) / 256 < 4096 ? (tot + 255) / 256 : 4096);
    hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, g, splits);
  }
  return launch_status("tvq_gemm");
}

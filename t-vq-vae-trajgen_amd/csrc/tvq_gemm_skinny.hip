// Skinny GEMMs of the MaskGIT transformer and the decoder Linear (tvq_gemm dispatches
// here first):
//   C[M][N] = epi(alpha * A[M][K] B[K][N]),  A rows k-contiguous, K <= 512, any M, N,
//   B either k-contiguous (B(k,n) = W[n][k]: Linear forward X W^T) or n-contiguous
//   (B(k,n) = W[k][n]: the input gradient dY W).
// M is large (batch * tokens: 6,400 - 99,328 rows) while N, K <= 512.  On the
// v_mfma_f32_32x32x2_f32 A operand a lane holds row (l & 31), so k is permuted to give
// every lane a contiguous k range it reads with 16-B loads straight from HBM: within a K
// chunk of KC, lane half h takes k = KC*c + (KC/2)*h + t at MFMA step t (B uses the same
// order).  Each wave owns one 32 x 32 output tile on one accumulator.
//   * gemm_rb2_kernel (K <= 128, N <= 256): one tile per wave, the block's 32-column B
//     slice staged once through LDS into registers.
//   * gemm_skinny_kernel (K <= 512): a block stages its [K x 32*WN] B slice in the exact
//     B-fragment order (every fragment read is one contiguous 1-KB ds_read_b128 per
//     wave) and walks M persistently, the next step's A rows loading (ping-pong
//     registers) while the current one multiplies.
// Measured at the transformer's shapes (tools/gemm_bench.py, graph-replayed; ROCm 7.2):
// these beat the generic staged kernel by 0-40 % (largest on the HF K = 256 / 32 forms);
// what is left is load / store latency that one 32 x 32 x K tile per wave cannot hide
// (tools/mfma_probe.hip: the same tile pattern with B free of cost reaches 66 TFLOP/s).
#include <math.h>
#include <stdlib.h>

#include "tvq_gemm.h"

namespace tvq {

__device__ __forceinline__ int crow32(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

template <int KC, int WN, bool B_KCONTIG, bool HAS_R, bool HAS_C>
__global__ __launch_bounds__(256) void gemm_skinny_kernel(GemmArgs g) {
  constexpr int WM = 4 / WN;
  constexpr int HK = KC / 2;  // contiguous k per lane per chunk
  constexpr int T4 = HK / 4;
  constexpr int BN = 32 * WN;
  constexpr int TM = 32 * WM;
  // [chunk][wn][t4][lane][4]: B fragments, ds_read_b128 order; declared float4 so the
  // staging stores are ds_write_b128 (as float, hipcc split them into 4-way-conflicted
  // ds_write2_b32 pairs at a 16-B lane stride)
  extern __shared__ float4 Wsv[];
  float* Ws = reinterpret_cast<float*>(Wsv);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int nch = (g.K + KC - 1) / KC;
  const int n0 = blockIdx.y * BN;
  {  // stage B[k][n0 .. n0+BN) (zero outside K / N) slot by slot: contiguous LDS stores
     // (a scattered, bank-conflicted image write measured slower than these row reads)
    const int slots = nch * WN * T4 * 64;
    for (int e = tid; e < slots; e += 256) {
      const int l = e & 63, rest = e >> 6;
      const int t4 = rest % T4, jw = (rest / T4) % WN, c = rest / (T4 * WN);
      const int n = n0 + 32 * jw + (l & 31);
      const int k = c * KC + (l >> 5) * HK + 4 * t4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (n < g.N && k < g.K) {
        if (B_KCONTIG) {
          v = *(const float4*)(g.B + (int64_t)n * g.sbn + k);
        } else {
          const float* p = g.B + (int64_t)k * g.sbk + n;
          v.x = p[0];
          v.y = p[g.sbk];
          v.z = p[2 * g.sbk];
          v.w = p[3 * g.sbk];
        }
      }
      Wsv[e] = v;
    }
  }
  __syncthreads();
  const int ncol = n0 + 32 * wn + r32;
  const float bv = (g.bias && ncol < g.N) ? g.bias[ncol] : 0.f;
  const int mtiles = (g.M + TM - 1) / TM;
  const int mine = (int)blockIdx.x < mtiles ? (mtiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int total = mine * nch;  // (tile, chunk) steps of this block, in order
  // branch-free loads (a select right after a load would make the wave wait for it):
  // rows past M are clamped (never stored); k past K re-reads the row's first float4,
  // which multiplies the zero-filled k >= K entries of the staged B (K % 4 == 0)
  auto load_a = [&](float (&dst)[HK], int s) {
    const int q = s / nch, c = s - q * nch;
    int row = ((int)blockIdx.x + q * (int)gridDim.x) * TM + wm * 32 + r32;
    row = row < g.M ? row : g.M - 1;
    const int k0 = c * KC + h * HK;
    const float* src = g.A + (int64_t)row * g.sam;
#pragma unroll
    for (int t = 0; t < HK; t += 4) {
      const float4 v = *(const float4*)(src + (k0 + t < g.K ? k0 + t : 0));
      dst[t] = v.x; dst[t + 1] = v.y; dst[t + 2] = v.z; dst[t + 3] = v.w;
    }
  };
  floatx16 acc;
  float rv[16], cv[16];  // the tile's residual / accumulated C, requested with its last chunk
  const int ncl = ncol < g.N ? ncol : g.N - 1;
  auto compute = [&](const float (&a)[HK], int s) {
    const int q = s / nch, c = s - q * nch;
    if (c == 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    }
    if ((HAS_R || HAS_C) && c == nch - 1) {  // loads overlap the chunk's MFMAs
      const int mb = ((int)blockIdx.x + q * (int)gridDim.x) * TM + wm * 32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int m = mb + crow32(r, h);
        m = m < g.M ? m : g.M - 1;
        if (HAS_R) rv[r] = g.R[(int64_t)(g.rmod > 0 ? m % g.rmod : m) * g.ldr + ncl];
        if (HAS_C) cv[r] = g.C[(int64_t)m * g.ldc + ncl];
      }
    }
    const float* wf = Ws + ((c * WN + wn) * T4) * 256 + 4 * lane;
#pragma unroll
    for (int t4 = 0; t4 < T4; ++t4) {
      const float4 b4 = *(const float4*)(wf + t4 * 256);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * t4], b4.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * t4 + 1], b4.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * t4 + 2], b4.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * t4 + 3], b4.w, acc, 0, 0, 0);
    }
    if (c != nch - 1) return;
    // epilogue: register r -> row crow32(r, h) of the wave's 32-row tile, column ncol;
    // values combined in every lane, stores predicated (see gemm_rb2_kernel)
    const int mb = ((int)blockIdx.x + q * (int)gridDim.x) * TM + wm * 32;
    const bool colok = ncol < g.N;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = mb + crow32(r, h);
      const bool ok = colok && m < g.M;
      float v = acc[r] * g.alpha + bv;
      const int64_t ci = (int64_t)m * g.ldc + ncol;
      if (g.pre && ok) g.pre[ci] = v;
      if (g.act == 1) v = gelu_erf(v);
      if (g.gate) v *= *g.gate;
      if (HAS_R) v += rv[r];
      if (HAS_C) v += cv[r];
      if (ok) g.C[ci] = v;
    }
  };
  float a0[HK], a1[HK];
  if (total > 0) load_a(a0, 0);
  for (int s = 0; s < total; s += 2) {
    if (s + 1 < total) load_a(a1, s + 1);
    compute(a0, s);
    if (s + 1 >= total) break;
    if (s + 2 < total) load_a(a0, s + 2);
    compute(a1, s + 1);
  }
}

// K <= 128, one 32 x 32 tile per wave (no persistence: the hardware interleaves the
// resident waves' load / MFMA / store phases).  The block's 4 waves share one 32-column
// slice of B: it is staged with coalesced 16-B loads into a padded [32][KP + 4] LDS tile
// and copied into each wave's registers; each wave then loads its 32 A rows, runs K/2
// MFMAs and stores (measured the fastest of the forms in this file at the transformer
// shapes; tools/mfma_probe.hip).
template <int KH, bool B_KCONTIG, bool HAS_R, bool HAS_C>
__global__ __launch_bounds__(256) void gemm_rb2_kernel(GemmArgs g, int nblk, int xcd) {
  constexpr int KP = 2 * KH;
  constexpr int P = KP + 4;
  __shared__ float Bs[32 * P];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  int mblk = (int)blockIdx.x, nb = (int)blockIdx.y;
  if (xcd) {  // 1-D grid: the column blocks of one row block share an XCD (tvq_gemm.h)
    xcd_tile((int)blockIdx.x, nblk, &mblk, &nb);
    if (mblk * 128 >= g.M) return;
  }
  const int n0 = nb * 32;
  if (B_KCONTIG) {
    for (int e = tid; e < 32 * KP / 4; e += 256) {
      const int n = e / (KP / 4), k = (e - n * (KP / 4)) * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (n0 + n < g.N && k < g.K) v = *(const float4*)(g.B + (int64_t)(n0 + n) * g.sbn + k);
      *(float4*)(Bs + n * P + k) = v;
    }
  } else {
    for (int e = tid; e < KP * 32; e += 256) {
      const int k = e >> 5, n = e & 31;
      Bs[n * P + k] = (k < g.K && n0 + n < g.N) ? g.B[(int64_t)k * g.sbk + n0 + n] : 0.f;
    }
  }
  __syncthreads();
  float b[KH];
#pragma unroll
  for (int t = 0; t < KH; t += 4) {
    const float4 v = *(const float4*)(Bs + r32 * P + h * KH + t);
    b[t] = v.x; b[t + 1] = v.y; b[t + 2] = v.z; b[t + 3] = v.w;
  }
  const int mt = mblk * 4 + wid;
  if (mt * 32 >= g.M) return;
  int row = mt * 32 + r32;
  row = row < g.M ? row : g.M - 1;
  const float* src = g.A + (int64_t)row * g.sam;
  float a[KH];
#pragma unroll
  for (int t = 0; t < KH; t += 4) {  // k >= K re-reads k = 0 and meets b = 0
    const int k = h * KH + t;
    const float4 v = *(const float4*)(src + (k < g.K ? k : 0));
    a[t] = v.x; a[t + 1] = v.y; a[t + 2] = v.z; a[t + 3] = v.w;
  }
  // the epilogue's operands (bias, gate, residual / accumulated C) requested before the
  // MFMA chain, so their round trip overlaps it instead of following it: every lane loads
  // and combines unconditionally (rows / columns clamped), only the stores are predicated
  // -- a load used under a branch would be sunk past the MFMAs
  const int ncol = n0 + r32;
  const int ncl = ncol < g.N ? ncol : g.N - 1;
  const float bv = g.bias ? g.bias[ncl] : 0.f;
  const float gv = g.gate ? *g.gate : 1.f;
  float rv[16], cv[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    int m = mt * 32 + crow32(r, h);
    m = m < g.M ? m : g.M - 1;
    if (HAS_R) rv[r] = g.R[(int64_t)(g.rmod > 0 ? m % g.rmod : m) * g.ldr + ncl];
    if (HAS_C) cv[r] = g.C[(int64_t)m * g.ldc + ncl];
  }
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
  for (int t = 0; t < KH; ++t) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t], b[t], acc, 0, 0, 0);
  const bool colok = ncol < g.N;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = mt * 32 + crow32(r, h);
    const bool ok = colok && m < g.M;
    float v = acc[r] * g.alpha + bv;
    const int64_t ci = (int64_t)m * g.ldc + ncol;
    if (g.pre && ok) g.pre[ci] = v;
    if (g.act == 1) v = gelu_erf(v);
    if (g.gate) v *= gv;
    if (HAS_R) v += rv[r];
    if (HAS_C) v += cv[r];
    if (ok) g.C[ci] = v;
  }
}

template <int KH, bool BKC, bool HR, bool HC>
static void launch_rb2_e(const GemmArgs& g, int xcd, hipStream_t st) {
  const int mb = (g.M + 127) / 128, nb = (g.N + 31) / 32;
  if (xcd)
    hipLaunchKernelGGL((gemm_rb2_kernel<KH, BKC, HR, HC>), dim3(xcd_grid(mb, nb)), dim3(256), 0, st,
                       g, nb, 1);
  else
    hipLaunchKernelGGL((gemm_rb2_kernel<KH, BKC, HR, HC>), dim3(mb, nb), dim3(256), 0, st, g, nb, 0);
}

template <int KH, bool BKC>
static void launch_rb2(const GemmArgs& g, hipStream_t st) {
  constexpr int xcd = 1;  // XCD-aware tile map
  if (g.R && g.accumulate) launch_rb2_e<KH, BKC, true, true>(g, xcd, st);
  else if (g.R) launch_rb2_e<KH, BKC, true, false>(g, xcd, st);
  else if (g.accumulate) launch_rb2_e<KH, BKC, false, true>(g, xcd, st);
  else launch_rb2_e<KH, BKC, false, false>(g, xcd, st);
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

template <int KC, int WN, bool BKC, bool HR, bool HC>
static void launch_skinny_e(const GemmArgs& g, hipStream_t st) {
  const int nch = (g.K + KC - 1) / KC;
  const size_t lds = (size_t)nch * KC * 32 * WN * sizeof(float);
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)gemm_skinny_kernel<KC, WN, BKC, HR, HC>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
    return true;
  }();
  (void)attr;
  const int nb = (g.N + 32 * WN - 1) / (32 * WN);
  const int mtiles = (g.M + 32 * (4 / WN) - 1) / (32 * (4 / WN));
  int gx = 512 / nb;  // two resident blocks per CU, persistent over M
  if (gx < 1) gx = 1;
  if (gx > mtiles) gx = mtiles;
  hipLaunchKernelGGL((gemm_skinny_kernel<KC, WN, BKC, HR, HC>), dim3(gx, nb), dim3(256), lds, st, g);
}

template <int KC, int WN, bool BKC>
static void launch_skinny(const GemmArgs& g, hipStream_t st) {
  if (g.R && g.accumulate) launch_skinny_e<KC, WN, BKC, true, true>(g, st);
  else if (g.R) launch_skinny_e<KC, WN, BKC, true, false>(g, st);
  else if (g.accumulate) launch_skinny_e<KC, WN, BKC, false, true>(g, st);
  else launch_skinny_e<KC, WN, BKC, false, false>(g, st);
}

template <int KC, bool BKC>
static void launch_wn(const GemmArgs& g, int wn, hipStream_t st) {
  if (wn == 4) launch_skinny<KC, 4, BKC>(g, st);
  else if (wn == 2) launch_skinny<KC, 2, BKC>(g, st);
  else launch_skinny<KC, 1, BKC>(g, st);
}

bool gemm_skinny(const GemmArgs& g, hipStream_t st) {
  if (g.sak != 1 || g.K > 512 || (g.K & 3) || (g.sam & 3) || !aligned16(g.A)) return false;
  const bool bkc = g.sbk == 1;
  if (bkc && ((g.sbn & 3) || !aligned16(g.B))) return false;
  if (!bkc && g.sbn != 1) return false;
  if (g.K <= 128 && g.N <= 256) {
    if (g.K <= 32) {
      if (bkc) launch_rb2<16, true>(g, st); else launch_rb2<16, false>(g, st);
    } else if (g.K <= 64) {
      if (bkc) launch_rb2<32, true>(g, st); else launch_rb2<32, false>(g, st);
    } else {
      if (bkc) launch_rb2<64, true>(g, st); else launch_rb2<64, false>(g, st);
    }
    return true;
  }
  const int kc = g.K <= 32 ? 32 : 64;
  const int kp = (g.K + kc - 1) / kc * kc;
  int wn = 4;  // B slice [kp][32*wn] within 64 KB of LDS, and no wider than N needs
  while (wn > 1 && (size_t)kp * 32 * wn * 4 > 64 * 1024) wn >>= 1;
  while (wn > 1 && 32 * (wn / 2) >= g.N) wn >>= 1;
  if (kc == 32) {
    if (bkc) launch_wn<32, true>(g, wn, st);
    else launch_wn<32, false>(g, wn, st);
  } else {
    if (bkc) launch_wn<64, true>(g, wn, st);
    else launch_wn<64, false>(g, wn, st);
  }
  return true;
}

}  // namespace tvq

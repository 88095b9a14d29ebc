// Direct-operand MFMA GEMMs (operands go global -> registers, no LDS staging, no barrier in
// the main loop).  tvq_gemm offers every call here first:
//
//   gemm_dk_kernel  the input gradient dY W: A rows k-contiguous (sak == 1), B(k,n) =
//                   W[k][n] n-contiguous, K <= 1024 (transformer / decoder shapes: M =
//                   tokens 6,144 - 99,328, N, K <= 512).  The Linear forward X W^T stays
//                   on gemm_rb2 / gemm_skinny (measured faster there).
//   gemm_kt_kernel  the weight gradient dW = dY^T X: A(m,k) = A[k][m], B(k,n) = B[k][n]
//                   (sam == 1, sbn == 1), K = tokens.
//
// Why direct: at these shapes a 32 x 32 x K tile per wave is a long dependent MFMA chain
// (K = 128: 64 x 64 cycles) fed by one load phase, and M = 6,400 gives fewer waves than
// SIMDs.  Here the 4 waves of a block split K between them (a wave runs 1/4 of the chain)
// and add their partial tiles through LDS in a fixed order, so a block is 4x as many
// short, independent chains; each wave issues all loads of a chunk before using any.
//
// gemm_dk_kernel uses v_mfma_f32_16x16x4_f32 (lane l supplies A[l & 15][k = l >> 4],
// B[k = l >> 4][l & 15]; acc r of lane l is C[4 (l >> 4) + r][l & 15]).  k is permuted
// inside each 16-k group j: lane quad q holds k = 16 j + 4 q + i at MFMA step 4 j + i, so
// one 16-byte load gives a lane its 4 steps and a wave's load covers 16 rows x 64
// contiguous bytes (the 32x32x2 layout touches 64 rows per load).  The same permutation
// is applied to B, so every product is formed exactly once.
//
// gemm_kt_kernel uses v_mfma_f32_32x32x2_f32 (lane l supplies A[l & 31][k = l >> 5]):
// with m (n) contiguous in memory each operand load is two 128-byte token rows.  K is
// split over the block's 4 waves and over `splits` blocks per 32 x 32 tile; the split
// tiles go to slabs that one all-CU gemm_direct_reduce launch sums in split order (an
// in-launch last-block finish with write-through slabs measured 1.2-1.7x slower here).
//
// Determinism: every sum has a fixed order (per wave sequential in k, waves 0..3 in LDS,
// slabs 0..S-1), independent of scheduling; results are run-to-run bitwise identical.
#include <math.h>
#include <stdlib.h>

#include "tvq_gemm.h"

namespace tvq {

__device__ __forceinline__ float epi_value(const GemmArgs& g, int m, int n, float v) {
  v *= g.alpha;
  if (g.bias) v += g.bias[n];
  const int64_t ci = (int64_t)m * g.ldc + n;
  if (g.pre) g.pre[ci] = v;
  if (g.act == 1) v = gelu_erf(v);
  if (g.gate) v *= *g.gate;
  if (g.R) v += g.R[(int64_t)(g.rmod > 0 ? m % g.rmod : m) * g.ldr + n];
  if (g.accumulate) v += g.C[ci];
  return v;
}

// ---------------------------------------------------------------------------------------
// gemm_dk_kernel<TNW, KS, BKC>: block = 4 waves = (4 / KS) row tiles x KS k-slices.
// Wave tile 32 rows x 32*TNW columns = 2 x 2*TNW fragments of 16 x 16.  kw = k span of
// one slice (multiple of 16).  1-D grid over (row block, column block) by xcd_tile.
template <int TNW, int KS, bool BKC, int DK_G>
__global__ __launch_bounds__(256) void gemm_dk_kernel(GemmArgs g, int kw, int nblk) {
  constexpr int RT = 4 / KS;
  constexpr int NF = 2 * TNW;  // column fragments
  constexpr int RED = KS > 1 ? (KS - 1) * RT * 2 * NF * 4 * 64 : 1;
  __shared__ float red[RED];
  int mb, nb;
  xcd_tile((int)blockIdx.x, nblk, &mb, &nb);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int rt = wid % RT, ks = wid / RT;
  const int r16 = lane & 15, q = lane >> 4;
  const int m0 = (mb * RT + rt) * 32;
  if (mb * RT * 32 >= g.M) return;  // padding block of the XCD map (whole block)
  const int n0 = nb * 32 * TNW;
  const int kb = ks * kw;
  const int ke = min(g.K, kb + kw);
  const int ng = kb < ke ? (ke - kb + 15) / 16 : 0;

  // clamped row / column pointers (rows past M and columns past N are never stored)
  const float* arow[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) arow[i] = g.A + (int64_t)min(m0 + 16 * i + r16, g.M - 1) * g.sam;
  const float* bcol[NF];
#pragma unroll
  for (int c = 0; c < NF; ++c) {
    const int n = min(n0 + 16 * c + r16, g.N - 1);
    bcol[c] = g.B + (BKC ? (int64_t)n * g.sbn : (int64_t)n);
  }
  // group j: this lane's k = kb + 16 j + 4 q (+0..3); past ke -> address k = 0 (valid,
  // K % 4 == 0) and the A values are zeroed by a select where they are used.  Groups go
  // in chunks of DK_G whose loads are all issued before the first is used (the k span of
  // a slice is 1-4 groups at the transformer's shapes: one memory round trip; DK_G =
  // min(4, groups per slice), so no chunk loads a group it does not use).
  float4 a[DK_G][2], b[DK_G][NF];
  floatx4 acc[2][NF];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int c = 0; c < NF; ++c) acc[i][c] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int j0 = 0; j0 < ng; j0 += DK_G) {
#pragma unroll
    for (int jj = 0; jj < DK_G; ++jj) {
      int k = kb + 16 * (j0 + jj) + 4 * q;
      k = k < ke ? k : 0;
#pragma unroll
      for (int i = 0; i < 2; ++i) a[jj][i] = *(const float4*)(arow[i] + k);
#pragma unroll
      for (int c = 0; c < NF; ++c) {
        if (BKC) {
          b[jj][c] = *(const float4*)(bcol[c] + k);
        } else {
          const float* p = bcol[c] + (int64_t)k * g.sbk;
          b[jj][c].x = p[0];
          b[jj][c].y = p[g.sbk];
          b[jj][c].z = p[2 * g.sbk];
          b[jj][c].w = p[3 * g.sbk];
        }
      }
    }
#pragma unroll
    for (int jj = 0; jj < DK_G; ++jj) {
      const bool ok = kb + 16 * (j0 + jj) + 4 * q < ke;
      float av[2][4];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        av[i][0] = ok ? a[jj][i].x : 0.f;
        av[i][1] = ok ? a[jj][i].y : 0.f;
        av[i][2] = ok ? a[jj][i].z : 0.f;
        av[i][3] = ok ? a[jj][i].w : 0.f;
      }
#pragma unroll
      for (int c = 0; c < NF; ++c)
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][c] = mfma16x16x4(av[i][0], b[jj][c].x, acc[i][c]);
#pragma unroll
      for (int c = 0; c < NF; ++c)
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][c] = mfma16x16x4(av[i][1], b[jj][c].y, acc[i][c]);
#pragma unroll
      for (int c = 0; c < NF; ++c)
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][c] = mfma16x16x4(av[i][2], b[jj][c].z, acc[i][c]);
#pragma unroll
      for (int c = 0; c < NF; ++c)
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][c] = mfma16x16x4(av[i][3], b[jj][c].w, acc[i][c]);
    }
  }
  if (KS > 1) {
    if (ks > 0) {
      float* dst = red + ((ks - 1) * RT + rt) * (2 * NF * 4 * 64) + lane;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int c = 0; c < NF; ++c)
#pragma unroll
          for (int r = 0; r < 4; ++r) dst[((i * NF + c) * 4 + r) * 64] = acc[i][c][r];
    }
    __syncthreads();
    if (ks > 0) return;
    // fixed order ((slice 0 + 1) + 2) + 3, one fragment at a time
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int c = 0; c < NF; ++c) {
#pragma unroll
        for (int s = 1; s < KS; ++s) {
          const float* src = red + ((s - 1) * RT + rt) * (2 * NF * 4 * 64) + lane;
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][c][r] += src[((i * NF + c) * 4 + r) * 64];
        }
        __builtin_amdgcn_sched_barrier(0);
      }
  }
  // epilogue: acc[i][c][r] -> row m0 + 16 i + 4 q + r, column n0 + 16 c + r16
#pragma unroll
  for (int c = 0; c < NF; ++c) {
    const int n = n0 + 16 * c + r16;
    if (n >= g.N) continue;
    const float bv = g.bias ? g.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + 16 * i + 4 * q + r;
        if (m >= g.M) continue;
        float v = acc[i][c][r] * g.alpha + bv;
        const int64_t ci = (int64_t)m * g.ldc + n;
        if (g.pre) g.pre[ci] = v;
        if (g.act == 1) v = gelu_erf(v);
        if (g.gate) v *= *g.gate;
        if (g.R) v += g.R[(int64_t)(g.rmod > 0 ? m % g.rmod : m) * g.ldr + n];
        if (g.accumulate) v += g.C[ci];
        g.C[ci] = v;
      }
  }
}

// ---------------------------------------------------------------------------------------
// gemm_kt_kernel: one 32 x 32 tile per block, split z over K in spans of g.kper; wave w
// takes the w-th quarter of the span (kq = kper / 4, even).  1-D grid: xcd_tile over
// (split, tile) when the split count is a multiple of 8 (the tiles of one k span share
// an XCD's L2), else tile-fastest.
constexpr int KT_C = 32;  // MFMA steps (2 k each) per chunk: a chunk's loads are all in flight

__global__ __launch_bounds__(256) void gemm_kt_kernel(GemmArgs g, int tiles_n, int tiles, int S,
                                                       int xcd) {
  __shared__ float red[4 * 16 * 64];
  int z, tile;
  if (xcd) {
    xcd_tile((int)blockIdx.x, tiles, &z, &tile);
  } else {
    z = (int)blockIdx.x / tiles;
    tile = (int)blockIdx.x - z * tiles;
  }
  if (z >= S) return;  // padding block of the XCD map
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * 32, n0 = tn * 32;
  const int kq = g.kper / 4;
  const int kb = z * g.kper + wid * kq;
  const int ke = min(g.K, kb + kq);
  const int steps = kb < ke ? (ke - kb + 1) / 2 : 0;
  const float* pa = g.A + min(m0 + r32, g.M - 1);
  const float* pb = g.B + min(n0 + r32, g.N - 1);
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  // chunk c covers steps [c*KT_C, (c+1)*KT_C); step s: k = kb + 2 s + h.  Every load of a
  // chunk is issued before any is used (one memory round trip per chunk, the next chunk's
  // loads in flight while this one multiplies); past ke -> address kb (valid), A zeroed
  // by a select at use.
  float a[KT_C], b[KT_C], an[KT_C], bn[KT_C];
  auto load = [&](float(&ad)[KT_C], float(&bd)[KT_C], int s0) {
#pragma unroll
    for (int u = 0; u < KT_C; ++u) {
      int k = kb + 2 * (s0 + u) + h;
      k = k < ke ? k : kb;
      ad[u] = pa[(int64_t)k * g.sak];
      bd[u] = pb[(int64_t)k * g.sbk];
    }
  };
  auto mul = [&](const float(&ad)[KT_C], const float(&bd)[KT_C], int s0) {
#pragma unroll
    for (int u = 0; u < KT_C; ++u) {
      const float av = kb + 2 * (s0 + u) + h < ke ? ad[u] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bd[u], acc, 0, 0, 0);
    }
  };
  if (steps > 0) load(a, b, 0);
  for (int s = 0; s < steps; s += 2 * KT_C) {
    if (s + KT_C < steps) load(an, bn, s + KT_C);
    mul(a, b, s);
    if (s + KT_C >= steps) break;
    if (s + 2 * KT_C < steps) load(a, b, s + 2 * KT_C);
    mul(an, bn, s + KT_C);
  }
  // the 4 waves' partial tiles -> LDS; thread e then owns tile elements e, e + 256, ...
  // (row-major, so the global stores coalesce): wave sum in the fixed order 0 + 1 + 2 + 3
#pragma unroll
  for (int r = 0; r < 16; ++r) red[(wid * 16 + r) * 64 + lane] = acc[r];
  __syncthreads();
  float v[4];
  int mm[4], nn[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int e = tid + 256 * j, row = e >> 5, col = e & 31;
    const int ln = col + 32 * ((row >> 2) & 1), r = (row & 3) + 4 * (row >> 3);
    v[j] = ((red[r * 64 + ln] + red[(16 + r) * 64 + ln]) + red[(32 + r) * 64 + ln]) +
           red[(48 + r) * 64 + ln];
    mm[j] = m0 + row;
    nn[j] = n0 + col;
  }
  if (S == 1) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (mm[j] < g.M && nn[j] < g.N) g.C[(int64_t)mm[j] * g.ldc + nn[j]] = epi_value(g, mm[j], nn[j], v[j]);
    return;
  }
  const int64_t tot = (int64_t)g.M * g.N;
  float* slab = g.slab + (int64_t)z * tot;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (mm[j] < g.M && nn[j] < g.N) {
      float* d = slab + (int64_t)mm[j] * g.N + nn[j];
      if (g.cnt) st_wt(d, v[j]);
      else *d = v[j];
    }
  if (!g.cnt) return;
  // the last-arriving split block of this tile sums the slabs in split order
  if (!last_block(g.cnt + tile, S)) return;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (mm[j] >= g.M || nn[j] >= g.N) continue;
    const int64_t i = (int64_t)mm[j] * g.N + nn[j];
    float t = 0.f;
#pragma unroll 4
    for (int zz = 0; zz < S; ++zz) t += ld_wt(g.slab + (int64_t)zz * tot + i);
    g.C[(int64_t)mm[j] * g.ldc + nn[j]] = epi_value(g, mm[j], nn[j], t);
  }
}

__global__ void gemm_direct_reduce_kernel(GemmArgs g, int splits) {
  const int64_t tot = (int64_t)g.M * g.N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < tot;
       i += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
#pragma unroll 8
    for (int z = 0; z < splits; ++z) s += g.slab[(int64_t)z * tot + i];
    const int m = (int)(i / g.N), n = (int)(i - (int64_t)m * g.N);
    g.C[(int64_t)m * g.ldc + n] = epi_value(g, m, n, s);
  }
}

// ---------------------------------------------------------------------------------------
static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Size thresholds below which the staged generic kernel takes the call (default 0: the
// direct kernels measured equal or faster at every step shape, profiles/r02_gemm_ab.txt).
static int dk_min_k() { return 0; }
static int kt_min_tiles() { return 0; }
static bool direct_off() { return false; }

template <int TNW, int KS, int G>
static void launch_dk(const GemmArgs& g, int kw, hipStream_t st) {
  constexpr int RT = 4 / KS;
  const int mblk = (g.M + 32 * RT - 1) / (32 * RT), nblk = (g.N + 32 * TNW - 1) / (32 * TNW);
  hipLaunchKernelGGL((gemm_dk_kernel<TNW, KS, false, G>), dim3(xcd_grid(mblk, nblk)), dim3(256), 0,
                     st, g, kw, nblk);
}

template <int KS, int G>
static void launch_dk_tnw(const GemmArgs& g, int tnw, int kw, hipStream_t st) {
  if (tnw == 2) launch_dk<2, KS, G>(g, kw, st);
  else launch_dk<1, KS, G>(g, kw, st);
}

template <int KS>
static void launch_dk_g(const GemmArgs& g, int tnw, int kw, hipStream_t st) {
  const int ng = kw / 16;
  if (ng >= 4) launch_dk_tnw<KS, 4>(g, tnw, kw, st);
  else if (ng >= 2) launch_dk_tnw<KS, 2>(g, tnw, kw, st);
  else launch_dk_tnw<KS, 1>(g, tnw, kw, st);
}

// split count of the weight-gradient form: one 64-k chunk per wave where that gives at
// most ~1024 blocks, at most 32 slabs per tile
int gemm_direct_splits(int64_t M, int64_t N, int64_t K) {
  if (direct_off()) return 1;
  const int64_t tiles = ((M + 31) / 32) * ((N + 31) / 32);
  int64_t s = (K + 4 * 2 * KT_C - 1) / (4 * 2 * KT_C);  // one chunk per wave ...
  if (s > 1024 / tiles) s = 1024 / tiles;             // ... up to ~1024 blocks
  if (s > 32) s = 32;
  return s < 1 ? 1 : (int)s;
}

// Launches a direct kernel for `g` when one fits (returns true), else false.  `ws`: slab
// workspace of gemm_direct_workspace floats (the wgrad form with splits > 1 needs it).
bool gemm_direct(GemmArgs g, float* ws, hipStream_t st) {
  if (direct_off()) return false;
  // dk: the input gradient dY W (B n-contiguous).  The Linear forward (B k-contiguous)
  // stays on gemm_rb2 / gemm_skinny, measured faster there (profiles/r02_gemm_ab.txt).
  if (g.sak == 1 && g.sbn == 1 && g.sbk != 1 && g.K <= 1024 && (g.K & 3) == 0 &&
      (g.sam & 3) == 0 && aligned16(g.A) && g.K >= dk_min_k()) {
    const int KS = g.K >= 64 ? 4 : (g.K >= 32 ? 2 : 1);
    int kw = (g.K + KS - 1) / KS;
    kw = (kw + 15) / 16 * 16;
    const int RT = 4 / KS;
    const int64_t mb = (g.M + 32 * RT - 1) / (32 * RT);
    int tnw = 2;  // wave tile 32 x 64 while that leaves >= 512 blocks
    if (32 >= g.N || mb * ((g.N + 63) / 64) < 512) tnw = 1;
    if (KS == 4) launch_dk_g<4>(g, tnw, kw, st);
    else if (KS == 2) launch_dk_g<2>(g, tnw, kw, st);
    else launch_dk_g<1>(g, tnw, kw, st);
    return true;
  }
  if (g.sam == 1 && g.sbn == 1 && g.K >= 256 &&
      ((g.M + 31) / 32) * ((g.N + 31) / 32) >= kt_min_tiles()) {
    int splits = gemm_direct_splits(g.M, g.N, g.K);
    if (splits > 1 && !ws) return false;
    int kper = (g.K + splits - 1) / splits;
    kper = (kper + 7) / 8 * 8;  // 4 waves x an even k count
    splits = (g.K + kper - 1) / kper;
    g.kper = kper;
    g.slab = splits > 1 ? ws : nullptr;
    const int tiles_n = (g.N + 31) / 32;
    const int tiles = ((g.M + 31) / 32) * tiles_n;
    // slabs are summed by a separate all-CU launch: measured faster than the in-launch
    // last-block finish (lf_dw 10.9 vs 18.3 us, hf_head_dw 33.2 vs 40.5 us)
    g.cnt = nullptr;
    const int xcd = splits % 8 == 0;
    const unsigned grid = xcd ? xcd_grid(splits, tiles) : (unsigned)(tiles * splits);
    hipLaunchKernelGGL(gemm_kt_kernel, dim3(grid), dim3(256), 0, st, g, tiles_n, tiles, splits, xcd);
    if (splits > 1 && !g.cnt) {
      const int64_t tot = (int64_t)g.M * g.N;
      const int blocks = (int)((tot + 255) / 256 < 2048 ? (tot + 255) / 256 : 2048);
      hipLaunchKernelGGL(gemm_direct_reduce_kernel, dim3(blocks), dim3(256), 0, st, g, splits);
    }
    return true;
  }
  return false;
}

}  // namespace tvq

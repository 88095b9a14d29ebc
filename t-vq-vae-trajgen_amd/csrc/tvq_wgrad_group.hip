// Grouped weight-gradient GEMM: dW_d (+)= dY_d^T X_d for a list of Linear layers in ONE
// launch (+ one ordered slab-sum launch).
//
// A transformer backward produces one weight gradient per Linear (q|k|v, out, ff1, ff2 per
// layer).  Each is a small output (128 x 128 .. 384 x 128) over a long K (= tokens, 6,400
// LF / 24,832 HF): alone it cannot fill 256 CUs, so tvq_gemm runs it as a latency-bound
// split-K launch pair (~11-14 us each for 0.2 GFLOP).  Nothing on the critical path reads
// these gradients before the optimizer step, so the trainer defers them to the end of the
// backward (timevqvae.hip.wgrad.grouped) and issues the whole set here: the LF prior's 16
// weight gradients are 5.03 GFLOP in one launch that fills the chip.
//
// Tiling: a block owns a (32 TW) x (32 TW) output tile of one descriptor over one k span
// of `kper`; its 4 waves split the span and each computes the whole tile on
// v_mfma_f32_32x32x2_f32 (TW x TW accumulators: lane l supplies A[m0 + 32 i + (l & 31)]
// [k = l >> 5], i.e. each operand load is two 128-byte token rows of dY / X).  A wave
// issues a chunk's loads (KC steps) before multiplying, with the next chunk in flight; the
// chunk loop has no branches (past the span: address clamped, A zeroed by a select), so
// the loads of the next chunk stay in flight across it.  The 4 partial tiles are added
// through LDS in wave order; split tiles go to the descriptor's slab z and
// wgrad_group_reduce sums slabs 0..S-1 in order, then adds C.
//
// A launch's plan depends on the descriptors it holds (see wg_splits); the caller groups
// records the same way whatever the streams (timevqvae.hip.wgrad tags).  Every sum has a
// fixed order independent of scheduling: results are run-to-run identical.
//
// Bias gradients ride along: a descriptor with a bias output (db_m = sum_k dY(m, k), the
// Linear's bias gradient) has its n-tile-0 blocks also sum the dY values they already load,
// in the same fixed order as the tile (steps in order, then the two lane halves, then the
// waves (w0 + w2) + (w1 + w3)), into a per-split bias slab that the reduce launch sums;
// no separate column-sum launch per Linear.
//
// XCD map: block b runs on XCD b % 8; logical index L = (b % 8) * per + b / 8 walks
// (descriptor, split, tile), so one XCD holds whole splits: a split's dY / X token rows
// are fetched into one L2 and re-read from it by every tile of that split.
#include <alloca.h>
#include <stdint.h>
#include <stdlib.h>

#include "tvq_common.h"

namespace tvq {

constexpr int WG_MAXD = 24;

struct WgDesc {
  const float* A;  // dY: A(m, k) = A[k * lda + m]   (m = output feature, k = token)
  const float* B;  // X:  B(k, n) = B[k * ldb + n]   (n = input feature)
  float* C;        // dW: C[m * ldc + n]
  float* Cb;       // optional db: Cb[m] (+)= sum_k A(m, k)
  int lda, ldb, ldc;
  int M, N, K;
  int kper;        // k span of one split (multiple of 8 KC)
  int S;           // splits
  int tiles, tiles_n;
  int blk0;        // first logical block of this descriptor (tiles * S of them)
  int rb0;         // first block of this descriptor in the reduce launch
  int rbb0;        // first block of its bias sum in the reduce launch
  int accumulate;  // C += result
  int64_t slab;    // its S slabs of M x N partials in the workspace
  int64_t bslab;   // its S bias slabs of M partials (Cb, S > 1)
};

struct WgGroup {
  WgDesc d[WG_MAXD];
  float* ws;
  int n, per, blocks;
  int rbias;  // first bias block of the reduce launch
};

// the bias partial of a block: per-lane sums v[i] of rows m0 + row(i, lane) over this
// wave's steps -> the two lane halves (h = 0, 1) -> the waves (w0 + w2) + (w1 + w3) -> the
// split's slab row (S > 1) or Cb (+)=.  ROWS: rows per tile; row(i, lane) as the caller's.
template <int NV, int ROWS, typename RowOf>
__device__ __forceinline__ void wg_bias_store(const WgGroup& G, const WgDesc& d, int z, int m0,
                                             const float (&v)[NV], RowOf row_of, float* bred) {
  const int tid = (int)threadIdx.x, lane = tid & 63, wid = tid >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const float t = v[i] + __shfl_xor(v[i], 32);  // h0 + h1 (commutative: same in both)
    if (lane < 32) bred[wid * ROWS + row_of(i, lane)] = t;
  }
  __syncthreads();
  for (int r = tid; r < ROWS; r += 256) {
    const int m = m0 + r;
    if (m >= d.M) continue;
    const float s = (bred[r] + bred[2 * ROWS + r]) + (bred[ROWS + r] + bred[3 * ROWS + r]);
    if (d.S > 1) {
      G.ws[d.bslab + (int64_t)z * d.M + m] = s;
    } else {
      float* c = d.Cb + m;
      *c = d.accumulate ? s + *c : s;
    }
  }
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t wg_rsrc(const float* p, int64_t floats) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0, (int)(floats * 4), 0x00020000);
}

// Byte offset of token row k (wave-uniform; each lane adds its row h and column through
// its base voffset).  It goes into the range-checked voffset, so rows past K load as 0;
// rows past the wave's span (inside the tensor) are zeroed at use.
__device__ __forceinline__ int wg_row(int k, int ld) { return k * ld * 4; }

template <int TW, int KC>
__global__ __launch_bounds__(256, 2) void wgrad_group_kernel(WgGroup G) {
  constexpr int WSZ = TW * TW * 16 * 64;  // one wave's partial tile in LDS
  __shared__ float red[4 * WSZ];
  __shared__ float bred[4 * 32 * TW];
  const int b = (int)blockIdx.x;
  const int L = (b & 7) * G.per + (b >> 3);
  if (L >= G.blocks) return;  // padding block of the XCD map (whole block)
  int di = 0;
  for (int i = 1; i < G.n; ++i) di = G.d[i].blk0 <= L ? i : di;
  const WgDesc& d = G.d[di];
  const int l = L - d.blk0;
  const int z = l / d.tiles, t = l - z * d.tiles;
  const int tm = t / d.tiles_n, tn = t - tm * d.tiles_n;
  const int m0 = tm * 32 * TW, n0 = tn * 32 * TW;
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar k bounds
  const int r32 = lane & 31, h = lane >> 5;
  const int kq = d.kper >> 2;
  const int kb = z * d.kper + wid * kq;
  const int ke = min(d.K, kb + kq);
  const int steps = kb < ke ? (ke - kb + 1) >> 1 : 0;
  const int nch = (steps + KC - 1) / KC;
  const int lda = d.lda, ldb = d.ldb, K = d.K;
  const auto ra = wg_rsrc(d.A, (int64_t)K * lda), rb = wg_rsrc(d.B, (int64_t)K * ldb);
  // per-lane byte offsets (row h, clamped column): rows past M / columns past N are never
  // stored
  int va[TW], vb[TW];
#pragma unroll
  for (int i = 0; i < TW; ++i) {
    va[i] = (h * lda + min(m0 + 32 * i + r32, d.M - 1)) * 4;
    vb[i] = (h * ldb + min(n0 + 32 * i + r32, d.N - 1)) * 4;
  }
  floatx16 acc[TW][TW];
  float bs[TW];  // bias partials (used by n-tile-0 blocks of a descriptor with Cb)
#pragma unroll
  for (int i = 0; i < TW; ++i) {
    bs[i] = 0.f;
#pragma unroll
    for (int j = 0; j < TW; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  }

  // step s: this lane's k = kb + 2 s + h; past ke: A zeroed by a select.  The chunk loop
  // has no data-dependent branch: the next chunk's loads are always in flight while this
  // one multiplies (the one past the last chunk is clamped and never used).
  float a0[KC][TW], b0[KC][TW], a1[KC][TW], b1[KC][TW];
  auto load = [&](float(&ad)[KC][TW], float(&bd)[KC][TW], int s0) {
#pragma unroll
    for (int u = 0; u < KC; ++u) {
      const int k = kb + 2 * (s0 + u);
      const int oa = wg_row(k, lda), ob = wg_row(k, ldb);
#pragma unroll
      for (int i = 0; i < TW; ++i) {
        ad[u][i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ra, va[i] + oa, 0, 0));
        bd[u][i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rb, vb[i] + ob, 0, 0));
      }
    }
  };
  auto mul = [&](const float(&ad)[KC][TW], const float(&bd)[KC][TW], int s0) {
#pragma unroll
    for (int u = 0; u < KC; ++u) {
      const bool ok = kb + 2 * (s0 + u) + h < ke;
#pragma unroll
      for (int i = 0; i < TW; ++i) {
        const float av = ok ? ad[u][i] : 0.f;
        bs[i] += av;
#pragma unroll
        for (int j = 0; j < TW; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bd[u][j], acc[i][j], 0, 0, 0);
      }
    }
  };
  // sched_barrier: keeps each chunk's loads together ahead of the previous chunk's MFMAs
  // (left alone, the scheduler sinks every load next to its use: one load round trip per
  // step)
  if (nch > 0) load(a0, b0, 0);
  for (int c = 0; c < nch; c += 2) {
    load(a1, b1, (c + 1) * KC);
    __builtin_amdgcn_sched_barrier(0);
    mul(a0, b0, c * KC);
    __builtin_amdgcn_sched_barrier(0);
    if (c + 1 >= nch) break;
    load(a0, b0, (c + 2) * KC);
    __builtin_amdgcn_sched_barrier(0);
    mul(a1, b1, (c + 1) * KC);
    __builtin_amdgcn_sched_barrier(0);
  }

  if (d.Cb && tn == 0)  // block-uniform
    wg_bias_store<TW, 32 * TW>(G, d, z, m0, bs, [](int i, int ln) { return 32 * i + ln; }, bred);
  // the 4 waves' partial tiles -> LDS; thread e then owns tile elements e, e + 256, ...
  // (row-major, so the global stores coalesce): (w0 + w2) + (w1 + w3), the wide form's order
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int j = 0; j < TW; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[wid * WSZ + ((i * TW + j) * 16 + r) * 64 + lane] = acc[i][j][r];
  __syncthreads();
  const int64_t ldc = d.ldc;
  float* slab = d.S > 1 ? G.ws + d.slab + (int64_t)z * d.M * d.N : nullptr;
#pragma unroll
  for (int q = 0; q < TW * TW * 4; ++q) {
    const int e = tid + 256 * q;
    const int row = e / (32 * TW), col = e - row * (32 * TW);
    const int i = row >> 5, j = col >> 5, rr = row & 31, cc = col & 31;
    const int ln = cc + 32 * ((rr >> 2) & 1), r = (rr & 3) + 4 * (rr >> 3);
    const int o = ((i * TW + j) * 16 + r) * 64 + ln;
    const float v = (red[o] + red[2 * WSZ + o]) + (red[WSZ + o] + red[3 * WSZ + o]);
    const int m = m0 + row, n = n0 + col;
    if (m < d.M && n < d.N) {
      if (slab) {
        slab[(int64_t)m * d.N + n] = v;
      } else {
        float* c = d.C + m * ldc + n;
        *c = d.accumulate ? v + *c : v;
      }
    }
  }
}

// Wide form for 16-byte-aligned outputs of at least 64 x 64: a 128 (m) x 64 (n) tile from
// ONE float4 of dY and ONE float2 of X per lane and step (lane l = (h, r): dY row k at
// m0 + 4 r, X row k at n0 + 2 r): 8 MFMAs per 2 loads, 32 FLOP per loaded byte (the TW
// form: 16).  MFMA j x jj multiplies the rows {m0 + 4 r + j} by the columns {n0 + 2 r + jj},
// a permutation of the tile that the store undoes.
template <int KC>
__global__ __launch_bounds__(256, 2) void wgrad_wide_kernel(WgGroup G) {
  constexpr int WSZ = 8 * 16 * 64;  // one wave's partial tile in LDS
  __shared__ float red[2 * WSZ];
  __shared__ float bred[4 * 128];
  const int b = (int)blockIdx.x;
  const int L = (b & 7) * G.per + (b >> 3);
  if (L >= G.blocks) return;  // padding block of the XCD map (whole block)
  int di = 0;
  for (int i = 1; i < G.n; ++i) di = G.d[i].blk0 <= L ? i : di;
  const WgDesc& d = G.d[di];
  const int l = L - d.blk0;
  const int z = l / d.tiles, t = l - z * d.tiles;
  const int tm = t / d.tiles_n, tn = t - tm * d.tiles_n;
  const int m0 = tm * 128, n0 = tn * 64;
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar k bounds
  const int r32 = lane & 31, h = lane >> 5;
  const int kq = d.kper >> 2;
  const int kb = z * d.kper + wid * kq;
  const int ke = min(d.K, kb + kq);
  const int steps = kb < ke ? (ke - kb + 1) >> 1 : 0;
  const int nch = (steps + KC - 1) / KC;
  const int lda = d.lda, ldb = d.ldb, K = d.K;
  const auto ra = wg_rsrc(d.A, (int64_t)K * lda), rb = wg_rsrc(d.B, (int64_t)K * ldb);
  // clamped (M % 4 == 0, N % 2 == 0): rows past M / columns past N are never stored
  const int va = (h * lda + min(m0 + 4 * r32, d.M - 4)) * 4;
  const int vb = (h * ldb + min(n0 + 2 * r32, d.N - 2)) * 4;
  floatx16 acc[4][2];
  float bs[4] = {0.f, 0.f, 0.f, 0.f};  // bias partials of rows m0 + 4 r + j
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[j][jj][e] = 0.f;
  float4 a0[KC], a1[KC];
  float2 b0[KC], b1[KC];
  auto load = [&](float4(&ad)[KC], float2(&bd)[KC], int s0) {
#pragma unroll
    for (int u = 0; u < KC; ++u) {
      const int k = kb + 2 * (s0 + u);
      ad[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ra, va + wg_row(k, lda), 0, 0));
      bd[u] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rb, vb + wg_row(k, ldb), 0, 0));
    }
  };
  auto mul = [&](const float4(&ad)[KC], const float2(&bd)[KC], int s0) {
#pragma unroll
    for (int u = 0; u < KC; ++u) {
      const bool ok = kb + 2 * (s0 + u) + h < ke;
      const float av[4] = {ok ? ad[u].x : 0.f, ok ? ad[u].y : 0.f, ok ? ad[u].z : 0.f,
                           ok ? ad[u].w : 0.f};
      const float bv[2] = {bd[u].x, bd[u].y};
#pragma unroll
      for (int j = 0; j < 4; ++j) bs[j] += av[j];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
          acc[j][jj] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j], bv[jj], acc[j][jj], 0, 0, 0);
    }
  };
  // sched_barrier: keeps each chunk's loads together ahead of the previous chunk's MFMAs
  // (left alone, the scheduler sinks every load next to its use: one load round trip per
  // step)
  if (nch > 0) load(a0, b0, 0);
  for (int c = 0; c < nch; c += 2) {
    load(a1, b1, (c + 1) * KC);
    __builtin_amdgcn_sched_barrier(0);
    mul(a0, b0, c * KC);
    __builtin_amdgcn_sched_barrier(0);
    if (c + 1 >= nch) break;
    load(a0, b0, (c + 2) * KC);
    __builtin_amdgcn_sched_barrier(0);
    mul(a1, b1, (c + 1) * KC);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (d.Cb && tn == 0)  // block-uniform
    wg_bias_store<4, 128>(G, d, z, m0, bs, [](int j, int ln) { return 4 * ln + j; }, bred);
  // (w0 + w2) + (w1 + w3): waves 2, 3 -> LDS, waves 0, 1 add; wave 1 -> LDS, wave 0 adds
  float* slot = red + (wid & 1) * WSZ + lane;
  if (wid >= 2) {
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int e = 0; e < 16; ++e) slot[(q * 16 + e) * 64] = acc[q >> 1][q & 1][e];
  }
  __syncthreads();
  if (wid < 2) {
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[q >> 1][q & 1][e] += slot[(q * 16 + e) * 64];
  }
  __syncthreads();
  if (wid == 1) {
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int e = 0; e < 16; ++e) slot[(q * 16 + e) * 64] = acc[q >> 1][q & 1][e];
  }
  __syncthreads();
  if (wid != 0) return;
  const float* o1 = red + WSZ + lane;
  // acc e of lane (h, r): MFMA row 8 (e / 4) + 4 h + e % 4, column r -> tile row
  // 4 (MFMA row) + j, columns 2 r + {0, 1}
  const int n = n0 + 2 * r32;
  float* slab = d.S > 1 ? G.ws + d.slab + (int64_t)z * d.M * d.N : nullptr;
  const int64_t ldc = d.ldc;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float v0 = acc[j][0][e] + o1[((2 * j) * 16 + e) * 64];
      const float v1 = acc[j][1][e] + o1[((2 * j + 1) * 16 + e) * 64];
      const int m = m0 + 4 * (8 * (e >> 2) + 4 * h + (e & 3)) + j;
      if (m >= d.M || n >= d.N) continue;
      if (slab) {
        *reinterpret_cast<float2*>(slab + (int64_t)m * d.N + n) = make_float2(v0, v1);
      } else {
        float* c = d.C + m * ldc + n;
        c[0] = d.accumulate ? v0 + c[0] : v0;
        c[1] = d.accumulate ? v1 + c[1] : v1;
      }
    }
}

// slabs 0..S-1 summed in order, then C (+)= sum; one 256-element chunk of one split
// descriptor per block
__global__ __launch_bounds__(256) void wgrad_group_reduce_kernel(WgGroup G) {
  const int b = (int)blockIdx.x;
  if (b >= G.rbias) {  // bias slabs: 256 rows of one descriptor's bias per block
    int di = -1;
    for (int i = 0; i < G.n; ++i) di = (G.d[i].Cb && G.d[i].S > 1 && G.d[i].rbb0 <= b) ? i : di;
    if (di < 0) return;
    const WgDesc& d = G.d[di];
    const int m = (b - d.rbb0) * 256 + (int)threadIdx.x;
    if (m >= d.M) return;
    const float* p = G.ws + d.bslab + m;
    float s = 0.f;
    for (int z = 0; z < d.S; ++z) s += p[(int64_t)z * d.M];
    float* c = d.Cb + m;
    *c = d.accumulate ? s + *c : s;
    return;
  }
  int di = 0;
  for (int i = 1; i < G.n; ++i) di = G.d[i].rb0 <= b ? i : di;
  const WgDesc& d = G.d[di];
  const int64_t e = (int64_t)(b - d.rb0) * 256 + threadIdx.x;
  if (d.S <= 1 || e >= (int64_t)d.M * d.N) return;
  const float* p = G.ws + d.slab + e;
  const int64_t tot = (int64_t)d.M * d.N;
  float s = 0.f;
#pragma unroll 8
  for (int z = 0; z < d.S; ++z) s += p[z * tot];
  const int m = (int)(e / d.N), n = (int)(e - (int64_t)m * d.N);
  float* c = d.C + (int64_t)m * d.ldc + n;
  *c = d.accumulate ? s + *c : s;
}

// ---------------------------------------------------------------------------------------
// Tile classes: 4 = the wide 128 x 64 form, 2 = 64 x 64, 1 = 32 x 32.  MFMA steps per
// chunk: 8 at 64 x 64 and 128 x 64 (2 waves per SIMD without spills), 16 at 32 x 32.
__host__ __device__ constexpr int wg_kc(int tw) { return tw == 1 ? 16 : 8; }

// Plans are made per launch: a launch holds one tile class (wide 128 x 64 = 4, 64 x 64 = 2,
// 32 x 32 = 1) and at most WG_MAXD descriptors, in the caller's order.  Its split count S
// is chosen from the launch's work units (64 x 64 tiles for classes 4 and 2, 32 x 32 for
// class 1) so that it has about TVQ_WG_UNITS (default 1000, resp. 1024) unit-splits: the
// LF prior's 16 Linears + its head (100 units) get S = 10, i.e. 500 wide blocks, one round
// at 2 per CU; a lone 256 x 256 Linear gets short spans over many blocks.  Every
// descriptor of the launch uses S (its k span: K / S rounded up to whole chunks of the 4
// waves, 8 KC).  Classes 4 and 2 count the same units and sum in the same order, so a
// descriptor's bits do not depend on which of the two its alignment selects.
static int wg_units(int64_t M, int64_t N, int tw) {
  const int u = tw == 1 ? 32 : 64;
  return (int)(((M + u - 1) / u) * ((N + u - 1) / u));
}

static int wg_class(int64_t M, int64_t N, bool wide_ok) {
  constexpr bool wide_on = true;
  if (M <= 32 || N <= 32) return 1;
  return (wide_on && wide_ok && M % 4 == 0 && N % 2 == 0) ? 4 : 2;
}

static int wg_splits(int units, int tw) {
  constexpr int t2 = 1000, t1 = 1024;  // ~work units per launch (tile classes 2/4, 1)
  int64_t s = ((tw == 1 ? t1 : t2) + units / 2) / (units > 0 ? units : 1);
  return (int)(s < 1 ? 1 : (s > 64 ? 64 : s));
}

static void wg_span(int64_t K, int S, int tw, int* kper, int* splits) {
  const int q = 8 * wg_kc(tw);
  int64_t kp = (K + S - 1) / S;
  kp = (kp + q - 1) / q * q;
  *kper = (int)kp;
  *splits = (int)((K + kp - 1) / kp);
}

static bool wide_aligned(const float* A, int64_t lda, const float* B, int64_t ldb) {
  return ((uintptr_t)A & 15) == 0 && lda % 4 == 0 && ((uintptr_t)B & 7) == 0 && ldb % 2 == 0;
}

// an upper bound (the alignment that picks a class is not known here): S <= 64 and
// S <= ceil(K / 64) for every descriptor; room for a bias slab per descriptor
static int64_t wg_smax(int64_t K) { return (K + 63) / 64 < 64 ? (K + 63) / 64 : 64; }

extern "C" int64_t tvq_wgrad_group_workspace(int64_t n, const int64_t* M, const int64_t* N,
                                             const int64_t* K) {
  int64_t need = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t s = wg_smax(K[i]);
    if (s > 1) need += s * M[i] * (N[i] + 1);
  }
  return need;
}

extern "C" int tvq_wgrad_group(int64_t n, const float* const* dY, const int64_t* ldy,
                               const float* const* X, const int64_t* ldx, float* const* dW,
                               const int64_t* ldw, const int64_t* M, const int64_t* N,
                               const int64_t* K, int64_t accumulate, float* workspace,
                               tvq_stream_t stream) {
  return tvq_wgrad_group_bias(n, dY, ldy, X, ldx, dW, ldw, nullptr, M, N, K, accumulate,
                              workspace, stream);
}

extern "C" int tvq_wgrad_group_bias(int64_t n, const float* const* dY, const int64_t* ldy,
                                    const float* const* X, const int64_t* ldx, float* const* dW,
                                    const int64_t* ldw, float* const* dB, const int64_t* M,
                                    const int64_t* N, const int64_t* K, int64_t accumulate,
                                    float* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(n >= 0 && dY && ldy && X && ldx && dW && ldw && M && N && K,
                "tvq_wgrad_group: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  for (int64_t j = 0; j < n; ++j)
    TVQ_CHECK_ARG(dY[j] && X[j] && dW[j] && M[j] > 0 && N[j] > 0 && K[j] > 0 && ldy[j] >= M[j] &&
                      ldx[j] >= N[j] && ldw[j] >= N[j] &&
                      (K[j] + 64) * (ldy[j] > ldx[j] ? ldy[j] : ldx[j]) < ((int64_t)1 << 29) &&
                      M[j] * ldw[j] < ((int64_t)1 << 31),
                  "tvq_wgrad_group: bad descriptor %lld", (long long)j);
  int64_t* slab_of = (int64_t*)alloca(sizeof(int64_t) * (n > 0 ? n : 1));
  int64_t* bslab_of = (int64_t*)alloca(sizeof(int64_t) * (n > 0 ? n : 1));
  int* cls = (int*)alloca(sizeof(int) * (n > 0 ? n : 1));
  int64_t slab0 = 0;
  for (int64_t j = 0; j < n; ++j) {  // each descriptor's slabs at its workspace-bound offset
    slab_of[j] = slab0;
    const int64_t s = wg_smax(K[j]);
    if (s > 1) slab0 += s * M[j] * N[j];
    cls[j] = wg_class(M[j], N[j], wide_aligned(dY[j], ldy[j], X[j], ldx[j]));
  }
  for (int64_t j = 0; j < n; ++j) {  // then the bias slabs
    bslab_of[j] = slab0;
    const int64_t s = wg_smax(K[j]);
    if (s > 1) slab0 += s * M[j];
  }
  TVQ_CHECK_ARG(slab0 == 0 || workspace, "tvq_wgrad_group: workspace required");
  // one launch pair per chunk of <= WG_MAXD descriptors of one class, in order on `stream`
  // (the outputs are disjoint: the launches may run in any order)
  for (int tw : {4, 2, 1}) {
    int64_t j = 0;
    while (true) {
      int64_t idx[WG_MAXD];
      int cnt = 0, units = 0;
      for (; j < n && cnt < WG_MAXD; ++j)
        if (cls[j] == tw) {
          idx[cnt++] = j;
          units += wg_units(M[j], N[j], tw);
        }
      if (cnt == 0) break;
      const int S0 = wg_splits(units, tw);
      WgGroup G;
      G.n = cnt;
      G.ws = workspace;
      int blk = 0, rb = 0;
      const int tsm = 32 * tw, tsn = tw == 4 ? 64 : 32 * tw;
      for (int i = 0; i < cnt; ++i) {
        const int64_t q = idx[i];
        WgDesc& d = G.d[i];
        d.A = dY[q];
        d.B = X[q];
        d.C = dW[q];
        d.Cb = dB ? dB[q] : nullptr;
        d.lda = (int)ldy[q];
        d.ldb = (int)ldx[q];
        d.ldc = (int)ldw[q];
        d.M = (int)M[q];
        d.N = (int)N[q];
        d.K = (int)K[q];
        wg_span(K[q], S0, tw, &d.kper, &d.S);
        d.tiles_n = (int)((N[q] + tsn - 1) / tsn);
        d.tiles = (int)((M[q] + tsm - 1) / tsm) * d.tiles_n;
        d.blk0 = blk;
        d.rb0 = rb;
        d.accumulate = (int)accumulate;
        d.slab = slab_of[q];
        d.bslab = bslab_of[q];
        blk += d.tiles * d.S;
        if (d.S > 1) rb += (int)((M[q] * N[q] + 255) / 256);
      }
      G.rbias = rb;
      for (int i = 0; i < cnt; ++i) {
        WgDesc& d = G.d[i];
        d.rbb0 = rb;
        if (d.Cb && d.S > 1) rb += (d.M + 255) / 256;
      }
      G.blocks = blk;
      G.per = (blk + 7) / 8;
      const unsigned grid = (unsigned)(8 * G.per);
      if (tw == 4)
        hipLaunchKernelGGL((wgrad_wide_kernel<wg_kc(4)>), dim3(grid), dim3(256), 0, st, G);
      else if (tw == 2)
        hipLaunchKernelGGL((wgrad_group_kernel<2, wg_kc(2)>), dim3(grid), dim3(256), 0, st, G);
      else
        hipLaunchKernelGGL((wgrad_group_kernel<1, wg_kc(1)>), dim3(grid), dim3(256), 0, st, G);
      if (rb > 0) hipLaunchKernelGGL(wgrad_group_reduce_kernel, dim3((unsigned)rb), dim3(256), 0, st, G);
    }
  }
  return launch_status("tvq_wgrad_group");
}

}  // namespace tvq

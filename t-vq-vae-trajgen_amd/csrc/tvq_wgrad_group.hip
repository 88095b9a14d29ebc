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
// issues a chunk's loads (KC steps) before multiplying, with the next chunk in flight.
// The 4 partial tiles are added through LDS in wave order; split tiles go to slab z of
// the workspace and wgrad_group_reduce sums slabs 0..S-1 in order, then adds C.
// Deterministic: every sum has a fixed order independent of scheduling.
//
// XCD map: block b runs on XCD b % 8; logical index L = (b % 8) * per + b / 8 walks
// (split, tile) split-major, so one XCD holds whole splits: a split's dY / X token rows are
// fetched into one L2 and re-read from it by every tile of that split.
#include <stdlib.h>

#include "tvq_common.h"

namespace tvq {

constexpr int WG_MAXD = 24;

struct WgDesc {
  const float* A;  // dY: A(m, k) = A[k * lda + m]   (m = output feature, k = token)
  const float* B;  // X:  B(k, n) = B[k * ldb + n]   (n = input feature)
  float* C;        // dW: C[m * ldc + n]
  int lda, ldb, ldc;
  int M, N, K;
  int kper;        // k span of one split (multiple of 8)
  int tiles_n;     // output tiles along n
  int tile0;       // first tile of this descriptor in the group's tile space
  int rb0;         // first block of this descriptor in the reduce launch
  int accumulate;  // C += result
  int64_t slab;    // offset of this descriptor's M x N partials inside one slab
};

struct WgGroup {
  WgDesc d[WG_MAXD];
  float* ws;    // S slabs of `tot` floats
  int64_t tot;
  int n, S, tiles, per;
};

__device__ __forceinline__ int wg_find_tile(const WgGroup& G, int t) {
  int di = 0;
  for (int i = 1; i < G.n; ++i) di = G.d[i].tile0 <= t ? i : di;
  return di;
}

template <int TW, int KC>
__global__ __launch_bounds__(256, 2) void wgrad_group_kernel(WgGroup G) {
  constexpr int WSZ = TW * TW * 16 * 64;  // one wave's partial tile in LDS
  __shared__ float red[4 * WSZ];
  const int b = (int)blockIdx.x;
  const int L = (b & 7) * G.per + (b >> 3);
  const int z = L / G.tiles, t = L - z * G.tiles;
  if (z >= G.S) return;  // padding block of the XCD map (whole block)
  const WgDesc& d = G.d[wg_find_tile(G, t)];
  const int lt = t - d.tile0;
  const int tm = lt / d.tiles_n, tn = lt - tm * d.tiles_n;
  const int m0 = tm * 32 * TW, n0 = tn * 32 * TW;
  const int tid = (int)threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  const int kq = d.kper >> 2;
  const int kb = z * d.kper + wid * kq;
  const int ke = min(d.K, kb + kq);
  const int steps = kb < ke ? (ke - kb + 1) >> 1 : 0;
  const int64_t lda = d.lda, ldb = d.ldb;
  // clamped row / column pointers (rows past M and columns past N are never stored)
  const float* pa[TW];
  const float* pb[TW];
#pragma unroll
  for (int i = 0; i < TW; ++i) {
    pa[i] = d.A + min(m0 + 32 * i + r32, d.M - 1);
    pb[i] = d.B + min(n0 + 32 * i + r32, d.N - 1);
  }
  floatx16 acc[TW][TW];
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int j = 0; j < TW; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // step s: k = kb + 2 s + h; steps past `steps` are skipped (wave-uniform branch); a
  // lane's k past ke (odd span) -> address kb and A zeroed by a select at use
  float a0[KC][TW], b0[KC][TW], a1[KC][TW], b1[KC][TW];
  auto load = [&](float(&ad)[KC][TW], float(&bd)[KC][TW], int s0) {
#pragma unroll
    for (int u = 0; u < KC; ++u) {
      if (s0 + u < steps) {
        int k = kb + 2 * (s0 + u) + h;
        k = k < ke ? k : kb;
#pragma unroll
        for (int i = 0; i < TW; ++i) {
          ad[u][i] = pa[i][k * lda];
          bd[u][i] = pb[i][k * ldb];
        }
      }
    }
  };
  auto mul = [&](const float(&ad)[KC][TW], const float(&bd)[KC][TW], int s0) {
#pragma unroll
    for (int u = 0; u < KC; ++u) {
      if (s0 + u < steps) {
        const bool ok = kb + 2 * (s0 + u) + h < ke;
#pragma unroll
        for (int i = 0; i < TW; ++i) {
          const float av = ok ? ad[u][i] : 0.f;
#pragma unroll
          for (int j = 0; j < TW; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bd[u][j], acc[i][j], 0, 0, 0);
        }
      }
    }
  };
  if (steps > 0) load(a0, b0, 0);
  for (int s = 0; s < steps; s += 2 * KC) {
    if (s + KC < steps) load(a1, b1, s + KC);
    mul(a0, b0, s);
    if (s + KC >= steps) break;
    if (s + 2 * KC < steps) load(a0, b0, s + 2 * KC);
    mul(a1, b1, s + KC);
  }

  // the 4 waves' partial tiles -> LDS; thread e then owns tile elements e, e + 256, ...
  // (row-major, so the global stores coalesce): ((w0 + w1) + w2) + w3
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int j = 0; j < TW; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[wid * WSZ + ((i * TW + j) * 16 + r) * 64 + lane] = acc[i][j][r];
  __syncthreads();
  const int64_t ldc = d.ldc;
  float* slab = G.S > 1 ? G.ws + (int64_t)z * G.tot + d.slab : nullptr;
#pragma unroll
  for (int q = 0; q < TW * TW * 4; ++q) {
    const int e = tid + 256 * q;
    const int row = e / (32 * TW), col = e - row * (32 * TW);
    const int i = row >> 5, j = col >> 5, rr = row & 31, cc = col & 31;
    const int ln = cc + 32 * ((rr >> 2) & 1), r = (rr & 3) + 4 * (rr >> 3);
    const int o = ((i * TW + j) * 16 + r) * 64 + ln;
    const float v = ((red[o] + red[WSZ + o]) + red[2 * WSZ + o]) + red[3 * WSZ + o];
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

// slabs 0..S-1 summed in order, then C (+)= sum; one 256-element chunk of one descriptor
// per block
__global__ __launch_bounds__(256) void wgrad_group_reduce_kernel(WgGroup G) {
  const int b = (int)blockIdx.x;
  int di = 0;
  for (int i = 1; i < G.n; ++i) di = G.d[i].rb0 <= b ? i : di;
  const WgDesc& d = G.d[di];
  const int64_t e = (int64_t)(b - d.rb0) * 256 + threadIdx.x;
  if (e >= (int64_t)d.M * d.N) return;
  const float* p = G.ws + d.slab + e;
  float s = 0.f;
#pragma unroll 8
  for (int z = 0; z < G.S; ++z) s += p[(int64_t)z * G.tot];
  const int m = (int)(e / d.N), n = (int)(e - (int64_t)m * d.N);
  float* c = d.C + (int64_t)m * d.ldc + n;
  *c = d.accumulate ? s + *c : s;
}

// ---------------------------------------------------------------------------------------
static int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

struct WgPlan {
  int TW, S, kper, tiles;
  int64_t tot;
};

// Tile width, split count and k span for descriptors [0, n): 64 x 64 tiles unless some
// output is <= 32 wide; about TVQ_WG_BLOCKS (default 2048: 4 rounds of the 2 blocks per
// CU the 64 KB LDS / ~200 VGPR footprint allows) blocks, at most 64 slabs, k spans of at
// least 64 (16 MFMA steps per wave).
static WgPlan wg_plan(int64_t n, const int64_t* M, const int64_t* N, const int64_t* K) {
  WgPlan p;
  p.TW = 2;
  int64_t kmax = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (M[i] <= 32 || N[i] <= 32) p.TW = 1;
    if (K[i] > kmax) kmax = K[i];
  }
  const int ts = 32 * p.TW;
  p.tiles = 0;
  p.tot = 0;
  for (int64_t i = 0; i < n; ++i) {
    p.tiles += (int)(((M[i] + ts - 1) / ts) * ((N[i] + ts - 1) / ts));
    p.tot += M[i] * N[i];
  }
  const int target = env_int("TVQ_WG_BLOCKS", p.TW == 2 ? 2048 : 4096);
  int64_t s = (target + p.tiles / 2) / p.tiles;
  if (s > 64) s = 64;
  if (s < 1) s = 1;
  int64_t kper = (kmax + s - 1) / s;
  kper = (kper + 7) / 8 * 8;
  if (kper < 64) kper = 64;
  p.kper = (int)kper;
  p.S = (int)((kmax + kper - 1) / kper);
  return p;
}

extern "C" int64_t tvq_wgrad_group_workspace(int64_t n, const int64_t* M, const int64_t* N,
                                             const int64_t* K) {
  int64_t best = 0;
  for (int64_t c0 = 0; c0 < n; c0 += WG_MAXD) {
    const int64_t c = n - c0 < WG_MAXD ? n - c0 : WG_MAXD;
    const WgPlan p = wg_plan(c, M + c0, N + c0, K + c0);
    const int64_t need = p.S > 1 ? p.S * p.tot : 0;
    if (need > best) best = need;
  }
  return best;
}

extern "C" int tvq_wgrad_group(int64_t n, const float* const* dY, const int64_t* ldy,
                               const float* const* X, const int64_t* ldx, float* const* dW,
                               const int64_t* ldw, const int64_t* M, const int64_t* N,
                               const int64_t* K, int64_t accumulate, float* workspace,
                               tvq_stream_t stream) {
  TVQ_CHECK_ARG(n >= 0 && dY && ldy && X && ldx && dW && ldw && M && N && K,
                "tvq_wgrad_group: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  for (int64_t c0 = 0; c0 < n; c0 += WG_MAXD) {  // chunks run in order on `stream`
    const int64_t c = n - c0 < WG_MAXD ? n - c0 : WG_MAXD;
    const WgPlan p = wg_plan(c, M + c0, N + c0, K + c0);
    TVQ_CHECK_ARG(p.S == 1 || workspace, "tvq_wgrad_group: workspace required");
    WgGroup G;
    G.n = (int)c;
    G.S = p.S;
    G.tiles = p.tiles;
    G.tot = p.tot;
    G.ws = workspace;
    const int ts = 32 * p.TW;
    int tile0 = 0, rb0 = 0;
    int64_t off = 0;
    for (int64_t i = 0; i < c; ++i) {
      const int64_t j = c0 + i;
      TVQ_CHECK_ARG(dY[j] && X[j] && dW[j] && M[j] > 0 && N[j] > 0 && K[j] > 0 &&
                        ldy[j] >= M[j] && ldx[j] >= N[j] && ldw[j] >= N[j] &&
                        K[j] * (ldy[j] > ldx[j] ? ldy[j] : ldx[j]) < ((int64_t)1 << 31) &&
                        M[j] * ldw[j] < ((int64_t)1 << 31),
                    "tvq_wgrad_group: bad descriptor %lld", (long long)j);
      WgDesc& d = G.d[i];
      d.A = dY[j];
      d.B = X[j];
      d.C = dW[j];
      d.lda = (int)ldy[j];
      d.ldb = (int)ldx[j];
      d.ldc = (int)ldw[j];
      d.M = (int)M[j];
      d.N = (int)N[j];
      d.K = (int)K[j];
      d.kper = p.kper;
      d.tiles_n = (int)((N[j] + ts - 1) / ts);
      d.tile0 = tile0;
      d.rb0 = rb0;
      d.accumulate = (int)accumulate;
      d.slab = off;
      tile0 += (int)((M[j] + ts - 1) / ts) * d.tiles_n;
      rb0 += (int)((M[j] * N[j] + 255) / 256);
      off += M[j] * N[j];
    }
    const int64_t logical = (int64_t)p.tiles * p.S;
    G.per = (int)((logical + 7) / 8);
    const unsigned grid = (unsigned)(8 * G.per);
    if (p.TW == 2)
      hipLaunchKernelGGL((wgrad_group_kernel<2, 16>), dim3(grid), dim3(256), 0, st, G);
    else
      hipLaunchKernelGGL((wgrad_group_kernel<1, 16>), dim3(grid), dim3(256), 0, st, G);
    if (p.S > 1)
      hipLaunchKernelGGL(wgrad_group_reduce_kernel, dim3((unsigned)rb0), dim3(256), 0, st, G);
  }
  return launch_status("tvq_wgrad_group");
}

}  // namespace tvq

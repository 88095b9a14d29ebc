// Deterministic reduction primitives shared by the backward kernels.
//
// reduce_rows  out[j] (+)= sum_{p<P} in[p*ld + j]   (column sums of a P x N slab):
//              two levels of 256-thread blocks (64 columns x 4 row groups, fixed
//              combine order), coalesced along j; replaces one-thread-per-column
//              loops that were latency bound (split-K / wgrad slabs, LayerNorm and
//              RMSNorm gamma partials, Linear bias gradients).
//              Optional split output: rows of length L -> out1 (first L-1 columns,
//              dense) and out2 (last column): the fused conv weight|bias gradient.
// group_by     stable counting sort of int indices in [0, V): offsets[V+1] and a
//              permutation (positions grouped by value in increasing position
//              order) -> segmented sums in a fixed order with no float atomics
//              (VQ embed_sum, nn.Embedding backward).
#include "tvq_common.h"
#include "tvq_reduce.h"

namespace tvq {

constexpr int RR_COLS = 64, RR_GROUPS = 4, RR_ROWS = 64;

// column block j0..j0+63, rows [p0, p1) of `in` (row stride ld): 4 row groups strided
// by 4 each, combined (g0+g1)+(g2+g3) -- the fixed order of every level
template <bool WT>
__device__ __forceinline__ float rr_colsum(const float* __restrict__ in, int64_t p0, int64_t p1,
                                           int64_t ld, int64_t j, int64_t N, float (*sh)[RR_COLS],
                                           int c, int g) {
  float s = 0.f;
  if (j < N) {
    // 16 rows' loads in flight per thread (the adds stay in row order): the slabs here are
    // 64-256 rows tall, and 4 in flight left the sum bound by load latency (42 us for the
    // band-end batch of the fused ResBlocks' 256-row weight-gradient slabs, now 22 us).
    // (32 in flight, or a masked 16-row tail, measured slower.)
    int64_t p = p0 + g;
    for (; p + 15 * RR_GROUPS < p1; p += 16 * RR_GROUPS) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const float* a = in + (p + u * RR_GROUPS) * ld + j;
        v[u] = WT ? ld_wt(a) : *a;
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) s += v[u];
    }
    for (; p < p1; p += RR_GROUPS) s += WT ? ld_wt(in + p * ld + j) : in[p * ld + j];
  }
  sh[g][c] = s;
  __syncthreads();
  const float t = (sh[0][c] + sh[1][c]) + (sh[2][c] + sh[3][c]);
  __syncthreads();
  return t;
}

__device__ __forceinline__ void rr_store(float t, int64_t j, float* __restrict__ out,
                                         float* __restrict__ out2, int64_t L, int accumulate) {
  if (L > 0) {  // split output: [rows][L] -> out (L-1 cols) | out2 (last col)
    const int64_t r = j / L, col = j - r * L;
    float* d = col < L - 1 ? out + r * (L - 1) + col : out2 + r;
    if (col < L - 1 || out2) *d = accumulate ? *d + t : t;
  } else {
    out[j] = accumulate ? out[j] + t : t;
  }
}

// direct: one level, rows [0, P) -> out.  !direct: level 1 (row block blockIdx.y ->
// scratch row); with `cnt` the last row block of column block x then runs level 2 over
// the R scratch rows (same order as the separate level-2 launch) and writes out.
__global__ __launch_bounds__(256) void reduce_rows_kernel(const float* __restrict__ in, int64_t P,
                                                          int64_t N, int64_t ld, int rows_per_blk,
                                                          float* __restrict__ out,
                                                          float* __restrict__ out2, int64_t L,
                                                          int accumulate, int direct,
                                                          float* __restrict__ scratch,
                                                          int* __restrict__ cnt) {
  __shared__ float sh[RR_GROUPS][RR_COLS];
  const int c = threadIdx.x % RR_COLS, g = threadIdx.x / RR_COLS;
  const int64_t j = (int64_t)blockIdx.x * RR_COLS + c;
  const int64_t p0 = (int64_t)blockIdx.y * rows_per_blk;
  const int64_t p1 = min(P, p0 + rows_per_blk);
  const float t = rr_colsum<false>(in, p0, p1, ld, j, N, sh, c, g);
  if (direct) {
    if (g == 0 && j < N) rr_store(t, j, out, out2, L, accumulate);
    return;
  }
  if (g == 0 && j < N) {
    if (cnt) st_wt(scratch + (int64_t)blockIdx.y * N + j, t);
    else scratch[(int64_t)blockIdx.y * N + j] = t;
  }
  if (cnt && last_block(cnt + blockIdx.x, (int)gridDim.y)) {
    const float u = rr_colsum<true>(scratch, 0, gridDim.y, N, j, N, sh, c, g);
    if (g == 0 && j < N) rr_store(u, j, out, out2, L, accumulate);
  }
}

// one launch (each thread sums <= RR_ONE / 4 rows) when the slab is short; the
// two-level split only pays for tall slabs, where one block column would serialise
constexpr int64_t RR_ONE = 256;

int64_t reduce_rows_scratch(int64_t P, int64_t N) {
  const int64_t R = (P + RR_ROWS - 1) / RR_ROWS;
  return (R > 1 && P > RR_ONE) ? R * N : 0;
}

void reduce_rows(const float* in, int64_t P, int64_t N, int64_t ld, float* out, float* out2,
                 int64_t L, int accumulate, float* scratch, hipStream_t st) {
  const unsigned gx = (unsigned)((N + RR_COLS - 1) / RR_COLS);
  const int64_t R = (P + RR_ROWS - 1) / RR_ROWS;
  if (R <= 1 || P <= RR_ONE || scratch == nullptr) {  // single level: one block column per 64 cols
    hipLaunchKernelGGL(reduce_rows_kernel, dim3(gx, 1), dim3(256), 0, st, in, P, N, ld, (int)P,
                       out, out2, L, accumulate, 1, nullptr, nullptr);
    return;
  }
  int* cnt = counters(gx, FIN_REDUCE);
  hipLaunchKernelGGL(reduce_rows_kernel, dim3(gx, (unsigned)R), dim3(256), 0, st, in, P, N, ld,
                     RR_ROWS, out, out2, L, accumulate, 0, scratch, cnt);
  if (!cnt)
    hipLaunchKernelGGL(reduce_rows_kernel, dim3(gx, 1), dim3(256), 0, st, scratch, R, N, N, (int)R,
                       out, out2, L, accumulate, 1, nullptr, nullptr);
}

// Batched single-level column sums: blockIdx.x runs over the jobs' column blocks (each job
// takes ceil(N / cols) consecutive blocks, found by a scalar scan of the job list); each
// block is exactly reduce_rows_kernel's direct path.  Up to RR_BATCH jobs per launch (the
// band-end batch of a stage1 band is ~80 slabs: one launch, was four of 24).
constexpr int RR_BATCH = 96;
struct RrJobK {  // 40 bytes: RR_BATCH of them stay inside a 4 KB kernel-argument block
  const float* in;
  float* out;
  float* out2;
  int P, N, L, accumulate;
};
struct RrBatch {
  RrJobK job[RR_BATCH];
  int n;
};
static_assert(sizeof(RrBatch) <= 3900, "reduce_rows batch kernel arguments");

// the job of block `blk` and its first block (wave-uniform scan)
__device__ __forceinline__ int rr_job_of(const RrBatch& b, int blk, int cols, int& first) {
  int j = 0, b0 = 0;
  for (; j + 1 < b.n; ++j) {
    const int nb = (b.job[j].N + cols - 1) / cols;
    if (blk < b0 + nb) break;
    b0 += nb;
  }
  first = b0;
  return j;
}

__global__ __launch_bounds__(256) void reduce_rows_batch_kernel(RrBatch b) {
  __shared__ float sh[RR_GROUPS][RR_COLS];
  int first;
  const int j = rr_job_of(b, (int)blockIdx.x, RR_COLS, first);
  const RrJobK& jb = b.job[j];
  const int c = threadIdx.x % RR_COLS, g = threadIdx.x / RR_COLS;
  const int64_t col = (int64_t)(blockIdx.x - first) * RR_COLS + c;
  const float t = rr_colsum<false>(jb.in, 0, jb.P, jb.N, col, jb.N, sh, c, g);
  if (g == 0 && col < jb.N) rr_store(t, col, jb.out, jb.out2, jb.L, jb.accumulate);
}

// The same sums four adjacent columns per thread with 16-byte loads (N % 4 == 0, aligned
// slab): 256 columns per block, each column summed in exactly rr_colsum's row order
// ((g0 + g1) + (g2 + g3) over row groups of stride 4, rows in order within a group), so
// the results are bitwise those of the scalar kernel with a quarter of the load
// instructions (the band-end batch of the conv weight-gradient slabs reads 140-200 MB).
__global__ __launch_bounds__(256) void reduce_rows_batch4_kernel(RrBatch b) {
  __shared__ float4 sh[RR_GROUPS][RR_COLS];
  int first;
  const int j = rr_job_of(b, (int)blockIdx.x, 4 * RR_COLS, first);
  const RrJobK& jb = b.job[j];
  const int c = threadIdx.x % RR_COLS, g = threadIdx.x / RR_COLS;
  const int64_t col = ((int64_t)(blockIdx.x - first) * RR_COLS + c) * 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (col < jb.N) {
    const float* in = jb.in + col;
    int64_t p = g;
    for (; p + 15 * RR_GROUPS < jb.P; p += 16 * RR_GROUPS) {
      float4 v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = *reinterpret_cast<const float4*>(in + (p + u * RR_GROUPS) * jb.N);
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        s.x += v[u].x;
        s.y += v[u].y;
        s.z += v[u].z;
        s.w += v[u].w;
      }
    }
    for (; p < jb.P; p += RR_GROUPS) {
      const float4 v = *reinterpret_cast<const float4*>(in + p * jb.N);
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
  }
  sh[g][c] = s;
  __syncthreads();
  if (g != 0 || col >= jb.N) return;
  const float4 a = sh[0][c], b1 = sh[1][c], c2 = sh[2][c], d3 = sh[3][c];
  const float t[4] = {(a.x + b1.x) + (c2.x + d3.x), (a.y + b1.y) + (c2.y + d3.y),
                      (a.z + b1.z) + (c2.z + d3.z), (a.w + b1.w) + (c2.w + d3.w)};
#pragma unroll
  for (int q = 0; q < 4; ++q) rr_store(t[q], col + q, jb.out, jb.out2, jb.L, jb.accumulate);
}

void reduce_rows_batch(const RrJob* jobs, int n, hipStream_t st) {
  // 16-byte form for the jobs whose slabs allow it, the scalar form for the rest
  for (int wide = 1; wide >= 0; --wide) {
    RrJob sel[RR_BATCH];
    int k = 0;
    auto flush = [&]() {
      if (k == 0) return;
      RrBatch b;
      b.n = k;
      const int cols = wide ? 4 * RR_COLS : RR_COLS;
      int blocks = 0;
      for (int i = 0; i < k; ++i) {
        b.job[i] = {sel[i].in, sel[i].out, sel[i].out2, (int)sel[i].P, (int)sel[i].N,
                    (int)sel[i].L, sel[i].accumulate};
        blocks += (int)((sel[i].N + cols - 1) / cols);
      }
      if (wide)
        hipLaunchKernelGGL(reduce_rows_batch4_kernel, dim3((unsigned)blocks), dim3(256), 0, st, b);
      else
        hipLaunchKernelGGL(reduce_rows_batch_kernel, dim3((unsigned)blocks), dim3(256), 0, st, b);
      k = 0;
    };
    for (int i = 0; i < n; ++i) {
      const bool w4 = jobs[i].N % 4 == 0 && ((uintptr_t)jobs[i].in & 15) == 0;
      if (w4 != (wide == 1)) continue;
      sel[k++] = jobs[i];
      if (k == RR_BATCH) flush();
    }
    flush();
  }
}

// ---------------------------------------------------------------- group-by
// tokens per histogram / placement chunk (512 measured no faster in the step: gb_scan 11.7 vs
// 10.6 us, hist / place 8 vs 6.4 us)
constexpr int GB_CHUNK = 256;
// rows per segmented-sum chunk: one 4-wave block (32 rows per wave); every value has at least
// one chunk (an empty value's chunk writes its zero row), skewed values many
constexpr int SEG_CH = 128;
__host__ __device__ __forceinline__ int seg_chunks_of(int n) { return n > 0 ? (n + SEG_CH - 1) / SEG_CH : 1; }
static int64_t seg_max_chunks(int64_t M, int64_t V) { return (M + SEG_CH - 1) / SEG_CH + V; }
__host__ __device__ __forceinline__ int* seg_chunk_infos(int* seg_start, int64_t V) {
  const uintptr_t p = reinterpret_cast<uintptr_t>(seg_start + V + 1);
  return reinterpret_cast<int*>((p + 15) & ~(uintptr_t)15);
}
// chunk descriptors (int4 per chunk: value, first sorted row, rows, first chunk | count << 16)
// for the nc chunks of value v whose rows start at sorted position r0: one load per block
__device__ __forceinline__ void seg_chunk_info(int* info, int v, int r0, int n, int cs, int nc) {
  for (int i = 0; i < nc; ++i) {
    const int a = r0 + i * SEG_CH;
    const int4 d = make_int4(v, a, min(n - i * SEG_CH, SEG_CH), cs | (nc << 16));
    reinterpret_cast<int4*>(info)[cs + i] = d;
  }
}

template <typename IT>
__global__ __launch_bounds__(256) void gb_hist_kernel(const IT* __restrict__ idx, int64_t M, int V,
                                                      int* __restrict__ hist) {
  extern __shared__ int h[];
  for (int v = threadIdx.x; v < V; v += 256) h[v] = 0;
  __syncthreads();
  const int64_t m0 = (int64_t)blockIdx.x * GB_CHUNK;
  for (int64_t m = m0 + threadIdx.x; m < min(M, m0 + GB_CHUNK); m += 256) {
    const int v = (int)idx[m];
    if (v >= 0 && v < V) atomicAdd(&h[v], 1);  // integer: exact
  }
  __syncthreads();
  for (int v = threadIdx.x; v < V; v += 256) hist[(int64_t)blockIdx.x * V + v] = h[v];
}

// one block: per-value totals over chunks, exclusive scan -> offsets[V+1];
// chunk_off[chunk][v] = offsets[v] + sum_{c' < chunk} hist[c'][v] (chunk-major: the threads
// of consecutive values read / write consecutive words; a value-major layout measured 2.6x
// slower, 27.6 vs 10.6 us)
__device__ __forceinline__ int wave_incl_scan(int x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

// Exclusive block scan (1024 threads) of two per-thread counters; returns the totals.
__device__ __forceinline__ void block_excl_scan2(int& a, int& b, int& tot_a, int& tot_b) {
  __shared__ int wa[16], wb[16];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int ia = wave_incl_scan(a), ib = wave_incl_scan(b);
  if (lane == 63) { wa[wid] = ia; wb[wid] = ib; }
  __syncthreads();
  int pa = 0, pb = 0;
  tot_a = 0;
  tot_b = 0;
  for (int w = 0; w < 16; ++w) {
    if (w < wid) { pa += wa[w]; pb += wb[w]; }
    tot_a += wa[w];
    tot_b += wb[w];
  }
  a = pa + ia - a;
  b = pb + ib - b;
}

// Column totals over chunks, a parallel exclusive scan over values (integer, so any
// order is exact), then per-chunk offsets.  One block of 1024 threads; each thread owns
// `per` consecutive values.
__global__ __launch_bounds__(1024) void gb_scan_kernel(const int* __restrict__ hist, int chunks,
                                                       int V, int* __restrict__ chunk_off,
                                                       int* __restrict__ offsets,
                                                       int* __restrict__ seg_start,
                                                       int* __restrict__ chunk_v,
                                                       int32_t* __restrict__ counts,
                                                       float* __restrict__ countsf) {
  extern __shared__ int tot[];  // [V]
  const int per = (V + 1023) / 1024;
  const int v0 = threadIdx.x * per;
  int t_loc = 0, s_loc = 0;
  for (int u = 0; u < per; ++u) {
    const int v = v0 + u;
    if (v >= V) break;
    int s = 0;
#pragma unroll 16
    for (int c = 0; c < chunks; ++c) s += hist[(int64_t)c * V + v];
    tot[v] = s;
    if (counts) {  // the per-value counts (the VQ statistics' counts / cluster sizes)
      counts[v] = s;
      countsf[v] = (float)s;
    }
    t_loc += s;
    s_loc += seg_chunks_of(s);
  }
  int all_t, all_s;
  block_excl_scan2(t_loc, s_loc, all_t, all_s);
  int run = t_loc, segs = s_loc;
  for (int u = 0; u < per; ++u) {
    const int v = v0 + u;
    if (v >= V) break;
    offsets[v] = run;
    if (seg_start) seg_start[v] = segs;
    int s = run;
#pragma unroll 16
    for (int c = 0; c < chunks; ++c) {
      const int h = hist[(int64_t)c * V + v];
      chunk_off[(int64_t)c * V + v] = s;
      s += h;
    }
    const int nc = seg_chunks_of(tot[v]);
    if (chunk_v) seg_chunk_info(chunk_v, v, run, tot[v], segs, nc);
    run += tot[v];
    segs += nc;
  }
  if (threadIdx.x == 0) {
    offsets[V] = all_t;
    if (seg_start) seg_start[V] = all_s;
  }
}

// The whole stable counting sort in one 1024-thread block (M <= GB1_MAX_M, V <= 1024: every
// group-by of the training step).  The indices go to LDS as 16-bit values; wave w owns a
// contiguous token range and counts it into its own histogram row (integer LDS atomics:
// exact); thread v then turns the 16 rows of value v into the waves' running offsets
// (exclusive block scan of the per-value totals and of the chunk counts), and each wave
// places its tokens in token order: the lanes holding the same value are found by AND-ing
// the ballots of the value's bits, a lane's rank among them is a popcount, and the highest
// such lane advances the wave's offset.  Same offsets / perm as the 3-launch path.
// Measured in the joint step (round 4, profiles/r04e_step_kernels.csv): one block is the
// fastest form for the class-embedding group-bys (M = 256: 4.5 us against ~15 for the three
// launches) but loses on the token group-bys (M = 6144 / 24576: 16-47 / 88-115 us), a long
// serial chain on one CU that shares it with the step's other three streams.  Above
// GB1_MAX_M the three-launch sort runs instead.
constexpr int GB1_MAX_M = 2048, GB1_MAX_V = 1024, GB1_T = 1024;
template <typename IT>
__global__ __launch_bounds__(GB1_T) void gb_sort1_kernel(const IT* __restrict__ idx, int M, int V,
                                                         int* __restrict__ offsets,
                                                         int* __restrict__ perm,
                                                         int* __restrict__ seg_start,
                                                         int* __restrict__ chunk_v,
                                                         int32_t* __restrict__ counts,
                                                         float* __restrict__ countsf) {
  extern __shared__ int gb1_smem[];
  int* hist = gb1_smem;  // [16][V]: counts, then each wave's running offsets
  unsigned short* vals = reinterpret_cast<unsigned short*>(gb1_smem + 16 * V);  // [M]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int per = ((M + 15) / 16 + 63) / 64 * 64;  // tokens per wave (multiple of 64)
  for (int i = tid; i < 16 * V; i += GB1_T) hist[i] = 0;
  // 8 loads in flight per thread (a load -> LDS store per iteration waits a full memory
  // round trip each time: 24 of them for M = 24576)
  for (int m0i = 0; m0i < M; m0i += 8 * GB1_T) {
    int v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int m = m0i + u * GB1_T + tid;
      v[u] = m < M ? (int)idx[m] : -1;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int m = m0i + u * GB1_T + tid;
      if (m < M) vals[m] = (unsigned short)(v[u] >= 0 && v[u] < V ? v[u] : 0xFFFF);
    }
  }
  __syncthreads();
  const int m0 = w * per, m1 = min(M, m0 + per);
  for (int m = m0 + lane; m < m1; m += 64) {
    const int v = vals[m];
    if (v != 0xFFFF) atomicAdd(&hist[w * V + v], 1);
  }
  __syncthreads();
  int tot = 0;
  if (tid < V)
    for (int k = 0; k < 16; ++k) tot += hist[k * V + tid];
  int nc = tid < V ? seg_chunks_of(tot) : 0;
  int ex_t = tot, ex_c = nc, all_t, all_s;
  block_excl_scan2(ex_t, ex_c, all_t, all_s);
  if (tid < V) {
    offsets[tid] = ex_t;
    seg_start[tid] = ex_c;
    if (counts) {
      counts[tid] = tot;
      countsf[tid] = (float)tot;
    }
    seg_chunk_info(chunk_v, tid, ex_t, tot, ex_c, nc);
    int run = ex_t;
    for (int k = 0; k < 16; ++k) {
      const int c = hist[k * V + tid];
      hist[k * V + tid] = run;
      run += c;
    }
  }
  if (tid == 0) {
    offsets[V] = all_t;
    seg_start[V] = all_s;
  }
  __syncthreads();
  const int nbits = V > 1 ? 32 - __clz(V - 1) : 0;
  const unsigned long long below = (1ull << lane) - 1ull;
  for (int g0 = m0; g0 < m1; g0 += 64) {
    const int m = g0 + lane;
    const int v = m < m1 ? (int)vals[m] : 0xFFFF;
    const bool ok = v != 0xFFFF;
    unsigned long long eq = __ballot(ok);
    for (int b = 0; b < nbits; ++b) {
      const bool bit = (v >> b) & 1;
      const unsigned long long bal = __ballot(bit);
      eq &= bit ? bal : ~bal;
    }
    if (ok) {
      const int base = hist[w * V + v];
      perm[base + __popcll(eq & below)] = m;
      if ((eq >> lane) == 1ull) hist[w * V + v] = base + __popcll(eq);
    }
  }
}

// stable placement: rank of m among equal values earlier in its chunk = the count in the
// chunk's earlier waves (per-wave LDS histograms, integer atomics: exact) + the lanes below
// it in its own wave holding the same value (AND of the value bits' ballots, popcount)
template <typename IT>
__global__ __launch_bounds__(GB_CHUNK) void gb_place_kernel(const IT* __restrict__ idx, int64_t M,
                                                            int V, const int* __restrict__ chunk_off,
                                                            int* __restrict__ perm) {
  constexpr int NWV = GB_CHUNK / 64;  // one token per thread
  extern __shared__ int cw[];         // [NWV][V]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < NWV * V; i += GB_CHUNK) cw[i] = 0;
  const int64_t m = (int64_t)blockIdx.x * GB_CHUNK + tid;
  int v = m < M ? (int)idx[m] : -1;
  const bool ok = v >= 0 && v < V;
  if (!ok) v = 0;
  __syncthreads();
  if (ok) atomicAdd(&cw[w * V + v], 1);
  const int nbits = V > 1 ? 32 - __clz(V - 1) : 0;
  unsigned long long eq = __ballot(ok);
  for (int b = 0; b < nbits; ++b) {
    const bool bit = (v >> b) & 1;
    const unsigned long long bal = __ballot(bit);
    eq &= bit ? bal : ~bal;
  }
  __syncthreads();
  if (!ok) return;
  int r = __popcll(eq & ((1ull << lane) - 1ull));
  for (int k = 0; k < w; ++k) r += cw[k * V + v];
  perm[chunk_off[(int64_t)blockIdx.x * V + v] + r] = (int)m;
}

// the same placement for V > GB_PLACE_MAX_V (the per-wave histograms would not fit LDS):
// rank by scanning the chunk's earlier indices
constexpr int GB_PLACE_MAX_V = 4096;
template <typename IT>
__global__ __launch_bounds__(256) void gb_place_wide_kernel(const IT* __restrict__ idx, int64_t M,
                                                            int V, const int* __restrict__ chunk_off,
                                                            int* __restrict__ perm) {
  __shared__ int vals[GB_CHUNK];
  const int64_t m0 = (int64_t)blockIdx.x * GB_CHUNK;
  const int n = (int)min((int64_t)GB_CHUNK, M - m0);
  for (int i = threadIdx.x; i < n; i += 256) vals[i] = (int)idx[m0 + i];
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += 256) {
    const int v = vals[i];
    if (v < 0 || v >= V) continue;
    int r = 0;
    for (int k = 0; k < i; ++k) r += (vals[k] == v);
    perm[chunk_off[(int64_t)blockIdx.x * V + v] + r] = (int)(m0 + i);
  }
}

int64_t group_by_scratch_ints(int64_t M, int64_t V) {
  const int64_t chunks = (M + GB_CHUNK - 1) / GB_CHUNK;
  // hist + chunk_off (3-launch path) | seg_start | (16-B aligned) chunk descriptors
  return 2 * chunks * V + (V + 1) + 4 + 4 * seg_max_chunks(M, V);
}

template <typename IT>
static void group_by_t(const IT* idx, int64_t M, int64_t V, int* offsets, int* perm, int* scratch,
                       hipStream_t st, int32_t* counts, float* countsf) {
  const int chunks = (int)((M + GB_CHUNK - 1) / GB_CHUNK);
  int* hist = scratch;
  int* coff = scratch + (int64_t)chunks * V;
  int* seg_start = coff + (int64_t)chunks * V;
  int* chunk_v = seg_chunk_infos(seg_start, V);
  if (M <= GB1_MAX_M && V <= GB1_MAX_V) {
    const size_t lds = (size_t)16 * V * 4 + (size_t)M * 2;  // <= 68 KB
    TVQ_PLAN("group_by sort1 M%lld V%lld", (long long)M, (long long)V);
    hipLaunchKernelGGL(gb_sort1_kernel<IT>, dim3(1), dim3(GB1_T), lds, st, idx, (int)M, (int)V,
                       offsets, perm, seg_start, chunk_v, counts, countsf);
    return;
  }
  TVQ_PLAN("group_by 3-launch M%lld V%lld", (long long)M, (long long)V);
  hipLaunchKernelGGL(gb_hist_kernel<IT>, dim3(chunks), dim3(256), V * sizeof(int), st, idx, M,
                     (int)V, hist);
  hipLaunchKernelGGL(gb_scan_kernel, dim3(1), dim3(1024), V * sizeof(int), st, hist, chunks, (int)V,
                     coff, offsets, seg_start, chunk_v, counts, countsf);
  if (V <= GB_PLACE_MAX_V)
    hipLaunchKernelGGL(gb_place_kernel<IT>, dim3(chunks), dim3(GB_CHUNK),
                       (size_t)(GB_CHUNK / 64) * V * sizeof(int), st, idx, M, (int)V, coff, perm);
  else
    hipLaunchKernelGGL(gb_place_wide_kernel<IT>, dim3(chunks), dim3(256), 0, st, idx, M, (int)V,
                       coff, perm);
}

void group_by_i32(const int32_t* idx, int64_t M, int64_t V, int* offsets, int* perm, int* scratch,
                  hipStream_t st, int32_t* counts, float* countsf) {
  group_by_t<int32_t>(idx, M, V, offsets, perm, scratch, st, counts, countsf);
}
void group_by_i64(const int64_t* idx, int64_t M, int64_t V, int* offsets, int* perm, int* scratch,
                  hipStream_t st) {
  group_by_t<int64_t>(idx, M, V, offsets, perm, scratch, st, nullptr, nullptr);
}

// Segmented row sums in one launch: block c takes chunk c of the sorted rows (SEG_CH rows of
// ONE value, chunk_v[c]); its 4 waves sum 32 rows each in order (the wave's row indices read
// once and broadcast by shuffles, 16 rows' loads in flight before any add), then wave 0 adds
// the wave partials in wave order.  A value with one chunk (nearly all) is written directly;
// a skewed value (the MaskGIT mask token, a collapsed code) publishes its chunk partials
// (write-through) and the block that draws its last ticket sums them in chunk order, so the
// result never depends on arrival order (bitwise reproducible).  Without a counter pool
// the partials are summed by seg_combine_kernel instead (same order).
template <int ND>
__device__ __forceinline__ void seg_rows_wave(const SegRows& s, const int* __restrict__ perm,
                                              int r0, int n, int v, float (&acc)[ND]) {
  const int lane = threadIdx.x & 63;
  const int pm = lane < n ? perm[r0 + lane] : 0;
#pragma unroll
  for (int i = 0; i < ND; ++i) acc[i] = 0.f;
  const bool drop = s.drop_p > 0.f && (int64_t)v != s.mask_id;
  const uint64_t seed = drop ? mix_seed(s.seed_ptr, s.offset) : 0ull;
  const float sc = drop ? 1.0f / (1.0f - s.drop_p) : 1.0f;
  constexpr int U = ND <= 2 ? 16 : 8;  // rows in flight
  for (int rb = 0; rb < n; rb += U) {
    float x[U][ND];
    int mm[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int m = __shfl(pm, rb + u < n ? rb + u : 0, 64);
      mm[u] = m;
      const int64_t b = m / s.N, nn = m - b * s.N;
      const float* row = s.src + b * s.sB + nn * s.sN;
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        const int d = lane + 64 * i;
        x[u][i] = row[(int64_t)(d < s.D ? d : 0) * s.sD];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (rb + u >= n) break;
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        const int d = lane + 64 * i;
        float xv = x[u][i];
        if (drop) xv = uniform01(seed, (uint64_t)((int64_t)mm[u] * s.D + d)) >= s.drop_p ? xv * sc : 0.f;
        acc[i] += xv;
      }
    }
  }
}

template <int ND>
__global__ __launch_bounds__(256) void seg_sum_kernel(SegRows s, const int* __restrict__ offsets,
                                                      const int* __restrict__ perm,
                                                      const int* __restrict__ seg_start,
                                                      const int* __restrict__ chunk_v, int V,
                                                      float* __restrict__ part,
                                                      float* __restrict__ out, int accumulate,
                                                      int* __restrict__ cnt) {
  __shared__ float red[3][64 * ND];
  __shared__ float cmb[256];
  const int c = blockIdx.x;
  const int total = seg_start[V];
  const int4 d4 = reinterpret_cast<const int4*>(chunk_v)[c < total ? c : 0];
  if (c >= total) return;  // block-uniform
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int v = d4.x, r0 = d4.y, r1 = d4.y + d4.z;
  const int cs = d4.w & 0xFFFF, ce = cs + (d4.w >> 16);
  const int rw = r0 + 32 * w, n = max(0, min(r1 - rw, 32));
  float acc[ND];
  seg_rows_wave<ND>(s, perm, rw, n, v, acc);
  if (w > 0) {
#pragma unroll
    for (int i = 0; i < ND; ++i) red[w - 1][lane + 64 * i] = acc[i];
  }
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int i = 0; i < ND; ++i) {
      const int d = lane + 64 * i;
      const float t = ((acc[i] + red[0][d]) + red[1][d]) + red[2][d];
      if (d >= s.D) continue;
      if (ce - cs == 1) {
        const int64_t e = (int64_t)v * s.D + d;
        out[e] = accumulate ? out[e] + t : t;
      } else if (cnt) {
        st_wt(part + (int64_t)c * s.D + d, t);
      } else {
        part[(int64_t)c * s.D + d] = t;
      }
    }
  }
  if (ce - cs == 1 || !cnt) return;  // block-uniform
  if (!last_block(cnt + v, ce - cs)) return;
  // the value's chunk partials in chunk order: thread (j, d) sums chunks cs + j, + J, ...
  // (16 in flight), then the J partial sums in a fixed pairwise tree
  int J = 1;
  while (2 * J * s.D <= 256) J *= 2;
  for (int d0 = 0; d0 < s.D; d0 += 256 / J) {
    const int j = threadIdx.x / (256 / J), d = d0 + threadIdx.x % (256 / J);
    float t = 0.f;
    if (d < s.D) {
      int k = cs + j;
      for (; k + 15 * J < ce; k += 16 * J) {
        float q[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) q[u] = ld_wt(part + (int64_t)(k + u * J) * s.D + d);
#pragma unroll
        for (int u = 0; u < 16; ++u) t += q[u];
      }
      for (; k < ce; k += J) t += ld_wt(part + (int64_t)k * s.D + d);
    }
    cmb[threadIdx.x] = t;
    __syncthreads();
    for (int h = J / 2; h >= 1; h >>= 1) {
      if (j < h) cmb[threadIdx.x] += cmb[threadIdx.x + h * (256 / J)];
      __syncthreads();
    }
    if (j == 0 && d < s.D) {
      const int64_t e = (int64_t)v * s.D + d;
      out[e] = accumulate ? out[e] + cmb[threadIdx.x] : cmb[threadIdx.x];
    }
    __syncthreads();
  }
}

// seg_sum_kernel's combine as a launch (no counter pool): values with > 1 chunk
__global__ __launch_bounds__(256) void seg_combine_kernel(const float* __restrict__ part,
                                                          const int* __restrict__ seg_start, int V,
                                                          int D, float* __restrict__ out,
                                                          int accumulate) {
  __shared__ float cmb[256];
  const int v = blockIdx.x;
  const int cs = seg_start[v], ce = seg_start[v + 1];
  if (ce - cs <= 1) return;
  int J = 1;
  while (2 * J * D <= 256) J *= 2;
  for (int d0 = 0; d0 < D; d0 += 256 / J) {
    const int j = threadIdx.x / (256 / J), d = d0 + threadIdx.x % (256 / J);
    float t = 0.f;
    if (d < D) {
      int k = cs + j;
      for (; k + 15 * J < ce; k += 16 * J) {
        float q[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) q[u] = part[(int64_t)(k + u * J) * D + d];
#pragma unroll
        for (int u = 0; u < 16; ++u) t += q[u];
      }
      for (; k < ce; k += J) t += part[(int64_t)k * D + d];
    }
    cmb[threadIdx.x] = t;
    __syncthreads();
    for (int h = J / 2; h >= 1; h >>= 1) {
      if (j < h) cmb[threadIdx.x] += cmb[threadIdx.x + h * (256 / J)];
      __syncthreads();
    }
    if (j == 0 && d < D) {
      const int64_t e = (int64_t)v * D + d;
      out[e] = accumulate ? out[e] + cmb[threadIdx.x] : cmb[threadIdx.x];
    }
    __syncthreads();
  }
}

int64_t seg_rowsum_scratch_floats(int64_t M, int64_t V, int64_t D) {
  // (the chunk descriptors live in the group-by scratch, seg_chunk_infos)
  return seg_max_chunks(M, V) * D;
}

void seg_rowsum(const SegRows& s, const int* offsets, const int* perm, const int* seg_start,
                int64_t M, int64_t V, float* out, int accumulate, float* part, hipStream_t st) {
  const int max_chunks = (int)seg_max_chunks(M, V);
  const int* chunk_v = seg_chunk_infos(const_cast<int*>(seg_start), V);
  int* cnt = counters(V, FIN_REDUCE);
  const dim3 grid((unsigned)max_chunks);
#define SEG_L(NDV) hipLaunchKernelGGL(seg_sum_kernel<NDV>, grid, dim3(256), 0, st, s, offsets, perm, \
                                      seg_start, chunk_v, (int)V, part, out, accumulate, cnt)
  if (s.D <= 64) SEG_L(1);
  else if (s.D <= 128) SEG_L(2);
  else if (s.D <= 256) SEG_L(4);
  else SEG_L(8);
#undef SEG_L
  if (!cnt)
    hipLaunchKernelGGL(seg_combine_kernel, dim3((unsigned)V), dim3(256), 0, st, part, seg_start,
                       (int)V, s.D, out, accumulate);
}

int* group_by_seg_start(int* scratch, int64_t M, int64_t V) {
  const int64_t chunks = (M + GB_CHUNK - 1) / GB_CHUNK;
  return scratch + 2 * chunks * V;
}

}  // namespace tvq

using namespace tvq;

extern "C" int64_t tvq_reduce_rows_workspace(int64_t P, int64_t N) {
  return reduce_rows_scratch(P, N);
}

extern "C" int tvq_reduce_rows(const float* in, int64_t P, int64_t N, int64_t ld, float* out,
                               int64_t accumulate, float* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(in && out && P > 0 && N > 0 && ld >= N, "tvq_reduce_rows: bad arguments");
  TVQ_CHECK_ARG(reduce_rows_scratch(P, N) == 0 || workspace, "tvq_reduce_rows: needs workspace");
  reduce_rows(in, P, N, ld, out, nullptr, 0, (int)accumulate, workspace, (hipStream_t)stream);
  return launch_status("tvq_reduce_rows");
}

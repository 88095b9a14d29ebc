// The LF MaskGIT prior's whole forward in eval mode (iterative decoding, maskgit.py:294-355
// first_pass -> masked_prediction -> BidirectionalTransformer.forward_lf,
// bidirectional_transformer.py:166-192 with the x-transformers encoder of :92-110) as ONE
// launch per decoding step: one wave per sequence, every activation in registers.
//
//   x = cat(cls_emb[c], tok_emb[s] + pos_emb[:n])              (embed_assemble)
//   x = LayerNorm_gamma(x W_in^T)                              (project_in, post_emb_norm)
//   depth x { x += Attn(RMSNorm(x)) W_o^T ; x += W2 GELU(W1 RMSNorm(x) + b1) + b2 }
//   x = RMSNorm(x) W_out^T                                     (final_norm, project_out)
//   h = LayerNorm_{w,b,1e-12}(GELU(x W_p^T + b_p))              (pred_head; W_p W_out composed)
//   logits[:, i-1, k] = h_i . tok_emb[k] + bias[i-1, k],  i = 1..n, k < K   (tied logits)
//
// Layout ("token on the lane"): the sequence (n + 1 <= 32 tokens, cls first) sits on the 32
// columns of v_mfma_f32_32x32x2_f32 tiles, lane l owning token l & 31 and, in its 16
// accumulator registers per tile, feature rows crow(r, h) (h = l >> 5) of that token.  A
// Linear y^T = W x^T then takes W as the A operand (lane = output feature, k = the step's
// feature, straight from L1/L2 with 16-B loads) and x^T as the B operand: the B value of
// step t is register t of the lane's own token -- the previous layer's output, never moved.
// The same registers are the A operand of x W^T (token on the lane as the ROW), which is
// how V comes out feature-on-the-lane for O^T = V^T P^T.  So attention is
//   S^T = K Q^T (A = K regs, B = Q regs: one query per lane, its keys in registers),
//   softmax over the registers + one xor-32 shuffle,
//   O^T = V^T P^T (A = V regs, B = P regs),
// and the out-projection / FF consume O^T / GELU(u)^T from registers.  Norm statistics
// are a register sum + one xor-32 shuffle.  Per step and sequence this is 7936 MFMAs
// (config.yaml LF prior: depth 4, width 128, 2 heads x 64, ff 128, K = 512; 8448 less
// project_in, folded into the embedding tables, and project_out, composed into pred_head); the
// unfused path ran ~30 launches per step, each streaming activations through HBM.
//
// Weights: every Linear's 32-row tiles are consumed in one fixed order (project_in, per
// layer q/k/v per head and the head's out-projection columns, ff1, ff2, then the composed
// project_out / pred_head weight, the tied-logit code tiles).  prior_pack_kernel writes them once per call
// into a stream in the MFMA operand order (tile -> 16-B group T4 -> lane): every load is one
// coalesced 1-KB row, and each wave loads the first groups of tile i+1 while it multiplies
// tile i, so a tile never starts on an L2 round trip.  (A 4-wave block staging the stream
// through a 2 x 16 KB LDS ring with one barrier per tile measured slower: 591 vs 431 us per
// launch for the unpipelined direct loads, the barriers and LDS reads exposed at one wave
// per SIMD.)
//
// Arithmetic follows the unfused kernels' formulas (rmsnorm_fwd, layernorm_fwd, the GEMM
// epilogue order (acc + bias) + residual, attention_fwd's softmax); sums over features run
// in a different order (fp32, within the 1e-4 parity bar, tests/test_prior_eval.py).
#include <math.h>
#include <stdlib.h>

#include "tvq_common.h"
#include "tvq_gemm.h"
#include "tvq_race.h"

namespace tvq {

constexpr int PE_D = 128;     // prior width (hidden_dim == embed_dim), heads x 64 == 128
constexpr int PE_MAXDEPTH = 8;
constexpr int PE_FIXED = 5, PE_PER_LAYER = 10, PE_TAIL = 7;

struct PriorLayer {
  const float *g_attn, *wq, *wk, *wv, *wo, *g_ff, *w1, *b1, *w2, *b2;
};
struct PriorArgs {
  const int64_t* s;
  int64_t ss;  // row stride of s
  const int64_t* cls;  // (B) class index, nullptr: the null class n_classes
  int n_classes, B, n, K, depth;
  const float *tok_emb, *pos_emb, *cls_emb, *w_in, *post_gamma;
  PriorLayer L[PE_MAXDEPTH];
  const float *g_final, *w_out, *wp, *bp, *ln_w, *ln_b, *bias;
  float ln_eps;
  float* logits;  // (B, n, K); in draw mode the debug copy of the logits, nullable
  // draw mode (sampled != null): the race of tvq_maskgit_sample on the logits in registers
  int64_t mask_id;
  const float* gumbel;
  const int64_t* seed_ptr;
  uint64_t offset;
  int64_t* sampled;
  float* selp;
  // project_in folded into the embedding tables (one-wave kernel): rows tok [0, K+1),
  // pos [K+1, K+1+n), cls [K+1+n, ...) of (table row) W_in^T, written by prior_fold_kernel
  float* ftab;
  // project_out (with final_norm's g) composed with pred_head's Linear: wc = W_p W_out diag(g)
  // (128 x 128, written by prior_headfold_kernel), packed as the 4 head tiles
  float* wc;
};

__device__ __forceinline__ floatx16 pe_mfma(float a, float b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int pe_crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ void pe_zero(floatx16& a) {
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = 0.f;
}

// GELU by gelu_as (tvq_common.h): branch-free, the library erff's range branches diverged
// across a wave's 64 values and the GELUs were a quarter of this kernel's VALU instructions
__device__ __forceinline__ float pe_gelu(float x) { return gelu_as(x); }

// ---- the weight-tile stream.  Tile idx (order of consumption) -> source rows.
struct PeTile {
  const float* w;  // row-major, ld = PE_D
  int row0, k0, ns, rows;  // first row, first column, MFMA steps (64: K=128, 32: K=64)
  const float* gk;  // per-column factor folded into the packed tile (an RMSNorm's g), or null
};
__device__ __forceinline__ int pe_ntiles(int depth, int K) {
  return 4 + 28 * depth + 4 + (K + 31) / 32;
}
__device__ __forceinline__ PeTile pe_tile(const PriorArgs& a, int idx) {
  if (idx < 4) return {a.w_in, 32 * idx, 0, 64, PE_D, nullptr};
  idx -= 4;
  if (idx < 28 * a.depth) {
    const PriorLayer& L = a.L[idx / 28];
    const int j = idx % 28;
    if (j < 20) {
      const int hd = j / 10, jj = j % 10;
      if (jj < 6) {  // q / k / v read RMSNorm_attn(x): its g is folded in
        const int u = jj / 3, m = jj % 3;
        return {m == 0 ? L.wq : (m == 1 ? L.wk : L.wv), 64 * hd + 32 * u, 0, 64, PE_D, L.g_attn};
      }
      return {L.wo, 32 * (jj - 6), 64 * hd, 32, PE_D, nullptr};
    }
    if (j < 24) return {L.w1, 32 * (j - 20), 0, 64, PE_D, L.g_ff};
    return {L.w2, 32 * (j - 24), 0, 64, PE_D, nullptr};
  }
  idx -= 28 * a.depth;
  if (idx < 4) return {a.wc, 32 * idx, 0, 64, PE_D, nullptr};  // W_p W_out diag(g_final)
  idx -= 4;
  return {a.tok_emb, 32 * idx, 0, 64, a.K, nullptr};  // code rows >= K are packed as zeros
}
// float4 offset of tile idx in the stream: 1024 per 64-step tile, 512 per 32-step tile
__device__ __forceinline__ int64_t pe_tile_off(int idx, int depth) {
  int64_t off = 0;
  if (idx > 4) {
    const int lt = min(idx - 4, 28 * depth);  // layer tiles before idx
    const int full = lt / 28, rem = lt % 28;
    const int outproj = 8 * full + (rem <= 6 ? 0 : min(rem - 6, 4)) + (rem <= 16 ? 0 : min(rem - 16, 4));
    off = (int64_t)1024 * idx - 512 * outproj;
  } else {
    off = (int64_t)1024 * idx;
  }
  return off;
}

// stream element e (float4) of tile t: group T4 = e / 64, lane l = e % 64 ->
// W[row0 + (l & 31)][k0 + 32*(T4>>2) + 8*(T4&3) + 4*(l>>5) .. +3]
// first: the stream's first tile (4 when project_in is folded into the tables)
__global__ __launch_bounds__(256) void prior_pack_kernel(PriorArgs a, float4* __restrict__ out,
                                                         int first) {
  const int idx = (int)blockIdx.x + first;
  const PeTile t = pe_tile(a, idx);
  float4* dst = out + pe_tile_off(idx, a.depth) - pe_tile_off(first, a.depth);
  const int n4 = t.ns / 4 * 64;
  for (int e = threadIdx.x; e < n4; e += 256) {
    const int T4 = e >> 6, l = e & 63;
    const int row = t.row0 + (l & 31);
    const int k = t.k0 + 32 * (T4 >> 2) + 8 * (T4 & 3) + 4 * (l >> 5);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < t.rows) v = *reinterpret_cast<const float4*>(t.w + (int64_t)row * PE_D + k);
    if (t.gk) {  // W[n][k] * g[k]: RMSNorm's per-feature g moved onto the Linear
      const float4 g = *reinterpret_cast<const float4*>(t.gk + k);
      v.x *= g.x; v.y *= g.y; v.z *= g.z; v.w *= g.w;
    }
    dst[e] = v;
  }
}

// project_in folded into the tables the embedding reads: row r of tok_emb (r < K+1), pos_emb
// (the next n) or cls_emb (the rest) times W_in^T -- cat(cls, tok + pos) W_in^T is then a
// gather and an add of projected rows (the same function up to fp32 reassociation), and the
// 256 project_in MFMAs per sequence and their 4 weight tiles leave the launch
__global__ __launch_bounds__(128) void prior_fold_kernel(PriorArgs a) {
  const int r = blockIdx.x, j = threadIdx.x;
  const int V = a.K + 1;
  const float* src = r < V ? a.tok_emb + (int64_t)r * PE_D
                   : (r < V + a.n ? a.pos_emb + (int64_t)(r - V) * PE_D
                                  : a.cls_emb + (int64_t)(r - V - a.n) * PE_D);
  const float* w = a.w_in + (int64_t)j * PE_D;
  float acc = 0.f;
#pragma unroll 8
  for (int k = 0; k < PE_D; k += 4) {
    const float4 x = *reinterpret_cast<const float4*>(src + k);
    const float4 y = *reinterpret_cast<const float4*>(w + k);
    acc = fmaf(x.x, y.x, acc);
    acc = fmaf(x.y, y.y, acc);
    acc = fmaf(x.z, y.z, acc);
    acc = fmaf(x.w, y.w, acc);
  }
  a.ftab[(int64_t)r * PE_D + j] = acc;
}

// final_norm -> project_out -> pred_head's Linear without a nonlinearity between the two
// Linears: wc[i][k] = (sum_j W_p[i][j] W_out[j][k]) g_final[k], one row per block, the j sum
// in order (the same function up to fp32 reassociation; 256 MFMAs per sequence
// and 4 weight tiles leave the launch)
__global__ __launch_bounds__(128) void prior_headfold_kernel(PriorArgs a) {
  const int i = blockIdx.x, k = threadIdx.x;
  const float* wp = a.wp + (int64_t)i * PE_D;
  float acc = 0.f;
#pragma unroll 8
  for (int j = 0; j < PE_D; ++j) acc = fmaf(wp[j], a.w_out[(int64_t)j * PE_D + k], acc);
  a.wc[(int64_t)i * PE_D + k] = acc * a.g_final[k];
}

// a per-feature vector (D floats) in the register layout: v[tile][r] = p[32*tile + crow(r,h)]
__device__ __forceinline__ void pe_load_vec(const float* __restrict__ p, int h, floatx16 (&v)[4]) {
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 x = *reinterpret_cast<const float4*>(p + 32 * t + 8 * q + 4 * h);
      v[t][4 * q] = x.x;
      v[t][4 * q + 1] = x.y;
      v[t][4 * q + 2] = x.z;
      v[t][4 * q + 3] = x.w;
    }
}

// Per-wave consumer of the stream (no LDS, no barrier): a tile's 16-B groups are one
// coalesced 1-KB row each; the first 4 groups of the NEXT tile are loaded while the current
// tile is multiplied, so each tile starts on operands already in registers and its other
// groups arrive (in order) behind them.
#ifndef PE_PRE
// 16-B groups of the next tile loaded during the current one (2 measured best of 1 / 2 / 4 / 8:
// the sampler batch 0.3 % faster than 4, 8 2.5 % slower; profiles/r06_prior_sched_ab.txt)
#define PE_PRE 2
#endif
struct PeStream {
  const float4* __restrict__ src;
  int64_t off;  // float4 offset of the current tile
  int idx, ntiles, depth, lane;
  float4 pre[PE_PRE];  // the current tile's first groups
};

__device__ __forceinline__ void pe_stream_begin(PeStream& st) {
  st.idx = 0;
  st.off = 0;
#pragma unroll
  for (int i = 0; i < PE_PRE; ++i) st.pre[i] = st.src[i * 64 + st.lane];
}

// acc += over NS MFMA steps t of the stream's current tile: (WA) A = W[row][kmap(t,h)],
// B = bv(t);  (!WA) A = bv(t), B = W[row][kmap(t,h)];  kmap(t,h) = 32*(t>>4) + crow(t&15, h).
template <bool WA, int NS, class BV>
__device__ __forceinline__ floatx16 pe_gemm(PeStream& st, BV bv, floatx16 acc) {
  constexpr int G = NS / 4;  // 16-B groups of the tile (>= 8)
  static_assert(G >= PE_PRE, "tile shorter than the prefetch");
  // wave-uniform tile offset in an SGPR: every load below is scalar base + the lane's
  // 16-byte slot + an immediate (no per-load address arithmetic on the VALU)
  const int off = __builtin_amdgcn_readfirstlane((int)st.off);
  const float4* cur = st.src + off;
  float4 rest[G - PE_PRE > 0 ? G - PE_PRE : 1];
#pragma unroll
  for (int i = 0; i < G - PE_PRE; ++i) rest[i] = cur[(PE_PRE + i) * 64 + st.lane];
  const int nidx = st.idx + 1;
  const int noff = off + G * 64;
  float4 nq[PE_PRE];
  if (nidx < st.ntiles) {
#pragma unroll
    for (int i = 0; i < PE_PRE; ++i) nq[i] = st.src[noff + i * 64 + st.lane];
  } else {
#pragma unroll
    for (int i = 0; i < PE_PRE; ++i) nq[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int T4 = 0; T4 < G; ++T4) {
    const float4 w4 = T4 < PE_PRE ? st.pre[T4] : rest[T4 - PE_PRE];
    const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float b = bv(4 * T4 + e);
      acc = WA ? pe_mfma(wv[e], b, acc) : pe_mfma(b, wv[e], acc);
    }
  }
#pragma unroll
  for (int i = 0; i < PE_PRE; ++i) st.pre[i] = nq[i];
  st.off = noff;
  st.idx = nidx;
  return acc;
}

// x-transformers RMSNorm (rmsnorm_fwd_kernel): x * (1 / max(|x|, 1e-12)) * sqrt(D) * g;
// g is folded into the packed weights of the Linears that read the norm (pe_tile), so only
// the per-token factor is applied here.
__device__ __forceinline__ void pe_rms(const floatx16 (&x)[4], floatx16 (&y)[4]) {
  float ss = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) ss = fmaf(x[t][r], x[t][r], ss);
  ss += __shfl_xor(ss, 32, 64);
  const float f = 1.0f / fmaxf(sqrtf(ss), 1e-12f) * sqrtf((float)PE_D);
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) y[t][r] = x[t][r] * f;
}

// 16 values of a per-feature vector for output tile ot: v[r] = p[32*ot + crow(r,h)]
__device__ __forceinline__ void pe_load_tile_vec(const float* __restrict__ p, int ot, int h,
                                                 floatx16& v) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 x = *reinterpret_cast<const float4*>(p + 32 * ot + 8 * q + 4 * h);
    v[4 * q] = x.x;
    v[4 * q + 1] = x.y;
    v[4 * q + 2] = x.z;
    v[4 * q + 3] = x.w;
  }
}

// y^T = W x^T + b (4 output tiles, K = 128); each tile's 16 bias values load while the
// tile's MFMAs run
__device__ __forceinline__ void pe_linear_bias(PeStream& st, const floatx16 (&x)[4],
                                               const float* __restrict__ bias, int h,
                                               floatx16 (&out)[4]) {
#pragma unroll
  for (int ot = 0; ot < 4; ++ot) {
    floatx16 bv, acc;
    pe_load_tile_vec(bias, ot, h, bv);
    pe_zero(acc);
    acc = pe_gemm<true, 64>(st, [&](int t) { return x[t >> 4][t & 15]; }, acc);
#pragma unroll
    for (int r = 0; r < 16; ++r) out[ot][r] = acc[r] + bv[r];
  }
}

// LayerNorm over the D features (layernorm_fwd_kernel): (x - mean) * rstd * w (+ b)
__device__ __forceinline__ void pe_layernorm(floatx16 (&x)[4], const float* __restrict__ w,
                                             const float* __restrict__ b, float eps, int h) {
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += x[t][r];
  s += __shfl_xor(s, 32, 64);
  const float mean = s / (float)PE_D;
  float v = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float d = x[t][r] - mean;
      v = fmaf(d, d, v);
    }
  v += __shfl_xor(v, 32, 64);
  const float rstd = 1.0f / sqrtf(v / (float)PE_D + eps);
  floatx16 wv[4], bv[4];
  pe_load_vec(w, h, wv);
  if (b) pe_load_vec(b, h, bv);
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float y = (x[t][r] - mean) * rstd * wv[t][r];
      if (b) y += bv[t][r];
      x[t][r] = y;
    }
}

// The tied logits + race of the one-wave kernel; the variants are compile-time so the
// product path (device noise, no logits copy) has no branch in its loop.  (Software-
// pipelining tile c + 1's MFMA chain against tile c's race in one basic block measured
// slower: 328 vs 317 us per launch, the extra live accumulator pushing values into AGPR
// moves.)  lout (tests): the logits.
template <bool INJ, bool LOUT>
__device__ __forceinline__ void pe_draw(PeStream& st, const floatx16 (&x)[4], RaceState& rs,
                                        const float* __restrict__ brow,
                                        const float* __restrict__ grow, uint32_t key,
                                        uint32_t ctr0, float* __restrict__ lout, bool store_ok,
                                        int K, int h) {
  auto bx = [&](int tt) { return x[tt >> 4][tt & 15]; };
  for (int c0 = 0; c0 < K; c0 += 32) {
    float v[16];  // the bias first: loads return in order, the stream prefetch comes next
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = brow[min(c0 + race_crow(r, h), K - 1)];
    floatx16 acc;
    pe_zero(acc);
    acc = pe_gemm<true, 64>(st, bx, acc);
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] += acc[r];
    if (LOUT) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int code = c0 + race_crow(r, h);
        if (store_ok && code < K) lout[code] = v[r];
      }
    }
    race_tile<INJ>(rs, v, c0, h, K, grow, key, ctr0);
  }
}

// one wave (64 threads) per sequence
__global__ __launch_bounds__(64) void prior_lf_eval_kernel(PriorArgs a,
                                                           const float4* __restrict__ wstream) {
  const int l = threadIdx.x & 63, r32 = l & 31, h = l >> 5;
  const bool seq_ok = true;
  const int b = blockIdx.x;
  const int n = a.n, ntok = a.n + 1;  // tokens incl. cls (<= 32)
  const bool live = r32 < ntok;
  PeStream st;
  st.src = wstream;
  st.ntiles = pe_ntiles(a.depth, a.K) - 4;  // project_in's tiles are folded into ftab
  st.depth = a.depth;
  st.lane = l;
  pe_stream_begin(st);
  // ---- project_in(embedding) from the folded tables: the cls row, then token + position
  // rows (zeros on the padding lanes)
  floatx16 x[4];
  {
    const int V = a.K + 1;
    const float* src;
    const float* pos = nullptr;
    if (r32 == 0) {
      const int64_t c = a.cls ? a.cls[b] : (int64_t)a.n_classes;
      src = a.ftab + (V + n + c) * PE_D;
    } else {
      const int i = live ? r32 - 1 : 0;
      src = a.ftab + a.s[(int64_t)b * a.ss + i] * PE_D;
      pos = a.ftab + (int64_t)(V + i) * PE_D;
    }
    pe_load_vec(src, h, x);
    if (pos) {
      floatx16 p[4];
      pe_load_vec(pos, h, p);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) x[t][r] += p[t][r];
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) x[t][r] = live ? x[t][r] : 0.f;
  }
  // ---- post_emb_norm (x-transformers LayerNorm: gamma only)
  pe_layernorm(x, a.post_gamma, nullptr, 1e-5f, h);
  // ---- encoder layers (pre-norm, eval: every branch runs)
  for (int li = 0; li < a.depth; ++li) {
    const PriorLayer L = a.L[li];
    floatx16 xn[4], y[4];
    // attention branch: y = concat_h(softmax(Q_h K_h^T / 8) V_h) W_o^T
    pe_rms(x, xn);  // g_attn folded into q / k / v
#pragma unroll
    for (int t = 0; t < 4; ++t) pe_zero(y[t]);
#pragma unroll
    for (int hd = 0; hd < 2; ++hd) {
      floatx16 q[2], k[2], v[2], s, o[2];
      auto bx = [&](int t) { return xn[t >> 4][t & 15]; };
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        pe_zero(q[u]);
        pe_zero(k[u]);
        pe_zero(v[u]);
        q[u] = pe_gemm<true, 64>(st, bx, q[u]);   // Q^T: token on the lane
        k[u] = pe_gemm<true, 64>(st, bx, k[u]);   // K^T: token on the lane
        v[u] = pe_gemm<false, 64>(st, bx, v[u]);  // V: feature on the lane
      }
      // S^T = K Q^T: lane = query, registers = keys crow(i, h)
      pe_zero(s);
#pragma unroll
      for (int t = 0; t < 32; ++t) s = pe_mfma(k[t >> 4][t & 15], q[t >> 4][t & 15], s);
      float mx = -INFINITY;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float sv = pe_crow(i, h) < ntok ? s[i] * 0.125f : -INFINITY;  // 64^-1/2
        s[i] = sv;
        mx = fmaxf(mx, sv);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      float sum = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float e = expf(s[i] - mx);
        s[i] = e;
        sum += e;
      }
      sum += __shfl_xor(sum, 32, 64);
      const float inv = 1.0f / sum;
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] *= inv;
      // O^T = V^T P^T: lane = query, registers = head features 32u + crow(r, h)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        pe_zero(o[u]);
#pragma unroll
        for (int t = 0; t < 16; ++t) o[u] = pe_mfma(v[u][t], s[t], o[u]);
      }
      // y += W_o[:, 64hd : 64hd + 64] O_h^T
#pragma unroll
      for (int ot = 0; ot < 4; ++ot)
        y[ot] = pe_gemm<true, 32>(st, [&](int t) { return o[t >> 4][t & 15]; }, y[ot]);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) x[t][r] = live ? y[t][r] + x[t][r] : 0.f;
    // feed-forward branch: y = W2 GELU(W1 xn + b1) + b2
    pe_rms(x, xn);  // g_ff folded into ff1
    floatx16 u[4];
    pe_linear_bias(st, xn, L.b1, h, u);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) u[t][r] = pe_gelu(u[t][r]);
    pe_linear_bias(st, u, L.b2, h, y);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) x[t][r] = live ? y[t][r] + x[t][r] : 0.f;
  }
  // ---- final_norm, project_out and pred_head: LayerNorm_{w,b}(GELU(RMSNorm(x) (W_p W_out)^T
  // + b_p)) (g_final folded into wc)
  {
    floatx16 xn[4], y[4];
    pe_rms(x, xn);
    pe_linear_bias(st, xn, a.bp, h, y);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) x[t][r] = pe_gelu(y[t][r]);
    pe_layernorm(x, a.ln_w, a.ln_b, a.ln_eps, h);
  }
  const int ldb = a.K + 1;
  if (a.sampled) {
    // ---- tied logits token-on-the-lane (the code tile as the A operand: registers = codes
    // crow(r, h)), drawn from by the race in registers (tvq_race.h); the cls lane and the
    // padding lanes run along and store nothing
    const int tok = r32;
    const bool tok_ok = tok >= 1 && tok <= n;
    const int64_t t = (int64_t)b * n + (tok_ok ? tok - 1 : 0);
    const float* brow = a.bias + (int64_t)(tok_ok ? tok - 1 : 0) * ldb;
    // every lane reads a valid row (t is clamped for the cls / padding lanes, which store
    // nothing): race_tile<true> dereferences it unconditionally
    const float* grow = a.gumbel ? a.gumbel + t * a.K : nullptr;
    const uint32_t key = a.gumbel ? 0u : race_key(mix_seed(a.seed_ptr, a.offset));
    // the variant is chosen on wave-uniform arguments only (the MFMA chains inside need every
    // lane); the cls / padding lanes' logits stores are predicated off inside
    float* lout = a.logits ? a.logits + t * a.K : nullptr;
    RaceState rs;
    race_init(rs);
    const uint32_t ctr0 = (uint32_t)t * (uint32_t)a.K;
    if (!a.gumbel && !a.logits)
      pe_draw<false, false>(st, x, rs, brow, nullptr, key, ctr0, nullptr, tok_ok, a.K, h);
    else if (!a.gumbel)
      pe_draw<false, true>(st, x, rs, brow, nullptr, key, ctr0, lout, tok_ok, a.K, h);
    else if (!a.logits)
      pe_draw<true, false>(st, x, rs, brow, grow, key, ctr0, nullptr, tok_ok, a.K, h);
    else
      pe_draw<true, true>(st, x, rs, brow, grow, key, ctr0, lout, tok_ok, a.K, h);
    int pick;
    float p;
    race_finish(rs, pick, p);
    if (h == 0 && tok_ok) {
      const int64_t s0 = a.s[(int64_t)b * a.ss + tok - 1];
      const bool known = s0 != a.mask_id;
      a.sampled[t] = known ? s0 : (int64_t)pick;
      a.selp[t] = known ? INFINITY : p;
    }
    return;
  }
  // ---- tied logits: lane = code, registers = tokens crow(r, h); the cls row is dropped
  float* out = a.logits + (int64_t)b * n * a.K;
  for (int c0 = 0; c0 < a.K; c0 += 32) {
    const int code = c0 + r32;
    floatx16 acc;
    pe_zero(acc);
    acc = pe_gemm<false, 64>(st, [&](int t) { return x[t >> 4][t & 15]; }, acc);
    if (seq_ok && code < a.K) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int tok = pe_crow(r, h);
        if (tok >= 1 && tok <= n)
          out[(int64_t)(tok - 1) * a.K + code] = acc[r] + a.bias[(int64_t)(tok - 1) * ldb + code];
      }
    }
  }
}

}  // namespace tvq

using namespace tvq;

// bytes of the packed weight stream tvq_prior_lf_eval needs as its workspace
extern "C" int64_t tvq_prior_lf_eval_workspace(int64_t depth, int64_t K, int64_t n,
                                               int64_t n_classes) {
  if (depth < 1 || depth > PE_MAXDEPTH || K < 1 || n < 1 || n_classes < 0) return -1;
  const int64_t tiles64 = 4 + 20 * depth + 4 + (K + 31) / 32;  // 64-step tiles
  const int64_t stream = (tiles64 * 1024 + depth * 8 * 512) * 16;
  // + the folded tables + the composed head weight
  return stream + (K + 1 + n + n_classes + 1) * PE_D * 4 + PE_D * PE_D * 4;
}

static int prior_lf_eval_launch(PriorArgs& a, const int64_t* s, int64_t B, int64_t n,
                                int64_t s_stride, const int64_t* cls_idx, int64_t n_classes,
                                int64_t width, const float* const* weights, int64_t depth,
                                int64_t K, float ln_eps, void* workspace, bool ready,
                                tvq_stream_t stream, const char* name) {
  TVQ_CHECK_ARG(s && weights && B >= 1 && n >= 1 && n + 1 <= 32 && K >= 1 &&
                    width == PE_D && depth >= 1 && depth <= PE_MAXDEPTH && n_classes >= 0,
                "tvq_prior_lf_eval: unsupported shape (width 128, n + 1 <= 32, depth <= 8)");
  a.s = s; a.ss = s_stride; a.cls = cls_idx; a.n_classes = (int)n_classes;
  a.B = (int)B; a.n = (int)n; a.K = (int)K; a.depth = (int)depth;
  const float* const* w = weights;
  a.tok_emb = w[0]; a.pos_emb = w[1]; a.cls_emb = w[2]; a.w_in = w[3]; a.post_gamma = w[4];
  for (int i = 0; i < depth; ++i) {
    const float* const* p = w + PE_FIXED + PE_PER_LAYER * i;
    a.L[i] = {p[0], p[1], p[2], p[3], p[4], p[5], p[6], p[7], p[8], p[9]};
  }
  const float* const* t = w + PE_FIXED + PE_PER_LAYER * depth;
  a.g_final = t[0]; a.w_out = t[1]; a.wp = t[2]; a.bp = t[3]; a.ln_w = t[4]; a.ln_b = t[5];
  a.bias = t[6];
  a.ln_eps = ln_eps;
  for (int i = 0; i < PE_FIXED + PE_PER_LAYER * depth + PE_TAIL; ++i)
    TVQ_CHECK_ARG(w[i] != nullptr && ((uintptr_t)w[i] & 15) == 0,
                  "tvq_prior_lf_eval: weight pointers must be non-null and 16-byte aligned");
  TVQ_CHECK_ARG(workspace && ((uintptr_t)workspace & 15) == 0,
                "tvq_prior_lf_eval: workspace must be non-null and 16-byte aligned");
  const int ntiles = 4 + 28 * (int)depth + 4 + (int)((K + 31) / 32);
  hipStream_t st = (hipStream_t)stream;
  float4* ws = reinterpret_cast<float4*>(workspace);
  // (A two-wave-per-sequence form -- heads / feed-forward halves split over two waves, the
  // residual stream exchanged through LDS -- measured slower in round 4: sampler batch 5.86
  // vs 5.57 ms, 356 vs 327 us per launch; the LDS exchanges, barriers and the work both
  // waves repeat cost more than the second wave hides, the one-wave kernel's MFMA pipe
  // being ~64 % busy already (profiles/r04_prior_pmc.txt).  Removed in round 5.)
  const int64_t tiles64 = 4 + 20 * depth + 4 + (K + 31) / 32;  // as the workspace
  a.ftab = reinterpret_cast<float*>(ws + tiles64 * 1024 + depth * 8 * 512);
  a.wc = a.ftab + (K + 1 + n + n_classes + 1) * PE_D;  // 16-B aligned (PE_D floats per row)
  if (!ready) {  // weights -> folded tables, the composed head weight, packed stream
    hipLaunchKernelGGL(prior_fold_kernel, dim3((unsigned)(K + 1 + n + n_classes + 1)), dim3(128),
                       0, st, a);
    hipLaunchKernelGGL(prior_headfold_kernel, dim3(PE_D), dim3(PE_D), 0, st, a);
    hipLaunchKernelGGL(prior_pack_kernel, dim3((unsigned)(ntiles - 4)), dim3(256), 0, st, a, ws, 4);
  }
  hipLaunchKernelGGL(prior_lf_eval_kernel, dim3((unsigned)B), dim3(64), 0, st, a,
                     (const float4*)ws);
  TVQ_PLAN("prior_lf_eval waves=1");
  return launch_status(name);
}

extern "C" int tvq_prior_lf_eval(const int64_t* s, int64_t B, int64_t n, int64_t s_stride,
                                 const int64_t* cls_idx, int64_t n_classes, int64_t width,
                                 const float* const* weights, int64_t depth, int64_t K,
                                 float ln_eps, float* logits, void* workspace,
                                 tvq_stream_t stream) {
  TVQ_CHECK_ARG(logits, "tvq_prior_lf_eval: null logits");
  PriorArgs a = {};
  a.logits = logits;
  return prior_lf_eval_launch(a, s, B, n, s_stride, cls_idx, n_classes, width, weights, depth, K,
                              ln_eps, workspace, false, stream, "tvq_prior_lf_eval");
}

extern "C" int tvq_prior_lf_eval_sample(const int64_t* s, int64_t B, int64_t n, int64_t s_stride,
                                        const int64_t* cls_idx, int64_t n_classes, int64_t width,
                                        const float* const* weights, int64_t depth, int64_t K,
                                        float ln_eps, int64_t mask_id, const float* gumbel,
                                        const int64_t* seed_ptr, uint64_t offset,
                                        int64_t* sampled, float* selp, float* logits,
                                        void* workspace, int64_t workspace_ready,
                                        tvq_stream_t stream) {
  TVQ_CHECK_ARG(sampled && selp, "tvq_prior_lf_eval_sample: null outputs");
  TVQ_CHECK_ARG(gumbel || seed_ptr, "tvq_prior_lf_eval_sample: need gumbel noise or a seed");
  TVQ_CHECK_ARG(gumbel || B * n * K < (int64_t)1 << 32, "tvq_prior_lf_eval_sample: B n K >= 2^32");
  PriorArgs a = {};
  a.logits = logits;
  a.mask_id = mask_id; a.gumbel = gumbel; a.seed_ptr = seed_ptr; a.offset = offset;
  a.sampled = sampled; a.selp = selp;
  TVQ_PLAN("prior_lf_eval_sample B=%lld n=%lld K=%lld", (long long)B, (long long)n, (long long)K);
  return prior_lf_eval_launch(a, s, B, n, s_stride, cls_idx, n_classes, width, weights, depth, K,
                              ln_eps, workspace, workspace_ready != 0, stream,
                              "tvq_prior_lf_eval_sample");
}

// x-transformers attention (bidirectional_transformer.py:92-110: heads x dim_head 64,
// softmax(Q K^T * scale), attention dropout) on the v_mfma_f32_32x32x2_f32 matrix cores.
//
// Sequences are short (LF 25, HF 97 tokens: the token counts do not depend on T), so a
// (batch, head) is padded to NT = ceil(S/32) tiles of 32 and handled whole: scores and
// probabilities live in registers, never in HBM.  Q/K/V/O/dO are read in the Linear
// layout [(b*S + s) * ld + h*64 + d] (no head transposes).
//
// Fragment maps (32x32x2 f32; lane l, r32 = l & 31, h = l >> 5; C/D register i holds
// row (i&3) + 8(i>>2) + 4h, column r32):
//   * a "row fragment" of a [rows][64] operand gives lane l row r32 and, at MFMA step t,
//     d = 32h + t: each lane reads 32 contiguous floats (the d order is permuted; the sum
//     over d is unchanged up to fp32 rounding order).
//   * forward: S^T = K Q^T (A = K rows, B = Q rows) puts one query per lane and its keys
//     in the 16 accumulator registers, so the softmax is a register reduction plus one
//     xor-32 shuffle, and P is already the A operand of P V (step = register i, key =
//     row(i, h)): no LDS at all.
//   * backward: S = Q K^T and dP = dO V^T (query in registers, key on the lane) feed
//     dV += P^T dO and dK += dS^T Q with no data movement; dQ = dS K needs the key on
//     the register side, so dS goes through LDS once (padded pitch, conflict-free).
//     Wave w of a (batch, head) group owns key tile w (dK, dV need no cross-wave sum),
//     then query tile w for dQ.
#include <float.h>
#include <math.h>

#include "tvq_common.h"

namespace tvq {

constexpr int ATT_DH = 64;

struct AttnArgs {
  const float* q; const float* k; const float* v;
  int64_t ldq, ldk, ldv;
  float* o; int64_t ldo;
  float* lse;  // [B*H*S]
  int B, H, S;
  float scale;
  float drop_p;
  const int64_t* seed_ptr;
  uint64_t offset;
};

struct AttnBwdArgs {
  AttnArgs f;
  const float* out; int64_t ldout;  // forward output O (for D_i = dO_i . O_i)
  const float* dout; int64_t ldd;
  float* dq; float* dk; float* dv; int64_t ldg;  // grads in the Q/K/V layout, stride ldg
};

__device__ __forceinline__ bool attn_keep(uint64_t seed, int64_t bh, int S, int i, int j, float p) {
  return uniform01(seed, ((uint64_t)bh * S + i) * S + j) >= p;
}

__device__ __forceinline__ floatx16 mfma32(float a, float b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int crow(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// 32 contiguous floats of row `row` (d = 32h .. 32h+31 of the head), zeros when row >= S
__device__ __forceinline__ void load_row_frag(float (&f)[32], const float* base, int64_t ld,
                                              int64_t row0, int row, int S, int h) {
  if (row < S) {
    const float* p = base + (row0 + row) * ld + 32 * h;
#pragma unroll
    for (int t = 0; t < 32; t += 4) {
      const float4 v = *(const float4*)(p + t);
      f[t] = v.x; f[t + 1] = v.y; f[t + 2] = v.z; f[t + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int t = 0; t < 32; ++t) f[t] = 0.f;
  }
}

__device__ __forceinline__ void zero16(floatx16& a) {
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = 0.f;
}

// one wave = one (batch*head, 32-query tile); 4 waves per block
template <int NT>
__global__ __launch_bounds__(256) void attention_fwd_kernel(AttnArgs a) {
  const int lane = threadIdx.x & 63, r32 = lane & 31, h = lane >> 5;
  const int item = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= a.B * a.H * NT) return;
  const int bh = item / NT, qt = item - bh * NT;
  const int b = bh / a.H, hh = bh - b * a.H;
  const int S = a.S;
  const int64_t row0 = (int64_t)b * S;
  const float* qb = a.q + hh * ATT_DH;
  const float* kb = a.k + hh * ATT_DH;
  const float* vb = a.v + hh * ATT_DH;
  const int q = qt * 32 + r32;  // this lane's query

  float qf[32], kf[32];
  load_row_frag(qf, qb, a.ldq, row0, q, S, h);
  floatx16 sc[NT];
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
    load_row_frag(kf, kb, a.ldk, row0, kt * 32 + r32, S, h);
    zero16(sc[kt]);
#pragma unroll
    for (int t = 0; t < 32; ++t) sc[kt] = mfma32(kf[t], qf[t], sc[kt]);
  }
  // softmax over keys: registers (keys crow(i,h) + 32kt) and the partner half (xor 32)
  float mx = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < NT; ++kt)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = kt * 32 + crow(i, h);
      const float s = key < S ? sc[kt][i] * a.scale : -INFINITY;
      sc[kt][i] = s;
      mx = fmaxf(mx, s);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int kt = 0; kt < NT; ++kt)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float e = expf(sc[kt][i] - mx);
      sc[kt][i] = e;
      sum += e;
    }
  sum += __shfl_xor(sum, 32, 64);
  const float inv = 1.0f / sum;
  if (h == 0 && q < S) a.lse[(int64_t)bh * S + q] = mx + logf(sum);
  const bool drop = a.drop_p > 0.f;
  const uint64_t seed = drop ? mix_seed(a.seed_ptr, a.offset) : 0ull;
  const float dscale = drop ? 1.0f / (1.0f - a.drop_p) : 1.0f;
#pragma unroll
  for (int kt = 0; kt < NT; ++kt)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float p = sc[kt][i] * inv;
      if (drop) {
        const int key = kt * 32 + crow(i, h);
        p = (q < S && key < S && attn_keep(seed, bh, S, q, key, a.drop_p)) ? p * dscale : 0.f;
      }
      sc[kt][i] = p;
    }
  // O = P V: A = P (query on the lane, key = crow(i, h) at step i), B = V[key][d]
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    floatx16 o;
    zero16(o);
#pragma unroll
    for (int kt = 0; kt < NT; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        int key = kt * 32 + crow(i, h);
        key = key < S ? key : S - 1;  // its probability is 0
        const float vv = vb[(row0 + key) * a.ldv + dt * 32 + r32];
        o = mfma32(sc[kt][i], vv, o);
      }
    // D rows = queries crow(i, h) of the tile, column = d
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int qq = qt * 32 + crow(i, h);
      if (qq < S) a.o[(row0 + qq) * a.ldo + hh * ATT_DH + dt * 32 + r32] = o[i];
    }
  }
}

// a group of NT waves = one (batch*head); wave w owns key tile w, then query tile w.
// LDS per group: dS [NT*32][NT*32 + 4], lse and D [NT*32].
template <int NT>
__global__ __launch_bounds__(256) void attention_bwd_kernel(AttnBwdArgs ab) {
  constexpr int G = NT == 1 ? 4 : 1;  // groups per block
  constexpr int SP = NT * 32;
  constexpr int PITCH = SP + 4;
  constexpr int GROUP_FLOATS = SP * PITCH + 2 * SP;
  extern __shared__ float sm[];
  const AttnArgs& a = ab.f;
  const int lane = threadIdx.x & 63, r32 = lane & 31, h = lane >> 5;
  const int wave = threadIdx.x >> 6;
  const int grp = wave / NT, w = wave - grp * NT;
  const int bh = blockIdx.x * G + grp;
  const bool live = bh < a.B * a.H;
  const int S = a.S;
  const int b = live ? bh / a.H : 0, hh = live ? bh - b * a.H : 0;
  const int64_t row0 = (int64_t)b * S;
  float* dSs = sm + grp * GROUP_FLOATS;
  float* Ls = dSs + SP * PITCH;
  float* Ds = Ls + SP;
  const float* qb = a.q + hh * ATT_DH;
  const float* kb = a.k + hh * ATT_DH;
  const float* vb = a.v + hh * ATT_DH;
  const float* ob = ab.out + hh * ATT_DH;
  const float* gb = ab.dout + hh * ATT_DH;

  float f0[32], f1[32];
  // prologue: D_q = dO_q . O_q and lse_q of query tile w
  if (live) {
    const int q = w * 32 + r32;
    load_row_frag(f0, gb, ab.ldd, row0, q, S, h);
    load_row_frag(f1, ob, ab.ldout, row0, q, S, h);
    float d = 0.f;
#pragma unroll
    for (int t = 0; t < 32; ++t) d = fmaf(f0[t], f1[t], d);
    d += __shfl_xor(d, 32, 64);
    if (h == 0) {
      Ds[q] = d;
      Ls[q] = q < S ? a.lse[(int64_t)bh * S + q] : 0.f;
    }
  }
  __syncthreads();
  if (live) {
    const bool drop = a.drop_p > 0.f;
    const uint64_t seed = drop ? mix_seed(a.seed_ptr, a.offset) : 0ull;
    const float dscale = drop ? 1.0f / (1.0f - a.drop_p) : 1.0f;
    const int key = w * 32 + r32;  // this lane's key (column of the S / dP tiles)
    float kf[32], vf[32];
    load_row_frag(kf, kb, a.ldk, row0, key, S, h);
    load_row_frag(vf, vb, a.ldv, row0, key, S, h);
    floatx16 dv[2], dk[2];
    zero16(dv[0]); zero16(dv[1]); zero16(dk[0]); zero16(dk[1]);
    for (int qt = 0; qt < NT; ++qt) {
      floatx16 s, dp;
      zero16(s);
      zero16(dp);
      load_row_frag(f0, qb, a.ldq, row0, qt * 32 + r32, S, h);
#pragma unroll
      for (int t = 0; t < 32; ++t) s = mfma32(f0[t], kf[t], s);
      load_row_frag(f1, gb, ab.ldd, row0, qt * 32 + r32, S, h);
#pragma unroll
      for (int t = 0; t < 32; ++t) dp = mfma32(f1[t], vf[t], dp);
      // P (dropped) and dS; register i: query qt*32 + crow(i, h), key `key`
      floatx16 pd, ds;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ql = qt * 32 + crow(i, h);
        float p = 0.f, g = 0.f;
        if (ql < S && key < S) {
          p = expf(s[i] * a.scale - Ls[ql]);
          float d = dp[i];
          float pp = p;
          if (drop) {
            const bool kp = attn_keep(seed, bh, S, ql, key, a.drop_p);
            pp = kp ? p * dscale : 0.f;
            d = kp ? d * dscale : 0.f;
          }
          g = p * (d - Ds[ql]);
          p = pp;
        }
        pd[i] = p;
        ds[i] = g;
        dSs[ql * PITCH + key] = g;
      }
      // dV += P^T dO, dK += dS^T Q: A = register i (k = query crow(i, h)), B = row gather
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int ql = qt * 32 + crow(i, h);
          const int qc = ql < S ? ql : S - 1;  // rows past S carry P = dS = 0
          const float go = gb[(row0 + qc) * ab.ldd + dt * 32 + r32];
          const float qv = qb[(row0 + qc) * a.ldq + dt * 32 + r32];
          dv[dt] = mfma32(pd[i], go, dv[dt]);
          dk[dt] = mfma32(ds[i], qv, dk[dt]);
        }
    }
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int kk = w * 32 + crow(i, h);
        if (kk < S) {
          const int64_t o = (row0 + kk) * ab.ldg + hh * ATT_DH + dt * 32 + r32;
          ab.dv[o] = dv[dt][i];
          ab.dk[o] = dk[dt][i] * a.scale;
        }
      }
  }
  __syncthreads();
  if (live) {
    // dQ for query tile w: A = dS[q][key] from LDS (key = kt*32 + 16h + s at step s),
    // B = K[key][d]
    const int q = w * 32 + r32;
    floatx16 dq[2];
    zero16(dq[0]);
    zero16(dq[1]);
#pragma unroll
    for (int kt = 0; kt < NT; ++kt) {
      float sv[16];
      const float* src = dSs + q * PITCH + kt * 32 + 16 * h;
#pragma unroll
      for (int s4 = 0; s4 < 16; s4 += 4) {
        const float4 v = *(const float4*)(src + s4);
        sv[s4] = v.x; sv[s4 + 1] = v.y; sv[s4 + 2] = v.z; sv[s4 + 3] = v.w;
      }
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          int kk = kt * 32 + 16 * h + s;
          kk = kk < S ? kk : S - 1;  // dS is 0 there
          dq[dt] = mfma32(sv[s], kb[(row0 + kk) * a.ldk + dt * 32 + r32], dq[dt]);
        }
    }
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qq = w * 32 + crow(i, h);
        if (qq < S) ab.dq[(row0 + qq) * ab.ldg + hh * ATT_DH + dt * 32 + r32] = dq[dt][i] * a.scale;
      }
  }
}

template <int NT>
static void launch_fwd(const AttnArgs& a, hipStream_t st) {
  const int items = a.B * a.H * NT;
  hipLaunchKernelGGL((attention_fwd_kernel<NT>), dim3((unsigned)((items + 3) / 4)), dim3(256), 0,
                     st, a);
}

template <int NT>
static void launch_bwd(const AttnBwdArgs& ab, hipStream_t st) {
  constexpr int G = NT == 1 ? 4 : 1;
  constexpr int SP = NT * 32;
  const size_t lds = (size_t)G * (SP * (SP + 4) + 2 * SP) * sizeof(float);
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)attention_bwd_kernel<NT>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    return true;
  }();
  (void)attr;
  const int groups = ab.f.B * ab.f.H;
  hipLaunchKernelGGL((attention_bwd_kernel<NT>), dim3((unsigned)((groups + G - 1) / G)),
                     dim3(64 * NT * G), lds, st, ab);
}

}  // namespace tvq

using namespace tvq;

static bool attn_ptr_ok(const void* p, int64_t ld) { return ((uintptr_t)p & 15) == 0 && (ld & 3) == 0; }

extern "C" int tvq_attention_fwd(const float* q, int64_t ldq, const float* k, int64_t ldk,
                                 const float* v, int64_t ldv, float* o, int64_t ldo, float* lse,
                                 int64_t B, int64_t H, int64_t S, int64_t Dh, float scale,
                                 float drop_p, const int64_t* seed_ptr, uint64_t offset,
                                 tvq_stream_t stream) {
  TVQ_CHECK_ARG(q && k && v && o && lse && B > 0 && H > 0, "tvq_attention_fwd: bad arguments");
  TVQ_CHECK_ARG(Dh == ATT_DH && S >= 1 && S <= 128, "tvq_attention_fwd: need Dh=64, S<=128");
  TVQ_CHECK_ARG(attn_ptr_ok(q, ldq) && attn_ptr_ok(k, ldk),
                "tvq_attention_fwd: q/k need 16-B aligned rows (ld % 4 == 0)");
  TVQ_CHECK_ARG(drop_p == 0.f || seed_ptr, "tvq_attention_fwd: dropout needs a seed");
  AttnArgs a;
  a.q = q; a.k = k; a.v = v; a.ldq = ldq; a.ldk = ldk; a.ldv = ldv;
  a.o = o; a.ldo = ldo; a.lse = lse;
  a.B = (int)B; a.H = (int)H; a.S = (int)S; a.scale = scale;
  a.drop_p = drop_p; a.seed_ptr = seed_ptr; a.offset = offset;
  hipStream_t st = (hipStream_t)stream;
  switch ((S + 31) / 32) {
    case 1: launch_fwd<1>(a, st); break;
    case 2: launch_fwd<2>(a, st); break;
    case 3: launch_fwd<3>(a, st); break;
    default: launch_fwd<4>(a, st); break;
  }
  return launch_status("tvq_attention_fwd");
}

extern "C" int tvq_attention_bwd(const float* q, int64_t ldq, const float* k, int64_t ldk,
                                 const float* v, int64_t ldv, const float* out, int64_t ldout,
                                 const float* dout, int64_t ldd,
                                 const float* lse, int64_t B, int64_t H, int64_t S, int64_t Dh,
                                 float scale, float drop_p, const int64_t* seed_ptr,
                                 uint64_t offset, float* dq, float* dk, float* dv, int64_t ldg,
                                 tvq_stream_t stream) {
  TVQ_CHECK_ARG(q && k && v && out && dout && lse && dq && dk && dv,
                "tvq_attention_bwd: bad arguments");
  TVQ_CHECK_ARG(Dh == ATT_DH && S >= 1 && S <= 128, "tvq_attention_bwd: need Dh=64, S<=128");
  TVQ_CHECK_ARG(attn_ptr_ok(q, ldq) && attn_ptr_ok(k, ldk) && attn_ptr_ok(v, ldv) &&
                    attn_ptr_ok(out, ldout) && attn_ptr_ok(dout, ldd),
                "tvq_attention_bwd: operands need 16-B aligned rows (ld % 4 == 0)");
  TVQ_CHECK_ARG(drop_p == 0.f || seed_ptr, "tvq_attention_bwd: dropout needs a seed");
  AttnBwdArgs ab;
  ab.f.q = q; ab.f.k = k; ab.f.v = v; ab.f.ldq = ldq; ab.f.ldk = ldk; ab.f.ldv = ldv;
  ab.f.o = nullptr; ab.f.ldo = 0; ab.f.lse = (float*)lse;
  ab.f.B = (int)B; ab.f.H = (int)H; ab.f.S = (int)S; ab.f.scale = scale;
  ab.f.drop_p = drop_p; ab.f.seed_ptr = seed_ptr; ab.f.offset = offset;
  ab.out = out; ab.ldout = ldout;
  ab.dout = dout; ab.ldd = ldd; ab.dq = dq; ab.dk = dk; ab.dv = dv; ab.ldg = ldg;
  hipStream_t st = (hipStream_t)stream;
  switch ((S + 31) / 32) {
    case 1: launch_bwd<1>(ab, st); break;
    case 2: launch_bwd<2>(ab, st); break;
    case 3: launch_bwd<3>(ab, st); break;
    default: launch_bwd<4>(ab, st); break;
  }
  return launch_status("tvq_attention_bwd");
}

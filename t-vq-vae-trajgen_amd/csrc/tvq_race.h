// Exponential-race sampling of one token's code from 32-code tiles of its logits held
// "token on the lane" (v_mfma_f32_32x32x2_f32 with the code table as the A operand: lane
// l holds token l & 31 and, in accumulator register r, code 32 c + crow(r, l >> 5) of
// tile c).  Shared by the fused sampling epilogues (tied_logits_sample_kernel for the HF
// prior, prior_lf_eval_kernel for the LF prior): the logits never reach HBM.
//
// Per token: the race argmax_k l_k + g_k (torch.multinomial's n_sample = 1 algorithm,
// tvq_common.h race_gumbel; ties to the lowest code), and p(pick) of the fp32 softmax --
// a running max with the exp terms of each tile summed in fp32 and rescaled / accumulated
// in double -- combined across the two lane halves at the end.
#pragma once
#include "tvq_common.h"

namespace tvq {

struct RaceState {
  float m;     // running max of the logits
  double s;    // sum of exp(l - m)
  float best;  // best race key
  float bl;    // its logit
  int bk;      // its code
};

__device__ __forceinline__ void race_init(RaceState& st) {
  st.m = -INFINITY;
  st.s = 0.0;
  st.best = -INFINITY;
  st.bl = -INFINITY;
  st.bk = 0x7fffffff;
}

__device__ __forceinline__ int race_crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// one tile's 16 logits v[r] = l(code0 + crow(r, h)), codes >= K masked out; noise from the
// injected row g (g[code], INJ) or the hash at counter ctr0 + code
template <bool INJ>
__device__ __forceinline__ void race_tile(RaceState& st, const float (&v)[16], int code0, int h,
                                          int K, const float* __restrict__ g, uint32_t key,
                                          uint32_t ctr0) {
  const bool full = code0 + 32 <= K;  // wave-uniform: no per-code guard on full tiles
  float tmax = -INFINITY;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int code = code0 + race_crow(r, h);
    const bool ok = full || code < K;
    // INJ: g must be a valid row for every lane; the index is clamped so no load (even a
    // speculated one) leaves the row
    const float noise = INJ ? g[ok ? code : 0] : race_gumbel(key, ctr0 + (uint32_t)code);
    const float rk = ok ? v[r] + noise : -INFINITY;
    tmax = fmaxf(tmax, ok ? v[r] : -INFINITY);
    if (rk > st.best) {  // codes increase along r and the tiles: the first of ties stays
      st.best = rk;
      st.bl = v[r];
      st.bk = code;
    }
  }
  // rescale to a new running max (an fp32 factor, like the terms)
  const float mn = fmaxf(st.m, tmax);
  st.s *= (double)(st.m > -INFINITY ? __expf(st.m - mn) : 1.0f);
  st.m = mn;
  float ts = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r)
    ts += (full || code0 + race_crow(r, h) < K) ? __expf(v[r] - st.m) : 0.f;
  st.s += (double)ts;
}

// merge another partial state of the same token into st (symmetric: both sides of a merge
// end with bitwise-equal states)
__device__ __forceinline__ void race_merge(RaceState& st, float om, double os, float ob,
                                           float obl, int ok) {
  const float M = fmaxf(st.m, om);
  const double a = st.m > -INFINITY ? st.s * exp((double)st.m - (double)M) : 0.0;
  const double c = om > -INFINITY ? os * exp((double)om - (double)M) : 0.0;
  st.s = a + c;  // fp addition commutes: both sides get the same bits
  st.m = M;
  if (ob > st.best || (ob == st.best && ok < st.bk)) {
    st.best = ob;
    st.bl = obl;
    st.bk = ok;
  }
}

// combine the lane halves (xor 32) into the token's state, in every lane
__device__ __forceinline__ void race_halves(RaceState& st) {
  const float om = __shfl_xor(st.m, 32, 64);
  const double os = __shfl_xor(st.s, 32, 64);
  const float ob = __shfl_xor(st.best, 32, 64);
  const float obl = __shfl_xor(st.bl, 32, 64);
  const int ok = __shfl_xor(st.bk, 32, 64);
  race_merge(st, om, os, ob, obl, ok);
}

__device__ __forceinline__ void race_result(const RaceState& st, int& pick, float& p) {
  pick = st.bk;
  p = (float)((double)__expf(st.bl - st.m) / st.s);
}

// combine the lane halves; every lane then holds the token's (pick, p(pick))
__device__ __forceinline__ void race_finish(RaceState& st, int& pick, float& p) {
  race_halves(st);
  race_result(st, pick, p);
}

}  // namespace tvq

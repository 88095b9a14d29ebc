/* TEST INFRASTRUCTURE ONLY — plain-C restatement of the reference VQ codebook.
 *
 * Follows timevqvae/models/vq.py (reference repo):
 *   vq.py:210-214  dist = -( sum(x^2) - 2 x.E^T + sum(E^2) )      (fp32, this order)
 *   vq.py:216-222  embed_ind = argmax(dist)  (temp 0 -> argmax, first index on ties)
 *   vq.py:225      quantize = E_old[embed_ind]
 *   vq.py:228-242  EMA: cs = cs*decay + n*(1-decay); ea = ea*decay + sum^T*(1-decay);
 *                  cs' = (cs+eps)/(sum(cs)+K*eps)*sum(cs); E = ea / cs'
 *   vq.py:246-247  perplexity = exp(-sum p log(p+1e-10)), p = counts/M
 * plus an fp64 top-2 distance gap per row, used by the tests to qualify
 * near-ties (an fp32 argmin can legitimately differ inside the rounding bound).
 *
 * Built by oracle/Makefile into oracle/build/libvq_ref.so; called via ctypes from
 * tests/ only.  Never linked into the product.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* x: (M, D) row-major; E: (K, D) row-major. */
void vqref_assign(const float *x, long M, long D, const float *E, long K,
                  int64_t *idx, float *dist_best, double *gap64) {
  float *ee = (float *)malloc(sizeof(float) * K);
  for (long k = 0; k < K; ++k) {
    float s = 0.f;
    for (long d = 0; d < D; ++d) s += E[k * D + d] * E[k * D + d];
    ee[k] = s;
  }
  for (long m = 0; m < M; ++m) {
    const float *xr = x + m * D;
    float xx = 0.f;
    for (long d = 0; d < D; ++d) xx += xr[d] * xr[d];
    float best = -INFINITY;
    long bi = 0;
    double b1 = INFINITY, b2 = INFINITY;
    for (long k = 0; k < K; ++k) {
      const float *er = E + k * D;
      float dot = 0.f;
      double dd = 0.0;
      for (long d = 0; d < D; ++d) {
        dot += xr[d] * er[d];
        double df = (double)xr[d] - (double)er[d];
        dd += df * df;
      }
      float dist = -((xx - 2.0f * dot) + ee[k]);
      if (dist > best) { best = dist; bi = k; }
      if (dd < b1) { b2 = b1; b1 = dd; } else if (dd < b2) { b2 = dd; }
    }
    idx[m] = bi;
    if (dist_best) dist_best[m] = best;
    if (gap64) gap64[m] = b2 - b1;
  }
  free(ee);
}

/* Training-mode EMA update, in place on cs (K), ea (K,D), E (K,D).
 * counts_out (K) receives the per-code counts of this batch. */
void vqref_ema(const float *x, const int64_t *idx, long M, long D, long K,
               float decay, float eps, float *cs, float *ea, float *E,
               float *counts_out, float *perplexity) {
  float *n = (float *)calloc(K, sizeof(float));
  float *s = (float *)calloc(K * D, sizeof(float));
  for (long m = 0; m < M; ++m) {
    long k = idx[m];
    n[k] += 1.f;
    for (long d = 0; d < D; ++d) s[k * D + d] += x[m * D + d];
  }
  const float a = 1.0f - decay; /* torch: alpha=(1-decay) in double -> float */
  float tot = 0.f;
  for (long k = 0; k < K; ++k) {
    cs[k] = fmaf(n[k], a, cs[k] * decay);
    for (long d = 0; d < D; ++d) ea[k * D + d] = fmaf(s[k * D + d], a, ea[k * D + d] * decay);
  }
  for (long k = 0; k < K; ++k) tot += cs[k];
  const float denom = tot + (float)K * eps;
  for (long k = 0; k < K; ++k) {
    float c = (cs[k] + eps) / denom * tot;
    for (long d = 0; d < D; ++d) E[k * D + d] = ea[k * D + d] / c;
  }
  float h = 0.f;
  for (long k = 0; k < K; ++k) {
    float p = n[k] / (float)M;
    h += p * logf(p + 1e-10f);
  }
  if (perplexity) *perplexity = expf(-h);
  if (counts_out) memcpy(counts_out, n, sizeof(float) * K);
  free(n);
  free(s);
}

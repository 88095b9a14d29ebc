/* TEST INFRASTRUCTURE ONLY — plain-C restatement of the reference ROCKET transform.
 *
 * Follows timevqvae/evaluation/rocket_functions.py (reference repo):
 *   :60-88   apply_kernel: output_length = L + 2p - (len-1)d; for i in [-p, L+p-(len-1)d):
 *            s = bias + sum_j w[j] * X[i + j d] over in-range indices (zero padding);
 *            max over i, ppv = count(s > 0) / output_length
 *   :91-126  apply_kernels: features [ppv_k, max_k] per kernel, 2 per kernel, kernels in
 *            order, weights packed back to back (offset = prefix sum of lengths)
 * float64 throughout, sums in j order without contraction (numba's fastmath may fuse or
 * reassociate; the tests' tolerances allow for it).  `threads` > 1 splits the examples
 * over pthreads (the reference's prange) for the CPU baseline.
 *
 * Built by oracle/Makefile into oracle/build/librocket_ref.so; called via ctypes from
 * tests/ and bench tooling only.  Never linked into the product.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>

typedef struct {
  const double* X;
  int64_t n, L, ldx;
  const double* w;
  const int32_t* len;
  const double* bias;
  const int32_t* dil;
  const int32_t* pad;
  int64_t nk;
  double* out;
  int64_t e0, e1;
} Job;

static void run(const Job* j) {
  for (int64_t e = j->e0; e < j->e1; ++e) {
    const double* x = j->X + e * j->ldx;
    int64_t a1 = 0;
    for (int64_t k = 0; k < j->nk; ++k) {
      const int len = j->len[k], d = j->dil[k], p = j->pad[k];
      const double* w = j->w + a1;
      const int64_t olen = (j->L + 2 * p) - (int64_t)(len - 1) * d;
      const int64_t end = (j->L + p) - (int64_t)(len - 1) * d;
      int64_t ppv = 0;
      double mx = -INFINITY;
      for (int64_t i = -p; i < end; ++i) {
        double s = j->bias[k];
        int64_t idx = i;
        for (int t = 0; t < len; ++t) {
          if (idx > -1 && idx < j->L) s = s + w[t] * x[idx];
          idx += d;
        }
        if (s > mx) mx = s;
        if (s > 0) ppv += 1;
      }
      j->out[e * 2 * j->nk + 2 * k] = (double)ppv / (double)olen;
      j->out[e * 2 * j->nk + 2 * k + 1] = mx;
      a1 += len;
    }
  }
}

static void* trun(void* a) {
  run((const Job*)a);
  return NULL;
}

void rocketref_apply(const double* X, int64_t n, int64_t L, int64_t ldx, const double* w,
                     const int32_t* len, const double* bias, const int32_t* dil,
                     const int32_t* pad, int64_t nk, double* out, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  Job jobs[256];
  pthread_t th[256];
  const int64_t per = (n + threads - 1) / threads;
  int started = 0;
  for (int t = 0; t < threads; ++t) {
    Job jb = {X, n, L, ldx, w, len, bias, dil, pad, nk, out, t * per, (t + 1) * per};
    if (jb.e0 >= n) break;
    if (jb.e1 > n) jb.e1 = n;
    jobs[t] = jb;
    if (threads == 1) {
      run(&jobs[t]);
    } else {
      pthread_create(&th[t], NULL, trun, &jobs[t]);
    }
    ++started;
  }
  if (threads > 1)
    for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
}

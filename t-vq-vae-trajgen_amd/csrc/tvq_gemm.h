// Shared between the generic staged GEMM (tvq_gemm.hip) and the skinny-GEMM family
// (tvq_gemm_skinny.hip) behind tvq_gemm.
#pragma once
#include "tvq_common.h"

namespace tvq {

struct GemmArgs {
  const float* A;
  const float* B;
  float* C;
  int M, N, K;
  int64_t sam, sak, sbk, sbn, ldc;
  const float* bias;
  const float* R;
  int64_t ldr;
  int64_t rmod;    // R row = m % rmod when > 0 (per-position bias broadcast over the batch)
  float* pre;      // optional: pre-activation output (ldc layout), for the GELU backward
  int act;         // 0 none, 1 GELU(erf)
  const float* gate;  // optional device scalar: the (activated) result times *gate, before
                      // R / accumulate (x-transformers layer dropout: keep = 0 or 1)
  int accumulate;  // C += result
  float alpha;
  int kper;        // K range per split
  float* slab;     // split-K partials [split][M][N] (nullptr: write C directly)
  int* cnt;        // split-K: one counter per (m, n) tile -> the last split block finishes
};

// XCD-aware tile map for a grid of xcd_grid(mt, nt) blocks: block b runs on XCD b % 8, so
// the nt column tiles of one row tile are given to blocks b, b + 8, ..., b + 8 (nt - 1):
// one XCD, consecutive in its dispatch order, so the row tile's A rows are fetched into
// that XCD's L2 once and re-read from it (a row-major grid spreads them over all eight
// L2s and re-streams A nt times).  Row tiles are padded to a multiple of 8; blocks with
// *mt >= mtiles have nothing to do.
static inline unsigned xcd_grid(int mtiles, int ntiles) {
  return (unsigned)(((mtiles + 7) / 8) * 8 * ntiles);
}
__device__ __forceinline__ void xcd_tile(int b, int ntiles, int* mt, int* nt) {
  const int x = b & 7, l = b >> 3;
  *mt = (l / ntiles) * 8 + x;
  *nt = l - (l / ntiles) * ntiles;
}

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f));
}

// Launches the skinny MFMA kernel for `g` when its strides / sizes fit one
// (tvq_gemm_skinny.hip); false: the caller uses the generic path.
bool gemm_skinny(const GemmArgs& g, hipStream_t stream);

// Direct-operand kernels (tvq_gemm_direct.hip), offered every call first; `ws` holds
// gemm_direct_splits(M, N, K) * M * N floats when that is > 1.
bool gemm_direct(GemmArgs g, float* ws, hipStream_t stream);
int gemm_direct_splits(int64_t M, int64_t N, int64_t K);

}  // namespace tvq

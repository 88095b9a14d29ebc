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
  int accumulate;  // C += result
  float alpha;
  int kper;        // K range per split
  float* slab;     // split-K partials [split][M][N] (nullptr: write C directly)
  int* cnt;        // split-K: one counter per (m, n) tile -> the last split block finishes
};

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f));
}

// Launches the skinny MFMA kernel for `g` when its strides / sizes fit one
// (tvq_gemm_skinny.hip); false: the caller uses the generic path.
bool gemm_skinny(const GemmArgs& g, hipStream_t stream);

}  // namespace tvq

// Internal (non-ABI) entry points of the conv engine used by other kernel files.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tvq {
// Deterministic split sum of a weight-gradient slab slab[s][n][kcols] (s < splits) into
// dw[n][kcols-1] (+ db[n] from the last column when db != null); batched into the open
// tvq_conv_wgrad_defer scope when there is one.  reduce_rows_scratch(splits, N*kcols)
// floats of scratch must follow the slab.
void conv_wgrad_finish(float* slab, int splits, int64_t N, int64_t kcols, float* dw, float* db,
                       int accumulate, hipStream_t st);
// out[0..N) (+)= sum of P contiguous rows of `in` -- a parameter gradient the optimizer
// alone reads (norm weights): batched into the open deferral scope when the scope takes
// it, else reduce_rows now (scratch: reduce_rows_scratch(P, N) floats)
void param_rows_finish(const float* in, int64_t P, int64_t N, float* out, int accumulate,
                       float* scratch, hipStream_t st);
// A weight's (n, c, tap) view (element w[n*wsn + c*wsc + tap]) packed [tap][c][n] from the
// open pack-cache scope, else into ws (N*C*KK floats), else unpacked when ws is null; the
// returned pointer's strides (n, c, tap) go to *sn, *sc, *st.
const float* conv_pack_view(const float* w, int N, int C, int KK, int64_t wsn, int64_t wsc,
                            float* ws, hipStream_t st, int64_t* sn, int64_t* sc, int64_t* stp);
}  // namespace tvq

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
// Two 3x3 weight (+ bias) gradients of one (B, C, 3, 8) -> N shape in one launch (the fused LF
// ResBlock's pair); false (nothing launched) when the shape is not conv_wgrad_w8's.
// ws0 / ws1: tvq_conv_workspace(4, ...) floats each, alive until the deferral scope's flush.
bool conv_wgrad_w8_pair(const float* x0, const float* dy0, float* ws0, float* dw0, float* db0,
                        const float* x1, const float* dy1, float* ws1, float* dw1, float* db1,
                        int64_t B, int64_t C, int64_t N, int accumulate, hipStream_t st);
// n <= 4 such gradients on (B, C, 3, 16) maps in one launch (the fused RB<32, 16> ResBlocks),
// each into its own conv_wgrad_w16_slab_floats slab, summed by the deferral scope's flush.
bool conv_wgrad_w8_fits(int64_t B, int64_t C, int64_t N);
void conv_wgrad_w8_multi(int n, const float* const* x, const float* const* dy, float* const* ws,
                         float* const* dw, float* const* db, int64_t B, int64_t C, int64_t N,
                         int accumulate, hipStream_t st);
bool conv_wgrad_w16_fits(int64_t B, int64_t C, int64_t N);
int64_t conv_wgrad_w16_slab_floats(int64_t B, int64_t C, int64_t N);
void conv_wgrad_w16_multi(int n, const float* const* x, const float* const* dy, float* const* ws,
                          float* const* dw, float* const* db, int64_t B, int64_t C, int64_t N,
                          int accumulate, hipStream_t st);
}  // namespace tvq

/* tvq.h — C ABI of libtvq_hip.so, the gfx950 (MI355X) hot path of TimeVQVAE.
 *
 * The reference (SynthAIr/T-VQ-VAE-TrajGen) is pure Python/PyTorch and has no
 * FFI; its boundary is the nn.Module API of timevqvae.models.{vq,vq_vae,
 * maskgit,bidirectional_transformer}.  This header is the thin C layer BELOW that
 * API: the product's Python modules (t-vq-vae-trajgen_amd/timevqvae) keep the
 * reference signatures and call these entry points through ctypes.  Each entry
 * cites the reference operation it replaces (paths relative to the reference
 * repo root).
 *
 * Conventions
 *   - raw device pointers, element counts/strides in elements, fp32 data,
 *     int64 indices (torch.long);
 *   - every call is asynchronous on `stream` (a hipStream_t; pass torch's current
 *     stream), performs no allocation and no host synchronisation, and is
 *     therefore capturable into a hipGraph;
 *   - return 0 (TVQ_OK) or a negative status; tvq_last_error() gives the message
 *     (thread-local).
 */
#ifndef TVQ_H
#define TVQ_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TVQ_OK 0
#define TVQ_ERR_ARG -1
#define TVQ_ERR_LAUNCH -2

typedef void* tvq_stream_t; /* hipStream_t */

const char* tvq_last_error(void);
int tvq_abi_version(void);

/* ---------------------------------------------------------------- VQ codebook
 * Replaces EuclideanCodebook.forward (timevqvae/models/vq.py:197-251) and the
 * straight-through + commitment loss of VectorQuantize.forward (vq.py:357-366).
 * x is (B,N,D) with arbitrary element strides (sB,sN,sD): quantize() passes the
 * 'b c h w -> b (h w) c' VIEW of the NCHW latent (train_utils.py:338-358) so no
 * transpose is materialised; `quant` is written with the same strides.
 */

/* ee[k] = sum_d E[k,d]^2 (vq.py:213). E: (K,D) row-major. */
int tvq_vq_sqnorm(const float* E, int64_t K, int64_t D, float* ee, tvq_stream_t stream);

/* Number of per-block commit partials tvq_vq_assign writes (workspace size). */
int64_t tvq_vq_assign_nblocks(int64_t M);

/* dist = -((sum x^2 - 2 x.E^T) + ee) (vq.py:210-214), idx = argmax (first index
 * on ties, vq.py:216-222), q = E[idx] with the pre-update codebook (vq.py:225).
 * training!=0: quant = x + (q - x) (straight-through value, vq.py:358) and
 * commit_partial[blk] = sum (quant - x)^2 over the block's rows (vq.py:364);
 * training==0: quant = q, commit_partial may be NULL.
 * D must be one of 32, 64, 128. */
int tvq_vq_assign(const float* x, int64_t B, int64_t N, int64_t D, int64_t sB, int64_t sN,
                  int64_t sD, const float* E, const float* ee, int64_t K, int training,
                  float* quant, int64_t* idx, int32_t* idx32, float* commit_partial,
                  tvq_stream_t stream);

/* Per-code batch statistics, deterministic (no float atomics): counts[k] (int32),
 * cs_batch[k] = counts (float) = onehot.sum(0) (vq.py:228) and, if es_batch is
 * non-NULL, es_batch[k,:] = sum of rows assigned to k = (x^T onehot)^T (vq.py:233),
 * summed in row order.  es_batch: (K,D) row-major. */
int tvq_vq_stats(const float* x, int64_t B, int64_t N, int64_t D, int64_t sB, int64_t sN,
                 int64_t sD, const int32_t* idx32, int64_t K, int32_t* counts, float* cs_batch,
                 float* es_batch, tvq_stream_t stream);

/* EMA blend in place (vq.py:231,236 ema_inplace):
 *   cluster_size = cluster_size*decay + cs_batch*(1-decay)
 *   embed_avg    = embed_avg*decay    + es_batch*(1-decay)
 * (cs_batch/es_batch may have been all-reduced across ranks in between,
 *  vq.py:229,234 — the reference's sync_codebook hook). */
int tvq_vq_ema(const float* cs_batch, const float* es_batch, int64_t K, int64_t D, float decay,
               float* cluster_size, float* embed_avg, tvq_stream_t stream);

/* Laplace-smoothed normalisation (vq.py:237-242):
 *   embed = embed_avg / ((cs+eps)/(sum cs + K*eps) * sum cs)
 * plus perplexity = exp(-sum p log(p+1e-10)), p = counts/M (vq.py:246-247), and,
 * when commit_partial != NULL, commit = sum(partials)/(M*D) (F.mse_loss mean).
 * Any of embed_avg/embed may be NULL to skip the normalisation (eval mode). */
int tvq_vq_finalize(const float* cluster_size, const float* embed_avg, int64_t K, int64_t D,
                    float eps, float* embed, const int32_t* counts, int64_t M,
                    float* perplexity, const float* commit_partial, int64_t nparts,
                    float* commit, tvq_stream_t stream);

/* Backward of the straight-through + commitment loss (vq.py:358,364) over n
 * densely-stored elements sharing one layout:
 *   dx = dquant + (2*gcommit[0]/numel) * (x - quant) */
int tvq_vq_backward(const float* x, const float* quant, const float* dquant,
                    const float* gcommit, int64_t n, int64_t numel, float* dx,
                    tvq_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* TVQ_H */

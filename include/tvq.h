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
/* Source stamp compiled in by csrc/Makefile: the first 16 hex digits of the sha1 of every
 * csrc *.hip / *.h (sorted by name) followed by include/tvq.h.  The same 16 digits follow the
 * literal "tvq_source_hash=" in the library file, so a loader can read the stamp without
 * mapping the library. */
const char* tvq_source_hash(void);
/* The EXTRA build defines the library was compiled with (A/B builds; "" by default).  Kept
 * out of the source stamp so an A/B build still names the sources it came from. */
const char* tvq_build_extra(void);
/* Register a zeroed pool of n int32 counters on `device` (a HIP device index).  The
 * kernels that finish a grid-level reduction in their last-arriving block (BatchNorm /
 * Snake statistics, column sums, split-K slabs) take slots from it and leave them
 * zero.  Without a pool, those reductions use a separate finishing launch (same
 * result).  Call before the first launch on that device, outside graph capture. */
int tvq_counter_pool(int64_t device, int32_t* zeroed, int64_t n);
/* Bracket a hipGraph capture (begin = 1 / 0): slots taken inside are pinned for the
 * process lifetime (a graph replays with its capture-time slots), taken from the top
 * half of the pool, which eager launches never use. */
int tvq_counter_capture(int64_t begin);
/* Step glue (no reference counterpart; replaces the PyTorch elementwise launches a step
 * graph held): p[0..n) = value (FusedAdamW.zero_grad of the flat gradient buffer);
 * p[0] += value (the dropout seed advance of hip/rng.py); out = ((a + b) + c) + d and
 * out_ab = a + b elementwise over n floats, c / d / out / out_ab nullable (the logged loss
 * sums of stage1.py:170-198, maskgit.py:155-192). */
int tvq_fill(float* p, int64_t n, float value, tvq_stream_t stream);
int tvq_fill_i64(int64_t* p, int64_t n, int64_t value, tvq_stream_t stream);
/* p[0] = a and (q non-NULL) q[0] = b in one launch. */
int tvq_fill2(float* p, float a, float* q, float b, tvq_stream_t stream);
int tvq_add_i64(int64_t* p, int64_t value, tvq_stream_t stream);
int tvq_sum4(const float* a, const float* b, const float* c, const float* d, float* out,
             float* out_ab, int64_t n, tvq_stream_t stream);
/* Dispatch trace (tests / diagnosis; no reference counterpart).  tvq_plan_trace(1) clears
 * the log and starts recording one line per launch decision of the host-side plans (conv
 * kernel variant and its K stage / split plan, fused ResBlock kernels, VQ assignment row
 * groups); tvq_plan_trace(0) stops.  tvq_plan_read copies the newline-separated log into
 * buf (NUL-terminated, at most cap-1 bytes) and returns its full length. */
int tvq_plan_trace(int64_t on);
int64_t tvq_plan_read(char* buf, int64_t cap);

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

/* Stochastic assignment (EuclideanCodebook.forward with svq_temp > 0, vq.py:216-222 via
 * softmax_sample vq.py:51-56): idx ~ Categorical(logits = dist / temp), drawn as Gumbel-max
 * argmax(dist/temp + g) in the same pass as tvq_vq_assign.  g = -log(-log u) with u from
 * the device seed (*seed_ptr, offset, m*K + k), or injected: gumbel (M, K) row-major, for
 * tests.  temp == 0 is tvq_vq_assign (deterministic argmax).  Other arguments as
 * tvq_vq_assign. */
int tvq_vq_assign_svq(const float* x, int64_t B, int64_t N, int64_t D, int64_t sB, int64_t sN,
                      int64_t sD, const float* E, const float* ee, int64_t K, int training,
                      float temp, const float* gumbel, const int64_t* seed_ptr, uint64_t offset,
                      float* quant, int64_t* idx, int32_t* idx32, float* commit_partial,
                      tvq_stream_t stream);
/* tvq_vq_assign_svq that, when training, also writes x token-major to token_rows
 * (M x D floats, row m = x[m / N, m % N, :]; NULL: not written), so that tvq_vq_stats
 * can read contiguous rows (pass token_rows with B = 1, N = M, sN = D, sD = 1) instead of
 * gathering D-strided elements of an NCHW latent. */
int tvq_vq_assign_rows(const float* x, int64_t B, int64_t N, int64_t D, int64_t sB, int64_t sN,
                       int64_t sD, const float* E, const float* ee, int64_t K, int training,
                       float temp, const float* gumbel, const int64_t* seed_ptr, uint64_t offset,
                       float* quant, int64_t* idx, int32_t* idx32, float* commit_partial,
                       float* token_rows, tvq_stream_t stream);

/* Per-code batch statistics, deterministic (no float atomics): a stable group-by
 * (counting sort) of idx32, then per-code row sums in row order.
 * counts[k] (int32), cs_batch[k] = counts (float) = onehot.sum(0) (vq.py:228) and, if
 * es_batch is non-NULL, es_batch[k,:] = (x^T onehot)^T (vq.py:233), (K,D) row-major.
 * workspace: tvq_vq_stats_workspace(M, K) int32s. */
int64_t tvq_vq_stats_workspace(int64_t M, int64_t K);
int tvq_vq_stats(const float* x, int64_t B, int64_t N, int64_t D, int64_t sB, int64_t sN,
                 int64_t sD, const int32_t* idx32, int64_t K, int32_t* counts, float* cs_batch,
                 float* es_batch, int32_t* workspace, tvq_stream_t stream);

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


/* ------------------------------------------------------------ STFT / iSTFT
 * time_to_timefreq + zero_pad_{high,low}_freq(copy=True) + the stage1 targets
 * (train_utils.py:293-321,361-386; vq_vae.py:179-180; stage1.py:101-113) in one
 * pass: x (B,C,T) -> raw (B,2C,3,T+1) = time_to_timefreq(x), enc_l/enc_h the
 * band-copied encoder inputs, tgt_l/tgt_h (B,C,T) = interp(istft(band(stft(x))));
 * any output may be NULL. */
int tvq_stft_encode(const float* x, int64_t B, int64_t C, int64_t T, float* raw, float* enc_l,
                    float* enc_h, float* tgt_l, float* tgt_h, tvq_stream_t stream);

/* VQVAEDecoder tail (vq_vae.py:258-262): zero_pad band mask (band 0 = LF keeps
 * bin 0, 1 = HF keeps bins 1,2, 2 = none: plain timefreq_to_time) -> istft ->
 * nn.Upsample(Tout, 'linear') (identity when Tout == W-1).
 * h (B,2C,3,W) -> y (B,C,Tout).  bwd: dy (B,C,Tout) -> dh (B,2C,3,W). */
int tvq_istft_decode(const float* h, int64_t B, int64_t C, int64_t W, int64_t band, int64_t Tout,
                     float* y, tvq_stream_t stream);
int tvq_istft_decode_bwd(const float* dy, int64_t B, int64_t C, int64_t W, int64_t band,
                         int64_t Tout, float* dh, tvq_stream_t stream);

/* ----------------------------------------------------------- convolutions
 * nn.Conv2d / nn.ConvTranspose2d / nn.Conv1d of VQVAEEncBlock, ResBlock,
 * VQVAEDecBlock, the decoder tail and Upscale (vq_vae.py:13-121,238-251;
 * bidirectional_transformer.py:12-30).  NCHW fp32; supported kernels:
 * (KH,KW,SW) = (3,4,2) [replicate or zero pad], (3,3,1), (1,1,1), (1,3,1);
 * padding (KH/2, (KW-1)/2).  Epilogue of the forward conv: + bias, optional
 * dropout (counter-based mask keyed by (*seed_ptr, offset) and the flat output
 * index: the device seed advances once per step so graph replays differ) and + residual
 * (ResBlock: proj(x) + Dropout(conv(..)), vq_vae.py:52,62).
 * workspace: floats sized by tvq_conv_workspace(op, ...); nullable for the forward ops and
 * the non-replicate dgrads (then no weight repack and no split-K).  It holds the
 * replicate-pad canvas (dgrad), the tap-major repacked weight and split-K partials. */
int tvq_conv_out_width(int64_t Win, int64_t KW, int64_t SW, int64_t transposed);
/* engine selection (process-wide) bits: 1 = halo-tile kernel for fwd/dgrad convs with
 * few gathered channels (whose padded image and weight panel fit in 64 KB of LDS),
 * 2 = halo-tile weight gradient, 4 = halo-tile wherever it fits, 8 = no 32x32-MFMA
 * wide-channel tile, 16 / 32 = its K stage BK = 32 / 16 (default 64), 64 = its 4-wave
 * block (default 12 waves), 128 = its 64-channel variant for narrow maps (default off),
 * 256 = no direct small transposed-gather kernel, 512 = no stride-2 small-channel conv
 * kernels (conv_s2f / conv_s2t), 1024 = no stride-2 small-channel weight-gradient kernel,
 * 2048 = no few-output wide-input kernel (conv_n16: 128 -> <= 16 channels on (B, 128, 3, 32));
 * 0 forces the staged GEMMs (with the stride-2 kernels); < 0 only queries.  Default 3.
 * Returns the previous setting. */
int tvq_conv_config(int64_t halo);

/* Per-step weight-pack cache for the staged-GEMM convs (their weights are repacked to
 * [tap][c][n] on every call otherwise).  begin(id, arena, cap, stream) opens a scope: it
 * repacks every (weight, view) recorded under `id` into `arena` with a few batched
 * launches on `stream`; inside the scope a recorded weight is read from its arena slot and
 * a new one is packed into a fresh slot and recorded (arena full -> the per-call path).
 * Each id keeps its own entries (two graph segments with their own caches each repack only
 * their weights); beginning an id with another arena drops its entries, release(id) frees
 * them.  The weights must not change between begin and end (open it around
 * forward+backward, not the optimizer step); one scope is open at a time (process-wide
 * host state).  entries() = the last scope's recorded count. */
int tvq_conv_packcache_begin(int64_t id, float* arena, int64_t cap_floats, tvq_stream_t stream);
int tvq_conv_packcache_end(void);
int tvq_conv_packcache_release(int64_t id);
/* pause(1) / pause(0): convs between them bypass the open scope (weights computed inside it). */
int tvq_conv_packcache_pause(int64_t on);
int64_t tvq_conv_packcache_entries(void);

/* Deferred weight-gradient reductions: between begin() and flush(stream), the split sums
 * of tvq_conv2d_wgrad / tvq_convT2d_wgrad (<= 256 splits) are recorded instead of launched,
 * and flush() runs them all in a few batched launches on `stream` -- bit for bit the same
 * sums.  Until the flush the callers' workspaces must stay allocated and dw / db are not
 * final.  Process-wide host state, one scope at a time. */
int tvq_conv_wgrad_defer_begin(void);
int tvq_conv_wgrad_defer_flush(tvq_stream_t stream);
/* The same scope, recording only the reductions issued on `stream` -- the conv weight
 * gradients and the RMSNorm / LayerNorm weight gradients accumulated into a flat gradient
 * (tvq_rmsnorm_bwd / tvq_layernorm_bwd with accumulate = 1); those issued on other streams
 * run at once.  Flush on the same `stream`. */
int tvq_wgrad_defer_begin_stream(tvq_stream_t stream);
/* paused != 0: calls inside the scope reduce immediately (a gradient needed at once) */
int tvq_conv_wgrad_defer_pause(int64_t paused);
/* op: 0 conv2d fwd, 1 convT2d fwd, 2 conv2d dgrad, 3 convT2d dgrad, 4 conv2d wgrad,
 * 5 convT2d wgrad; (Ci, Co, Wi) = the layer's input channels, output channels, input
 * width.  Returns the workspace size in floats (>= 1), -1 for a bad op. */
int64_t tvq_conv_workspace(int64_t op, int64_t B, int64_t Ci, int64_t H, int64_t Wi, int64_t Co,
                           int64_t KH, int64_t KW, int64_t SW, int64_t replicate);
int tvq_conv2d_fwd(const float* x, int64_t B, int64_t Ci, int64_t H, int64_t Wi, const float* w,
                   const float* bias, int64_t Co, int64_t KH, int64_t KW, int64_t SW,
                   int64_t replicate, float* y, const float* residual, float drop_p,
                   const int64_t* seed_ptr, uint64_t offset, float* workspace,
                   tvq_stream_t stream);
int tvq_convT2d_fwd(const float* x, int64_t B, int64_t Ci, int64_t H, int64_t Wi, const float* w,
                    const float* bias, int64_t Co, int64_t KH, int64_t KW, int64_t SW, float* y,
                    const float* residual, float* workspace, tvq_stream_t stream);
/* Eval-mode conv (/ transposed conv) [-> GELU] -> BatchNorm2d from its running statistics
 * -> Snake (snake_a nullable) in one launch: VQVAEDecBlock.block / ResBlock.convs[1:4] /
 * Upscale's Conv1d -> GELU -> BN (pre_gelu = 1) while sampling (vq_vae.py:31-48,98-118,
 * bidirectional_transformer.py:37-52); tvq_conv2d_fwd / tvq_convT2d_fwd followed by
 * tvq_gelu_fwd and tvq_bn_eval_fwd up to the Snake's sin^2 evaluation (~1e-7 relative).
 * Shapes whose conv path has no fused epilogue run the eval BN as a second launch.
 * Workspace as the plain forward's. */
int tvq_conv2d_fwd_bn_eval(const float* x, int64_t B, int64_t Ci, int64_t H, int64_t Wi,
                           const float* w, const float* bias, int64_t Co, int64_t KH, int64_t KW,
                           int64_t SW, int64_t replicate, int64_t pre_gelu, const float* bn_w,
                           const float* bn_b,
                           const float* running_mean, const float* running_var, float eps,
                           const float* snake_a, float* y, float* workspace, tvq_stream_t stream);
int tvq_convT2d_fwd_bn_eval(const float* x, int64_t B, int64_t Ci, int64_t H, int64_t Wi,
                            const float* w, const float* bias, int64_t Co, int64_t KH, int64_t KW,
                            int64_t SW, const float* bn_w, const float* bn_b,
                            const float* running_mean, const float* running_var, float eps,
                            const float* snake_a, float* y, float* workspace,
                            tvq_stream_t stream);
int tvq_conv2d_dgrad(const float* dy, int64_t B, int64_t Co, int64_t H, int64_t Wo,
                     const float* w, int64_t Ci, int64_t KH, int64_t KW, int64_t SW,
                     int64_t replicate, float* dx, int64_t Wi, float* workspace,
                     tvq_stream_t stream);
int tvq_convT2d_dgrad(const float* dy, int64_t B, int64_t Co, int64_t H, int64_t Wo,
                      const float* w, int64_t Ci, int64_t KH, int64_t KW, int64_t SW, float* dx,
                      int64_t Wi, float* workspace, tvq_stream_t stream);
/* weight gradient (+ the bias gradient sum dY into db when non-NULL, as an extra
 * ones-column of the same GEMM); splits over positions reduced in a fixed order */
int tvq_conv2d_wgrad(const float* x, int64_t B, int64_t Ci, int64_t H, int64_t Wi,
                     const float* dy, int64_t Co, int64_t Wo, int64_t KH, int64_t KW, int64_t SW,
                     int64_t replicate, float* dw, float* db, int64_t accumulate, float* workspace,
                     tvq_stream_t stream);
int tvq_convT2d_wgrad(const float* x, int64_t B, int64_t Ci, int64_t H, int64_t Wi,
                      const float* dy, int64_t Co, int64_t Wo, int64_t KH, int64_t KW, int64_t SW,
                      float* dw, int64_t accumulate, float* workspace, tvq_stream_t stream);
/* bias gradients: out[c] (+)= sum_{b,p} x[b,c,p] */
int64_t tvq_channel_sum_workspace(int64_t B, int64_t C, int64_t HW);
int tvq_channel_sum(const float* x, int64_t B, int64_t C, int64_t HW, float* out,
                    int64_t accumulate, float* workspace, tvq_stream_t stream);

/* ------------------------------------------------ BatchNorm + SnakeActivation
 * nn.BatchNorm2d/1d (momentum 0.1) followed by SnakeActivation
 * x + (1/a) sin(a x)^2 (train_utils.py:421-448) when snake_a != NULL
 * (VQVAEEncBlock/DecBlock block.1-2, ResBlock convs.2-3).  fp64 statistics.
 * scale_shift: 2*C floats kept for the backward; workspace: tvq_bn_workspace bytes. */
int64_t tvq_bn_workspace(int64_t B, int64_t C, int64_t HW);
int tvq_bn_train_fwd(const float* x, int64_t B, int64_t C, int64_t HW, const float* w,
                     const float* b, float* running_mean, float* running_var,
                     int64_t* num_batches_tracked, float momentum, float eps,
                     const float* snake_a, float* y, float* save_mean, float* save_invstd,
                     float* scale_shift, void* workspace, tvq_stream_t stream);
int tvq_bn_eval_fwd(const float* x, int64_t B, int64_t C, int64_t HW, const float* w,
                    const float* b, const float* running_mean, const float* running_var,
                    float eps, const float* snake_a, float* y, float* scale_shift,
                    tvq_stream_t stream);
int tvq_bn_bwd(const float* dy, const float* x, int64_t B, int64_t C, int64_t HW, const float* w,
               const float* snake_a, const float* save_mean, const float* save_invstd,
               const float* scale_shift, float* dx, float* dw, float* db, float* da,
               int64_t accumulate, void* workspace, tvq_stream_t stream);
/* standalone Snake (ResBlock convs.0, vq_vae.py:31); a: (C,) */
int tvq_snake_fwd(const float* x, int64_t B, int64_t C, int64_t HW, const float* a, float* y,
                  tvq_stream_t stream);
int64_t tvq_snake_workspace(int64_t B, int64_t C, int64_t HW);
/* dx = Snake'(x) dy (+ dx_add, nullable: the ResBlock skip path's gradient of the same x,
 * summed here instead of by a separate autograd add); da (+)= its per-channel sum */
int tvq_snake_bwd(const float* dy, const float* x, int64_t B, int64_t C, int64_t HW,
                  const float* a, const float* dx_add, float* dx, float* da, int64_t accumulate,
                  void* workspace, tvq_stream_t stream);
/* backward of the dropout fused in tvq_conv2d_fwd (same seed, same flat index) */
int tvq_dropout_bwd(const float* dy, int64_t n, float p, const int64_t* seed_ptr,
                    uint64_t offset, float* dx, tvq_stream_t stream);

/* ---- fused ResBlock (vq_vae.py:13-62), C_in == C_out = C in {8,16,32}, H = 3,
 * W in {16,32,64}, C*W <= 1024 (csrc/tvq_resblock.hip), and C = 64, W = 8 (the LF band's
 * 64-channel maps, csrc/tvq_resblock_w8.hip: weights from L2, the weight gradients by the
 * image-batched tvq_conv2d_wgrad inside tvq_resblock_bwd):
 *   y = x + Dropout_p(conv2(Snake_a2(BN(conv1(Snake_a1(x)) + b1))) + b2)
 * replaces tvq_snake_fwd + tvq_conv2d_fwd + tvq_bn_train_fwd + tvq_conv2d_fwd(residual,
 * dropout) and their backward.  Weights (C,C,3,3), a1/a2/biases/BN params (C,). */
/* bytes of workspace for B images, or -1 when the shape is not supported */
int64_t tvq_resblock_workspace(int64_t B, int64_t C, int64_t H, int64_t W);
/* floats of the `h` buffer the training forward fills and the backward reads: B*C*3*W (the
 * conv1 output) for C in {8,16,32}; 3*B*C*3*W for C = 64, W = 8 (conv1 output | Snake_a1(x) |
 * Snake_a2(BN(h)), the weight gradients' inputs); -1 when the shape is not supported */
int64_t tvq_resblock_saved_floats(int64_t B, int64_t C, int64_t H, int64_t W);
/* training forward: h (B,C,3,W) = conv1 output (kept for backward), y (B,C,3,W), save
 * (4C floats) = batch mean | invstd | BN scale | BN shift; running stats updated in place
 * (momentum, unbiased var, num_batches_tracked += 1) */
int tvq_resblock_train_fwd(const float* x, int64_t B, int64_t C, int64_t H, int64_t W,
                           const float* a1, const float* w1, const float* b1, const float* bn_w,
                           const float* bn_b, float* running_mean, float* running_var,
                           int64_t* num_batches_tracked, float momentum, float eps,
                           const float* a2, const float* w2, const float* b2, float drop_p,
                           const int64_t* seed_ptr, uint64_t offset, float* h, float* y,
                           float* save, void* workspace, tvq_stream_t stream);
/* eval forward (BN from the running statistics, no dropout), one launch */
int tvq_resblock_eval_fwd(const float* x, int64_t B, int64_t C, int64_t H, int64_t W,
                          const float* a1, const float* w1, const float* b1, const float* bn_w,
                          const float* bn_b, const float* running_mean,
                          const float* running_var, float eps, const float* a2, const float* w2,
                          const float* b2, float* y, tvq_stream_t stream);
/* backward from dy: dx and every parameter gradient (written, or added when accumulate);
 * dbn_w / dbn_b may be NULL.  The workspace must stay alive until an open
 * tvq_conv_wgrad_defer scope is flushed (the weight-gradient slab sums are batched there). */
int tvq_resblock_bwd(const float* dy, const float* x, const float* h, int64_t B, int64_t C,
                     int64_t H, int64_t W, const float* a1, const float* w1, const float* bn_w,
                     const float* save, const float* a2, const float* w2, float drop_p,
                     const int64_t* seed_ptr, uint64_t offset, float* dx, float* da1, float* dw1,
                     float* db1, float* dbn_w, float* dbn_b, float* da2, float* dw2, float* db2,
                     int64_t accumulate, void* workspace, tvq_stream_t stream);
/* Two consecutive identity ResBlocks of the encoder / decoder stacks (vq_vae.py:143-170,
 * 211-251: n_resnet_blocks = 2 per level) as one chain: forward rb_fwd1(1) | rb_fwd21 |
 * rb_fwd2(2), backward rb_bwd2(2) | rb_bwd12 | rb_bwd1(1), the middle launch running one
 * block's last kernel and the other's first on the same images with the activation handed
 * over in registers; bitwise equal to the two blocks' tvq_resblock_train_fwd / _bwd.
 * Parameter arrays (host arrays of device pointers): p = {a1, w1, b1, bn_w, bn_b, a2, w2, b2},
 * rs = {running_mean, running_var}, q = {a1, w1, bn_w, save, a2, w2},
 * g = {da1, dw1, db1, dbn_w, dbn_b, da2, dw2, db2}.  Each block has its own workspace
 * (tvq_resblock_workspace bytes) and saved buffers; y1 (block 1's output) is block 2's
 * input, dy1 receives the gradient at it.  C = 64, W = 8 (tvq_resblock_w8.hip): w8_fwd21 /
 * w8_bwd12, the BN finish launches between.  1 when the shape takes this path (C in
 * {8, 16, 32} or the C = 64 LF maps), else 0. */
int tvq_resblock_pair_supported(int64_t B, int64_t C, int64_t H, int64_t W);
int tvq_resblock_pair_train_fwd(const float* x, int64_t B, int64_t C, int64_t H, int64_t W,
                                const float* const* p1, const float* const* p2,
                                float* const* rs1, float* const* rs2, int64_t* nbt1,
                                int64_t* nbt2, float momentum, float eps, float drop_p,
                                const int64_t* seed_ptr, uint64_t offset1, uint64_t offset2,
                                float* h1, float* y1, float* save1, float* h2, float* y2,
                                float* save2, void* ws1, void* ws2, tvq_stream_t stream);
int tvq_resblock_pair_bwd(const float* dy, const float* x, int64_t B, int64_t C, int64_t H,
                          int64_t W, const float* const* q1, const float* const* q2,
                          const float* h1, const float* y1, const float* h2, float drop_p,
                          const int64_t* seed_ptr, uint64_t offset1, uint64_t offset2, float* dx,
                          float* dy1, float* const* g1, float* const* g2, int64_t accumulate,
                          void* ws1, void* ws2, tvq_stream_t stream);
/* Fused projection ResBlock (in_channels != out_channels, the 1x1 `proj` on the skip) on the
 * LF band's W = 8 maps: Ci -> Co in {64 -> 128, 128 -> 64}, H = 3 (csrc/tvq_resblock_w8p.hip;
 * reference vq_vae.py:13-62):
 *   y = (proj(x) + bp) + Dropout_p(conv2(Snake_a2(BN(conv1(Snake_a1(x)) + b1))) + b2)
 * workspace: tvq_resblock_proj_workspace bytes (0 = shape unsupported); saved: the
 * backward's activations (h | Snake_a1(x) | Snake_a2(BN(h))), tvq_resblock_proj_saved_floats
 * floats; save: 4 Co floats (batch mean | invstd | scale | shift).  The backward writes dx and
 * every parameter gradient ((+)= with accumulate), the conv / proj weight-gradient slab sums
 * joining an open deferral scope (tvq_conv_wgrad_defer_begin). */
int64_t tvq_resblock_proj_workspace(int64_t B, int64_t Ci, int64_t Co, int64_t H, int64_t W);
int64_t tvq_resblock_proj_saved_floats(int64_t B, int64_t Ci, int64_t Co, int64_t H, int64_t W);
int tvq_resblock_proj_train_fwd(const float* x, int64_t B, int64_t Ci, int64_t Co, int64_t H,
                                int64_t W, const float* a1, const float* w1, const float* b1,
                                const float* bn_w, const float* bn_b, float* running_mean,
                                float* running_var, int64_t* nbt, float momentum, float eps,
                                const float* a2, const float* w2, const float* b2,
                                const float* wp, const float* bp, float drop_p,
                                const int64_t* seed_ptr, uint64_t offset, float* saved, float* y,
                                float* save, void* workspace, tvq_stream_t stream);
int tvq_resblock_proj_eval_fwd(const float* x, int64_t B, int64_t Ci, int64_t Co, int64_t H,
                               int64_t W, const float* a1, const float* w1, const float* b1,
                               const float* bn_w, const float* bn_b, const float* running_mean,
                               const float* running_var, float eps, const float* a2,
                               const float* w2, const float* b2, const float* wp,
                               const float* bp, float* y, tvq_stream_t stream);
int tvq_resblock_proj_bwd(const float* dy, const float* x, const float* saved, int64_t B,
                          int64_t Ci, int64_t Co, int64_t H, int64_t W, const float* a1,
                          const float* w1, const float* bn_w, const float* save, const float* a2,
                          const float* w2, const float* wp, float drop_p,
                          const int64_t* seed_ptr, uint64_t offset, float* dx, float* da1,
                          float* dw1, float* db1, float* dbn_w, float* dbn_b, float* da2,
                          float* dw2, float* db2, float* dwp, float* dbp, int64_t accumulate,
                          void* workspace, tvq_stream_t stream);

/* deterministic column sums of a P x N slab: out[j] (+)= sum_p in[p*ld + j]
 * (workspace: tvq_reduce_rows_workspace floats, may be 0). */
int64_t tvq_reduce_rows_workspace(int64_t P, int64_t N);
int tvq_reduce_rows(const float* in, int64_t P, int64_t N, int64_t ld, float* out,
                    int64_t accumulate, float* workspace, tvq_stream_t stream);

/* ------------------------------------------------------------- dense GEMM
 * nn.Linear and friends: C[m,n] = epi(alpha * sum_k A(m,k) B(k,n)),
 * A(m,k) = A[m*sam + k*sak], B(k,n) = B[k*sbk + n*sbn]; epi: + bias[n]
 * (pre-activation copy to `pre` if non-NULL), act (0 none, 1 GELU-erf),
 * times *gate (device scalar, if non-NULL: x-transformers layer dropout fused into
 * the branch's output Linear), + R[(rmod ? m % rmod : m)*ldr + n] (residual, or the per-position logits bias
 * of bidirectional_transformer.py:187), accumulate (C +=).  Workspace
 * (tvq_gemm_workspace floats) enables deterministic split-K. */
int64_t tvq_gemm_workspace(int64_t M, int64_t N, int64_t K);
int tvq_gemm(const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk, int64_t sbn,
             float* C, int64_t ldc, int64_t M, int64_t N, int64_t K, float alpha,
             const float* bias, const float* R, int64_t ldr, int64_t rmod, int64_t act, float* pre,
             int64_t accumulate, const float* gate, float* workspace, tvq_stream_t stream);
/* Grouped weight gradients of n Linear layers (the dW part of nn.Linear's backward,
 * issued together at the end of a backward instead of one tvq_gemm per layer):
 *   dW_i[m*ldw_i + n] (+)= sum_k dY_i[k*ldy_i + m] X_i[k*ldx_i + n],
 * m < M_i (out features), n < N_i (in features), k < K_i (tokens).  Host arrays of
 * length n (device pointers in dY / X / dW).  Each sum has a fixed order (results are
 * run-to-run bitwise identical).  Workspace: tvq_wgrad_group_workspace floats. */
int64_t tvq_wgrad_group_workspace(int64_t n, const int64_t* M, const int64_t* N, const int64_t* K);
int tvq_wgrad_group(int64_t n, const float* const* dY, const int64_t* ldy, const float* const* X,
                    const int64_t* ldx, float* const* dW, const int64_t* ldw, const int64_t* M,
                    const int64_t* N, const int64_t* K, int64_t accumulate, float* workspace,
                    tvq_stream_t stream);
/* The same with each layer's bias gradient in the same launch pair (replaces one column-sum
 * launch per Linear, bias_grad_rows / tvq_channel_sum): dB_i[m] (+)= sum_k dY_i[k*ldy_i + m]
 * for the i with dB_i != NULL (dB: host array of n device pointers, entries may be NULL;
 * dB itself may be NULL).  Fixed order: run-to-run bitwise identical. */
int tvq_wgrad_group_bias(int64_t n, const float* const* dY, const int64_t* ldy,
                         const float* const* X, const int64_t* ldx, float* const* dW,
                         const int64_t* ldw, float* const* dB, const int64_t* M, const int64_t* N,
                         const int64_t* K, int64_t accumulate, float* workspace,
                         tvq_stream_t stream);

/* ------------------------------------------------------ losses, optimizer
 * F.mse_loss (kind 0) / F.l1_loss (kind 1) means (stage1.py:129,133); backward
 * gives d/d target (the reconstruction is the second argument there). */
int64_t tvq_loss_workspace(int64_t n);
int tvq_loss_fwd(const float* input, const float* target, int64_t n, int64_t kind, float* out,
                 float* workspace, tvq_stream_t stream);
int tvq_loss_bwd(const float* input, const float* target, int64_t n, int64_t kind,
                 const float* gout, float* dtarget, tvq_stream_t stream);
/* torch.optim.AdamW step over a flat buffer (stage1.py:230, stage2.py:113) holding
 * nseg parameter segments.  torch skips a parameter whose .grad is None (Lightning
 * zero_grad(set_to_none=True); x-transformers layer dropout leaves a skipped branch
 * without grads, bidirectional_transformer.py:104-108) and keeps state['step'] per
 * parameter, so each segment has a gate and its own step count:
 *   tvq_adamw_gates: gates[s] = (*gate_ptrs[s] != 0) (gate_ptrs[s] = 0: always 1);
 *   tvq_adamw_begin: lr_step = device {lr, step}: writes lr when lr >= 0 (pass -1 inside
 *     a captured graph and set lr[0] before each replay), counts the step, and
 *     seg_step[s] += 1 where gates[s] != 0;
 *   tvq_adamw: chunks = int64 [nchunks][3] {start, len <= tvq_adamw_chunk(), segment};
 *     segments with gates[s] == 0 are left untouched. */
int64_t tvq_adamw_chunk(void);
int tvq_adamw_gates(const int64_t* gate_ptrs, int64_t nseg, float* gates, tvq_stream_t stream);
int tvq_adamw_begin(float* lr_step, float lr, const float* gates, float* seg_step, int64_t nseg,
                    tvq_stream_t stream);
int tvq_adamw(float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
              const int64_t* chunks, int64_t nchunks, const float* lr_step, const float* gates,
              const float* seg_step, float beta1, float beta2, float eps, float weight_decay,
              tvq_stream_t stream);
/* The same, and with zero_grads != 0 each chunk also zeroes the gradient values it has read
 * (the next step's zero_grad folded into the update: FusedAdamW(zero_after_step=True)). */
int tvq_adamw_zero(float* params, float* grads, float* exp_avg, float* exp_avg_sq,
                   const int64_t* chunks, int64_t nchunks, const float* lr_step,
                   const float* gates, const float* seg_step, float beta1, float beta2, float eps,
                   float weight_decay, int64_t zero_grads, tvq_stream_t stream);
/* Two optimizers' steps in two launches (both step-count updates, then both updates):
 * for k in {0, 1} exactly tvq_adamw_begin(lr_step[k], lr[k], gates[k], seg_step[k], nseg[k])
 * followed by tvq_adamw_zero(params[k], ... , zero_grads).  Host arrays of length 2. */
int tvq_adamw2(float* const* params, float* const* grads, float* const* exp_avg,
               float* const* exp_avg_sq, const int64_t* const* chunks, const int64_t* nchunks,
               float* const* lr_step, const float* lr, const float* const* gates,
               float* const* seg_step, const int64_t* nseg, const float* beta1,
               const float* beta2, const float* eps, const float* weight_decay,
               int64_t zero_grads, tvq_stream_t stream);
/* x-transformers layer dropout (random() < p skips a branch) drawn on the device for
 * n <= 256 branches: keep[i] = U(seed, offset, i) >= p; touched[i] = keep[i], or
 * max(touched[i], keep[i]) when accumulate (a second pass of the prior in one step). */
int tvq_layer_drop(const int64_t* seed_ptr, uint64_t offset, float p, int64_t n, float* keep,
                   float* touched, int64_t accumulate, tvq_stream_t stream);

/* ------------------------------------------------ MaskGIT transformer
 * x-transformers internals used by BidirectionalTransformer
 * (bidirectional_transformer.py:92-110; restated):
 * RMSNorm F.normalize(x)*sqrt(D)*g; LayerNorm (post_emb_norm gamma-only, pred_head
 * affine eps 1e-12, bidirectional_transformer.py:115); attention softmax(QK^T*scale)
 * with dropout, head_dim 64, seq <= 104 (path: 25 / 97), Q/K/V/O in the Linear layout
 * [(b*S+s)*ld + h*64 + d]; lse: [B*H*S] saved for the backward. */
int tvq_rmsnorm_fwd(const float* x, int64_t M, int64_t D, const float* g, float scale, float* y,
                    float* inv_norm, tvq_stream_t stream);
int64_t tvq_norm_bwd_workspace(int64_t M, int64_t D);
int tvq_rmsnorm_bwd(const float* dy, const float* x, int64_t M, int64_t D, const float* g,
                    float scale, const float* inv_norm, const float* dres, float* dx, float* dg,
                    int64_t accumulate, float* workspace, tvq_stream_t stream);
/* Token-embedding assembly (bidirectional_transformer.py:185,229-231): out (B, n+1, D1+D2)
 * = cat(cls (B, D1+D2), [t1 | t2] + pos[:n], dim=1), t1/t2 read through (b, j, d) strides
 * (t2 NULL with D2 = 0 for the LF prior).  Backward: dcls / dt1 / dt2 (same strides, each
 * NULL to skip) = the matching slices of dout; dpos (n, D1+D2) (+)= sum over b in order. */
int tvq_embed_assemble(const float* cls, const float* t1, int64_t s1b, int64_t s1n, int64_t s1d,
                       int64_t D1, const float* t2, int64_t s2b, int64_t s2n, int64_t s2d,
                       int64_t D2, const float* pos, int64_t B, int64_t n, float* out,
                       tvq_stream_t stream);
int tvq_embed_assemble_bwd(const float* dout, int64_t B, int64_t n, int64_t D1, int64_t D2,
                           float* dcls, float* dt1, int64_t s1b, int64_t s1n, int64_t s1d,
                           float* dt2, int64_t s2b, int64_t s2n, int64_t s2d, float* dpos,
                           int64_t accumulate, tvq_stream_t stream);
/* Training class conditioning (bidirectional_transformer.py:124-150): idx[b] = y[b] if
 * u_b > p else null_id; u_b = rnd[b] (injected) or the device counter RNG at (seed, offset). */
int tvq_class_index(const int64_t* y, int64_t B, float p, int64_t null_id, const int64_t* seed_ptr,
                    uint64_t offset, const float* rnd, int64_t* idx, tvq_stream_t stream);
/* Upscale's layout change fused into the nearest upsample (bidirectional_transformer.py:
 * 25-27): x (B, Lin, D) -> y (B, D, Lout), and its backward dy (B, D, Lout) -> dx (B, Lin, D). */
int tvq_upsample_nearest_t(const float* x, int64_t B, int64_t Lin, int64_t D, int64_t Lout,
                           float* y, tvq_stream_t stream);
int tvq_upsample_nearest_t_bwd(const float* dy, int64_t B, int64_t Lin, int64_t D, int64_t Lout,
                               float* dx, tvq_stream_t stream);
/* out[j*ldo + d] (+)= sum_b in[b*sb + j*sj + d] (j < n, d < D; b in order): batch sums of
 * per-position tables, e.g. the tied-logits bias gradient (bidirectional_transformer.py:187). */
int tvq_batch_colsum(const float* in, int64_t B, int64_t sb, int64_t n, int64_t sj, int64_t D,
                     float* out, int64_t ldo, int64_t accumulate, tvq_stream_t stream);
/* y[i] = x[i] * s[0] (s a device scalar; the gradient of a layer-dropout-gated branch). */
int tvq_scale_by(const float* x, int64_t n, const float* s, float* y, tvq_stream_t stream);
int tvq_layernorm_fwd(const float* x, int64_t M, int64_t D, const float* gamma, const float* beta,
                      float eps, float* y, float* mean, float* rstd, tvq_stream_t stream);
int tvq_layernorm_bwd(const float* dy, const float* x, int64_t M, int64_t D, const float* gamma,
                      const float* mean, const float* rstd, float* dx, float* dgamma,
                      float* dbeta, int64_t accumulate, float* workspace, tvq_stream_t stream);
int tvq_attention_fwd(const float* q, int64_t ldq, const float* k, int64_t ldk, const float* v,
                      int64_t ldv, float* o, int64_t ldo, float* lse, int64_t B, int64_t H,
                      int64_t S, int64_t Dh, float scale, float drop_p, const int64_t* seed_ptr,
                      uint64_t offset, tvq_stream_t stream);
int tvq_attention_bwd(const float* q, int64_t ldq, const float* k, int64_t ldk, const float* v,
                      int64_t ldv, const float* out, int64_t ldout, const float* dout, int64_t ldd,
                      const float* lse, int64_t B,
                      int64_t H, int64_t S, int64_t Dh, float scale, float drop_p,
                      const int64_t* seed_ptr, uint64_t offset, float* dq, float* dk, float* dv,
                      int64_t ldg, tvq_stream_t stream);
/* nn.Embedding lookups (tok_emb, pos/class emb) with the token-embedding dropout of
 * _token_emb_dropout (bidirectional_transformer.py:152-164: dropout only where
 * idx != mask_id); backward: deterministic per-row segmented sum. */
int tvq_embedding_fwd(const int64_t* idx, int64_t M, int64_t D, const float* table, float* out,
                      int64_t ldo, int64_t mask_id, float drop_p, const int64_t* seed_ptr,
                      uint64_t offset, tvq_stream_t stream);
int64_t tvq_embedding_bwd_workspace(int64_t M, int64_t V);
int tvq_embedding_bwd(const int64_t* idx, int64_t M, int64_t D, const float* g, int64_t ldg,
                      int64_t V, float* tgrad, int64_t accumulate, int64_t mask_id, float drop_p,
                      const int64_t* seed_ptr, uint64_t offset, int32_t* workspace,
                      tvq_stream_t stream);
/* embed[:, 1:, :] of the priors (the class token dropped before the head,
 * bidirectional_transformer.py:188,233): backward == 0: y (B, n, D) from x (B, n+1, D);
 * backward != 0: its adjoint, y (B, n+1, D) from x (B, n, D) with zero class rows.  D % 4 == 0,
 * 16-byte aligned. */
int tvq_drop_first_token(const float* x, int64_t B, int64_t n, int64_t D, float* y,
                         int64_t backward, tvq_stream_t stream);
/* F.cross_entropy(logits[~keep], s[~keep]) (maskgit.py:183-191); out = {loss, count}. */
int64_t tvq_masked_ce_workspace(int64_t M);
int tvq_masked_ce_fwd(const float* logits, int64_t ldl, int64_t M, int64_t K,
                      const int64_t* target, const bool* keep, float* lse, float* out,
                      float* workspace, tvq_stream_t stream);
int tvq_masked_ce_bwd(const float* logits, int64_t ldl, int64_t M, int64_t K,
                      const int64_t* target, const bool* keep, const float* lse,
                      const float* stats, const float* gout, float* dlogits, int64_t ldd,
                      tvq_stream_t stream);
/* MaskGIT._randomly_mask_tokens (maskgit.py:194-216) on device: cosine schedule,
 * per-row top-k of U[0,1) scores; ratio (float64, as np.random.uniform draws it) / rand
 * may be given (testing) or NULL (device RNG). */
int tvq_mask_tokens(const int64_t* s, int64_t B, int64_t n, int64_t mask_id,
                    const int64_t* seed_ptr, uint64_t offset, const double* ratio,
                    const float* rand, int64_t* s_M, bool* keep, tvq_stream_t stream);
/* Upscale's F.interpolate(mode='nearest') (bidirectional_transformer.py:27) and GELU. */
int tvq_upsample_nearest(const float* x, int64_t R, int64_t Lin, int64_t Lout, float* y,
                         tvq_stream_t stream);
int tvq_upsample_nearest_bwd(const float* dy, int64_t R, int64_t Lin, int64_t Lout, float* dx,
                             tvq_stream_t stream);
int tvq_gelu_fwd(const float* x, int64_t n, float* y, tvq_stream_t stream);
/* The priors' FeedForward branch in training (x-transformers FeedForward in the pre-norm
 * residual, bidirectional_transformer.py:92-110, ff_mult 1), D = 128, M token rows:
 *   pre = xn W1^T + b1 (M x 128), hd = Dropout_p(GELU(pre)) (the mask: uniform01 of
 *   (seed, offset) at m * 128 + j >= p), y = r + gate * (hd W2^T + b2)   (gate nullable: 1)
 * one launch; 16-byte aligned pointers.  tvq_ffn_bwd: from gy = dL/dy the pre-activation
 * gradient d_pre (M x 128, for the W1 / b1 gradients), d(xn) and, when gate and gy_gated are
 * both non-null, gy_gated = gate * gy (M x 128): the W2 / b2 gradients are the caller's,
 * hd^T (gate gy) and colsum(gate gy), so a dropped branch (gate 0) gets zero there.
 * p in [0, 1). */
int tvq_ffn_fwd(const float* xn, const float* r, int64_t M, int64_t D, const float* W1,
                const float* b1, const float* W2, const float* b2, const float* gate, float p,
                const int64_t* seed_ptr, uint64_t offset, float* y, float* pre, float* hd,
                tvq_stream_t stream);
int tvq_ffn_bwd(const float* gy, const float* pre, int64_t M, int64_t D, const float* W1,
                const float* W2, const float* gate, float p, const int64_t* seed_ptr,
                uint64_t offset, float* d_pre, float* dxn, float* gy_gated, tvq_stream_t stream);
int tvq_gelu_bwd(const float* dy, const float* x, int64_t n, float* dx, tvq_stream_t stream);
/* The priors' attention branch in training (x-transformers pre-norm layer with RMSNorm,
 * bidirectional_transformer.py:92-110), D = 128, 2 heads of 64, S <= 32 tokens per sequence,
 * B sequences of row-major (B*S, 128) token rows (csrc/tvq_xattn.hip):
 *   xn = RMSNorm_g(x) (x / max(|x|, 1e-12) * nscale * g), [q|k|v] = xn [Wq;Wk;Wv]^T (Wqkv:
 *   384 x 128 row-major), per head P = Dropout_p(softmax(q k^T / 8)) (the mask of
 *   tvq_attention_fwd), o = P v, y = x + gate * (o Wo^T)   (gate nullable: 1)
 * one launch; it also writes xn (B*S x 128), inv (B*S: 1 / max(|x|, 1e-12)), qkv (B*S x 384),
 * o (B*S x 128) and lse (B*2*S) for the backward and the weight gradients.
 * tvq_attn_branch_bwd: from gy = dL/dy: dx (the residual and RMSNorm paths), dqkv (B*S x 384;
 * the caller's dWqkv = dqkv^T xn), gy_gated = gate * gy (when gate and gy_gated are both
 * non-null; the caller's dWo = gy_gated^T o, else gy^T o), dg (written, or added when
 * accumulate: then batched into an open tvq_wgrad_defer scope).  workspace:
 * tvq_attn_branch_workspace(B, 128) floats.  16-byte aligned rows; p in [0, 1). */
int64_t tvq_attn_branch_workspace(int64_t B, int64_t D);
int tvq_attn_branch_fwd(const float* x, int64_t B, int64_t S, int64_t D, int64_t heads,
                        const float* g, float nscale, const float* Wqkv, const float* Wo,
                        const float* gate, float drop_p, const int64_t* seed_ptr, uint64_t offset,
                        float* y, float* xn, float* inv, float* qkv, float* o, float* lse,
                        tvq_stream_t stream);
int tvq_attn_branch_bwd(const float* gy, const float* x, int64_t B, int64_t S, int64_t D,
                        int64_t heads, const float* g, float nscale, const float* inv,
                        const float* Wqkv, const float* Wo, const float* gate, float drop_p,
                        const int64_t* seed_ptr, uint64_t offset, const float* qkv, const float* o,
                        const float* lse, float* dx, float* dqkv, float* gy_gated, float* dg,
                        int64_t accumulate, float* workspace, tvq_stream_t stream);


/* ---------------------------------------------------------------- fused LF prior (eval)
 * BidirectionalTransformer.forward_lf (bidirectional_transformer.py:166-192, the
 * x-transformers encoder of :92-110) in eval mode, as used by MaskGIT.first_pass
 * (maskgit.py:294-355): embedding (cls row + token + position), project_in, post_emb_norm,
 * `depth` pre-norm RMSNorm layers (2 heads x 64 attention, ff 128 + GELU), final norm,
 * project_out, pred_head (Linear + GELU + LayerNorm(eps ln_eps)) and the tied logits
 * h . tok_emb[:K]^T + bias[:, :K], one wave per sequence.  s: (B, n) tokens (row stride
 * s_stride), n + 1 <= 32; cls_idx: (B) class indices or NULL (the null class n_classes);
 * width must be 128.  weights: a HOST array of 5 + 10*depth + 7 device pointers, in order
 *   tok_emb (K+1, 128), pos_emb (n+1, 128), class_condition_emb (n_classes+1, 128),
 *   project_in W (128, 128), post_emb_norm gamma (128),
 *   per layer: attn RMSNorm g, to_q, to_k, to_v (128, 128), to_out (128, 128),
 *              ff RMSNorm g, ff.0.0 W (128, 128), b (128), ff.2 W (128, 128), b (128),
 *   final_norm g, project_out W, pred_head.0 W, b, pred_head.2 W, b, bias (n, K+1).
 * logits: (B, n, K).  workspace: tvq_prior_lf_eval_workspace(depth, K, n, n_classes) bytes
 * (16-B aligned)
 * receive the weights repacked once per call into the kernel's operand order. */
int64_t tvq_prior_lf_eval_workspace(int64_t depth, int64_t K, int64_t n, int64_t n_classes);
int tvq_prior_lf_eval(const int64_t* s, int64_t B, int64_t n, int64_t s_stride,
                      const int64_t* cls_idx, int64_t n_classes, int64_t width,
                      const float* const* weights, int64_t depth, int64_t K, float ln_eps,
                      float* logits, void* workspace, tvq_stream_t stream);
/* tvq_prior_lf_eval followed by the categorical draw of tvq_maskgit_sample (same race, same
 * noise counters) in the same launch: the tied logits are drawn from in registers and never
 * written (logits, nullable, receives them for checking).  s doubles as the tokens whose
 * mask_id entries are drawn (the others are kept, p = +inf).  workspace_ready != 0: the
 * workspace already holds this call's weights packed (an earlier call with the same weights,
 * e.g. the previous decoding step): the packing launches are skipped. */
int tvq_prior_lf_eval_sample(const int64_t* s, int64_t B, int64_t n, int64_t s_stride,
                             const int64_t* cls_idx, int64_t n_classes, int64_t width,
                             const float* const* weights, int64_t depth, int64_t K, float ln_eps,
                             int64_t mask_id, const float* gumbel, const int64_t* seed_ptr,
                             uint64_t offset, int64_t* sampled, float* selp, float* logits,
                             void* workspace, int64_t workspace_ready, tvq_stream_t stream);

/* ---------------------------------------------------------------- MaskGIT sampling
 * One iterative-decoding step of MaskGIT.first_pass / second_pass (maskgit.py:294-411):
 * tvq_maskgit_sample draws, for every token equal to mask_id, a code from
 * Categorical(logits) as Categorical.sample runs it (maskgit.py:307-315 ->
 * torch.multinomial's n_sample = 1 exponential race: argmax_k l_k + Gumbel_k, ties to the
 * lowest k), keeps the other tokens, and writes p(sampled) (fp32 softmax, double sum; +inf
 * for kept tokens, maskgit.py:320-326).  logits (B, n, K) with batch/token strides (sb, sn).
 * tvq_maskgit_remask: confidence = log(p + 1e-5) + temperature * Gumbel, re-mask exactly
 * the k lowest-confidence tokens of each row (mask_by_random_topk, maskgit.py:238-267,
 * ties by index) -> s_out (nullable) and/or masking (uint8, nullable).
 * Noise: gumbel (B*n*K Gumbel values, row-major) / u_gumbel (B*n uniforms) when given,
 * else the counter hash of (*seed_ptr, offset, element).
 * tvq_tied_logits_sample: tvq_maskgit_sample of logits = h W[:K]^T + bias[i, :K] (the
 * priors' tied output head, bidirectional_transformer.py:186-191; row m = b n + i) without
 * writing the logits: h (M, D), D 64 or 128; W (>= K, D); bias (n, ldb); h, W and the
 * workspace (tvq_tied_logits_sample_workspace(K, D, n) bytes) 16-byte aligned.
 * logits_out (M, K, nullable) receives the logits the draw used. */
int tvq_maskgit_sample(const float* logits, int64_t sb, int64_t sn, int64_t B, int64_t n,
                       int64_t K, const int64_t* s_in, int64_t mask_id, const float* gumbel,
                       const int64_t* seed_ptr, uint64_t offset, int64_t* sampled, float* selp,
                       tvq_stream_t stream);
int64_t tvq_tied_logits_sample_workspace(int64_t K, int64_t D, int64_t n);
int tvq_tied_logits_sample(const float* h, int64_t M, int64_t D, const float* W, int64_t K,
                           const float* bias, int64_t n, int64_t ldb, const int64_t* s_in,
                           int64_t mask_id, const float* gumbel, const int64_t* seed_ptr,
                           uint64_t offset, int64_t* sampled, float* selp, float* logits_out,
                           void* workspace, tvq_stream_t stream);
int tvq_maskgit_remask(const float* selp, int64_t B, int64_t n, int64_t k, float temperature,
                       const float* u_gumbel, const int64_t* seed_ptr, uint64_t offset,
                       const int64_t* sampled, int64_t mask_id, int64_t* s_out, uint8_t* masking,
                       tvq_stream_t stream);
/* out[b, d, p] = E[idx[b, p], d]: the codebook lookup of decode_token_ind_to_timeseries
 * (maskgit.py:461-469: F.embedding + 'b n c -> b c (h w)') written in NCHW. */
int tvq_codebook_gather_nchw(const int64_t* idx, int64_t B, int64_t P, int64_t D, const float* E,
                             float* out, tvq_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * ROCKET features (evaluation/rocket_functions.py:60-126 apply_kernel / apply_kernels, the
 * reference's numba CPU transform used by the FID/IS evaluation, sampler.py:184-189).
 * X (n, L) float64 row stride ldx; the kernels as generate_kernels (:21-57) returns them:
 * weights (sum of lengths) float64 packed back to back, woff[k] = offset of kernel k's
 * weights, lengths (1..16), biases float64, dilations (>= 1), paddings; out (n, 2 nk)
 * float64 = [ppv_k, max_k] per kernel.  float64, unfused multiply/add in the reference's
 * order: equal to its interpreted loop bit for bit.  Kernels outside the contract get NaN
 * features.  L <= 8192. */
int tvq_rocket_apply(const double* X, int64_t n, int64_t L, int64_t ldx, const double* weights,
                     const int32_t* woff, const int32_t* lengths, const double* biases,
                     const int32_t* dilations, const int32_t* paddings, int64_t nk, double* out,
                     tvq_stream_t stream);

/* ---- FID feature statistics (evaluation/eval_utils.py:56-81 calculate_fid; csrc/tvq_fid.hip):
 * mu (D) = z.mean(0) and cov (D x D) = np.cov(z, rowvar=False) (divisor N-1) of the rows of
 * z (N x D, float64, row-major), fixed summation order.  The matrix square root of
 * cov1 @ cov2 stays on the host (float64 scipy.linalg.sqrtm, as the reference). */
int tvq_fid_moments(const double* z, int64_t N, int64_t D, double* mu, double* cov,
                    tvq_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * FidelityEnhancer / Unet1D eval forward (models/fidelity_enhancer.py:284-498, the
 * sampler's post-decode refinement, generation/sampler.py:156-169).  (B, C, L) fp32.
 * tvq_fe_ws_weight: WeightStandardizedConv2d weight (:102-106), per output row of n = Ci*K.
 * tvq_fe_conv1d: nn.Conv1d(Ci, Co, K, stride S, padding P) (zero, or replicate when
 *   replicate != 0, :386-392); up2 != 0 reads x nearest-upsampled by 2 (Upsample, :85-89);
 *   bias and residual (added after the bias) nullable; Lout = tvq_fe_conv1d_out_len(...).
 * tvq_fe_group_norm_snake: GroupNorm(G, C, eps) -> Snake(a) (+ residual), Block.forward
 *   (:193-204) and ResnetBlock's skip add (:231).
 * tvq_fe_channel_layernorm: LayerNorm over C, gamma only (:119-127) (+ residual).
 * tvq_fe_linear_attention / tvq_fe_attention: LinearAttention (:234-260) / Attention
 *   (:263-283) core on to_qkv's output (B, 3 H dh, n) -> (B, H dh, n); dh must be 32.
 * tvq_fe_cat_interp: cat(interp(a -> L), interp(b -> L)) on channels, linear,
 *   align_corners=False (Unet1D skips :434-452; Cb = 0 interpolates a alone, :495-497). */
int64_t tvq_fe_conv1d_out_len(int64_t Lin, int64_t K, int64_t S, int64_t P, int64_t up2);
int tvq_fe_ws_weight(const float* w, int64_t Co, int64_t n, float eps, float* out,
                     tvq_stream_t stream);
int tvq_fe_conv1d(const float* x, int64_t B, int64_t Ci, int64_t Lin, const float* w,
                  const float* bias, int64_t Co, int64_t K, int64_t S, int64_t P, int64_t up2,
                  int64_t replicate, const float* residual, float* y, int64_t Lout,
                  tvq_stream_t stream);
int tvq_fe_group_norm_snake(const float* x, int64_t B, int64_t C, int64_t L, int64_t G,
                            const float* gamma, const float* beta, const float* a, float eps,
                            const float* residual, float* y, tvq_stream_t stream);
int tvq_fe_channel_layernorm(const float* x, int64_t B, int64_t C, int64_t L, const float* g,
                             float eps, const float* residual, float* y, tvq_stream_t stream);
int tvq_fe_linear_attention(const float* qkv, int64_t B, int64_t H, int64_t dh, int64_t n,
                            float* out, tvq_stream_t stream);
/* tvq_fe_linear_attention_fused: the same from the block input x (B, C, n) and the to_qkv
 * weight (3 H dh, C): q/k/v computed in LDS (bitwise equal to tvq_fe_conv1d + the core). */
int tvq_fe_linear_attention_fused(const float* x, int64_t B, int64_t C, int64_t n,
                                  const float* wqkv, int64_t H, int64_t dh, float* out,
                                  tvq_stream_t stream);
int tvq_fe_attention(const float* qkv, int64_t B, int64_t H, int64_t dh, int64_t n, float* out,
                     tvq_stream_t stream);
int tvq_fe_cat_interp(const float* a, int64_t Ca, int64_t La, const float* b, int64_t Cb,
                      int64_t Lb, int64_t B, int64_t L, float* out, tvq_stream_t stream);

/* ---- FidelityEnhancer training (Stage3, trainers/stage3.py:197-231; csrc/tvq_fe_train.hip).
 * The Unet1D convolutions train on the conv engine (tvq_conv2d_* with H = 1; kinds k7 and
 * k4/s2 for the init conv and Downsample, k3 replicate for the final convs). */
/* WeightStandardizedConv2d backward: w (O, n) rows, g = dL/d(standardised w) -> dw */
int tvq_fe_ws_weight_bwd(const float* w, int64_t O, int64_t n, float eps, const float* g,
                         float* dw, int64_t accumulate, tvq_stream_t stream);
/* y = Dropout_p(Snake_a(GroupNorm_G(x))) (+ residual); mean / rstd (B*G) saved */
int tvq_fe_gn_snake_train_fwd(const float* x, int64_t B, int64_t C, int64_t L, int64_t G,
                              const float* gamma, const float* beta, const float* a, float eps,
                              float drop_p, const int64_t* seed_ptr, uint64_t offset,
                              const float* residual, float* y, float* mean, float* rstd,
                              tvq_stream_t stream);
/* backward from dy: dx, and per element (B, C, L) terms whose channel sums are dgamma
 * (tgam), dbeta (tbet) and da (tda) */
int tvq_fe_gn_snake_bwd(const float* dy, const float* x, int64_t B, int64_t C, int64_t L,
                        int64_t G, const float* gamma, const float* beta, const float* a,
                        const float* mean, const float* rstd, float drop_p,
                        const int64_t* seed_ptr, uint64_t offset, float* dx, float* tgam,
                        float* tbet, float* tda, tvq_stream_t stream);
/* channel LayerNorm backward: dx and tg = dy * xhat (channel sums = dg) */
int tvq_fe_channel_layernorm_bwd(const float* dy, const float* x, int64_t B, int64_t C,
                                 int64_t L, const float* g, float eps, float* dx, float* tg,
                                 tvq_stream_t stream);
/* attention cores backward: qkv (B, 3 H dh, n) as to_qkv wrote it, dout (B, H dh, n) ->
 * dqkv (B, 3 H dh, n); dh = 32; full attention n <= ~70 (LDS) */
int tvq_fe_linear_attention_bwd(const float* qkv, const float* dout, int64_t B, int64_t H,
                                int64_t dh, int64_t n, float* dqkv, tvq_stream_t stream);
int tvq_fe_attention_bwd(const float* qkv, const float* dout, int64_t B, int64_t H, int64_t dh,
                         int64_t n, float* dqkv, tvq_stream_t stream);
/* tvq_fe_cat_interp backward: gout (B, Ca + Cb, L) -> da (B, Ca, La), db (B, Cb, Lb) */
int tvq_fe_cat_interp_bwd(const float* gout, int64_t Ca, int64_t La, int64_t Cb, int64_t Lb,
                          int64_t B, int64_t L, float* da, float* db, tvq_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Trajectory data format (utils/data_utils.py:84-110 get_data; scripts/generate.py:14-20
 * post_processed_generated_trajectories).  X (N, Fc = L*F) float64, columns [t0 f0, t0 f1,
 * ...] as np.stack(flight.data[features].values.ravel()) builds them.
 * tvq_minmax_fit: sklearn MinMaxScaler(feature_range=(lo, hi)).fit, per column (NaN
 *   skipped): data_min/data_max/scale/min_ (Fc float64 each); workspace of
 *   tvq_minmax_fit_workspace(Fc) doubles.
 * tvq_minmax_transform: out (N, F, L) float32 = transpose((X * scale + min_) as (N, L, F)),
 *   sklearn's float64 arithmetic, then the torch.FloatTensor cast: bit-equal.
 * tvq_minmax_inverse: out (N, L*F) float32 from x (N, F, L) float32: numpy's in-place
 *   `X -= min_; X /= scale_` on the float32 array (float64 op, float32 store), bit-equal. */
int64_t tvq_minmax_fit_workspace(int64_t Fc);
int tvq_minmax_fit(const double* X, int64_t N, int64_t Fc, double lo, double hi, double* data_min,
                   double* data_max, double* scale, double* min_, double* workspace,
                   tvq_stream_t stream);
int tvq_minmax_transform(const double* X, int64_t N, int64_t L, int64_t F, const double* scale,
                         const double* min_, float* out, tvq_stream_t stream);
int tvq_minmax_inverse(const float* x, int64_t N, int64_t L, int64_t F, const double* scale,
                       const double* min_, float* out, tvq_stream_t stream);

/* ---- Training EncBlock / DecBlock conv with the BatchNorm statistics in its epilogue
 * (reference vq_vae.py:65-121: Conv2d(3x4, stride (1,2), replicate) / ConvTranspose2d ->
 * BatchNorm2d -> Snake).  tvq_conv_bnstats_blocks: the per-block partials per channel that
 * tvq_conv2d_fwd_bnstats writes for this shape (transposed: ConvTranspose2d), 0 when the shape
 * does not take the stride-2 kernels.  tvq_conv2d_fwd_bnstats: y = conv(x) + bias as
 * tvq_conv2d_fwd / tvq_convT2d_fwd, plus part[(n blocks + blk) 2 + k] = (sum, sum of squares)
 * of y over block blk's outputs of channel n (fp64).  tvq_bn_train_apply_part: the BatchNorm
 * (+ Snake) training forward of tvq_bn_train_fwd from those partials (one launch). */
int64_t tvq_conv_bnstats_blocks(int64_t B, int64_t Ci, int64_t H, int64_t Wi, int64_t Co,
                                int64_t KH, int64_t KW, int64_t SW, int64_t transposed);
int tvq_conv2d_fwd_bnstats(const float* x, int64_t B, int64_t Ci, int64_t H, int64_t Wi,
                           const float* w, const float* bias, int64_t Co, int64_t KH, int64_t KW,
                           int64_t SW, int64_t replicate, int64_t transposed, float* y,
                           double* part, tvq_stream_t stream);
int tvq_bn_train_apply_part(const float* x, int64_t B, int64_t C, int64_t HW, const double* part,
                            int64_t nblk, const float* w, const float* b, float* running_mean,
                            float* running_var, int64_t* num_batches_tracked, float momentum,
                            float eps, const float* snake_a, float* y, float* save_mean,
                            float* save_invstd, float* scale_shift, tvq_stream_t stream);

/* ---- Upscale's first conv on the nearest-upsampled LF tokens (tvq_upscale.hip;
 * reference bidirectional_transformer.py:12-30 Upscale.forward: interpolate(nearest, m) ->
 * Conv1d(d, H, 3, padding 1) [-> GELU [-> BatchNorm1d eval]]), computed on the n-token grid:
 * Z = x Wcat^T with Wcat = [W_0; W_1; W_2] (3 H, d), then out[f j + r] = b + A_{j-1 or j}
 * + B_j + C_{j or j+1}; the backward forms the per-token window sums S = [S_0 | S_1 | S_2]
 * of dY, dx = S Wcat, dWcat = S^T x.  f = m / n >= 2 (integer), n <= 64, m <= 240. */
/* Wcat[(t H + c) d + k] = w[(c d + k) 3 + t] for w (H, d, 3). */
int tvq_ups_pack(const float* w, int64_t H, int64_t D, float* wcat, tvq_stream_t stream);
/* dw[(c d + k) 3 + t] (+)= dwcat[(t H + c) d + k]. */
int tvq_ups_wscatter(const float* dwcat, int64_t H, int64_t D, float* dw, int64_t accumulate,
                     tvq_stream_t stream);
/* z (B n, 3 H) -> out (B, H, f n).  mode 0: out = GELU(v) and pre = v (training, the
 * erff GELU of tvq_gelu_fwd); 1: out = v; 2: out = BN_eval(GELU(v)) from the running
 * statistics (sampling).  v = conv + bias (bias may be NULL). */
int tvq_ups_combine(const float* z, int64_t B, int64_t n, int64_t f, int64_t H,
                    const float* bias, int64_t mode, const float* bn_w, const float* bn_b,
                    const float* bn_rm, const float* bn_rv, float bn_eps, float* out, float* pre,
                    tvq_stream_t stream);
/* s (B n, 3 H) = window sums of dY1 = dy (B, H, f n) [* GELU'(pre) when pre != NULL];
 * part (B, H) (optional) = per-image sums of dY1 (the bias gradient's partials). */
int tvq_ups_sums(const float* dy, const float* pre, int64_t B, int64_t n, int64_t f, int64_t H,
                 float* s, float* part, tvq_stream_t stream);
/* The HF prior's project_in with Upscale's second conv folded in (training; reference
 * bidirectional_transformer.py:194-231 + x-transformers ContinuousTransformerWrapper.project_in):
 * z (B, m+1, d) = cat(Cp, v^T + R + P) with v (B, d, m) = conv(u, W_l W2) + W_l b2, R (B m, d) =
 * th W_h^T, P (m, d) = pos[:m] W_in^T, Cp (B, d) = cls W_in^T; the backward splits dz into
 * dv (B, d, m), dR (B m, d) and dCp (B, d).  d (m + 1) <= 16384. */
int tvq_hfe_assemble(const float* v, const float* R, const float* P, const float* Cp, int64_t B,
                     int64_t m, int64_t d, float* z, tvq_stream_t stream);
int tvq_hfe_assemble_bwd(const float* dz, int64_t B, int64_t m, int64_t d, float* dv, float* dR,
                         float* dCp, tvq_stream_t stream);
/* The priors' training loss head in one launch (+ a count, a transpose and a final launch):
 * logits = h W[:K]^T + bias[m mod n] (bidirectional_transformer.py:186-191), the masked
 * cross-entropy of maskgit.py:183-191 and, for the backward that starts at this loss with the
 * root gradient *gscale, dlogits = keep ? 0 : (softmax - onehot(target)) * gscale / cnt and
 * dh = dlogits W[:K] -- the logits never reach memory.  h (M, 128), W (>= K, 128), bias (n,
 * ldb >= K), target int64 (M), keep bool (M); out = {loss, cnt}.  K in {64, 128, 256, 512};
 * workspace: tvq_tied_logits_ce_workspace(M, K) floats. */
int64_t tvq_tied_logits_ce_workspace(int64_t M, int64_t K);
int tvq_tied_logits_ce(const float* h, int64_t M, int64_t D, const float* W, int64_t K,
                       const float* bias, int64_t n, int64_t ldb, const int64_t* target,
                       const bool* keep, const float* gscale, float* dlogits, float* dh,
                       float* out, float* workspace, tvq_stream_t stream);
/* out[0] = a[0] / b[0] (device scalars). */
int tvq_scalar_ratio(const float* a, const float* b, float* out, tvq_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* TVQ_H */

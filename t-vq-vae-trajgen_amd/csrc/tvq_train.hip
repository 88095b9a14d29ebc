// Stage1 losses (stage1.py:129-135) and the fused AdamW step (stage1.py:229-236).
//
// Losses: F.mse_loss(x_l, xhat_l) and F.l1_loss(x_h, xhat_h), means over all
// elements; two-stage deterministic reductions.  Backward writes d/d xhat.
// AdamW follows torch.optim.AdamW (single-tensor path) operation for operation:
//   p *= 1 - lr*wd;  m = lerp(m, g, 1-b1);  v = v*b2 + (1-b2) g^2;
//   p -= (lr / (1-b1^t)) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
// with lr and t read from device memory (graph-replay friendly); one launch
// covers a whole flat parameter buffer.
#include <math.h>

#include "tvq_common.h"

namespace tvq {

// kind 0: sum (a-b)^2, kind 1: sum |a-b|
__global__ __launch_bounds__(256) void loss_partial_kernel(const float* __restrict__ a,
                                                           const float* __restrict__ b, int64_t n,
                                                           int kind, float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float d = a[i] - b[i];
    s += kind == 0 ? d * d : fabsf(d);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void loss_final_kernel(const float* __restrict__ part, int nparts,
                                                         int64_t n, float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) s += part[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) out[0] = s / (float)n;
}

// d/d target of mean loss(input, target): mse: 2(t - x)/n * g ; l1: sign(t - x)/n * g
__global__ void loss_bwd_kernel(const float* __restrict__ input, const float* __restrict__ target,
                                int64_t n, int kind, const float* __restrict__ gout,
                                float* __restrict__ dtarget) {
  const float g = gout[0] / (float)n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float d = target[i] - input[i];
    dtarget[i] = kind == 0 ? 2.0f * d * g : (d > 0.f ? g : (d < 0.f ? -g : 0.f));
  }
}

// One block per chunk of one parameter segment (chunk = {start, len, segment}).  A
// segment whose gate is 0 this step is skipped whole: torch.optim.AdamW leaves a
// parameter whose .grad is None untouched (no decay, no moment update, no step count),
// which is what x-transformers' layer dropout produces for a skipped branch.
constexpr int ADAMW_CHUNK = 4096;

struct AdamArgs {  // one optimizer's flat buffers and hyper-parameters
  float *p, *m, *v;
  const float* g;
  const int64_t* chunks;
  const float *lr_step, *gates;
  float* seg_step;
  float b1, b2, eps, wd;
  float* gz;  // the gradient again when the update zeroes what it reads, else null
  int nchunks;
};

__device__ __forceinline__ void adamw_chunk(float* __restrict__ p, const float* __restrict__ g,
                                            float* __restrict__ m, float* __restrict__ v,
                                            const int64_t* __restrict__ chunks,
                                            const float* __restrict__ lr_step,
                                            const float* __restrict__ gates,
                                            const float* __restrict__ seg_step, float b1,
                                            float b2, float eps, float wd,
                                            float* __restrict__ gz, int chunk) {
  const int64_t start = chunks[3 * chunk];
  const int len = (int)chunks[3 * chunk + 1];
  const int seg = (int)chunks[3 * chunk + 2];
  if (gates[seg] == 0.f) {
    // a gated-off segment is not updated, but its gradient is still cleared (the next
    // step's zero_grad), so a non-finite value left by a dropped branch cannot survive
    // until the gate reopens
    if (gz)
      for (int j = threadIdx.x; j < len; j += 256) gz[start + j] = 0.f;
    return;
  }
  const double lr = lr_step[0];
  const double t = seg_step[seg];
  const double bc1 = 1.0 - pow((double)b1, t);
  const double bc2 = 1.0 - pow((double)b2, t);
  const float step_size = (float)(lr / bc1);
  const float bc2s = (float)sqrt(bc2);
  const float decay = (float)(1.0 - lr * (double)wd);
  const float w1 = 1.0f - b1, w2 = 1.0f - b2;
  for (int j = threadIdx.x; j < len; j += 256) {
    const int64_t i = start + j;
    const float gi = g[i];
    if (gz) gz[i] = 0.f;  // the next step's zero_grad, done where the gradient is read
    float pi = p[i] * decay;
    float mi = m[i];
    mi = mi + w1 * (gi - mi);
    float vi = v[i] * b2 + w2 * gi * gi;
    const float denom = sqrtf(vi) / bc2s + eps;
    pi = pi - step_size * (mi / denom);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
  }
}

__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p,
                                                    const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    const int64_t* __restrict__ chunks,
                                                    const float* __restrict__ lr_step,
                                                    const float* __restrict__ gates,
                                                    const float* __restrict__ seg_step, float b1,
                                                    float b2, float eps, float wd,
                                                    float* __restrict__ gz) {
  adamw_chunk(p, g, m, v, chunks, lr_step, gates, seg_step, b1, b2, eps, wd, gz, blockIdx.x);
}

// two optimizers' updates in one launch: blocks [0, a0.nchunks) update the first
struct AdamPair {
  AdamArgs o[2];
};
__global__ __launch_bounds__(256) void adamw2_kernel(AdamPair a) {
  const int k = (int)blockIdx.x >= a.o[0].nchunks ? 1 : 0;
  const AdamArgs& o = a.o[k];
  adamw_chunk(o.p, o.g, o.m, o.v, o.chunks, o.lr_step, o.gates, o.seg_step, o.b1, o.b2, o.eps,
              o.wd, o.gz, (int)blockIdx.x - (k ? a.o[0].nchunks : 0));
}

// gates[s] = *gate_ptr[s] (1 where the segment has no gate); then the per-segment step
// counts advance where the gate is set (torch keeps state['step'] per parameter)
__global__ void adamw_gates_kernel(const int64_t* __restrict__ gate_ptrs, int64_t nseg,
                                   float* __restrict__ gates) {
  for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < nseg;
       s += (int64_t)gridDim.x * blockDim.x) {
    const float* gp = (const float*)gate_ptrs[s];
    gates[s] = gp ? (*gp != 0.f ? 1.f : 0.f) : 1.f;
  }
}

__device__ __forceinline__ void adamw_begin(float* __restrict__ lr_step, float lr,
                                            const float* __restrict__ gates,
                                            float* __restrict__ seg_step, int64_t nseg,
                                            int64_t s) {
  if (s == 0) {
    if (lr >= 0.f) lr_step[0] = lr;
    lr_step[1] += 1.0f;
  }
  if (s < nseg && gates[s] != 0.f) seg_step[s] += 1.0f;
}

__global__ void adamw_begin_kernel(float* __restrict__ lr_step, float lr,
                                   const float* __restrict__ gates, float* __restrict__ seg_step,
                                   int64_t nseg) {
  adamw_begin(lr_step, lr, gates, seg_step, nseg, blockIdx.x * (int64_t)blockDim.x + threadIdx.x);
}

// both optimizers' step counts (blockIdx.y = optimizer)
__global__ void adamw_begin2_kernel(AdamPair a, float lr0, float lr1, int64_t nseg0,
                                    int64_t nseg1) {
  const int k = blockIdx.y;
  const AdamArgs& o = a.o[k];
  adamw_begin(const_cast<float*>(o.lr_step), k ? lr1 : lr0, o.gates, o.seg_step, k ? nseg1 : nseg0,
              blockIdx.x * (int64_t)blockDim.x + threadIdx.x);
}

// layer-dropout decisions of one x-transformers layer stack (random() < p skips a
// branch): keep[i] = U(seed, offset, i) >= p; touched[i] = keep[i] (first pass of the
// step) or max(touched[i], keep[i]) (a later pass: CFG runs the prior twice)
__global__ void layer_drop_kernel(const int64_t* seed_ptr, uint64_t offset, float p, int n,
                                  float* __restrict__ keep, float* __restrict__ touched,
                                  int accumulate) {
  const int i = threadIdx.x;
  if (i >= n) return;
  const uint64_t seed = mix_seed(seed_ptr, offset);
  const float k = uniform01(seed, (uint64_t)i) >= p ? 1.f : 0.f;
  keep[i] = k;
  touched[i] = accumulate ? fmaxf(touched[i], k) : k;
}

static int blocks_for(int64_t n, int cap) {
  int64_t b = (n + 255) / 256;
  if (b < 1) b = 1;
  return (int)(b < cap ? b : cap);
}

}  // namespace tvq

using namespace tvq;

extern "C" int64_t tvq_loss_workspace(int64_t n) { return blocks_for(n, 1024); }

extern "C" int tvq_loss_fwd(const float* input, const float* target, int64_t n, int64_t kind,
                            float* out, float* workspace, tvq_stream_t stream) {
  TVQ_CHECK_ARG(input && target && out && workspace && n > 0 && (kind == 0 || kind == 1),
                "tvq_loss_fwd: bad arguments");
  const int nb = blocks_for(n, 1024);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(loss_partial_kernel, dim3(nb), dim3(256), 0, st, input, target, n, (int)kind,
                     workspace);
  hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(256), 0, st, workspace, nb, n, out);
  return launch_status("tvq_loss_fwd");
}

extern "C" int tvq_loss_bwd(const float* input, const float* target, int64_t n, int64_t kind,
                            const float* gout, float* dtarget, tvq_stream_t stream) {
  TVQ_CHECK_ARG(input && target && gout && dtarget && n > 0, "tvq_loss_bwd: bad arguments");
  hipLaunchKernelGGL(loss_bwd_kernel, dim3(blocks_for(n, 4096)), dim3(256), 0, (hipStream_t)stream,
                     input, target, n, (int)kind, gout, dtarget);
  return launch_status("tvq_loss_bwd");
}

extern "C" int64_t tvq_adamw_chunk(void) { return ADAMW_CHUNK; }

extern "C" int tvq_adamw_gates(const int64_t* gate_ptrs, int64_t nseg, float* gates,
                               tvq_stream_t stream) {
  TVQ_CHECK_ARG(gate_ptrs && gates && nseg > 0, "tvq_adamw_gates: bad arguments");
  hipLaunchKernelGGL(adamw_gates_kernel, dim3(blocks_for(nseg, 64)), dim3(256), 0,
                     (hipStream_t)stream, gate_ptrs, nseg, gates);
  return launch_status("tvq_adamw_gates");
}

// lr_step: device float[2] = {lr, step}; sets lr (when >= 0), counts the step, and
// advances the step count of every segment whose gate is set.
extern "C" int tvq_adamw_begin(float* lr_step, float lr, const float* gates, float* seg_step,
                               int64_t nseg, tvq_stream_t stream) {
  TVQ_CHECK_ARG(lr_step && gates && seg_step && nseg > 0, "tvq_adamw_begin: bad arguments");
  hipLaunchKernelGGL(adamw_begin_kernel, dim3(blocks_for(nseg, 64)), dim3(256), 0,
                     (hipStream_t)stream, lr_step, lr, gates, seg_step, nseg);
  return launch_status("tvq_adamw_begin");
}

extern "C" int tvq_adamw_zero(float* params, float* grads, float* exp_avg, float* exp_avg_sq,
                              const int64_t* chunks, int64_t nchunks, const float* lr_step,
                              const float* gates, const float* seg_step, float beta1, float beta2,
                              float eps, float weight_decay, int64_t zero_grads,
                              tvq_stream_t stream) {
  TVQ_CHECK_ARG(params && grads && exp_avg && exp_avg_sq && chunks && lr_step && gates &&
                    seg_step && nchunks >= 0,
                "tvq_adamw: bad arguments");
  if (nchunks == 0) return TVQ_OK;
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)nchunks), dim3(256), 0, (hipStream_t)stream,
                     params, grads, exp_avg, exp_avg_sq, chunks, lr_step, gates, seg_step, beta1,
                     beta2, eps, weight_decay, zero_grads ? grads : nullptr);
  return launch_status("tvq_adamw");
}

// Two FusedAdamW updates (their begin + update) as two launches instead of four: the same
// arithmetic per optimizer as tvq_adamw_begin + tvq_adamw_zero.
extern "C" int tvq_adamw2(float* const* params, float* const* grads, float* const* exp_avg,
                          float* const* exp_avg_sq, const int64_t* const* chunks,
                          const int64_t* nchunks, float* const* lr_step, const float* lr,
                          const float* const* gates, float* const* seg_step, const int64_t* nseg,
                          const float* beta1, const float* beta2, const float* eps,
                          const float* weight_decay, int64_t zero_grads, tvq_stream_t stream) {
  TVQ_CHECK_ARG(params && grads && exp_avg && exp_avg_sq && chunks && nchunks && lr_step && lr &&
                    gates && seg_step && nseg && beta1 && beta2 && eps && weight_decay,
                "tvq_adamw2: bad arguments");
  AdamPair a;
  for (int k = 0; k < 2; ++k) {
    TVQ_CHECK_ARG(params[k] && grads[k] && exp_avg[k] && exp_avg_sq[k] && chunks[k] && lr_step[k] &&
                      gates[k] && seg_step[k] && nchunks[k] >= 0 && nseg[k] >= 0,
                  "tvq_adamw2: bad optimizer %d", k);
    a.o[k] = {params[k], exp_avg[k], exp_avg_sq[k], grads[k], chunks[k], lr_step[k], gates[k],
              seg_step[k], beta1[k], beta2[k], eps[k], weight_decay[k],
              zero_grads ? grads[k] : nullptr, (int)nchunks[k]};
  }
  hipStream_t st = (hipStream_t)stream;
  const int64_t nmax = nseg[0] > nseg[1] ? nseg[0] : nseg[1];
  hipLaunchKernelGGL(adamw_begin2_kernel, dim3((unsigned)blocks_for(nmax + 1, 1 << 20), 2),
                     dim3(256), 0, st, a, lr[0], lr[1], nseg[0], nseg[1]);
  if (nchunks[0] + nchunks[1] > 0)
    hipLaunchKernelGGL(adamw2_kernel, dim3((unsigned)(nchunks[0] + nchunks[1])), dim3(256), 0, st,
                       a);
  return launch_status("tvq_adamw2");
}

extern "C" int tvq_adamw(float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                         const int64_t* chunks, int64_t nchunks, const float* lr_step,
                         const float* gates, const float* seg_step, float beta1, float beta2,
                         float eps, float weight_decay, tvq_stream_t stream) {
  return tvq_adamw_zero(params, const_cast<float*>(grads), exp_avg, exp_avg_sq, chunks, nchunks,
                        lr_step, gates, seg_step, beta1, beta2, eps, weight_decay, 0, stream);
}

extern "C" int tvq_layer_drop(const int64_t* seed_ptr, uint64_t offset, float p, int64_t n,
                              float* keep, float* touched, int64_t accumulate,
                              tvq_stream_t stream) {
  TVQ_CHECK_ARG(keep && touched && n > 0 && n <= 256, "tvq_layer_drop: bad arguments");
  hipLaunchKernelGGL(layer_drop_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, seed_ptr,
                     offset, p, (int)n, keep, touched, (int)accumulate);
  return launch_status("tvq_layer_drop");
}

// ---------------------------------------------------------------- step glue
// The few elementwise ops a training step still needed from PyTorch (zero the flat
// gradients, advance the dropout seed, add up the logged losses) as HIP launches, so a
// replayed step graph holds no at::native kernel.
namespace tvq {
__global__ __launch_bounds__(256) void fill_f32_kernel(float* __restrict__ p, int64_t n, float v,
                                                       int vec) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  if (vec) {
    float4* q = reinterpret_cast<float4*>(p);
    const float4 f = make_float4(v, v, v, v);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n / 4; i += stride) q[i] = f;
    for (int64_t i = n / 4 * 4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) p[i] = v;
  } else {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) p[i] = v;
  }
}

__global__ __launch_bounds__(256) void fill_i64_kernel(int64_t* __restrict__ p, int64_t n,
                                                       int64_t v) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    p[i] = v;
}

__global__ void add_i64_kernel(int64_t* __restrict__ p, int64_t v) {
  if (threadIdx.x == 0) p[0] += v;
}

// out = ((a + b) + c) + d elementwise (c, d nullable), out_ab = a + b (nullable): the
// evaluation order of Python's `a + b + c + d`
__global__ __launch_bounds__(256) void sum4_kernel(const float* __restrict__ a,
                                                   const float* __restrict__ b,
                                                   const float* __restrict__ c,
                                                   const float* __restrict__ d,
                                                   float* __restrict__ out,
                                                   float* __restrict__ out_ab, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float ab = a[i] + b[i];
    float t = ab;
    if (c) t = t + c[i];
    if (d) t = t + d[i];
    if (out) out[i] = t;
    if (out_ab) out_ab[i] = ab;
  }
}
}  // namespace tvq

extern "C" int tvq_fill(float* p, int64_t n, float value, tvq_stream_t stream) {
  TVQ_CHECK_ARG(p && n >= 0, "tvq_fill: bad arguments");
  if (n == 0) return TVQ_OK;
  const int vec = ((uintptr_t)p & 15) == 0;
  int64_t blocks = ((vec ? n / 4 : n) + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 2048 ? 2048 : blocks);
  hipLaunchKernelGGL(fill_f32_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, p,
                     n, value, vec);
  return launch_status("tvq_fill");
}

// p[0] = a, q[0] = b in one launch (two optimizers' learning rates before a replay)
__global__ void fill2_kernel(float* __restrict__ p, float a, float* __restrict__ q, float b) {
  if (threadIdx.x == 0) p[0] = a;
  if (threadIdx.x == 1 && q) q[0] = b;
}

extern "C" int tvq_fill2(float* p, float a, float* q, float b, tvq_stream_t stream) {
  TVQ_CHECK_ARG(p, "tvq_fill2: bad arguments");
  hipLaunchKernelGGL(fill2_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, p, a, q, b);
  return launch_status("tvq_fill2");
}

extern "C" int tvq_fill_i64(int64_t* p, int64_t n, int64_t value, tvq_stream_t stream) {
  TVQ_CHECK_ARG(p && n >= 0, "tvq_fill_i64: bad arguments");
  if (n == 0) return TVQ_OK;
  int64_t blocks = (n + 255) / 256;
  blocks = blocks > 2048 ? 2048 : blocks;
  hipLaunchKernelGGL(fill_i64_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, p,
                     n, value);
  return launch_status("tvq_fill_i64");
}

extern "C" int tvq_add_i64(int64_t* p, int64_t value, tvq_stream_t stream) {
  TVQ_CHECK_ARG(p, "tvq_add_i64: bad arguments");
  hipLaunchKernelGGL(add_i64_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, p, value);
  return launch_status("tvq_add_i64");
}

extern "C" int tvq_sum4(const float* a, const float* b, const float* c, const float* d, float* out,
                        float* out_ab, int64_t n, tvq_stream_t stream) {
  TVQ_CHECK_ARG(a && b && (out || out_ab) && n > 0 && (c || !d), "tvq_sum4: bad arguments");
  const int64_t blocks = (n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024;
  hipLaunchKernelGGL(sum4_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a, b, c,
                     d, out, out_ab, n);
  return launch_status("tvq_sum4");
}

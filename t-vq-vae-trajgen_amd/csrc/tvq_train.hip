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

__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                             float* __restrict__ m, float* __restrict__ v, int64_t n,
                             const float* __restrict__ lr_step, float b1, float b2, float eps,
                             float wd) {
  const double lr = lr_step[0];
  const double t = lr_step[1];
  const double bc1 = 1.0 - pow((double)b1, t);
  const double bc2 = 1.0 - pow((double)b2, t);
  const float step_size = (float)(lr / bc1);
  const float bc2s = (float)sqrt(bc2);
  const float decay = (float)(1.0 - lr * (double)wd);
  const float w1 = 1.0f - b1, w2 = 1.0f - b2;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i];
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

__global__ void adamw_begin_kernel(float* __restrict__ lr_step, float lr) {
  if (lr >= 0.f) lr_step[0] = lr;
  lr_step[1] += 1.0f;
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

// lr_step: device float[2] = {lr, step}; tvq_adamw_begin sets lr and increments step.
extern "C" int tvq_adamw_begin(float* lr_step, float lr, tvq_stream_t stream) {
  TVQ_CHECK_ARG(lr_step, "tvq_adamw_begin: bad arguments");
  hipLaunchKernelGGL(adamw_begin_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, lr_step, lr);
  return launch_status("tvq_adamw_begin");
}

extern "C" int tvq_adamw(float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                         int64_t n, const float* lr_step, float beta1, float beta2, float eps,
                         float weight_decay, tvq_stream_t stream) {
  TVQ_CHECK_ARG(params && grads && exp_avg && exp_avg_sq && lr_step && n >= 0,
                "tvq_adamw: bad arguments");
  if (n == 0) return TVQ_OK;
  hipLaunchKernelGGL(adamw_kernel, dim3(blocks_for(n, 4096)), dim3(256), 0, (hipStream_t)stream,
                     params, grads, exp_avg, exp_avg_sq, n, lr_step, beta1, beta2, eps,
                     weight_decay);
  return launch_status("tvq_adamw");
}

// Shared helpers for the TimeVQVAE gfx950 kernels (CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tvq.h"

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace tvq {

// thread-local last-error message returned by tvq_last_error()
void set_error(const char* fmt, ...);

// k zeroed int32 counters from the current device's pool (tvq_counter_pool), or nullptr
// when no pool is registered / fused finishes are disabled (TVQ_FUSED_FINISH=0): the
// caller then falls back to a separate finishing launch.  Slots are handed out round
// robin; a kernel returns every counter it used to zero before it exits.
enum FinishClass { FIN_NORM = 0, FIN_REDUCE = 1, FIN_GEMM = 2, FIN_CONV = 3 };
int* counters(int64_t k, FinishClass cls);

inline int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return TVQ_ERR_LAUNCH;
  }
  return TVQ_OK;
}

// Dispatch trace (tvq_plan_trace / tvq_plan_read): while on, every host-side plan records
// the kernel variant it launched ("conv_t32 bk16 nw12 tn128", "conv_wgrad_s2 S=256
// spr=2", ...), so a test can confirm which kernel a shape took.  Off by default: one
// branch per launch.
extern bool g_plan_trace;
void plan_note_impl(const char* fmt, ...);
#define TVQ_PLAN(...)                                   \
  do {                                                  \
    if (::tvq::g_plan_trace) ::tvq::plan_note_impl(__VA_ARGS__); \
  } while (0)

#define TVQ_CHECK_ARG(cond, ...)          \
  do {                                    \
    if (!(cond)) {                        \
      ::tvq::set_error(__VA_ARGS__);      \
      return TVQ_ERR_ARG;                 \
    }                                     \
  } while (0)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum, deterministic (fixed tree).  `red` needs blockDim/64 floats.
// Returns the total in every thread.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

// Grid-level finish without a second launch: every block of a group publishes its
// partial results, then takes a ticket; the block that draws the last ticket combines
// the group's partials in a fixed order, so the result does not depend on arrival
// order.  The L2s of the 8 XCDs are not coherent, so the partials are published with
// write-through stores (st_wt: agent-scope relaxed atomic store, `sc1`), drained with
// s_waitcnt vmcnt(0) by every storing wave before the block's barrier, and read back with
// ld_wt (`sc1` loads that do not hit a stale L1/L2 line): the hand-off form of
// cdna_hip_programming.md §6 Guideline 16 (R1) in which the write-through stores and their
// drain stand in for the producer's release.  TVQ_TICKET selects the ticket's ordering:
//   2: agent-scope acq_rel fetch_add -- release / acquire in the HIP memory model's own
//      terms; the release writes back the XCD's whole L2 in every block (measured: joint
//      step 6.58 vs 5.75 ms, profiles/r03_ticket_ab.txt);
//   1 (default): relaxed ticket, and the last block alone takes an agent-scope acquire
//      fence before it reads the partials;
//   0: relaxed ticket between wavefront-scope fences (compiler ordering only).
// The last block re-zeroes the counter for the next launch.
#ifndef TVQ_TICKET
#define TVQ_TICKET 1
#endif
template <typename T>
__device__ __forceinline__ void st_wt(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ T ld_wt(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Returns the same value in every thread of the block.
// REQUIREMENT (TVQ_TICKET 0/1): every partial a last block reads must have been stored with
// st_wt by its producer (a plain store may sit in the producing XCD's L2, and the reader's
// ld_wt on another XCD would see stale data with no error); only TVQ_TICKET=2 orders plain
// stores by itself.  Build with -DTVQ_TICKET=2 (EXTRA=-DTVQ_TICKET=2) to check a suspect
// producer: the results must be bitwise equal to the default build's.
__device__ __forceinline__ bool last_block(int* counter, int total) {
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's st_wt stores are done
  __syncthreads();
  if (threadIdx.x == 0) {
#if TVQ_TICKET == 2
    const int t = __hip_atomic_fetch_add(counter, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
#else
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const int t = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#endif
    s_last = t == total - 1;
    if (s_last) {
#if TVQ_TICKET == 1
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
      __hip_atomic_store(counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  return s_last != 0;
}

// q = n / d by one v_mul_hi_u32 with m = ceil(2^32 / d): exact while n * d < 2^32
// (callers check that bound on the host); d == 1 is encoded as m = 0
struct Div16 {
  uint32_t d, m;
};
static inline Div16 make_div16(int64_t d) {
  Div16 r;
  r.d = (uint32_t)d;
  r.m = (uint32_t)(((1ull << 32) + (uint64_t)d - 1) / (uint64_t)d);
  return r;
}
__device__ __forceinline__ int div16(int n, const Div16& v) {
  return v.m ? (int)__umulhi((uint32_t)n, v.m) : n;
}

__device__ __forceinline__ floatx4 mfma16x16x4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float snake_f(float x, float a, float inv_a) {
  float s = sinf(a * x);
  return x + inv_a * (s * s);
}

// sin(y)^2 for Snake epilogues fused into other kernels: Cody-Waite reduction by pi/2 in
// three fp32 parts (exact enough for |y| < 2^17; Snake arguments are a * BatchNorm output)
// and the Cephes single-precision sin / cos polynomials on [-pi/4, pi/4] (relative error
// ~1e-7); the quadrant's sign drops out of the square.  Unlike sinf it has no Payne-Hanek
// path, whose registers would otherwise be reserved in every kernel that inlines it.
__device__ __forceinline__ float sin2_cw(float y) {
  const float k = rintf(y * 0.636619772f);
  float r = fmaf(-k, 1.57079637e+00f, y);
  r = fmaf(-k, -4.37113883e-08f, r);
  r = fmaf(-k, -1.71512451e-15f, r);
  const float z = r * r;
  const float sn = fmaf(fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f) * z, r, r);
  const float cs = fmaf(fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z,
                             4.166664568298827e-2f) * z, z, fmaf(-0.5f, z, 1.0f));
  return ((int)k & 1) ? cs * cs : sn * sn;
}

// GELU(x) = x/2 (1 + erf(x / sqrt 2)) with erf by Abramowitz-Stegun 7.1.26 (|error| <=
// 1.5e-7, branch-free: one reciprocal, one exp, a degree-5 polynomial) for eval-path
// epilogues; within fp32 noise of the exact form at the tests' 1e-4 / 1e-6 bars.  The
// training path keeps the library erff.
__device__ __forceinline__ float gelu_as(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = 1.0f - p * t * __expf(-z * z);  // erf(|x| / sqrt 2)
  return 0.5f * x * (1.0f + copysignf(e, x));
}

// counter-based RNG (Philox-lite / splitmix hash) for dropout masks: uniform in [0,1)
__device__ __forceinline__ uint32_t hash_u32(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (uint32_t)(x >> 32);
}
// dropout stream key: device-resident seed (advanced once per training step, so
// hipGraph replays draw fresh masks) mixed with a host offset (call site / call count)
__device__ __forceinline__ uint64_t mix_seed(const int64_t* seed_ptr, uint64_t offset) {
  const uint64_t s = seed_ptr ? (uint64_t)(*seed_ptr) : 0ull;
  return (s * 0x9E3779B97F4A7C15ull) ^ (offset * 0xC2B2AE3D27D4EB4Full + 0x165667B19E3779F9ull);
}
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t ctr) {
  return (hash_u32(seed * 0xD1B54A32D192ED03ull + ctr) >> 8) * (1.0f / 16777216.0f);
}

// Categorical draws by exponential race -- torch.multinomial's own n_sample = 1 algorithm
// (argmax_k p_k / q_k, q_k ~ Exp(1)), which Categorical.sample calls -- in log form:
// argmax_k l_k + g_k with g_k = -log q_k (Gumbel), ties to the lowest k.  One draw per
// (token, code), so the noise is a cheap 32-bit counter hash keyed by the call's stream
// key; u = (2j + 1) 2^-24 is exact in fp32 and strictly inside (0, 1), and q is clamped
// away from 0, so g is finite: a code whose fp32 softmax probability is 0 (l_k < max - 103)
// can never win, g being within [-2.9, 17.4].
__device__ __forceinline__ uint32_t race_key(uint64_t seed) {
  return hash_u32(seed);
}
__device__ __forceinline__ float race_gumbel(uint32_t key, uint32_t ctr) {
  // the key enters as an affine map ctr * (key | 1) + key before lowbias32 (2 multiplies:
  // per (token, code) this is hot): two calls' counter ranges meet only at scattered
  // points, never as a shifted copy of one stream (which ctr + key alone would give)
  uint32_t x = ctr * (key | 1u) + key;
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  const float u = (float)((x >> 9) * 2u + 1u) * (1.0f / 16777216.0f);
  // raw v_log_f32 (log2; u >= 2^-24 and q >= 2^-25 are normal): -ln(-ln u) without the
  // library log's denormal scaling
  const float q = fmaxf(-0.69314718f * __builtin_amdgcn_logf(u), 2.9802322e-08f);
  return -0.69314718f * __builtin_amdgcn_logf(q);
}

}  // namespace tvq

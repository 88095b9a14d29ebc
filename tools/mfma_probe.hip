// Micro-probes for the skinny-GEMM design (tools/gemm_bench.py shapes), gfx950.
//   build: hipcc -O3 --offload-arch=gfx950 tools/mfma_probe.hip -o tools/mfma_probe
//   P1 MFMA chain: each wave issues n v_mfma_f32_32x32x2_f32 on 1 or 4 accumulators
//   P2 A loads, one row per lane (the MFMA A-operand pattern), 16 B per lane per load
//   P3 the same bytes with coalesced float4 loads (consecutive lanes, consecutive 16 B)
//   P4 epilogue stores: 32x32 tile per wave, 16 stores of 2 x 128 B
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float floatx16 __attribute__((ext_vector_type(16)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int NACC>
__global__ __launch_bounds__(256) void p_mfma(float* out, int n, float x) {
  floatx16 acc[NACC];
  for (int j = 0; j < NACC; ++j)
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  float a = x * threadIdx.x, b = x + threadIdx.x;
  for (int i = 0; i < n; i += NACC)
#pragma unroll
    for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[j], 0, 0, 0);
  float s = 0.f;
  for (int j = 0; j < NACC; ++j)
    for (int r = 0; r < 16; ++r) s += acc[j][r];
  if (s == 12345.f) out[threadIdx.x] = s;
}

// rows x 128 floats; each wave reads 32 rows (lane row l&31, half h reads cols 64h..64h+63)
__global__ __launch_bounds__(256) void p_rowload(const float* A, float* out, int rows) {
  const int lane = threadIdx.x & 63, wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int row = wave * 32 + (lane & 31);
  if (row >= rows) return;
  const float* p = A + (size_t)row * 128 + 64 * (lane >> 5);
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 64; t += 4) {
    float4 v = *(const float4*)(p + t);
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.f) out[row] = s;
}

__global__ __launch_bounds__(256) void p_coload(const float* A, float* out, int rows) {
  const int lane = threadIdx.x & 63, wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const float* p = A + (size_t)wave * 32 * 128;
  if (wave * 32 >= rows) return;
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    float4 v = *(const float4*)(p + (t * 64 + lane) * 4);
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.f) out[wave] = s;
}

// C rows x 128: wave tile 32 x 32 at (wave / 4 row tile, wave % 4 col tile)
__global__ __launch_bounds__(256) void p_store(float* C, int rows) {
  const int lane = threadIdx.x & 63, wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int mt = wave / 4, nt = wave % 4;
  if (mt * 32 >= rows) return;
  const int h = lane >> 5, col = nt * 32 + (lane & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    C[(size_t)m * 128 + col] = (float)r;
  }
}

// the GEMM tile pattern: wave tile 32 x 32 of C = A (rows x 128) B (128 x 128);
// MODE bit 1: load A (else registers), bit 2: store C (else one guarded store)
template <int MODE>
__global__ __launch_bounds__(256) void p_tile(const float* A, float* C, int rows) {
  const int lane = threadIdx.x & 63, wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int mt = wave / 4, nt = wave % 4;
  if (mt * 32 >= rows) return;
  const int r32 = lane & 31, h = lane >> 5;
  float a[64];
  if (MODE & 1) {
    const float* p = A + (size_t)(mt * 32 + r32) * 128 + 64 * h;
#pragma unroll
    for (int t = 0; t < 64; t += 4) {
      const float4 v = *(const float4*)(p + t);
      a[t] = v.x; a[t + 1] = v.y; a[t + 2] = v.z; a[t + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int t = 0; t < 64; ++t) a[t] = lane * 0.001f + t;
  }
  floatx16 acc;
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
  for (int t = 0; t < 64; ++t) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t], 0.5f + t, acc, 0, 0, 0);
  const int col = nt * 32 + r32;
  if (MODE & 2) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      C[(size_t)m * 128 + col] = acc[r];
    }
  } else {
    float s = 0.f;
    for (int r = 0; r < 16; ++r) s += acc[r];
    if (s == 12345.f) C[col] = s;
  }
}

int main() {
  const int rows = 25600;
  float *A, *C, *out;
  CK(hipMalloc(&A, (size_t)rows * 128 * 4));
  CK(hipMalloc(&C, (size_t)rows * 128 * 4));
  CK(hipMalloc(&out, (size_t)rows * 4));
  CK(hipMemset(A, 0, (size_t)rows * 128 * 4));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto timeit = [&](const char* name, auto launch, double work, const char* unit) {
    for (int i = 0; i < 200; ++i) launch();  // warm clocks
    hipDeviceSynchronize();
    hipEventRecord(e0);
    const int n = 200;
    for (int i = 0; i < n; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / n;
    printf("%-34s %9.2f us  %8.2f %s\n", name, us, work / (us * 1e-6) / 1e12, unit);
  };
  // P1: 1024 blocks x 4 waves = 4096 waves (4 per SIMD) x n MFMAs
  for (int n : {64, 256}) {
    const double fl = 4096.0 * n * 2 * 32 * 32 * 2;
    char nm[64];
    snprintf(nm, sizeof nm, "mfma 1acc n=%d (4 waves/SIMD)", n);
    timeit(nm, [&] { hipLaunchKernelGGL(p_mfma<1>, dim3(1024), dim3(256), 0, 0, out, n, 1.f); }, fl, "TFLOP/s");
    snprintf(nm, sizeof nm, "mfma 4acc n=%d (4 waves/SIMD)", n);
    timeit(nm, [&] { hipLaunchKernelGGL(p_mfma<4>, dim3(1024), dim3(256), 0, 0, out, n, 1.f); }, fl, "TFLOP/s");
    const double fl1 = 1024.0 * n * 2 * 32 * 32 * 2;
    snprintf(nm, sizeof nm, "mfma 1acc n=%d (1 wave/SIMD)", n);
    timeit(nm, [&] { hipLaunchKernelGGL(p_mfma<1>, dim3(256), dim3(256), 0, 0, out, n, 1.f); }, fl1, "TFLOP/s");
  }
  const double bytes = (double)rows * 128 * 4;
  timeit("A row-per-lane loads (MFMA layout)", [&] {
    hipLaunchKernelGGL(p_rowload, dim3(rows / 128), dim3(256), 0, 0, A, out, rows); }, bytes, "TB/s");
  timeit("A coalesced float4 loads", [&] {
    hipLaunchKernelGGL(p_coload, dim3(rows / 128), dim3(256), 0, 0, A, out, rows); }, bytes, "TB/s");
  timeit("C epilogue stores (2 x 128 B)", [&] {
    hipLaunchKernelGGL(p_store, dim3(rows / 32), dim3(256), 0, 0, C, rows); }, bytes, "TB/s");
  const double fl = 2.0 * rows * 128 * 128;
  timeit("tile: MFMA only", [&] {
    hipLaunchKernelGGL(p_tile<0>, dim3(rows / 32), dim3(256), 0, 0, A, C, rows); }, fl, "TFLOP/s");
  timeit("tile: load + MFMA", [&] {
    hipLaunchKernelGGL(p_tile<1>, dim3(rows / 32), dim3(256), 0, 0, A, C, rows); }, fl, "TFLOP/s");
  timeit("tile: MFMA + store", [&] {
    hipLaunchKernelGGL(p_tile<2>, dim3(rows / 32), dim3(256), 0, 0, A, C, rows); }, fl, "TFLOP/s");
  timeit("tile: load + MFMA + store", [&] {
    hipLaunchKernelGGL(p_tile<3>, dim3(rows / 32), dim3(256), 0, 0, A, C, rows); }, fl, "TFLOP/s");
  timeit("hipMemcpy D2D same bytes (r+w)", [&] { hipMemcpyAsync(C, A, (size_t)bytes, hipMemcpyDeviceToDevice, 0); },
         2 * bytes, "TB/s");
  return 0;
}

// Issue rate of the f16 MFMA shapes on one SIMD: one wave, 8 independent accumulators, back to back.
// hipcc --offload-arch=gfx950 -O3 -o tools/probes/mfma_rate tools/probes/mfma_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
#define ITERS 4096
__global__ void k16(float* out, int salt) {
  h4 a = {(_Float16)(threadIdx.x + salt), 1, 2, 3}, b = {1, 2, 3, (_Float16)salt};
  f4 acc[8] = {};
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, acc[j], 0, 0, 0);
  }
  float s = 0;
  for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[threadIdx.x] = s;
}
__global__ void k32(float* out, int salt) {
  h8 a = {(_Float16)(threadIdx.x + salt), 1, 2, 3, 4, 5, 6, 7}, b = {1, 2, 3, (_Float16)salt, 4, 5, 6, 7};
  f4 acc[8] = {};
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[j], 0, 0, 0);
  }
  float s = 0;
  for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[threadIdx.x] = s;
}
int main() {
  float* d;
  hipMalloc(&d, 256 * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);  // kHz
  for (int rep = 0; rep < 3; ++rep) {
    for (int which = 0; which < 2; ++which) {
      hipLaunchKernelGGL(which ? k32 : k16, dim3(1), dim3(64), 0, 0, d, rep);  // warm
      hipEventRecord(e0, 0);
      for (int l = 0; l < 10; ++l) hipLaunchKernelGGL(which ? k32 : k16, dim3(1), dim3(64), 0, 0, d, rep);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double n = 10.0 * ITERS * 8;
      printf("%s: %.3f ns per MFMA, %.1f cycles at %.0f MHz (K=%d)\n", which ? "16x16x32_f16" : "16x16x16_f16",
             ms * 1e6 / n, ms * 1e-3 / n * clk * 1e3, clk / 1e3, which ? 32 : 16);
    }
  }
  hipFree(d);
  return 0;
}

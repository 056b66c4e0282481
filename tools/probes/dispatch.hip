// Launch + dispatch cost of an (almost) empty kernel with the step kernel's per-wave footprint
// (one wave per SIMD: ~410 registers forced by the waves-per-EU attribute, 13 KB of LDS per wave),
// 4096 envs as 1024 one-wave blocks (the step kernel's shape) vs 256 four-wave blocks, timed with
// HIP events over back-to-back launches on one stream.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(1, 1))) void k(float* out, int flag) {
  __shared__ float lds[WAVES][3328];  // 13 KB per wave
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  lds[w][l] = (float)l;
  if (flag) out[blockIdx.x * 64 * WAVES + threadIdx.x] = lds[w][(l + 1) & 63];
}

template <int WAVES>
float run(float* o, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(k<WAVES>, dim3(1024 / WAVES), dim3(64 * WAVES), 0, 0, o, 0);
  hipEventRecord(a, 0);
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k<WAVES>, dim3(1024 / WAVES), dim3(64 * WAVES), 0, 0, o, 0);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  // one launch bracketed by its own events (the bench's method)
  float one = 0;
  for (int i = 0; i < 100; ++i) {
    hipEventRecord(a, 0);
    hipLaunchKernelGGL(k<WAVES>, dim3(1024 / WAVES), dim3(64 * WAVES), 0, 0, o, 0);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float m = 0;
    hipEventElapsedTime(&m, a, b);
    one += m;
  }
  printf("%d-wave blocks: %.2f us per launch back to back, %.2f us per event-bracketed launch\n", WAVES,
         ms * 1000.0f / iters, one * 10.0f);
  return ms;
}

int main() {
  float* o;
  hipMalloc(&o, 1024 * 64 * 4);
  run<1>(o, 2000);
  run<4>(o, 2000);
  run<1>(o, 2000);
  run<4>(o, 2000);
  return 0;
}

// Issue rate of v_pk_fma_f32 vs v_fma_f32 for ONE wave per SIMD (1024 waves, 256-thread
// blocks of 4 waves... one block per CU): independent chains, timed with s_memtime.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef float f2 __attribute__((ext_vector_type(2)));
template <int PK>
__global__ __launch_bounds__(256) void k(float* out, uint64_t* cyc, float s) {
  float a[16];
  f2 b[8];
  for (int i = 0; i < 16; ++i) a[i] = threadIdx.x * 0.001f + i;
  for (int i = 0; i < 8; ++i) b[i] = f2{a[2 * i], a[2 * i + 1]};
  uint64_t t0, t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int it = 0; it < 1000; ++it) {
    if (PK) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(b[i]) : "v"(f2{s, s}));
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(s));
    }
  }
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  float acc = 0;
  for (int i = 0; i < 16; ++i) acc += a[i];
  for (int i = 0; i < 8; ++i) acc += b[i].x + b[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  float* o; uint64_t* c; uint64_t h[256];
  hipMalloc(&o, 256 * 256 * 4); hipMalloc(&c, 256 * 8);
  for (int pk = 0; pk < 2; ++pk) {
    for (int rep = 0; rep < 2; ++rep) {
      if (pk) hipLaunchKernelGGL(k<1>, dim3(256), dim3(256), 0, 0, o, c, 1.0001f);
      else hipLaunchKernelGGL(k<0>, dim3(256), dim3(256), 0, 0, o, c, 1.0001f);
      hipDeviceSynchronize();
    }
    hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
    double m = 0; for (int i = 0; i < 256; ++i) m += h[i]; m /= 256;
    // 1000 iterations x 16 f32 FMAs per lane either way
    printf("%s: %.2f cycles per 16 FMAs per wave (%.2f per instruction)\n", pk ? "v_pk_fma_f32" : "v_fma_f32", m / 1000,
           m / 1000 / (pk ? 8 : 16));
  }
  return 0;
}

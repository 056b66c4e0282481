// Dependent-issue latency of the VALU forms the step kernel's serial chains use, for ONE
// wave per SIMD (256 blocks x 256 threads = one wave per SIMD on 256 CUs), s_memtime.
//   indep  : 16 independent v_fma_f32 chains (the issue-rate baseline)
//   fma    : one dependent v_fma_f32 chain
//   rsq    : dependent v_rsq_f32 -> v_fma_f32 pairs (the Cholesky pivot chain)
//   rcp    : dependent v_rcp_f32 -> v_mul_f32 pairs
//   dpp    : dependent v_add_f32 with a quad_perm DPP source (qsum)
//   perm16 : dependent v_permlane16_swap -> v_add_f32 pairs (rowsum4)
//   mulfma : dependent v_mul_f32 -> v_fma_f32 pairs
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, uint64_t* cyc, float s) {
  float a[16];
  for (int i = 0; i < 16; ++i) a[i] = threadIdx.x * 0.001f + i;
  float x = a[0], y = a[1];
  uint64_t t0, t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int it = 0; it < 1000; ++it) {
    if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(s));
    } else if (MODE == 1) {
#pragma unroll
      for (int i = 0; i < 16; ++i) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(s));
    } else if (MODE == 2) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_rsq_f32 %0, %0\n\tv_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(s));
    } else if (MODE == 3) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_rcp_f32 %0, %0\n\tv_mul_f32 %0, %0, %1" : "+v"(x) : "v"(s));
    } else if (MODE == 4) {
#pragma unroll
      for (int i = 0; i < 16; ++i) asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x));
    } else if (MODE == 5) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        asm volatile("v_mov_b32 %1, %0\n\tv_permlane16_swap_b32 %0, %1\n\tv_add_f32 %0, %0, %1" : "+v"(x), "+v"(y));
    } else if (MODE == 6) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_mul_f32 %0, %0, %1\n\tv_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(s));
    } else if (MODE == 7) {  // two interleaved dependent chains
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_fma_f32 %0, %0, %2, %2\n\tv_fma_f32 %1, %1, %2, %2" : "+v"(x), "+v"(y) : "v"(s));
    }
  }
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  float acc = x + y;
  for (int i = 0; i < 16; ++i) acc += a[i];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
double run(float* o, uint64_t* c) {
  uint64_t h[256];
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(256), 0, 0, o, c, 1.0001f);
    hipDeviceSynchronize();
  }
  hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < 256; ++i) m += h[i];
  return m / 256 / 1000;  // cycles per loop iteration (16 instructions)
}

int main() {
  float* o;
  uint64_t* c;
  hipMalloc(&o, 256 * 256 * 4);
  hipMalloc(&c, 256 * 8);
  printf("cycles per instruction, one wave per SIMD\n");
  printf("indep  v_fma x16 chains      %.2f\n", run<0>(o, c) / 16);
  printf("dep    v_fma chain           %.2f\n", run<1>(o, c) / 16);
  printf("dep    v_rsq+v_fma (per pair)%.2f\n", run<2>(o, c) / 8);
  printf("dep    v_rcp+v_mul (per pair)%.2f\n", run<3>(o, c) / 8);
  printf("dep    s_nop1+v_add_dpp      %.2f\n", run<4>(o, c) / 16);
  printf("dep    mov+permlane16+add    %.2f (per triple)\n", run<5>(o, c) / 8);
  printf("dep    v_mul+v_fma (per pair)%.2f\n", run<6>(o, c) / 8);
  printf("2 dep  v_fma chains (per ins)%.2f\n", run<7>(o, c) / 16);
  return 0;
}

// How the gfx950 SQ_INSTS_VALU_{FMA,ADD,MUL,TRANS}_F32 and SQ_INSTS_VALU_MFMA_MOPS_F32 counters tally
// packed-f32 (v_pk_*) and f32 MFMA instructions: one kernel per instruction kind, one wave, a known
// number of instructions (tools/profile_r03.sh runs it under rocprofv3 --pmc; the FP32 roofline of
// bench.py turns the step kernel's counters into FLOPs with these weights).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int ITERS = 1000;  // x 8 instructions
template <int MODE>
__global__ __launch_bounds__(64) void k(float* out, float s) {
  float a[8];
  f2 b[8];
  f4 acc = {0, 0, 0, 0};
  for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x * 0.001f + i; b[i] = f2{a[i], a[i] + 1}; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (MODE == 0) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(s));
      if (MODE == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(b[i]) : "v"(f2{s, s}));
      if (MODE == 2) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(s));
      if (MODE == 3) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(b[i]) : "v"(f2{s, s}));
      if (MODE == 4) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(s));
      if (MODE == 5) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(b[i]) : "v"(f2{s, s}));
      if (MODE == 6) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], s, acc, 0, 0, 0);
      if (MODE == 7) asm volatile("v_rcp_f32 %0, %0" : "+v"(a[i]));
    }
  }
  float r = acc.x + acc.y + acc.z + acc.w;
  for (int i = 0; i < 8; ++i) r += a[i] + b[i].x + b[i].y;
  out[threadIdx.x] = r;
}
int main() {
  float* o;
  hipMalloc(&o, 64 * 4);
  const char* names[8] = {"v_fma_f32", "v_pk_fma_f32", "v_add_f32", "v_pk_add_f32", "v_mul_f32", "v_pk_mul_f32",
                          "v_mfma_f32_16x16x4_f32", "v_rcp_f32"};
  hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, o, 1.0001f);
  hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, o, 1.0001f);
  hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, o, 1.0001f);
  hipLaunchKernelGGL(k<3>, dim3(1), dim3(64), 0, 0, o, 1.0001f);
  hipLaunchKernelGGL(k<4>, dim3(1), dim3(64), 0, 0, o, 1.0001f);
  hipLaunchKernelGGL(k<5>, dim3(1), dim3(64), 0, 0, o, 1.0001f);
  hipLaunchKernelGGL(k<6>, dim3(1), dim3(64), 0, 0, o, 1.0001f);
  hipLaunchKernelGGL(k<7>, dim3(1), dim3(64), 0, 0, o, 1.0001f);
  hipDeviceSynchronize();
  for (int m = 0; m < 8; ++m) printf("dispatch %d: %s x %d per wave\n", m + 1, names[m], 8 * ITERS);
  return 0;
}

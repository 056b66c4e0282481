// Semantics probe: DPP row_ror:k on gfx950 (which lane does lane i read from?)
#include <hip/hip_runtime.h>
#include <cstdio>
template <int CTRL>
__global__ void k(int* out) {
  int v = threadIdx.x;
  out[threadIdx.x] = __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false);
}
int main() {
  int* d; int h[64];
  (void)hipMalloc(&d, 64 * 4);
  hipLaunchKernelGGL(k<0x124>, dim3(1), dim3(64), 0, 0, d);
  (void)hipMemcpy(h, d, 256, hipMemcpyDeviceToHost);
  printf("row_ror:4  lanes 0..15 read from:"); for (int i = 0; i < 16; ++i) printf(" %d", h[i]); printf("\n");
  hipLaunchKernelGGL(k<0x128>, dim3(1), dim3(64), 0, 0, d);
  (void)hipMemcpy(h, d, 256, hipMemcpyDeviceToHost);
  printf("row_ror:8  lanes 0..15 read from:"); for (int i = 0; i < 16; ++i) printf(" %d", h[i]); printf("\n");
  hipLaunchKernelGGL(k<0x12C>, dim3(1), dim3(64), 0, 0, d);
  (void)hipMemcpy(h, d, 256, hipMemcpyDeviceToHost);
  printf("row_ror:12 lanes 0..15 read from:"); for (int i = 0; i < 16; ++i) printf(" %d", h[i]); printf("\n");
  return 0;
}

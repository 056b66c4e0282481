// Exhaustive check (all 2^32 f32 inputs) of the actuator net's softsign x / (|x| + 1):
// pm_softsign and pm_softsign2 (legged_tracking_amd/csrc/pmath.h, the product code) must
// be bit-identical to the IEEE division for every input (NaN for NaN / inf inputs).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/probes/softsign_div.hip -o tools/probes/sdiv
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#include "../../legged_tracking_amd/csrc/pmath.h"

__device__ __forceinline__ bool same(float a, float b) {
  return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
}

__global__ void check(unsigned long long* bad, uint32_t* example, uint64_t base) {
  const uint64_t idx = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t bits = (uint32_t)idx;
  const float x = __uint_as_float(bits);
  const float ref = x / (fabsf(x) + 1.0f);
  // a second input for the other half of the pair: the bit-reversed pattern
  const float y = __uint_as_float(__brev(bits));
  const float refy = y / (fabsf(y) + 1.0f);
  const float s = pm_softsign(x);
  const pm_f2 p = pm_softsign2(pm_f2{x, y});
  if (!same(s, ref)) { atomicAdd(&bad[0], 1ull); example[0] = bits; }
  if (!same(p.x, ref) || !same(p.y, refy)) { atomicAdd(&bad[1], 1ull); example[1] = bits; }
}

int main() {
  unsigned long long* bad;
  uint32_t* ex;
  if (hipMalloc(&bad, 16) != hipSuccess || hipMalloc(&ex, 8) != hipSuccess) return 2;
  (void)hipMemset(bad, 0, 16);
  (void)hipMemset(ex, 0, 8);
  const uint64_t chunk = 1ull << 30;
  for (uint64_t b = 0; b < (1ull << 32); b += chunk)
    hipLaunchKernelGGL(check, dim3(chunk / 256), dim3(256), 0, 0, bad, ex, b);
  unsigned long long h[2];
  uint32_t he[2];
  (void)hipMemcpy(h, bad, 16, hipMemcpyDeviceToHost);
  (void)hipMemcpy(he, ex, 8, hipMemcpyDeviceToHost);
  printf("pm_softsign  mismatches vs IEEE: %llu (e.g. 0x%08x)\n", h[0], he[0]);
  printf("pm_softsign2 mismatches vs IEEE: %llu (e.g. 0x%08x)\n", h[1], he[1]);
  return (h[0] || h[1]) ? 1 : 0;
}

// Exhaustive check (all 2^32 f32 inputs): is softsign x / (|x| + 1) computed with a
// hardware-reciprocal + FMA correction bit-identical to the IEEE division?
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/probes/softsign_div.hip -o /tmp/sdiv
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void check(unsigned long long* bad, uint32_t* example, uint64_t base) {
  uint64_t idx = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t bits = (uint32_t)idx;
  float x = __uint_as_float(bits);
  if (!isfinite(x)) return;
  float d = fabsf(x) + 1.0f;
  float ref = x / d;
  float r = __builtin_amdgcn_rcpf(d);
  // A: one correction step on the quotient
  float q = x * r;
  float e = fmaf(-q, d, x);
  float qa = fmaf(e, r, q);
  // B: refine the reciprocal first
  float rr = fmaf(fmaf(-d, r, 1.0f), r, r);
  float q2 = x * rr;
  float e2 = fmaf(-q2, d, x);
  float qb = fmaf(e2, rr, q2);
  if (__float_as_uint(qa) != __float_as_uint(ref)) { atomicAdd(&bad[0], 1ull); example[0] = bits; }
  if (__float_as_uint(qb) != __float_as_uint(ref)) { atomicAdd(&bad[1], 1ull); example[1] = bits; }
}

int main() {
  unsigned long long* bad; uint32_t* ex;
  hipMalloc(&bad, 16); hipMalloc(&ex, 8);
  hipMemset(bad, 0, 16); hipMemset(ex, 0, 8);
  const uint64_t chunk = 1ull << 30;
  for (uint64_t b = 0; b < (1ull << 32); b += chunk)
    hipLaunchKernelGGL(check, dim3(chunk / 256), dim3(256), 0, 0, bad, ex, b);
  unsigned long long h[2]; uint32_t he[2];
  hipMemcpy(h, bad, 16, hipMemcpyDeviceToHost); hipMemcpy(he, ex, 8, hipMemcpyDeviceToHost);
  printf("mismatches A (q-correction) = %llu (e.g. 0x%08x)\n", h[0], he[0]);
  printf("mismatches B (rcp refine + q-correction) = %llu (e.g. 0x%08x)\n", h[1], he[1]);
  return 0;
}

/*
 * pmath.h -- deterministic f32 transcendentals for the HIP kernels (product copy).
 *
 * Deterministic f32 sin/cos/asin/atan2 built only from IEEE-exact operations
 * (+ - * / sqrt, fmaf, rintf, fabsf, copysignf), so these kernels and the CPU
 * oracle (which carries its own copy, oracle/portable_math.h) produce
 * bit-identical height-scan inputs and rpy angles.  Algorithms: Cody-Waite reduction by pi/2 and
 * the single-precision minimax polynomials of the Cephes library (sinf/cosf,
 * asinf, atanf).  Accuracy ~1-2 ulp vs the correctly rounded value; torch's
 * own f32 functions differ from either at the ulp level, which the parity
 * tests absorb in their stated float tolerance.
 *
 * Compile with -ffp-contract=off: every a*b+c written below without fmaf must
 * stay two roundings.
 */
#ifndef GO1_PMATH_H
#define GO1_PMATH_H
#include <hip/hip_runtime.h>
#define PM_FN __device__ __forceinline__

#define PM_PIO2_HI 1.5703125f
#define PM_PIO2_MID 4.837512969970703125e-4f
#define PM_PIO2_LO 7.54978995489188216e-8f
#define PM_2_PI 0.636619772367581343f
#define PM_PIO2 1.57079632679489661923f
#define PM_PIO4 0.785398163397448309616f
#define PM_PI 3.14159265358979323846f

PM_FN float pm_sin_poly(float r) {
  float z = r * r;
  float p = fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
  return fmaf(p * z, r, r);
}

PM_FN float pm_cos_poly(float r) {
  float z = r * r;
  float p = fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
  return fmaf(p * z, z, fmaf(-0.5f, z, 1.0f));
}

/* sin and cos of x, |x| <= ~1e3 */
PM_FN void pm_sincosf(float x, float* s, float* c) {
  float j = rintf(x * PM_2_PI);
  float r = fmaf(-j, PM_PIO2_HI, x);
  r = fmaf(-j, PM_PIO2_MID, r);
  r = fmaf(-j, PM_PIO2_LO, r);
  /* bounded before the conversion: a NaN / huge argument must not be undefined behaviour */
  int q = ((int)fminf(fmaxf(j, -1.0e6f), 1.0e6f)) & 3;
  float sp = pm_sin_poly(r), cp = pm_cos_poly(r);
  /* quadrant by bit-test selects (a switch would become divergent branches):
     q = 0: (sp, cp), 1: (cp, -sp), 2: (-sp, -cp), 3: (-cp, sp) */
  const bool swap = q & 1, sneg = q & 2, cneg = (q ^ (q >> 1)) & 1;
  const float a = swap ? cp : sp, b = swap ? sp : cp;
  *s = sneg ? -a : a;
  *c = cneg ? -b : b;
}

PM_FN float pm_sinf(float x) { float s, c; pm_sincosf(x, &s, &c); return s; }
PM_FN float pm_cosf(float x) { float s, c; pm_sincosf(x, &s, &c); return c; }

/* asin / atan / atan2 with every case computed and the result selected: as if / else on the argument's range the
 * cases were exec-mask branches, one wave paying each arm (and its IEEE division) in turn.  The arithmetic of each
 * case is unchanged (atan's third case divides by 1.0, which is exact), so the results are bit for bit those of the
 * branching form and of oracle/portable_math.h. */
PM_FN float pm_asinf(float x) {
  const float a = fabsf(x);
  const bool big = a > 0.5f;
  const float zb = 0.5f * (1.0f - a);
  const float z = big ? zb : a * a, s = big ? sqrtf(zb) : a;
  float p = fmaf(fmaf(fmaf(fmaf(4.2163199048e-2f, z, 2.4181311049e-2f), z, 4.5470025998e-2f), z,
                      7.4953002686e-2f), z, 1.6666752422e-1f);
  float r = fmaf(p * z, s, s);
  r = big ? PM_PIO2 - (r + r) : r;
  return copysignf(r, x);
}

PM_FN float pm_atanf(float x) {
  const float a = fabsf(x);
  const bool big = a > 2.414213562373095f, mid = a > 0.4142135623730950f;
  const float y0 = big ? PM_PIO2 : (mid ? PM_PIO4 : 0.0f);
  const float num = big ? -1.0f : (mid ? a - 1.0f : a), den = big ? a : (mid ? a + 1.0f : 1.0f);
  const float t = num / den;
  float z = t * t;
  float p = fmaf(fmaf(fmaf(8.05374449538e-2f, z, -1.38776856032e-1f), z, 1.99777106478e-1f), z,
                 -3.33329491539e-1f);
  float r = y0 + fmaf(p * z, t, t);
  return copysignf(r, x);
}

PM_FN float pm_atan2f(float y, float x) {
  const float r0 = pm_atanf(y / x);  // (x = 0: inf or NaN, selected away below)
  const bool yneg = y < 0.0f || (y == 0.0f && __builtin_signbit(y));
  const float r1 = x < 0.0f ? (yneg ? r0 - PM_PI : r0 + PM_PI) : r0;
  const float rz = y == 0.0f ? (__builtin_signbit(x) ? copysignf(PM_PI, y) : copysignf(0.0f, y)) : copysignf(PM_PIO2, y);
  return x == 0.0f ? rz : r1;
}

/* ---- softsign x / (|x| + 1) of the actuator net, bit-identical to the IEEE quotient for
 * every f32 input (exhaustive check of both forms over all 2^32 inputs on gfx950:
 * tools/probes/softsign_div.hip).  Fast form: hardware reciprocal of d = |x| + 1 and one
 * FMA residual correction of the quotient, exact for all finite |x| < 2^126.  For
 * |x| >= 2^30 the IEEE quotient is exactly +-1 (|x| + 1 rounds to |x|), which is also what
 * the fast form returns for an input clamped to +-2^30, so the input is clamped there
 * (between 2^24 and 2^25 |x| + 1 can round UP, and the quotient is then not +-1);
 * fma(q, x - x, q) returns q for finite x and NaN for inf / NaN, as IEEE does. */
#ifndef GO1_FAST_SOFTSIGN
#define GO1_FAST_SOFTSIGN 1
#endif
typedef float pm_f2 __attribute__((ext_vector_type(2)));
#define PM_SOFTSIGN_LIM 1073741824.0f /* 2^30 */

PM_FN float pm_softsign(float x) {
#if GO1_FAST_SOFTSIGN
  const float xc = __builtin_amdgcn_fmed3f(x, -PM_SOFTSIGN_LIM, PM_SOFTSIGN_LIM);
  const float d = fabsf(xc) + 1.0f;
  const float r = __builtin_amdgcn_rcpf(d);
  const float q0 = xc * r;
  /* residual t = q0 d - x, q = q0 - t r: the same roundings as q0 + (x - q0 d) r, and the
     sign of a zero quotient survives (-0 -> -0) */
  const float q = fmaf(-fmaf(q0, d, -xc), r, q0);
  return fmaf(q, x - x, q);
#else
  return x / (fabsf(x) + 1.0f);
#endif
}

/* two softsigns in the halves of v_pk_mul / v_pk_fma (same roundings as pm_softsign) */
PM_FN pm_f2 pm_softsign2(pm_f2 x) {
#if GO1_FAST_SOFTSIGN
  /* one v_med3_f32 per half: fminf / fmaxf add a canonicalising v_max_f32 each (a NaN x
     becomes NaN again through the final fma with x - x, whatever the clamp returns) */
  const pm_f2 xc = {__builtin_amdgcn_fmed3f(x.x, -PM_SOFTSIGN_LIM, PM_SOFTSIGN_LIM),
                    __builtin_amdgcn_fmed3f(x.y, -PM_SOFTSIGN_LIM, PM_SOFTSIGN_LIM)};
  const pm_f2 d = {fabsf(xc.x) + 1.0f, fabsf(xc.y) + 1.0f};
  const pm_f2 r = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  const pm_f2 q0 = xc * r;
  const pm_f2 q = __builtin_elementwise_fma(-__builtin_elementwise_fma(q0, d, -xc), r, q0);
  return __builtin_elementwise_fma(q, x - x, q);
#else
  return pm_f2{x.x / (fabsf(x.x) + 1.0f), x.y / (fabsf(x.y) + 1.0f)};
#endif
}

#endif

// go1_step.hip -- MI355X (gfx950) fused Go1 trajectory-tracking step + C ABI.
//
// One launch = one LeggedRobot.step() for every env
// (go1_gym/envs/base/legged_robot_trajectory_tracking.py:64-169):
//   4 x [actuator-net torques (:957-996, :1311-1320) -> native articulated-body
//        integrator (replaces gym.simulate / fetch_results / refresh, :82-88)]
//   -> post-physics: kinematics (:130-136), height scan (:1918-1970), target and
//      command logic (:774-932), terminations (:198-216), RewardsCrawling terms
//      (:320-355), reset_idx (:218-296), observations (:357-475), epilogue (:148-153).
//
// Decomposition: one env = one quad of lanes, lane l = leg l (FL, FR, RL, RR).
// A 64-lane wave carries 16 envs; a block is one wave (4096 envs -> 256 blocks,
// one per CU).  Each lane runs its leg's three actuator-net evaluations, its
// leg's forward kinematics, contacts and ABA backward pass; the leg's
// articulated inertia and bias force are summed over the quad with DPP-level
// shuffles (__shfl_xor 1, 2), every lane of the quad solves the 6x6 base system
// redundantly (bit-identical), then runs its leg's forward pass.
// State is SoA row-major (n_envs, width) in HBM: a wave reads 16 contiguous env
// rows per field (coalesced); nothing is staged through LDS because no datum is
// shared between envs except the config/weights (scalar loads, SGPR-resident).
//
// Numerics: the post-physics section is compiled with FP contraction OFF and
// uses the deterministic transcendentals of pmath.h, so it is bit-identical to
// the CPU oracle (oracle/go1_oracle.c) given the same physical state; the
// integrator uses FMA contraction and native sin/cos (f32, compared with the
// oracle's f64 integrator within a tolerance).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <new>
#include <string>

#include "../../include/go1_mi355x.h"
#include "pmath.h"

#pragma clang fp contract(off)

#define NDOF 12
#define NB 17
#define EPB 16          // envs per block
#define TPB (EPB * 4)   // one wave
#define PI_F 3.14159265358979323846f
#define TWO_PI_F 6.28318548202514648438f  // (float)(2*pi), torch's f32 scalar

// ---------------------------------------------------------------- Philox
__device__ __forceinline__ void philox4x32(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t l0 = 0xD2511F53u * c[0], h0 = __umulhi(0xD2511F53u, c[0]);
    uint32_t l1 = 0xCD9E8D57u * c[2], h1 = __umulhi(0xCD9E8D57u, c[2]);
    uint32_t n0 = h1 ^ c[1] ^ k0, n2 = h0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = l1; c[2] = n2; c[3] = l0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}

struct Rng {
  const float* U;  // parity-mode uniforms or nullptr
  uint64_t seed, step;
  int e;
  __device__ float operator()(int slot) const {
    if (U) return U[(size_t)e * GO1_U_PER_ENV + slot];
    uint32_t c[4] = {(uint32_t)e, (uint32_t)slot >> 2, (uint32_t)step, (uint32_t)(step >> 32)};
    philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    return (float)(c[slot & 3] >> 8) * (1.0f / 16777216.0f);
  }
};

// ---------------------------------------------------------------- quad helpers
__device__ __forceinline__ float qsum(float v) {
  v = v + __shfl_xor(v, 1);
  v = v + __shfl_xor(v, 2);
  return v;
}

// ---------------------------------------------------------------- actuator net
// Bit-identical to go1o_actuator_eval: every output is an fmaf chain over k in
// increasing order seeded with the bias; softsign x / (|x| + 1) in IEEE division.
__device__ __forceinline__ float actuator_eval(const float* __restrict__ W, float x0, float x1, float x2, float x3,
                                               float x4, float x5) {
  float h1[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    float acc = W[192 + k];
    acc = fmaf(W[k * 6 + 0], x0, acc);
    acc = fmaf(W[k * 6 + 1], x1, acc);
    acc = fmaf(W[k * 6 + 2], x2, acc);
    acc = fmaf(W[k * 6 + 3], x3, acc);
    acc = fmaf(W[k * 6 + 4], x4, acc);
    acc = fmaf(W[k * 6 + 5], x5, acc);
    h1[k] = acc / (fabsf(acc) + 1.0f);
  }
  float out = W[1312];
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    float acc = W[1248 + k];
#pragma unroll
    for (int i = 0; i < 32; ++i) acc = fmaf(W[224 + k * 32 + i], h1[i], acc);
    float h2 = acc / (fabsf(acc) + 1.0f);
    out = fmaf(W[1280 + k], h2, out);
  }
  return out;
}

// ---------------------------------------------------------------- torch-order f32 math
__device__ __forceinline__ void quat_rotate_inverse_f(const float* q, const float* v, float* out) {
  float qw = q[3];
  float s = 2.0f * (qw * qw) - 1.0f;
  float a0 = v[0] * s, a1 = v[1] * s, a2 = v[2] * s;
  float c0 = q[1] * v[2] - q[2] * v[1];
  float c1 = q[2] * v[0] - q[0] * v[2];
  float c2 = q[0] * v[1] - q[1] * v[0];
  float b0 = c0 * qw * 2.0f, b1 = c1 * qw * 2.0f, b2 = c2 * qw * 2.0f;
  float d = q[0] * v[0] + q[1] * v[1] + q[2] * v[2];
  float e0 = q[0] * d * 2.0f, e1 = q[1] * d * 2.0f, e2 = q[2] * d * 2.0f;
  out[0] = a0 - b0 + e0;
  out[1] = a1 - b1 + e1;
  out[2] = a2 - b2 + e2;
}

__device__ __forceinline__ void quat_apply_yaw_inverse_f(const float* q, const float* v, float* out) {
  float qy[4] = {0.0f, 0.0f, q[2], q[3]};
  float n2 = fmaf(qy[3], qy[3], fmaf(qy[2], qy[2], fmaf(qy[1], qy[1], qy[0] * qy[0])));
  float n = sqrtf(n2);
  if (n < 1e-9f) n = 1e-9f;
#pragma unroll
  for (int i = 0; i < 4; ++i) qy[i] = qy[i] / n;
  quat_rotate_inverse_f(qy, v, out);
}

__device__ __forceinline__ float remainder_f(float a, float b) {
  float m = fmodf(a, b);
  if (m != 0.0f && ((b < 0.0f) != (m < 0.0f))) m += b;
  return m;
}

__device__ __forceinline__ float wrap_to_pi_f(float a) {
  a = remainder_f(a, TWO_PI_F);
  if (a > PI_F) a = a - TWO_PI_F;
  return a;
}

__device__ __forceinline__ void quat_to_rpy_f(const float* q, float* rpy) {
  float qx = q[0], qy = q[1], qz = q[2], qw = q[3];
  float sinr = 2.0f * (qw * qx + qy * qz);
  float cosr = qw * qw - qx * qx - qy * qy + qz * qz;
  float roll = pm_atan2f(sinr, cosr);
  float sinp = 2.0f * (qw * qy - qz * qx);
  float pitch = fabsf(sinp) >= 1.0f ? copysignf(PM_PIO2, sinp) : pm_asinf(sinp);
  float siny = 2.0f * (qw * qz + qx * qy);
  float cosy = qw * qw + qx * qx - qy * qy - qz * qz;
  float yaw = pm_atan2f(siny, cosy);
  rpy[0] = wrap_to_pi_f(remainder_f(roll, TWO_PI_F));
  rpy[1] = wrap_to_pi_f(remainder_f(pitch, TWO_PI_F));
  rpy[2] = wrap_to_pi_f(remainder_f(yaw, TWO_PI_F));
}

__device__ __forceinline__ float norm2_f(float x, float y) { return sqrtf(fmaf(y, y, x * x)); }
__device__ __forceinline__ float norm3_f(float x, float y, float z) { return sqrtf(fmaf(z, z, fmaf(y, y, x * x))); }
__device__ __forceinline__ float sq_f(float x) { return x * x; }
__device__ __forceinline__ float clampf(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }

// =====================================================================
//                  native articulated-body integrator (f32)
// =====================================================================
// Spatial vectors (angular; linear).  6x6 symmetric articulated inertia stored as
// [[A, B], [B^T, C]], A and C symmetric (xx xy xz yy yz zz), B row-major 3x3.
struct SI {
  float a[6], b[9], c[6];
};

#define S3(m, i, j) m[((i) == 0 ? ((j) == 0 ? 0 : (j) == 1 ? 1 : 2) : (i) == 1 ? ((j) == 0 ? 1 : (j) == 1 ? 3 : 4) : ((j) == 0 ? 2 : (j) == 1 ? 4 : 5))]

__device__ __forceinline__ void cross3(const float* a, const float* b, float* o) {
  float x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
  o[0] = x; o[1] = y; o[2] = z;
}

// y = M v for the symmetric spatial matrix
__device__ __forceinline__ void si_mul(const SI& M, const float* v, float* o) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    float s = 0.0f, t = 0.0f;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      s += S3(M.a, i, j) * v[j] + M.b[i * 3 + j] * v[3 + j];
      t += M.b[j * 3 + i] * v[j] + S3(M.c, i, j) * v[3 + j];
    }
    o[i] = s;
    o[3 + i] = t;
  }
}

__device__ __forceinline__ float si_get(const SI& M, int i, int j) {
  if (i < 3 && j < 3) return S3(M.a, i, j);
  if (i >= 3 && j >= 3) return S3(M.c, i - 3, j - 3);
  if (i < 3) return M.b[i * 3 + (j - 3)];
  return M.b[j * 3 + (i - 3)];
}

// rigid-body spatial inertia about the link origin
__device__ __forceinline__ void rigid_si(const float* body, float mscale, SI& I) {
  float m = body[0] * mscale;
  float c0 = body[1], c1 = body[2], c2 = body[3];
  float cc = c0 * c0 + c1 * c1 + c2 * c2;
  I.a[0] = body[4] * mscale + m * (cc - c0 * c0);
  I.a[1] = body[5] * mscale - m * c0 * c1;
  I.a[2] = body[6] * mscale - m * c0 * c2;
  I.a[3] = body[7] * mscale + m * (cc - c1 * c1);
  I.a[4] = body[8] * mscale - m * c1 * c2;
  I.a[5] = body[9] * mscale + m * (cc - c2 * c2);
  // B = m c~
  I.b[0] = 0.0f; I.b[1] = -m * c2; I.b[2] = m * c1;
  I.b[3] = m * c2; I.b[4] = 0.0f; I.b[5] = -m * c0;
  I.b[6] = -m * c1; I.b[7] = m * c0; I.b[8] = 0.0f;
  I.c[0] = m; I.c[1] = 0.0f; I.c[2] = 0.0f; I.c[3] = m; I.c[4] = 0.0f; I.c[5] = m;
}

// force cross product v x* f
__device__ __forceinline__ void crf(const float* v, const float* f, float* o) {
  float a[3], b[3], c[3];
  cross3(v, f, a);
  cross3(v + 3, f + 3, b);
  cross3(v, f + 3, c);
  o[0] = a[0] + b[0]; o[1] = a[1] + b[1]; o[2] = a[2] + b[2];
  o[3] = c[0]; o[4] = c[1]; o[5] = c[2];
}

// revolute joint about coordinate axis ax (0 = x, 1 = y): E = Rot(ax, q)^T
__device__ __forceinline__ void joint_E(int ax, float c, float s, float E[9]) {
  if (ax == 0) {
    E[0] = 1; E[1] = 0; E[2] = 0; E[3] = 0; E[4] = c; E[5] = s; E[6] = 0; E[7] = -s; E[8] = c;
  } else {
    E[0] = c; E[1] = 0; E[2] = -s; E[3] = 0; E[4] = 1; E[5] = 0; E[6] = s; E[7] = 0; E[8] = c;
  }
}

__device__ __forceinline__ void mat3_vec(const float* E, const float* v, float* o) {
  float x = E[0] * v[0] + E[1] * v[1] + E[2] * v[2];
  float y = E[3] * v[0] + E[4] * v[1] + E[5] * v[2];
  float z = E[6] * v[0] + E[7] * v[1] + E[8] * v[2];
  o[0] = x; o[1] = y; o[2] = z;
}

__device__ __forceinline__ void mat3T_vec(const float* E, const float* v, float* o) {
  float x = E[0] * v[0] + E[3] * v[1] + E[6] * v[2];
  float y = E[1] * v[0] + E[4] * v[1] + E[7] * v[2];
  float z = E[2] * v[0] + E[5] * v[1] + E[8] * v[2];
  o[0] = x; o[1] = y; o[2] = z;
}

// motion transform parent -> child
__device__ __forceinline__ void xm(const float* E, const float* r, const float* vin, float* vout) {
  float rw[3], t[3];
  cross3(r, vin, rw);
  t[0] = vin[3] - rw[0]; t[1] = vin[4] - rw[1]; t[2] = vin[5] - rw[2];
  float w[3], v[3];
  mat3_vec(E, vin, w);
  mat3_vec(E, t, v);
  vout[0] = w[0]; vout[1] = w[1]; vout[2] = w[2]; vout[3] = v[0]; vout[4] = v[1]; vout[5] = v[2];
}

// force transform child -> parent
__device__ __forceinline__ void xfT(const float* E, const float* r, const float* fin, float* fout) {
  float n[3], f[3], rf[3];
  mat3T_vec(E, fin, n);
  mat3T_vec(E, fin + 3, f);
  cross3(r, f, rf);
  fout[0] = n[0] + rf[0]; fout[1] = n[1] + rf[1]; fout[2] = n[2] + rf[2];
  fout[3] = f[0]; fout[4] = f[1]; fout[5] = f[2];
}

// X^T Ia X for X = [[E, 0], [-E r~, E]]: rotate blocks by E^T(.)E, then translate by r.
__device__ __forceinline__ void xform_inertia(const float* E, const float* r, const SI& In, SI& Out) {
  float A[9], B[9], C[9], T[9];
  // A' = E^T A E
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float s = 0.0f;
#pragma unroll
      for (int k = 0; k < 3; ++k) s += S3(In.a, i, k) * E[k * 3 + j];
      T[i * 3 + j] = s;
    }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float s = 0.0f;
#pragma unroll
      for (int k = 0; k < 3; ++k) s += E[k * 3 + i] * T[k * 3 + j];
      A[i * 3 + j] = s;
    }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float s = 0.0f;
#pragma unroll
      for (int k = 0; k < 3; ++k) s += In.b[i * 3 + k] * E[k * 3 + j];
      T[i * 3 + j] = s;
    }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float s = 0.0f;
#pragma unroll
      for (int k = 0; k < 3; ++k) s += E[k * 3 + i] * T[k * 3 + j];
      B[i * 3 + j] = s;
    }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float s = 0.0f;
#pragma unroll
      for (int k = 0; k < 3; ++k) s += S3(In.c, i, k) * E[k * 3 + j];
      T[i * 3 + j] = s;
    }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float s = 0.0f;
#pragma unroll
      for (int k = 0; k < 3; ++k) s += E[k * 3 + i] * T[k * 3 + j];
      C[i * 3 + j] = s;
    }
  // translate: A'' = A' + r~ B'^T - B' r~ - r~ C' r~ ; B'' = B' + r~ C'
  float rx[9] = {0.0f, -r[2], r[1], r[2], 0.0f, -r[0], -r[1], r[0], 0.0f};
  float RC[9], RBt[9], BR[9], RCR[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float s = 0.0f, t = 0.0f, u = 0.0f;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        s += rx[i * 3 + k] * C[k * 3 + j];
        t += rx[i * 3 + k] * B[j * 3 + k];
        u += B[i * 3 + k] * rx[k * 3 + j];
      }
      RC[i * 3 + j] = s;
      RBt[i * 3 + j] = t;
      BR[i * 3 + j] = u;
    }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float s = 0.0f;
#pragma unroll
      for (int k = 0; k < 3; ++k) s += RC[i * 3 + k] * rx[k * 3 + j];
      RCR[i * 3 + j] = s;
    }
  float Af[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) Af[i] = A[i] + RBt[i] - BR[i] - RCR[i];
  Out.a[0] = Af[0]; Out.a[1] = 0.5f * (Af[1] + Af[3]); Out.a[2] = 0.5f * (Af[2] + Af[6]);
  Out.a[3] = Af[4]; Out.a[4] = 0.5f * (Af[5] + Af[7]); Out.a[5] = Af[8];
#pragma unroll
  for (int i = 0; i < 9; ++i) Out.b[i] = B[i] + RC[i];
  Out.c[0] = C[0]; Out.c[1] = 0.5f * (C[1] + C[3]); Out.c[2] = 0.5f * (C[2] + C[6]);
  Out.c[3] = C[4]; Out.c[4] = 0.5f * (C[5] + C[7]); Out.c[5] = C[8];
}

__device__ __forceinline__ void si_add(SI& A, const SI& B) {
#pragma unroll
  for (int i = 0; i < 6; ++i) { A.a[i] += B.a[i]; A.c[i] += B.c[i]; }
#pragma unroll
  for (int i = 0; i < 9; ++i) A.b[i] += B.b[i];
}

// 6x6 SPD solve (Cholesky), identical instruction stream in every lane of a quad
__device__ __forceinline__ void solve6(const SI& M, const float* b, float* x) {
  float L[21];
#define LI(i, j) L[(i) * ((i) + 1) / 2 + (j)]
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j <= i; ++j) {
      float s = si_get(M, i, j);
#pragma unroll
      for (int k = 0; k < j; ++k) s -= LI(i, k) * LI(j, k);
      if (i == j) LI(i, i) = sqrtf(fmaxf(s, 1e-30f));
      else LI(i, j) = s / LI(j, j);
    }
  float y[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    float s = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) s -= LI(i, k) * y[k];
    y[i] = s / LI(i, i);
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    float s = y[i];
#pragma unroll
    for (int k = i + 1; k < 6; ++k) s -= LI(k, i) * x[k];
    x[i] = s / LI(i, i);
  }
#undef LI
}

__device__ __forceinline__ void quat_to_R(const float* q, float* R) {
  float x = q[0], y = q[1], z = q[2], w = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - z * w); R[2] = 2 * (x * z + y * w);
  R[3] = 2 * (x * y + z * w); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - x * w);
  R[6] = 2 * (x * z - y * w); R[7] = 2 * (y * z + x * w); R[8] = 1 - 2 * (x * x + y * y);
}

struct Terr {
  const float* tile;  // (2, nx, ny) or nullptr
  int nx, ny;
  float ox, oy, hs;
};

__device__ __forceinline__ float tile_at(const Terr& T, int layer, int i, int j) {
  i = min(max(i, 0), T.nx - 1);
  j = min(max(j, 0), T.ny - 1);
  return T.tile[((size_t)layer * T.nx + i) * T.ny + j];
}

__device__ __forceinline__ void height_query(const Terr& T, int layer, float x, float y, float& h, float& gx,
                                             float& gy) {
  if (!T.tile) {
    h = layer == 1 ? 0.0f : 1e9f;
    gx = gy = 0.0f;
    return;
  }
  float u = (x - T.ox) / T.hs, v = (y - T.oy) / T.hs;
  float fu = floorf(u), fv = floorf(v);
  int i = (int)fu, j = (int)fv;
  float a = u - fu, b = v - fv;
  float h00 = tile_at(T, layer, i, j), h10 = tile_at(T, layer, i + 1, j);
  float h01 = tile_at(T, layer, i, j + 1), h11 = tile_at(T, layer, i + 1, j + 1);
  h = (1 - a) * (1 - b) * h00 + a * (1 - b) * h10 + (1 - a) * b * h01 + a * b * h11;
  gx = ((1 - b) * (h10 - h00) + b * (h11 - h01)) / T.hs;
  gy = ((1 - a) * (h01 - h00) + a * (h11 - h10)) / T.hs;
}

struct CP {
  float k, d, kf, mu;
};

__device__ __forceinline__ void sphere_contact(const Terr& T, const CP& C, const float* p, const float* pv, float r,
                                               float* F) {
  F[0] = F[1] = F[2] = 0.0f;
#pragma unroll
  for (int layer = 1; layer >= 0; --layer) {
    float h, gx, gy;
    height_query(T, layer, p[0], p[1], h, gx, gy);
    float n[3], dv;
    if (layer == 1) {
      dv = h + r - p[2];
      n[0] = -gx; n[1] = -gy; n[2] = 1.0f;
    } else {
      dv = p[2] + r - h;
      n[0] = gx; n[1] = gy; n[2] = -1.0f;
    }
    if (dv <= 0.0f) continue;
    float inv = 1.0f / sqrtf(n[0] * n[0] + n[1] * n[1] + 1.0f);
    n[0] *= inv; n[1] *= inv; n[2] *= inv;
    float depth = dv * inv;
    float vn = pv[0] * n[0] + pv[1] * n[1] + pv[2] * n[2];
    float fn = C.k * depth - C.d * vn;
    if (fn <= 0.0f) continue;
    float vt[3] = {pv[0] - vn * n[0], pv[1] - vn * n[1], pv[2] - vn * n[2]};
    float vtn = sqrtf(vt[0] * vt[0] + vt[1] * vt[1] + vt[2] * vt[2]);
    float ft = fminf(C.kf * vtn, C.mu * fn);
    float s = vtn > 1e-9f ? ft / vtn : 0.0f;
    F[0] += fn * n[0] - s * vt[0];
    F[1] += fn * n[1] - s * vt[1];
    F[2] += fn * n[2] - s * vt[2];
  }
}

__device__ __forceinline__ void point_kin(const float* Rb, const float* pb, const float* vb, const float* lp, float* pw,
                                          float* vw) {
  float wl[3], vl[3];
  cross3(vb, lp, wl);
  vl[0] = vb[3] + wl[0]; vl[1] = vb[4] + wl[1]; vl[2] = vb[5] + wl[2];
  float t[3];
  mat3_vec(Rb, lp, t);
  pw[0] = pb[0] + t[0]; pw[1] = pb[1] + t[1]; pw[2] = pb[2] + t[2];
  mat3_vec(Rb, vl, vw);
}

__device__ __forceinline__ void point_force(const float* Rb, const float* lp, const float* F, float* fs) {
  float f[3], n[3];
  mat3T_vec(Rb, F, f);
  cross3(lp, f, n);
  fs[0] += n[0]; fs[1] += n[1]; fs[2] += n[2]; fs[3] += f[0]; fs[4] += f[1]; fs[5] += f[2];
}

// Physical state of one env as held by one lane of its quad.
struct Phys {
  float pos[3], quat[4], v[3], w[3];  // base (replicated in the quad)
  float q[3], qd[3];                   // this leg's joints
};

// One integrator step of length h.  cf: this lane's reported contact forces
// (thigh, calf, foot of its leg; base from the quad sum), written when cf_out.
__device__ void phys_substep(const go1_config* __restrict__ cfg, Phys& S, const float* tau, float h, const float* g,
                             float friction, float payload, const Terr& T, int leg, bool cf_out, float* cf_leg,
                             float* cf_base) {
#pragma clang fp contract(fast)
  const float* model = cfg->model;
  CP C = {cfg->contact_stiffness, cfg->contact_damping, cfg->friction_damping, friction};
  float R[9];
  quat_to_R(S.quat, R);
  float vb[6];
  mat3T_vec(R, S.w, vb);
  mat3T_vec(R, S.v, vb + 3);
  // ---- base rigid body (every lane of the quad, identical)
  const float* bb = model;  // base body block
  float mscale = (bb[0] + payload) / bb[0];
  SI I0;
  rigid_si(bb, mscale, I0);
  float p0[6], hm[6];
  si_mul(I0, vb, hm);
  crf(vb, hm, p0);
  // gravity on the base is applied once (lane-independent); trunk corners split 2 per lane
  float fbase[6] = {0, 0, 0, 0, 0, 0};
  {
    float gb[3];
    mat3T_vec(R, g, gb);
    float m = bb[0] * mscale;
    float fg[3] = {m * gb[0], m * gb[1], m * gb[2]}, cg[3];
    cross3(bb + 1, fg, cg);
    p0[0] -= cg[0]; p0[1] -= cg[1]; p0[2] -= cg[2]; p0[3] -= fg[0]; p0[4] -= fg[1]; p0[5] -= fg[2];
  }
  const float* th = model + 13 * 10 + 4 * 9 + 3 + 1;  // trunk half extents
  float Fb[3] = {0, 0, 0};
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    int cx = leg * 2 + k;
    float lp[3] = {(cx & 1) ? th[0] : -th[0], (cx & 2) ? th[1] : -th[1], (cx & 4) ? th[2] : -th[2]};
    float pw[3], vw[3], F[3];
    point_kin(R, S.pos, vb, lp, pw, vw);
    sphere_contact(T, C, pw, vw, 0.0f, F);
    point_force(R, lp, F, fbase);
    Fb[0] += F[0]; Fb[1] += F[1]; Fb[2] += F[2];
  }
  // ---- this leg: kinematics
  const float* origin = model + 13 * 10 + leg * 9;
  float E[3][9], vj[3][6], cj[3][6], Rw[3][9], pw_[3][3];
  {
    float Rp[9], pp[3], vp[6];
#pragma unroll
    for (int i = 0; i < 9; ++i) Rp[i] = R[i];
    pp[0] = S.pos[0]; pp[1] = S.pos[1]; pp[2] = S.pos[2];
#pragma unroll
    for (int i = 0; i < 6; ++i) vp[i] = vb[i];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int ax = j == 0 ? 0 : 1;
      const float* r = origin + j * 3;
      float s, c;
      sincosf(S.q[j], &s, &c);
      joint_E(ax, c, s, E[j]);
      xm(E[j], r, vp, vj[j]);
      vj[j][ax] += S.qd[j];
      float sq[3] = {0, 0, 0};
      sq[ax] = S.qd[j];
      cross3(vj[j], sq, cj[j]);
      cross3(vj[j] + 3, sq, cj[j] + 3);
      float rw[3];
      mat3_vec(Rp, r, rw);
      pw_[j][0] = pp[0] + rw[0]; pw_[j][1] = pp[1] + rw[1]; pw_[j][2] = pp[2] + rw[2];
      // Rw = Rp E^T
#pragma unroll
      for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b)
          Rw[j][a * 3 + b] = Rp[a * 3 + 0] * E[j][b * 3 + 0] + Rp[a * 3 + 1] * E[j][b * 3 + 1] +
                             Rp[a * 3 + 2] * E[j][b * 3 + 2];
#pragma unroll
      for (int i = 0; i < 9; ++i) Rp[i] = Rw[j][i];
      pp[0] = pw_[j][0]; pp[1] = pw_[j][1]; pp[2] = pw_[j][2];
#pragma unroll
      for (int i = 0; i < 6; ++i) vp[i] = vj[j][i];
    }
  }
  // ---- rigid inertias, bias and external forces
  SI IA[3];
  float pA[3][6];
  const float* foot = model + 13 * 10 + 4 * 9;
  const float foot_r = foot[3];
  const float thigh_r = model[13 * 10 + 4 * 9 + 3 + 1 + 3];
  const float calf_r = model[13 * 10 + 4 * 9 + 3 + 1 + 3 + 1];
  float cfl[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};  // thigh, calf, foot
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const float* B = model + 10 * (1 + leg * 3 + j);
    rigid_si(B, 1.0f, IA[j]);
    float hmj[6];
    si_mul(IA[j], vj[j], hmj);
    crf(vj[j], hmj, pA[j]);
    float gl[3], fext[6] = {0, 0, 0, 0, 0, 0};
    mat3T_vec(Rw[j], g, gl);
    float fg[3] = {B[0] * gl[0], B[0] * gl[1], B[0] * gl[2]}, cg[3];
    cross3(B + 1, fg, cg);
    fext[0] = cg[0]; fext[1] = cg[1]; fext[2] = cg[2]; fext[3] = fg[0]; fext[4] = fg[1]; fext[5] = fg[2];
    if (j == 1) {
      const float zs[3] = {-0.071f, -0.142f, -0.213f};
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        float lp[3] = {0.0f, 0.0f, zs[p]}, pw[3], vw[3], F[3];
        point_kin(Rw[j], pw_[j], vj[j], lp, pw, vw);
        sphere_contact(T, C, pw, vw, thigh_r, F);
        point_force(Rw[j], lp, F, fext);
        cfl[0][0] += F[0]; cfl[0][1] += F[1]; cfl[0][2] += F[2];
      }
    } else if (j == 2) {
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        float lp[3], rr;
        if (p < 2) { lp[0] = 0.0f; lp[1] = 0.0f; lp[2] = p == 0 ? -0.071f : -0.142f; rr = calf_r; }
        else { lp[0] = foot[0]; lp[1] = foot[1]; lp[2] = foot[2]; rr = foot_r; }
        float pw[3], vw[3], F[3];
        point_kin(Rw[j], pw_[j], vj[j], lp, pw, vw);
        sphere_contact(T, C, pw, vw, rr, F);
        point_force(Rw[j], lp, F, fext);
        int slot = p < 2 ? 1 : 2;
        cfl[slot][0] += F[0]; cfl[slot][1] += F[1]; cfl[slot][2] += F[2];
      }
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) pA[j][i] -= fext[i];
  }
  // ---- backward pass calf -> hip
  float U[3][6], D[3], u[3];
  SI Ip;
  float pp6[6];
#pragma unroll
  for (int j = 2; j >= 0; --j) {
    const int ax = j == 0 ? 0 : 1;
    const int dof = leg * 3 + j;
    float t = tau[j];
    float lo = cfg->hard_limits[dof * 2], hi = cfg->hard_limits[dof * 2 + 1];
    if (S.q[j] > hi) t -= cfg->limit_stiffness * (S.q[j] - hi) + cfg->limit_damping * S.qd[j];
    else if (S.q[j] < lo) t -= cfg->limit_stiffness * (S.q[j] - lo) + cfg->limit_damping * S.qd[j];
#pragma unroll
    for (int i = 0; i < 6; ++i) U[j][i] = si_get(IA[j], i, ax);
    D[j] = si_get(IA[j], ax, ax);
    u[j] = t - pA[j][ax];
    float invD = 1.0f / D[j];
    SI Ia;
    // Ia = IA - U U^T / D
    float Ua[3] = {U[j][0], U[j][1], U[j][2]}, Ul[3] = {U[j][3], U[j][4], U[j][5]};
    Ia.a[0] = IA[j].a[0] - Ua[0] * Ua[0] * invD; Ia.a[1] = IA[j].a[1] - Ua[0] * Ua[1] * invD;
    Ia.a[2] = IA[j].a[2] - Ua[0] * Ua[2] * invD; Ia.a[3] = IA[j].a[3] - Ua[1] * Ua[1] * invD;
    Ia.a[4] = IA[j].a[4] - Ua[1] * Ua[2] * invD; Ia.a[5] = IA[j].a[5] - Ua[2] * Ua[2] * invD;
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) Ia.b[a * 3 + b] = IA[j].b[a * 3 + b] - Ua[a] * Ul[b] * invD;
    Ia.c[0] = IA[j].c[0] - Ul[0] * Ul[0] * invD; Ia.c[1] = IA[j].c[1] - Ul[0] * Ul[1] * invD;
    Ia.c[2] = IA[j].c[2] - Ul[0] * Ul[2] * invD; Ia.c[3] = IA[j].c[3] - Ul[1] * Ul[1] * invD;
    Ia.c[4] = IA[j].c[4] - Ul[1] * Ul[2] * invD; Ia.c[5] = IA[j].c[5] - Ul[2] * Ul[2] * invD;
    float Iac[6], pa[6];
    si_mul(Ia, cj[j], Iac);
#pragma unroll
    for (int i = 0; i < 6; ++i) pa[i] = pA[j][i] + Iac[i] + U[j][i] * u[j] * invD;
    SI It;
    float pt[6];
    xform_inertia(E[j], origin + j * 3, Ia, It);
    xfT(E[j], origin + j * 3, pa, pt);
    if (j > 0) {
      si_add(IA[j - 1], It);
#pragma unroll
      for (int i = 0; i < 6; ++i) pA[j - 1][i] += pt[i];
    } else {
      Ip = It;
#pragma unroll
      for (int i = 0; i < 6; ++i) pp6[i] = pt[i];
    }
  }
  // ---- quad reduction: sum of the four legs' contributions and the trunk corners
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    Ip.a[i] = qsum(Ip.a[i]);
    Ip.c[i] = qsum(Ip.c[i]);
    pp6[i] = qsum(pp6[i] - fbase[i]);
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) Ip.b[i] = qsum(Ip.b[i]);
  si_add(I0, Ip);
  float rhs[6], a0[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) rhs[i] = -(p0[i] + pp6[i]);
  solve6(I0, rhs, a0);
  // ---- forward pass
  float qdd[3];
  {
    float ap[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) ap[i] = a0[i];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int ax = j == 0 ? 0 : 1;
      float aj[6];
      xm(E[j], origin + j * 3, ap, aj);
#pragma unroll
      for (int i = 0; i < 6; ++i) aj[i] += cj[j][i];
      float Ua = 0.0f;
#pragma unroll
      for (int i = 0; i < 6; ++i) Ua += U[j][i] * aj[i];
      qdd[j] = (u[j] - Ua) / D[j];
      aj[ax] += qdd[j];
#pragma unroll
      for (int i = 0; i < 6; ++i) ap[i] = aj[i];
    }
  }
  // ---- semi-implicit Euler (base identical in the quad)
  float wv[3], alb[3], aw[3], al[3];
  cross3(vb, vb + 3, wv);
  alb[0] = a0[3] + wv[0]; alb[1] = a0[4] + wv[1]; alb[2] = a0[5] + wv[2];
  mat3_vec(R, a0, aw);
  mat3_vec(R, alb, al);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    S.w[i] += h * aw[i];
    S.v[i] += h * al[i];
    S.pos[i] += h * S.v[i];
  }
  {
    float wn = sqrtf(S.w[0] * S.w[0] + S.w[1] * S.w[1] + S.w[2] * S.w[2]);
    float thh = 0.5f * h * wn;
    float sth, cth;
    sincosf(thh, &sth, &cth);
    float sc = thh > 1e-12f ? sth / wn : 0.5f * h;
    float dq[4] = {S.w[0] * sc, S.w[1] * sc, S.w[2] * sc, cth};
    float* q = S.quat;
    float nq[4];
    nq[3] = dq[3] * q[3] - dq[0] * q[0] - dq[1] * q[1] - dq[2] * q[2];
    nq[0] = dq[3] * q[0] + dq[0] * q[3] + dq[1] * q[2] - dq[2] * q[1];
    nq[1] = dq[3] * q[1] - dq[0] * q[2] + dq[1] * q[3] + dq[2] * q[0];
    nq[2] = dq[3] * q[2] + dq[0] * q[1] - dq[1] * q[0] + dq[2] * q[3];
    float inv = 1.0f / sqrtf(nq[0] * nq[0] + nq[1] * nq[1] + nq[2] * nq[2] + nq[3] * nq[3]);
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = nq[i] * inv;
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    S.qd[j] += h * qdd[j];
    S.q[j] += h * S.qd[j];
  }
  if (cf_out) {
#pragma unroll
    for (int i = 0; i < 9; ++i) cf_leg[i] = (&cfl[0][0])[i];
    cf_base[0] = qsum(Fb[0]);
    cf_base[1] = qsum(Fb[1]);
    cf_base[2] = qsum(Fb[2]);
  }
}

// =====================================================================
//                          the fused step kernel
// =====================================================================
struct KArgs {
  go1_state st;
  go1_terrain ter;
  go1_step_args a;
  int32_t* any_reset;
};

// reset_idx for one env, computed redundantly by the 4 lanes of its quad (:218-296)
__device__ void reset_env(const go1_config* __restrict__ c, const go1_terrain& ter, const Rng& rng, int e, int leg,
                          float* root, float* q, float* qd, float* strength, float* offset, float* traj) {
  float s = rng(0) * c->strength_range + c->strength_lo;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int d = leg * 3 + j;
    strength[j] = s;
    offset[j] = rng(1 + d) * c->offset_range + c->offset_lo;
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int d = leg * 3 + j;
    float f = c->reset_dof_range * rng(13 + d) + c->reset_dof_lo;
    q[j] = c->default_dof_pos[d] * f;
    qd[j] = 0.0f;
  }
#pragma unroll
  for (int i = 0; i < 13; ++i) root[i] = c->base_init_state[i];
  const float* eo = ter.env_origins + (size_t)e * 3;
  root[0] = root[0] + eo[0];
  root[1] = root[1] + eo[1];
  root[2] = root[2] + eo[2];
  if (c->custom_origins) {
    root[0] = root[0] + (c->x_init_range2 * rng(25) + c->x_init_lo);
    root[1] = root[1] + (c->y_init_range2 * rng(26) + c->y_init_lo);
    root[0] = root[0] + c->x_init_offset;
    root[1] = root[1] + c->y_init_offset;
  }
  float yaw = c->yaw_range2 * rng(27) + c->yaw_lo;
  float thh = yaw / 2.0f, sth, cth;
  pm_sincosf(thh, &sth, &cth);
  float qv[4] = {0.0f * sth, 0.0f * sth, 1.0f * sth, cth};
  float qn = sqrtf(fmaf(qv[3], qv[3], fmaf(qv[2], qv[2], fmaf(qv[1], qv[1], qv[0] * qv[0]))));
  if (qn < 1e-9f) qn = 1e-9f;
#pragma unroll
  for (int i = 0; i < 4; ++i) root[3 + i] = qv[i] / qn;
#pragma unroll
  for (int i = 0; i < 6; ++i) root[7 + i] = c->reset_vel_range * rng(28 + i) + c->reset_vel_lo;
  traj[0] = c->traj_base_x + root[0];
  traj[1] = c->traj_base_y + root[1];
  traj[2] = c->traj_base_z;
  traj[3] = c->traj_roll;
  traj[4] = c->traj_pitch;
  traj[5] = c->traj_yaw;
}

template <bool INJ>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(1, 1))) void go1_step_kernel(
    const go1_config* __restrict__ c, KArgs K) {
  const go1_state& st = K.st;
  const go1_step_args& A = K.a;
  const int n = c->n_envs;
  const int leg = threadIdx.x & 3;
  const int e = blockIdx.x * EPB + (threadIdx.x >> 2);
  if (e >= n) return;  // whole quads exit together
  const Rng rng = {A.uniforms, A.rng_seed, A.rng_step, e};
  const size_t d0 = (size_t)e * NDOF + leg * 3;

  // ---------------- load
  float act[3], root[13], q[3], qd[3], lag[GO1_LAG_SLOTS][3], eh[2][3], vh[2][3], strength[3], offset[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) act[j] = clampf(A.actions[d0 + j], -c->clip_actions, c->clip_actions);
#pragma unroll
  for (int i = 0; i < 13; ++i) root[i] = st.root[(size_t)e * 13 + i];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    q[j] = st.dof_pos[d0 + j];
    qd[j] = st.dof_vel[d0 + j];
    strength[j] = st.motor_strength[d0 + j];
    offset[j] = st.motor_offset[d0 + j];
#pragma unroll
    for (int s = 0; s < GO1_LAG_SLOTS; ++s) lag[s][j] = st.lag[(size_t)e * 84 + s * 12 + leg * 3 + j];
    eh[0][j] = st.pos_err_hist[(size_t)e * 24 + leg * 3 + j];
    eh[1][j] = st.pos_err_hist[(size_t)e * 24 + 12 + leg * 3 + j];
    vh[0][j] = st.vel_hist[(size_t)e * 24 + leg * 3 + j];
    vh[1][j] = st.vel_hist[(size_t)e * 24 + 12 + leg * 3 + j];
  }
  const float friction = st.friction[e], payload = st.payload[e];
  Terr T = {nullptr, c->hf_nx, c->hf_ny, 0.0f, 0.0f, c->horizontal_scale};
  if (c->terrain_kind == 1) {
    T.tile = K.ter.tiles + (size_t)K.ter.env_tile[e] * 2 * c->hf_nx * c->hf_ny;
    T.ox = K.ter.env_terrain_origin[(size_t)e * 3];
    T.oy = K.ter.env_terrain_origin[(size_t)e * 3 + 1];
  }

  // ---------------- decimation loop (:82-88)
  float scaled[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    scaled[j] = act[j] * c->action_scale;
    if (j == 0) scaled[j] = scaled[j] * c->hip_scale_reduction;
  }
  Phys P;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    P.pos[i] = root[i]; P.v[i] = root[7 + i]; P.w[i] = root[10 + i];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) P.quat[i] = root[3 + i];
  float torque[3], tgt[3];
  float cf_leg[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, cf_base[3] = {0, 0, 0};
  const int dec = c->decimation;
  for (int sub = 0; sub < dec; ++sub) {
    // _compute_torques (:957-996).  The weight pointer is laundered each sub-step so the
    // 1313 weights are re-read through the scalar cache instead of being hoisted into
    // (and spilled from) SGPRs for the whole loop.
    const float* W = c->actuator;
    asm volatile("" : "+s"(W));
#pragma unroll
    for (int s = 0; s < GO1_LAG_SLOTS - 1; ++s)
#pragma unroll
      for (int j = 0; j < 3; ++j) lag[s][j] = lag[s + 1][j];
#pragma unroll
    for (int j = 0; j < 3; ++j) lag[GO1_LAG_SLOTS - 1][j] = scaled[j];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int d = leg * 3 + j;
      tgt[j] = lag[0][j] + c->default_dof_pos[d];
      float err = q[j] - tgt[j] + offset[j];
      float t = actuator_eval(W, err, eh[0][j], eh[1][j], qd[j], vh[0][j], vh[1][j]);
      eh[1][j] = eh[0][j];
      eh[0][j] = err;
      vh[1][j] = vh[0][j];
      vh[0][j] = qd[j];
      t = t * strength[j];
      float lim = c->torque_limits[d];
      torque[j] = clampf(t, -lim, lim);
      if (A.dbg_torques) A.dbg_torques[((size_t)sub * n + e) * NDOF + d] = torque[j];
    }
    if (INJ) {
      const float* id = A.inj_dof + ((size_t)sub * n + e) * NDOF * 2;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        q[j] = id[(leg * 3 + j) * 2];
        qd[j] = id[(leg * 3 + j) * 2 + 1];
      }
    } else {
      const float h = c->sim_dt / (float)c->n_internal;
#pragma unroll
      for (int j = 0; j < 3; ++j) { P.q[j] = q[j]; P.qd[j] = qd[j]; }
      for (int k = 0; k < c->n_internal; ++k) {
        bool last = (sub == dec - 1) && (k == c->n_internal - 1);
        phys_substep(c, P, torque, h, A.sim_gravity, friction, payload, T, leg, last, cf_leg, cf_base);
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) { q[j] = P.q[j]; qd[j] = P.qd[j]; }
    }
  }
  float cf[NB * 3];  // only the entries this lane needs: base + its leg
  if (INJ) {
#pragma unroll
    for (int i = 0; i < 13; ++i) root[i] = A.inj_root[(size_t)e * 13 + i];
    const float* ic = A.inj_contact + (size_t)e * NB * 3;
#pragma unroll
    for (int i = 0; i < 3; ++i) cf_base[i] = ic[i];
#pragma unroll
    for (int b = 0; b < 3; ++b)
#pragma unroll
      for (int i = 0; i < 3; ++i) cf_leg[b * 3 + i] = ic[(2 + leg * 4 + b) * 3 + i];
  } else {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      root[i] = P.pos[i]; root[7 + i] = P.v[i]; root[10 + i] = P.w[i];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) root[3 + i] = P.quat[i];
  }
  (void)cf;
  if (A.contact_forces) {
    float* o = A.contact_forces + (size_t)e * NB * 3;
    if (leg == 0) { o[0] = cf_base[0]; o[1] = cf_base[1]; o[2] = cf_base[2]; }
    float* ol = o + (1 + leg * 4) * 3;
    ol[0] = 0.0f; ol[1] = 0.0f; ol[2] = 0.0f;  // hip: no contact geometry in the native model
#pragma unroll
    for (int i = 0; i < 9; ++i) ol[3 + i] = cf_leg[i];
  }

  // ================= post_physics_step (:114-169), contraction off =================
  int ep = st.episode_length[e] + 1;
  float qb[4] = {root[3], root[4], root[5], root[6]};
  float blv[3], bav[3], pg[3];
  quat_rotate_inverse_f(qb, root + 7, blv);
  quat_rotate_inverse_f(qb, root + 10, bav);
  quat_rotate_inverse_f(qb, A.gravity_vec, pg);
  float brot_prev[3] = {st.base_rotation[(size_t)e * 3], st.base_rotation[(size_t)e * 3 + 1],
                        st.base_rotation[(size_t)e * 3 + 2]};
  const float cam_pitch = brot_prev[1];

  // _plan_target_pose / _compute_relative_target_pose (:850-932)
  float traj[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) traj[i] = st.trajectory[(size_t)e * 6 + i];
  float rel_in[3] = {traj[0] - root[0], traj[1] - root[1], traj[2] - root[2]};
  float rel_lin[3], rpy[3], rel_rot[3];
  quat_apply_yaw_inverse_f(qb, rel_in, rel_lin);
  quat_to_rpy_f(qb, rpy);
#pragma unroll
  for (int i = 0; i < 3; ++i) rel_rot[i] = wrap_to_pi_f(traj[3 + i] - rpy[i]);
  float cmd[2] = {rel_lin[0], rel_lin[1]};

  // DR every rand_interval (:822-824)
  if (ep % c->rand_interval == 0) {
    float s = rng(34) * c->strength_range + c->strength_lo;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      strength[j] = s;
      offset[j] = rng(35 + leg * 3 + j) * c->offset_range + c->offset_lo;
    }
  }
  float rel_norm = norm2_f(rel_lin[0], rel_lin[1]);
  bool switched = rel_norm < c->switch_dist;
  int idx = st.curr_pose_index[e];
  if (switched) { idx += 1; if (idx > 0) idx = 0; }
  bool reached = switched && idx == 0;
  // collision count (:848): this lane's thigh + calf, base on lane 0
  float coll_l = (norm3_f(cf_leg[0], cf_leg[1], cf_leg[2]) > 0.1f ? 1.0f : 0.0f) +
                 (norm3_f(cf_leg[3], cf_leg[4], cf_leg[5]) > 0.1f ? 1.0f : 0.0f);
  if (leg == 0 && norm3_f(cf_base[0], cf_base[1], cf_base[2]) > 0.1f) coll_l += 1.0f;
  float coll = qsum(coll_l);

  // check_termination (:198-216)
  bool time_out = (float)ep > c->max_episode_length;
  bool reset = time_out;
  if (c->use_terminal_body_height && root[2] < c->terminal_body_height) reset = true;

  // rewards (:320-355, reward_crawling.py)
  const float* ldv = st.last_dof_vel + d0;
  const float* la = st.last_actions + d0;
  float t_tq = 0.0f, t_acc = 0.0f, t_ar = 0.0f, t_lim = 0.0f;
  {
    float x[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) x[j] = sq_f(torque[j]);
    t_tq = qsum((x[0] + x[1]) + x[2]);
#pragma unroll
    for (int j = 0; j < 3; ++j) x[j] = sq_f((ldv[j] - qd[j]) / c->dt);
    t_acc = qsum((x[0] + x[1]) + x[2]);
#pragma unroll
    for (int j = 0; j < 3; ++j) x[j] = sq_f(la[j] - act[j]);
    t_ar = qsum((x[0] + x[1]) + x[2]);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int d = leg * 3 + j;
      float lo = q[j] - c->dof_pos_limits[2 * d];
      float hi = q[j] - c->dof_pos_limits[2 * d + 1];
      float o = -(lo < 0.0f ? lo : 0.0f);
      x[j] = o + (hi > 0.0f ? hi : 0.0f);
    }
    t_lim = qsum((x[0] + x[1]) + x[2]);
  }
  float terms[GO1_NUM_TERMS];
  terms[0] = t_tq;
  terms[1] = t_acc;
  terms[2] = coll;
  terms[3] = t_ar;
  terms[4] = t_lim;
  terms[5] = sq_f(root[2] - c->base_height_target);
  terms[6] = sq_f(bav[0]) + sq_f(bav[1]);
  {
    float mag = norm2_f(rel_lin[0], rel_lin[1]);
    float lerr = sq_f(blv[0]) + sq_f(blv[1]);
    float r_e2e = expf(-lerr / c->tracking_sigma_lin);
    terms[7] = r_e2e * (mag < c->switch_dist ? 1.0f : 0.0f) * ((float)ep > c->t_reach ? 1.0f : 0.0f);
    float tx = rel_lin[0] / (mag + 1e-6f) * c->target_lin_vel;
    float ty = rel_lin[1] / (mag + 1e-6f) * c->target_lin_vel;
    float gate = mag > c->lin_reaching_criterion ? 1.0f : 0.0f;
    tx = tx * gate;
    ty = ty * gate;
    float le = sq_f(tx - blv[0]) + sq_f(ty - blv[1]);
    terms[8] = expf(-le / c->tracking_sigma_lin);
    float ta = rel_rot[2];
    float m = fabsf(ta);
    ta = ta / (m + 1e-6f) * c->target_ang_vel;
    ta = ta * (m > c->ang_reaching_criterion ? 1.0f : 0.0f);
    float ae = sq_f(ta - bav[2]);
    terms[9] = expf(-ae / c->tracking_sigma_ang);
  }
  float rew = 0.0f, pos = 0.0f, neg = 0.0f;
  float sums[GO1_NUM_SUMS];
#pragma unroll
  for (int k = 0; k < GO1_NUM_SUMS; ++k) sums[k] = st.episode_sums[(size_t)e * GO1_NUM_SUMS + k];
#pragma unroll
  for (int k = 0; k < GO1_NUM_TERMS; ++k) {
    float r = terms[k] * A.reward_scales[k];
    rew = rew + r;
    if (A.reward_scales[k] >= 0.0f) pos = pos + r; else neg = neg + r;
    sums[k] = sums[k] + r;
  }
  sums[10] = sums[10] + rew;
  sums[11] = sums[11] + pos;
  sums[12] = sums[12] + neg;
  if (A.dbg_terms && leg == 0)
#pragma unroll
    for (int k = 0; k < GO1_NUM_TERMS; ++k) A.dbg_terms[(size_t)e * GO1_NUM_TERMS + k] = terms[k];

  // ---- height scan (:1918-1965): uses the pre-reset root and the previous pitch
  const int x_start = c->measure_front_half ? GO1_GRID_X / 2 + 1 : 0;
  const int n_rows = GO1_GRID_X - x_start;
  const int n_pts = n_rows * GO1_GRID_Y;
  float hvals[2][28];  // this lane's points p = leg + 4 k, k < 28  (n_pts <= 231 needs debug path)
  const bool plane = c->terrain_kind == 0;
  float camx = 0.0f, camy = 0.0f;
  if (!plane) {
    float cos_p = pm_cosf(cam_pitch);
    camx = c->camera_offset_x * cos_p;
    camy = 0.0f * cos_p;
  }
  auto sample = [&](int i, int j, float& h0, float& h1) {
    if (plane) { h0 = 1.0f; h1 = 0.0f; return; }
    float px = c->height_grid_x[i] + root[0];
    float py = c->height_grid_y[j] + root[1];
    if (c->camera_zero) { px = px + camx; py = py + camy; }
    px = px - T.ox;
    py = py - T.oy;
    long ix = (long)(px / c->horizontal_scale);
    long iy = (long)(py / c->horizontal_scale);
    ix = ix < 0 ? 0 : (ix > c->hf_nx - 2 ? c->hf_nx - 2 : ix);
    iy = iy < 0 ? 0 : (iy > c->hf_ny - 2 ? c->hf_ny - 2 : iy);
    h0 = T.tile[(size_t)ix * c->hf_ny + iy];
    h1 = T.tile[((size_t)c->hf_nx + ix) * c->hf_ny + iy];
  };
#pragma unroll
  for (int k = 0; k < 28; ++k) {
    int p = leg + 4 * k;
    if (p < n_pts && k < 28) {
      int i = x_start + p / GO1_GRID_Y, j = p % GO1_GRID_Y;
      sample(i, j, hvals[0][k], hvals[1][k]);
    }
  }
  if (A.dbg_heights) {
    float* o = A.dbg_heights + (size_t)e * 2 * GO1_GRID_X * GO1_GRID_Y;
    for (int p = leg; p < GO1_GRID_X * GO1_GRID_Y; p += 4) {
      float h0, h1;
      sample(p / GO1_GRID_Y, p % GO1_GRID_Y, h0, h1);
      o[p] = h0;
      o[GO1_GRID_X * GO1_GRID_Y + p] = h1;
    }
  }

  // ---- reset_idx (:218-296)
  float traj_new[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) traj_new[i] = traj[i];
  if (reset) {
    reset_env(c, K.ter, rng, e, leg, root, q, qd, strength, offset, traj_new);
    idx = 0;
#pragma unroll
    for (int k = 0; k < GO1_NUM_SUMS; ++k) sums[k] = 0.0f;
#pragma unroll
    for (int s = 0; s < GO1_LAG_SLOTS; ++s)
#pragma unroll
      for (int j = 0; j < 3; ++j) lag[s][j] = 0.0f;
    cmd[0] = 0.0f;  // commands is a view of local_relative_linear, zeroed by reset_idx (:252, :802)
    cmd[1] = 0.0f;
  }
  const int coll_count = reset ? 0 : st.collision_count[e] + (int)coll;

  // ---- compute_observations (:357-475)
  float* o = A.obs + (size_t)e * GO1_NUM_OBS;
  const float clip = c->clip_obs;
  auto put = [&](int i, float v, float nv, bool noisy) {
    if (noisy && c->add_noise) v = v + (2.0f * rng(47 + i) - 1.0f) * nv;
    o[i] = clampf(v, -clip, clip);
  };
  if (leg == 0) {
    put(0, pg[0], c->noise_gravity, true);
    put(1, pg[1], c->noise_gravity, true);
    put(2, pg[2], c->noise_gravity, true);
    put(3, cmd[0] * 1.0f, 0.0f, false);
    put(4, cmd[1] * 1.0f, 0.0f, false);
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int d = leg * 3 + j;
    put(5 + d, (q[j] - c->default_dof_pos[d]) * c->obs_scale_dof_pos, c->noise_dof_pos, true);
    put(17 + d, qd[j] * c->obs_scale_dof_vel, c->noise_dof_vel, true);
    put(29 + d, act[j], 0.0f, false);
  }
  {
    const float zroot = root[2];
    const float cam_z = pm_sinf(cam_pitch) * c->camera_offset_norm;
#pragma unroll
    for (int k = 0; k < 28; ++k) {
      int p = leg + 4 * k;
      if (p < n_pts) {
#pragma unroll
        for (int layer = 0; layer < 2; ++layer) {
          float h = hvals[layer][k];
          if (c->camera_zero) {
            h = h - zroot;
            h = h - cam_z;
            h = clampf(h, -0.3f, 0.3f);
          } else {
            h = clampf(h, 0.0f, c->ceiling_height);
            h = h / c->ceiling_height;
            h = h - 0.5f;
          }
          o[41 + layer * n_pts + p] = clampf(h * c->obs_scale_heights, -clip, clip);
        }
      }
    }
  }
  if (leg == 0) {
    float* pv = A.priv + (size_t)e * GO1_NUM_PRIV;
    pv[0] = clampf((friction - c->priv_friction_shift) * c->priv_friction_scale, -clip, clip);
    pv[1] = clampf((st.restitution[e] - c->priv_rest_shift) * c->priv_rest_scale, -clip, clip);
  }

  // ---------------- write back (epilogue :148-153)
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    st.dof_pos[d0 + j] = q[j];
    st.dof_vel[d0 + j] = qd[j];
    st.last_actions[d0 + j] = act[j];
    st.last_dof_vel[d0 + j] = qd[j];
    st.motor_strength[d0 + j] = strength[j];
    st.motor_offset[d0 + j] = offset[j];
    st.joint_pos_target[d0 + j] = tgt[j];
#pragma unroll
    for (int s = 0; s < GO1_LAG_SLOTS; ++s) st.lag[(size_t)e * 84 + s * 12 + leg * 3 + j] = lag[s][j];
    st.pos_err_hist[(size_t)e * 24 + leg * 3 + j] = eh[0][j];
    st.pos_err_hist[(size_t)e * 24 + 12 + leg * 3 + j] = eh[1][j];
    st.vel_hist[(size_t)e * 24 + leg * 3 + j] = vh[0][j];
    st.vel_hist[(size_t)e * 24 + 12 + leg * 3 + j] = vh[1][j];
  }
  if (leg == 0) {
#pragma unroll
    for (int i = 0; i < 13; ++i) st.root[(size_t)e * 13 + i] = root[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) st.base_rotation[(size_t)e * 3 + i] = rpy[i];
#pragma unroll
    for (int i = 0; i < 6; ++i) st.trajectory[(size_t)e * 6 + i] = traj_new[i];
#pragma unroll
    for (int k = 0; k < GO1_NUM_SUMS; ++k) st.episode_sums[(size_t)e * GO1_NUM_SUMS + k] = sums[k];
    st.episode_length[e] = reset ? 0 : ep;
    st.curr_pose_index[e] = idx;
    st.collision_count[e] = coll_count;
    A.rew[e] = rew;
    A.reset[e] = reset;
    A.time_out[e] = time_out;
    if (A.dbg_commands) { A.dbg_commands[e * 2] = cmd[0]; A.dbg_commands[e * 2 + 1] = cmd[1]; }
    if (A.dbg_reached) A.dbg_reached[e] = reached;
  }
  // one atomic per wave when any env of the wave reset (extras["time_outs"] rebinding, :289-291)
  if (__ballot(reset && leg == 0) != 0ull && threadIdx.x == 0) atomicOr(K.any_reset, 1);
}

// extras["time_outs"] is rebound to time_out_buf only on steps where reset_idx ran.
__global__ void go1_finalize_kernel(int n, const int32_t* __restrict__ any_reset, int32_t* __restrict__ next_flag,
                                    const uint8_t* __restrict__ time_out, uint8_t* __restrict__ extras) {
  int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e == 0) *next_flag = 0;
  if (e < n && *any_reset) extras[e] = time_out[e];
}

// reset of masked envs (env.reset(), :46-55 of trajectory_tracking/__init__.py)
__global__ __launch_bounds__(TPB) void go1_reset_kernel(const go1_config* __restrict__ c, go1_state st,
                                                        go1_terrain ter, const uint8_t* __restrict__ mask,
                                                        const float* __restrict__ U, uint64_t seed, uint64_t step) {
  const int leg = threadIdx.x & 3;
  const int e = blockIdx.x * EPB + (threadIdx.x >> 2);
  if (e >= c->n_envs || !mask[e]) return;
  const Rng rng = {U, seed, step, e};
  float root[13], q[3], qd[3], strength[3], offset[3], traj[6];
  reset_env(c, ter, rng, e, leg, root, q, qd, strength, offset, traj);
  const size_t d0 = (size_t)e * NDOF + leg * 3;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    st.dof_pos[d0 + j] = q[j];
    st.dof_vel[d0 + j] = qd[j];
    st.motor_strength[d0 + j] = strength[j];
    st.motor_offset[d0 + j] = offset[j];
    st.last_actions[d0 + j] = 0.0f;
    st.last_dof_vel[d0 + j] = 0.0f;
#pragma unroll
    for (int s = 0; s < GO1_LAG_SLOTS; ++s) st.lag[(size_t)e * 84 + s * 12 + leg * 3 + j] = 0.0f;
  }
  if (leg == 0) {
#pragma unroll
    for (int i = 0; i < 13; ++i) st.root[(size_t)e * 13 + i] = root[i];
#pragma unroll
    for (int i = 0; i < 6; ++i) st.trajectory[(size_t)e * 6 + i] = traj[i];
#pragma unroll
    for (int k = 0; k < GO1_NUM_SUMS; ++k) st.episode_sums[(size_t)e * GO1_NUM_SUMS + k] = 0.0f;
    st.episode_length[e] = 0;
    st.curr_pose_index[e] = 0;
    st.collision_count[e] = 0;
  }
}

__global__ void go1_actuator_kernel(const go1_config* __restrict__ c, const float* __restrict__ x,
                                    float* __restrict__ out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* r = x + (size_t)i * 6;
  out[i] = actuator_eval(c->actuator, r[0], r[1], r[2], r[3], r[4], r[5]);
}

// =====================================================================
//                                C ABI
// =====================================================================
struct go1_handle {
  go1_config cfg;
  go1_config* d_cfg = nullptr;
  go1_state st;
  go1_terrain ter;
  bool bound = false, has_terrain = false;
  int32_t* d_flags = nullptr;  // any_reset double buffer
  uint64_t parity = 0;
};

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(x)                                                                      \
  do {                                                                                  \
    hipError_t _e = (x);                                                                \
    if (_e != hipSuccess) return fail(GO1_E_HIP, std::string(#x ": ") + hipGetErrorString(_e)); \
  } while (0)

extern "C" {

int go1_abi_version(void) { return GO1_ABI_VERSION; }

void go1_abi_sizes(int64_t out[4]) {
  out[0] = sizeof(go1_config);
  out[1] = sizeof(go1_state);
  out[2] = sizeof(go1_terrain);
  out[3] = sizeof(go1_step_args);
}

const char* go1_last_error(void) { return g_err.c_str(); }

int go1_create(const go1_config* cfg, go1_handle** out) {
  if (!cfg || !out) return fail(GO1_E_ARG, "go1_create: null argument");
  if (cfg->n_envs <= 0) return fail(GO1_E_ARG, "go1_create: n_envs must be > 0");
  if (cfg->decimation <= 0 || cfg->n_internal <= 0) return fail(GO1_E_ARG, "go1_create: decimation/n_internal");
  if (cfg->terrain_kind == 1 && (cfg->hf_nx < 2 || cfg->hf_ny < 2)) return fail(GO1_E_ARG, "go1_create: tile shape");
  if (cfg->rand_interval <= 0) return fail(GO1_E_ARG, "go1_create: rand_interval");
  if (!cfg->measure_front_half)
    return fail(GO1_E_ARG, "go1_create: only the 261-wide front-half height scan is on this path "
                           "(Cfg.terrain.measure_front_half, scripts/train.py:53)");
  go1_handle* h = new (std::nothrow) go1_handle();
  if (!h) return fail(GO1_E_ARG, "go1_create: out of host memory");
  h->cfg = *cfg;
  hipError_t e1 = hipMalloc(&h->d_cfg, sizeof(go1_config));
  hipError_t e2 = hipMalloc(&h->d_flags, 2 * sizeof(int32_t));
  if (e1 != hipSuccess || e2 != hipSuccess) {
    if (h->d_cfg) (void)hipFree(h->d_cfg);
    if (h->d_flags) (void)hipFree(h->d_flags);
    delete h;
    return fail(GO1_E_HIP, "go1_create: hipMalloc failed");
  }
  HIP_TRY(hipMemcpy(h->d_cfg, cfg, sizeof(go1_config), hipMemcpyHostToDevice));
  HIP_TRY(hipMemset(h->d_flags, 0, 2 * sizeof(int32_t)));
  *out = h;
  return GO1_OK;
}

int go1_bind(go1_handle* h, const go1_state* s) {
  if (!h || !s) return fail(GO1_E_ARG, "go1_bind: null argument");
  const void* p[] = {s->root, s->dof_pos, s->dof_vel, s->last_actions, s->last_dof_vel, s->lag, s->pos_err_hist,
                     s->vel_hist, s->motor_strength, s->motor_offset, s->friction, s->restitution, s->payload,
                     s->episode_length, s->curr_pose_index, s->trajectory, s->base_rotation, s->collision_count,
                     s->episode_sums, s->joint_pos_target};
  for (const void* q : p)
    if (!q) return fail(GO1_E_ARG, "go1_bind: every state plane must be non-null");
  h->st = *s;
  h->bound = true;
  return GO1_OK;
}

int go1_set_terrain(go1_handle* h, const go1_terrain* t) {
  if (!h || !t) return fail(GO1_E_ARG, "go1_set_terrain: null argument");
  if (!t->env_origins || !t->env_terrain_origin || !t->env_tile)
    return fail(GO1_E_ARG, "go1_set_terrain: env_origins / env_terrain_origin / env_tile required");
  if (h->cfg.terrain_kind == 1 && (!t->tiles || t->n_tiles <= 0))
    return fail(GO1_E_ARG, "go1_set_terrain: tunnel terrain needs tiles");
  h->ter = *t;
  h->has_terrain = true;
  return GO1_OK;
}

int go1_step(go1_handle* h, const go1_step_args* a, void* stream) {
  if (!h || !a) return fail(GO1_E_ARG, "go1_step: null argument");
  if (!h->bound || !h->has_terrain) return fail(GO1_E_STATE, "go1_step: call go1_bind and go1_set_terrain first");
  if (!a->actions || !a->obs || !a->priv || !a->rew || !a->reset || !a->time_out || !a->extras_time_outs)
    return fail(GO1_E_ARG, "go1_step: actions and every output buffer are required");
  bool inj = a->inj_dof != nullptr;
  if (inj && (!a->inj_root || !a->inj_contact)) return fail(GO1_E_ARG, "go1_step: partial injected state");
  hipStream_t s = (hipStream_t)stream;
  const int n = h->cfg.n_envs;
  int32_t* flag = h->d_flags + (h->parity & 1);
  int32_t* next = h->d_flags + ((h->parity + 1) & 1);
  h->parity++;
  KArgs K;
  K.st = h->st;
  K.ter = h->ter;
  K.a = *a;
  K.any_reset = flag;
  dim3 grid((n + EPB - 1) / EPB), block(TPB);
  if (a->ev_begin) HIP_TRY(hipEventRecord((hipEvent_t)a->ev_begin, s));
  if (inj) hipLaunchKernelGGL(go1_step_kernel<true>, grid, block, 0, s, h->d_cfg, K);
  else hipLaunchKernelGGL(go1_step_kernel<false>, grid, block, 0, s, h->d_cfg, K);
  HIP_TRY(hipGetLastError());
  if (a->ev_end) HIP_TRY(hipEventRecord((hipEvent_t)a->ev_end, s));
  hipLaunchKernelGGL(go1_finalize_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, flag, next, a->time_out,
                     a->extras_time_outs);
  HIP_TRY(hipGetLastError());
  return GO1_OK;
}

int go1_reset_envs(go1_handle* h, const uint8_t* mask, const float* uniforms, uint64_t rng_seed, uint64_t rng_step,
                   void* stream) {
  if (!h || !mask) return fail(GO1_E_ARG, "go1_reset_envs: null argument");
  if (!h->bound || !h->has_terrain) return fail(GO1_E_STATE, "go1_reset_envs: bind state and terrain first");
  const int n = h->cfg.n_envs;
  hipLaunchKernelGGL(go1_reset_kernel, dim3((n + EPB - 1) / EPB), dim3(TPB), 0, (hipStream_t)stream, h->d_cfg,
                     h->st, h->ter, mask, uniforms, rng_seed, rng_step);
  HIP_TRY(hipGetLastError());
  return GO1_OK;
}

int go1_actuator_net(go1_handle* h, const float* x, float* out, int32_t n_rows, void* stream) {
  if (!h || !x || !out || n_rows < 0) return fail(GO1_E_ARG, "go1_actuator_net: bad argument");
  if (n_rows == 0) return GO1_OK;
  hipLaunchKernelGGL(go1_actuator_kernel, dim3((n_rows + 255) / 256), dim3(256), 0, (hipStream_t)stream, h->d_cfg,
                     x, out, n_rows);
  HIP_TRY(hipGetLastError());
  return GO1_OK;
}

int go1_destroy(go1_handle* h) {
  if (!h) return GO1_OK;
  if (h->d_cfg) (void)hipFree(h->d_cfg);
  if (h->d_flags) (void)hipFree(h->d_flags);
  delete h;
  return GO1_OK;
}

}  // extern "C"

// go1_device.h -- device code shared by the MI355X Go1 step kernels (go1_step.hip: trajectory
// tracking; go1_velocity.hip: velocity tracking): Philox, lane-indexed selects, the actuator-net
// MFMA groups, torch-order f32 math, the native articulated-body integrator with implicit penalty
// contacts (phys_substep) and its helpers.  Included by one translation unit per library.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <new>
#include <string>

#include "../../include/go1_mi355x.h"
#include "go1_model_consts.h"
#include "go1_spec.h"
static_assert(GO1_MODEL_CONST_FLOATS == GO1_MODEL_FLOATS, "regenerate go1_model_consts.h");
#include "pmath.h"

#pragma clang fp contract(off)

#ifdef GO1_ISA_MARKS  // section markers for static instruction accounting (tools/isa_sections.py)
#define MARK(x) asm volatile("; MARK " #x)
#elif defined(GO1_STAMPS)
// Diagnostic build only (tools/stamps.py): every marker records (source line, s_memtime)
// into a buffer of its own, read back by go1_debug_stamps.  Never built into the product.
#define GO1_STAMP_WAVES 4096
#define GO1_STAMP_SLOTS 320
__device__ unsigned long long g_go1_stamps[GO1_STAMP_WAVES * GO1_STAMP_SLOTS];
__shared__ unsigned s_go1_stamp_k;
__device__ __forceinline__ void go1_stamp(unsigned line) {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  const unsigned i = s_go1_stamp_k;
  if (blockIdx.x < GO1_STAMP_WAVES && i < GO1_STAMP_SLOTS)
    g_go1_stamps[blockIdx.x * GO1_STAMP_SLOTS + i] = ((unsigned long long)line << 48) | (t & 0xffffffffffffull);
  s_go1_stamp_k = i + 1;
  __builtin_amdgcn_sched_barrier(0);
}
#define MARK(x) go1_stamp(__LINE__)
#else
#define MARK(x)
#endif
#define NDOF 12
#define NB 17
#define EPB 16          // envs per block of the reset kernel (4 lanes per env)
#define TPB 64          // one wave per block
#define HOLD_N 23       // post-physics inputs parked in LDS across the step kernel's sub-step loop
// LDS copy of the per-joint config arrays, contiguous in go1_config from default_dof_pos
// (checked at go1_create): default_dof_pos, dof_pos_limits, torque_limits, hard_limits,
// height_grid_x, height_grid_y, after the model block
#define LDS_DDP (GO1_MODEL_FLOATS)
#define LDS_DPL (LDS_DDP + 12)
#define LDS_TL (LDS_DPL + 24)
#define LDS_HL (LDS_TL + 12)
#define LDS_GX (LDS_HL + 24)
#define LDS_GY (LDS_GX + GO1_GRID_X)
#define LDS_FLOATS (LDS_GY + GO1_GRID_Y)
#define GO1_DIVERGED 1.0e4f
static_assert(offsetof(go1_config, height_grid_y) - offsetof(go1_config, default_dof_pos) ==
                  (LDS_GY - LDS_DDP) * sizeof(float),
              "per-joint config arrays must be contiguous in go1_config");  // |state component| treated as a diverged integrator
#define SEPB 4          // envs per wave of the step kernel (16 lanes per env: 4 roles x 4 legs)
#define PI_F 3.14159265358979323846f
#define TWO_PI_F 6.28318548202514648438f  // (float)(2*pi), torch's f32 scalar

// ---------------------------------------------------------------- Philox
__device__ __forceinline__ void philox4x32(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one v_mad_u64_u32 per product gives both halves (instead of v_mul_lo + v_mul_hi)
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t l0 = (uint32_t)p0, h0 = (uint32_t)(p0 >> 32), l1 = (uint32_t)p1, h1 = (uint32_t)(p1 >> 32);
    uint32_t n0 = h1 ^ c[1] ^ k0, n2 = h0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = l1; c[2] = n2; c[3] = l0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}

struct Rng {
  const float* U;  // parity-mode uniforms or nullptr
  uint64_t seed, step;
  int e;    // local env index (parity-mode uniforms)
  int gid;  // global env id (Philox counter): local index + go1_config.env_id_offset
  int ustride;  // parity-mode uniform row width (go1_config.u_per_env)
  __device__ float operator()(int slot) const {
    if (U) return U[(size_t)e * ustride + slot];
    uint32_t c[4] = {(uint32_t)gid, (uint32_t)slot >> 2, (uint32_t)step, (uint32_t)(step >> 32)};
    philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    return (float)(c[slot & 3] >> 8) * (1.0f / 16777216.0f);
  }
  // the four uniforms of slots 4 blk .. 4 blk + 3 (one Philox block), as operator() returns them
  __device__ void quad(int blk, float* u) const {
    if (U) {
#pragma unroll
      for (int k = 0; k < 4; ++k) u[k] = U[(size_t)e * ustride + 4 * blk + k];
      return;
    }
    uint32_t c[4] = {(uint32_t)gid, (uint32_t)blk, (uint32_t)step, (uint32_t)(step >> 32)};
    philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
    for (int k = 0; k < 4; ++k) u[k] = (float)(c[k] >> 8) * (1.0f / 16777216.0f);
  }
};

// ---------------------------------------------------------------- lane-indexed selects
// a[i] for a lane-dependent i in 0..3 as two levels of bit-test selects (v_cndmask): an
// equality chain (i == 0 ? .. : i == 1 ? ..) is turned into a switch with divergent branches
__device__ __forceinline__ float sel4(int i, float a0, float a1, float a2, float a3) {
  const bool lo = i & 1, hi = i & 2;
  return hi ? (lo ? a3 : a2) : (lo ? a1 : a0);
}
__device__ __forceinline__ float sel3(int i, const float* a) { return sel4(i, a[0], a[1], a[2], a[2]); }

// ---------------------------------------------------------------- quad helpers
// sum over the quad (lanes xor 1, 2) in the order (l0 + l1) + (l2 + l3); DPP quad_perm
// moves stay in the VALU (no LDS round trip)
__device__ __forceinline__ float qsum(float v) {
  // update_dpp(0, ., bound_ctrl) lets the compiler fold the move into the add (v_add_f32_dpp)
  v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, true));  // [1,0,3,2]
  v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, true));  // [2,3,0,1]
  return v;
}

// sum over the four 16-lane rows, (r0 + r1) + (r2 + r3): gfx950 v_permlane16/32_swap
__device__ __forceinline__ float rowsum4(float p) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(p), __float_as_uint(p), false, false);
  p = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(p), __float_as_uint(p), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// N independent row sums stage by stage (all permlane16 swaps, then their adds, then the
// permlane32 stage): one value at a time, every sum paid a register copy, a hazard nop and
// the full swap latency, twice
template <int N>
__device__ __forceinline__ void rowsum4_n(float* v) {
  float a[N], b[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[i]), __float_as_uint(v[i]), false, false);
    a[i] = __uint_as_float(r[0]);
    b[i] = __uint_as_float(r[1]);
  }
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = a[i] + b[i];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[i]), __float_as_uint(v[i]), false, false);
    a[i] = __uint_as_float(r[0]);
    b[i] = __uint_as_float(r[1]);
  }
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = a[i] + b[i];
}

// N values that two bodies split between the row pairs (body L on rows 0-1, body H on rows 2-3):
// the permlane16 stage sums each pair, then one permlane32 swap hands every lane both results --
// its two outputs are the low-half value (rows 0-1) and the high-half value (rows 2-3) on every
// lane.  Three VALU per value where two full row sums cost eight.
template <int N>
__device__ __forceinline__ void pairsum_rows_n(const float* v, float* lo, float* hi) {
  float a[N], b[N], s[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[i]), __float_as_uint(v[i]), false, false);
    a[i] = __uint_as_float(r[0]);
    b[i] = __uint_as_float(r[1]);
  }
#pragma unroll
  for (int i = 0; i < N; ++i) s[i] = a[i] + b[i];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(s[i]), __float_as_uint(s[i]), false, false);
    lo[i] = __uint_as_float(r[0]);
    hi[i] = __uint_as_float(r[1]);
  }
}

// ---------------------------------------------------------------- actuator net
// eval_actuator_network (:1311-1320) on the matrix cores.  One "group" = 16
// (env, joint) items; each item is carried by the 4 lanes {i, 16+i, 32+i, 48+i}
// of a wave (i = lane & 15, q = lane >> 4), exactly the v_mfma_f32_16x16x4_f32
// B-operand layout (B[k = q][item i]) and C/D layout (rows 4q..4q+3, column i).
//   layer 1: D = W1pad(32x8) . X(8x16): 2 M-tiles x 2 K-steps = 4 MFMA
//   layer 2: D = W2(32x32) . H1(32x16): each lane's layer-1 rows ARE its layer-2
//            B operand when the K-steps run over (m, r) with k = 16 m + 4 q + r,
//            so no data moves between the layers: 2 M-tiles x 8 K-steps = 16 MFMA
//   layer 3: per-lane fma over its 8 rows, then two xor-shuffles (16, 32).
// f32-input MFMA is bit-for-bit a k-ordered fmaf chain, and the oracle uses the
// same k order (oracle/go1_oracle.c go1o_actuator_eval): torques are bit-identical.
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

struct MlpFrag {
  float w1[2][2];  // [mo][s] = W1[16 mo + i][4 s + q]  (0 for k >= 6)
  float w2[2][8];  // [mo][4 m + r] = W2[16 mo + i][16 m + 4 q + r]
  f4 b1[2], b2[2]; // rows 4 q + r of tile mo
  float w3[2][4];  // w3[16 mo + 4 q + r]
  float b3;
};

__device__ __forceinline__ void mlp_load(const float* __restrict__ W, int lane, MlpFrag& F) {
  const int i = lane & 15, q = lane >> 4;
#pragma unroll
  for (int mo = 0; mo < 2; ++mo) {
#pragma unroll
    for (int sk = 0; sk < 2; ++sk) {
      const int k = 4 * sk + q;
      F.w1[mo][sk] = k < 6 ? W[(16 * mo + i) * 6 + k] : 0.0f;
    }
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) F.w2[mo][4 * m + r] = W[224 + (16 * mo + i) * 32 + 16 * m + 4 * q + r];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      F.b1[mo][r] = W[192 + 16 * mo + 4 * q + r];
      F.b2[mo][r] = W[1248 + 16 * mo + 4 * q + r];
      F.w3[mo][r] = W[1280 + 16 * mo + 4 * q + r];
    }
  }
  F.b3 = W[1312];
}

// The fragments wait out each sub-step's physics in LDS (round 6): the loop's register peak (the self-collision narrow
// phase, the capsule search, the trunk faces) is at the VGPR + AGPR limit, and 45 values held across it made the
// compiler spill.  mlp_unpark re-reads them through an opaque pointer before each evaluation (48 x 64 floats per wave).
#define MLP_PARK_FLOATS ((int)(sizeof(MlpFrag) / sizeof(float)))
__device__ __forceinline__ void mlp_park(const MlpFrag& F, float* s, int lane) {
  const float* f = reinterpret_cast<const float*>(&F);
#pragma unroll
  for (int k = 0; k < MLP_PARK_FLOATS; ++k) s[k * 64 + lane] = f[k];
}
__device__ __forceinline__ void mlp_unpark(MlpFrag& F, const float* s, int lane) {
  // an opaque lane index: no forwarding of the parked values (they would stay live in registers).  (An opaque
  // pointer would hide that s is LDS: the reads then compile to flat loads, with their longer latency.)
  asm volatile("" : "+v"(lane));
  float* f = reinterpret_cast<float*>(&F);
#pragma unroll
  for (int k = 0; k < MLP_PARK_FLOATS; ++k) f[k] = s[k * 64 + lane];
}

// b0 = X[k = q][item], b1v = X[k = 4 + q][item] (0 for q >= 2).  Returns the torque
// of item (lane & 15) in all four lanes of the item.  Needs all 64 lanes active.
__device__ __forceinline__ float mlp_group(const MlpFrag& F, float b0, float b1v) {
  f4 a1[2];
#pragma unroll
  for (int mo = 0; mo < 2; ++mo) {
    a1[mo] = __builtin_amdgcn_mfma_f32_16x16x4f32(F.w1[mo][0], b0, F.b1[mo], 0, 0, 0);
    a1[mo] = __builtin_amdgcn_mfma_f32_16x16x4f32(F.w1[mo][1], b1v, a1[mo], 0, 0, 0);
  }
  float h1[2][4];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 4; r += 2) {
      const f2 h = pm_softsign2(f2{a1[m][r], a1[m][r + 1]});
      h1[m][r] = h.x;
      h1[m][r + 1] = h.y;
    }
  f4 a2[2] = {F.b2[0], F.b2[1]};
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int mo = 0; mo < 2; ++mo)
        a2[mo] = __builtin_amdgcn_mfma_f32_16x16x4f32(F.w2[mo][4 * m + r], h1[m][r], a2[mo], 0, 0, 0);
  float h2[2][4];
#pragma unroll
  for (int mo = 0; mo < 2; ++mo)
#pragma unroll
    for (int r = 0; r < 4; r += 2) {
      const f2 h = pm_softsign2(f2{a2[mo][r], a2[mo][r + 1]});
      h2[mo][r] = h.x;
      h2[mo][r + 1] = h.y;
    }
  float p = 0.0f;
#pragma unroll
  for (int mo = 0; mo < 2; ++mo)
#pragma unroll
    for (int r = 0; r < 4; ++r) p = fmaf(F.w3[mo][r], h2[mo][r], p);
  return rowsum4(p) + F.b3;
}

// The three groups of a sub-step (joints 0..2) at once, layer by layer: 6 independent
// accumulator chains per layer keep the matrix pipe busy (one v_mfma_f32_16x16x4_f32 per
// 32 cycles per SIMD), and the softsign VALU of one group issues under the MFMAs of the
// next.  Each chain's k order is mlp_group's, so the torques are bit-identical to it.
__device__ __forceinline__ void mlp_group3(const MlpFrag& F, const float* b0, const float* b1v, float* t) {
  f4 a1[3][2];
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int mo = 0; mo < 2; ++mo) a1[g][mo] = __builtin_amdgcn_mfma_f32_16x16x4f32(F.w1[mo][0], b0[g], F.b1[mo], 0, 0, 0);
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int mo = 0; mo < 2; ++mo) a1[g][mo] = __builtin_amdgcn_mfma_f32_16x16x4f32(F.w1[mo][1], b1v[g], a1[g][mo], 0, 0, 0);
  float h1[3][2][4];
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        const f2 h = pm_softsign2(f2{a1[g][m][r], a1[g][m][r + 1]});
        h1[g][m][r] = h.x;
        h1[g][m][r + 1] = h.y;
      }
  f4 a2[3][2];
#pragma unroll
  for (int g = 0; g < 3; ++g) { a2[g][0] = F.b2[0]; a2[g][1] = F.b2[1]; }
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int mo = 0; mo < 2; ++mo)
          a2[g][mo] = __builtin_amdgcn_mfma_f32_16x16x4f32(F.w2[mo][4 * m + r], h1[g][m][r], a2[g][mo], 0, 0, 0);
#pragma unroll
  for (int g = 0; g < 3; ++g) {
    float p = 0.0f;
#pragma unroll
    for (int mo = 0; mo < 2; ++mo)
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        const f2 h = pm_softsign2(f2{a2[g][mo][r], a2[g][mo][r + 1]});
        p = fmaf(F.w3[mo][r], h.x, p);
        p = fmaf(F.w3[mo][r + 1], h.y, p);
      }
    t[g] = rowsum4(p) + F.b3;
  }
  // the matrix pipe takes one v_mfma_f32_16x16x4_f32 per 32 cycles and the wave may issue ~6 VALU
  // instructions in that gap: layer 1 first, then each layer-2 MFMA followed by softsign work
#pragma unroll
  for (int i = 0; i < 12; ++i) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
#pragma unroll
  for (int i = 0; i < 48; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
  }
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
  // fmodf is exact; so are its two cheap cases, which cover every angle this path wraps
  // (|a| < 2 |b|): a itself for |a| < |b|, and sign(a) (|a| - |b|) for |b| <= |a| < 2 |b|
  // (Sterbenz; the sign of a zero result is a's, as fmodf gives it).  The library's
  // iterative fmodf runs only for the rare larger |a|.
  const float aa = fabsf(a), ab = fabsf(b);
  float m = aa < ab ? a : copysignf(aa - ab, a);
  if (!(aa < 2.0f * ab)) m = fmodf(a, b);  // also NaN / inf inputs
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
// Everything from here to the step kernel is integrator code (compared with the f64
// oracle within a tolerance): FMA contraction on, including in the inlined helpers
// (a pragma inside phys_substep alone does not reach them).
#pragma clang fp contract(on)
// Spatial vectors (angular; linear).  6x6 symmetric articulated inertia stored as
// [[A, B], [B^T, C]], A and C symmetric (xx xy xz yy yz zz), B row-major 3x3.
struct SI {
  float a[6], b[9], c[6];
};

// Integrator-only fast math (hardware v_rcp_f32 / v_rsq_f32, ~1 ulp): the f32
// integrator is compared with the f64 oracle within a tolerance, never bitwise.
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
// hardware v_sin_f32 / v_cos_f32 on the angle in revolutions reduced to [0, 1) by v_fract_f32:
// 5 issue slots instead of the portable polynomial's ~25 (integrator only; absolute error
// ~1e-6, the step is compared with the f64 oracle within a tolerance)
__device__ __forceinline__ void hw_sincosf(float x, float* s, float* c) {
  const float r = __builtin_amdgcn_fractf(x * 0.159154943091895336f);
  *s = __builtin_amdgcn_sinf(r);
  *c = __builtin_amdgcn_cosf(r);
}
__device__ __forceinline__ float frsq(float x) { return __builtin_amdgcn_rsqf(x); }

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

// y = M v for a v whose components ax and 3 + ax are zero (c_j of a joint about axis ax)
__device__ __forceinline__ void si_mul_sparse(const SI& M, const float* v, int ax, float* o) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    float s = 0.0f, t = 0.0f;
    bool fs = true, ft = true;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if (j == ax) continue;
      s = fs ? S3(M.a, i, j) * v[j] : s + S3(M.a, i, j) * v[j];
      t = ft ? M.b[j * 3 + i] * v[j] : t + M.b[j * 3 + i] * v[j];
      fs = false; ft = false;
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if (j == ax) continue;
      s = s + M.b[i * 3 + j] * v[3 + j];
      t = t + S3(M.c, i, j) * v[3 + j];
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
  // structural zeros as -0.0: the compiler folds x + (-0.0) = x in si_add, not x + (+0.0)
  I.b[0] = -0.0f; I.b[1] = -m * c2; I.b[2] = m * c1;
  I.b[3] = m * c2; I.b[4] = -0.0f; I.b[5] = -m * c0;
  I.b[6] = -m * c1; I.b[7] = m * c0; I.b[8] = -0.0f;
  I.c[0] = m; I.c[1] = -0.0f; I.c[2] = -0.0f; I.c[3] = m; I.c[4] = -0.0f; I.c[5] = m;
}

// Rigid-body bias force v x* (I v) of a body (mass m, COM c, inertia Ic about the COM;
// model layout) from its momentum, without building the 6x6 inertia:
//   p = m (v + w x c),  L = Ic w + c x p,  v x* (L, p) = (w x L + v x p, w x p).
__device__ __forceinline__ void rigid_bias(const float* body, float mscale, const float* vel, float* o) {
  const float m = body[0] * mscale;
  const float* c = body + 1;
  const float* w = vel;
  const float* v = vel + 3;
  float wc[3], p[3], L[3], cp[3];
  cross3(w, c, wc);
#pragma unroll
  for (int i = 0; i < 3; ++i) p[i] = m * (v[i] + wc[i]);
  const float ixx = body[4] * mscale, ixy = body[5] * mscale, ixz = body[6] * mscale;
  const float iyy = body[7] * mscale, iyz = body[8] * mscale, izz = body[9] * mscale;
  cross3(c, p, cp);
  L[0] = ixx * w[0] + ixy * w[1] + ixz * w[2] + cp[0];
  L[1] = ixy * w[0] + iyy * w[1] + iyz * w[2] + cp[1];
  L[2] = ixz * w[0] + iyz * w[1] + izz * w[2] + cp[2];
  float a[3], b[3];
  cross3(w, L, a);
  cross3(v, p, b);
  o[0] = a[0] + b[0]; o[1] = a[1] + b[1]; o[2] = a[2] + b[2];
  cross3(w, p, o + 3);
}

// rigid_bias on a velocity given as (angular, linear) pairs, the result as pairs: the two
// products with w, w x L and w x p, run as one packed cross product of w with the (L, p) pairs
__device__ __forceinline__ void rigid_bias2(const float* body, const f2* vel, f2* o, float mscale = 1.0f) {
  const float m = body[0] * mscale;
  const float* c = body + 1;
  const float w[3] = {vel[0].x, vel[1].x, vel[2].x}, v[3] = {vel[0].y, vel[1].y, vel[2].y};
  float wc[3], p[3], L[3], cp[3], b[3];
  cross3(w, c, wc);
#pragma unroll
  for (int i = 0; i < 3; ++i) p[i] = m * (v[i] + wc[i]);
  const float ixx = body[4] * mscale, ixy = body[5] * mscale, ixz = body[6] * mscale;
  const float iyy = body[7] * mscale, iyz = body[8] * mscale, izz = body[9] * mscale;
  cross3(c, p, cp);
  L[0] = ixx * w[0] + ixy * w[1] + ixz * w[2] + cp[0];
  L[1] = ixy * w[0] + iyy * w[1] + iyz * w[2] + cp[1];
  L[2] = ixz * w[0] + iyz * w[1] + izz * w[2] + cp[2];
  const f2 X[3] = {f2{L[0], p[0]}, f2{L[1], p[1]}, f2{L[2], p[2]}};
  cross3(v, p, b);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
    const f2 wx = w[i1] * X[i2] - w[i2] * X[i1];
    o[i] = f2{wx.x + b[i], wx.y};
  }
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

// Revolute joint about coordinate axis ax (0 = x, 1 = y) by q: E = Rot(ax, q)^T maps
// parent coordinates to child coordinates.  Only (c, s) is kept; every product with E
// mixes two components.
__device__ __forceinline__ void rE(int ax, float c, float s, const float* v, float* o) {  // o = E v
  if (ax == 0) {
    float y = c * v[1] + s * v[2], z = c * v[2] - s * v[1];
    o[0] = v[0]; o[1] = y; o[2] = z;
  } else {
    float x = c * v[0] - s * v[2], z = s * v[0] + c * v[2];
    o[0] = x; o[1] = v[1]; o[2] = z;
  }
}

__device__ __forceinline__ void rET(int ax, float c, float s, const float* v, float* o) {  // o = E^T v
  if (ax == 0) {
    float y = c * v[1] - s * v[2], z = s * v[1] + c * v[2];
    o[0] = v[0]; o[1] = y; o[2] = z;
  } else {
    float x = c * v[0] + s * v[2], z = c * v[2] - s * v[0];
    o[0] = x; o[1] = v[1]; o[2] = z;
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

// Joint offsets are sparse in the Go1 model (go1_create checks it): hip (x, y, 0), thigh
// (0, y, 0), calf (0, 0, z).  `M` = mask of the components of r that may be non-zero
// (bit i = component i), a constant after inlining and unrolling, so the products with
// the zero components are never emitted (not even as 0 * x, which IEEE forbids folding).
__host__ __device__ __forceinline__ constexpr int offset_mask(int j) { return j == 0 ? 3 : (j == 1 ? 2 : 4); }
// which components of a x b can be non-zero, a and b with masks ma, mb
__device__ __forceinline__ constexpr int cross_mask(int ma, int mb) {
  int m = 0;
  for (int i = 0; i < 3; ++i) {
    const int p = (i + 1) % 3, q = (i + 2) % 3;
    if ((((ma >> p) & 1) && ((mb >> q) & 1)) || (((ma >> q) & 1) && ((mb >> p) & 1))) m |= 1 << i;
  }
  return m;
}
// component i of a x b (a_p b_q - a_q b_p) with only the terms the masks allow
__device__ __forceinline__ float cross_c(int ma, int mb, int i, const float* a, const float* b) {
  const int p = (i + 1) % 3, q = (i + 2) % 3;
  const bool t1 = ((ma >> p) & 1) && ((mb >> q) & 1), t2 = ((ma >> q) & 1) && ((mb >> p) & 1);
  if (t1 && t2) return a[p] * b[q] - a[q] * b[p];
  if (t1) return a[p] * b[q];
  if (t2) return -(a[q] * b[p]);
  return 0.0f;
}

// motion transform parent -> child: (w, v) -> (E w, E (v - r x w)), r with mask M
__device__ __forceinline__ void xm(int ax, float c, float s, int M, const float* r, const float* vin, float* vout) {
  const int cm = cross_mask(M, 7);
  float t[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) t[i] = ((cm >> i) & 1) ? vin[3 + i] - cross_c(M, 7, i, r, vin) : vin[3 + i];
  rE(ax, c, s, vin, vout);
  rE(ax, c, s, t, vout + 3);
}

// force transform child -> parent: (n, f) -> (E^T n + r x E^T f, E^T f), r with mask M
__device__ __forceinline__ void xfT(int ax, float c, float s, int M, const float* r, const float* fin, float* fout) {
  const int cm = cross_mask(M, 7);
  float n[3], f[3];
  rET(ax, c, s, fin, n);
  rET(ax, c, s, fin + 3, f);
#pragma unroll
  for (int i = 0; i < 3; ++i) fout[i] = ((cm >> i) & 1) ? n[i] + cross_c(M, 7, i, r, f) : n[i];
  fout[3] = f[0]; fout[4] = f[1]; fout[5] = f[2];
}

// Q = E^T M E for a full 3x3 M (row-major): rows of M E are E^T(row of M), then E^T per column.
__device__ __forceinline__ void rot_congruence(int ax, float c, float s, const float* M, float* Q) {
  float N[9];
#pragma unroll
  for (int i = 0; i < 3; ++i) rET(ax, c, s, M + 3 * i, N + 3 * i);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    float col[3] = {N[j], N[3 + j], N[6 + j]}, out[3];
    rET(ax, c, s, col, out);
    Q[j] = out[0]; Q[3 + j] = out[1]; Q[6 + j] = out[2];
  }
}

// Q = E^T M E for a symmetric M stored (xx xy xz yy yz zz) into a full 3x3 Q.  E^T rotates
// the two indices (p, r) other than the axis f by R = [[c, -s'], [s', c]] (s' = s for x,
// -s for y), so with c2 = c^2 - s'^2, s2 = 2 c s', h = (Mpp + Mrr) / 2, d = (Mpp - Mrr) / 2:
//   Qff = Mff, Qfp = c Mfp - s' Mfr, Qfr = s' Mfp + c Mfr,
//   Qpp = h + d c2 - Mpr s2, Qrr = h - d c2 + Mpr s2, Qpr = d s2 + Mpr c2.
__device__ __forceinline__ void rot_congruence_sym(int ax, float c, float s, float c2, float s2, const float* m,
                                                   float* Q) {
  const int f = ax, pI = ax == 0 ? 1 : 0, rI = 2;
  const float sp = ax == 0 ? s : -s;
  auto at = [&](int i, int j) -> float { return S3(m, i, j); };
  const float mff = at(f, f), mfp = at(f, pI), mfr = at(f, rI), mpp = at(pI, pI), mrr = at(rI, rI), mpr = at(pI, rI);
  const float h = 0.5f * (mpp + mrr), d = 0.5f * (mpp - mrr);
  const float qfp = c * mfp - sp * mfr, qfr = sp * mfp + c * mfr;
  const float qpp = h + d * c2 - mpr * s2, qrr = h - d * c2 + mpr * s2, qpr = d * s2 + mpr * c2;
  Q[f * 3 + f] = mff;
  Q[f * 3 + pI] = qfp; Q[pI * 3 + f] = qfp;
  Q[f * 3 + rI] = qfr; Q[rI * 3 + f] = qfr;
  Q[pI * 3 + pI] = qpp; Q[rI * 3 + rI] = qrr;
  Q[pI * 3 + rI] = qpr; Q[rI * 3 + pI] = qpr;
}

// X^T Ia X for X = [[E, 0], [-E r~, E]]: rotate the blocks by E^T(.)E, then translate by r
// (mask M):  A'' = A' + r~ B'^T - B' r~ - r~ C' r~ ,  B'' = B' + r~ C' ,  C'' = C'.
// RC = r~ C' has non-zero rows mc, BR = B' r~ non-zero columns mb, RCR = RC r~ both.
__device__ __forceinline__ void xform_inertia(int ax, float cq, float sq, int M, const float* r, const SI& In,
                                              SI& Out) {
  float A[9], B[9], C[9];
  const float sp = ax == 0 ? sq : -sq;
  const float c2 = cq * cq - sp * sp, s2 = 2.0f * cq * sp;
  rot_congruence_sym(ax, cq, sq, c2, s2, In.a, A);
  rot_congruence(ax, cq, sq, In.b, B);
  rot_congruence_sym(ax, cq, sq, c2, s2, In.c, C);
  // translation, with (M r~) row i = (row i of M) x r and r~ B'^T = -(B' r~)^T
  const int mc = cross_mask(M, 7), mb = cross_mask(7, M);
  float RC[9], BR[9], RCR[9];
#pragma unroll
  for (int j = 0; j < 3; ++j) {  // r~ C': column j = r x C'[:, j]
    const float col[3] = {C[j], C[3 + j], C[6 + j]};
#pragma unroll
    for (int i = 0; i < 3; ++i) RC[3 * i + j] = ((mc >> i) & 1) ? cross_c(M, 7, i, r, col) : 0.0f;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      BR[3 * i + j] = ((mb >> j) & 1) ? cross_c(7, M, j, B + 3 * i, r) : 0.0f;              // B' r~
      RCR[3 * i + j] = ((mc >> i) & (mb >> j) & 1) ? cross_c(7, M, j, RC + 3 * i, r) : 0.0f;  // r~ C' r~
    }
  // upper triangle of A'' = A' - BR^T - BR - RCR (symmetric); zero terms are skipped
  const int II[6] = {0, 0, 0, 1, 1, 2}, JJ[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
  for (int t = 0; t < 6; ++t) {
    const int i = II[t], j = JJ[t];
    float v = A[i * 3 + j];
    if ((mb >> i) & 1) v -= BR[j * 3 + i];
    if ((mb >> j) & 1) v -= BR[i * 3 + j];
    if ((mc >> i) & (mb >> j) & 1) v -= RCR[i * 3 + j];
    Out.a[t] = v;
    Out.c[t] = C[i * 3 + j];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) Out.b[3 * i + j] = ((mc >> i) & 1) ? B[3 * i + j] + RC[3 * i + j] : B[3 * i + j];
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
      if (i == j) LI(i, i) = frsq(fmaxf(s, 1e-30f));  // holds 1 / L_ii
      else LI(i, j) = s * LI(j, j);
    }
  float y[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    float s = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) s -= LI(i, k) * y[k];
    y[i] = s * LI(i, i);
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    float s = y[i];
#pragma unroll
    for (int k = i + 1; k < 6; ++k) s -= LI(k, i) * x[k];
    x[i] = s * LI(i, i);
  }
#undef LI
}

// ---- packed articulated-body algebra.  One wave alone issues a v_pk_fma_f32 (two FMAs) as
// fast as a v_fma_f32 (tools/probes/pk_rate.hip), and a spatial quantity pairs up by itself:
// a spatial vector is three (angular_i, linear_i) pairs, and a spatial inertia keeps its two
// symmetric 3 x 3 blocks as six (A_t, C_t) pairs -- every rotation, rank-1 update and sum of the
// articulated-body passes treats the two halves alike.  B (general 3 x 3) stays scalar.
struct SIP {
  f2 ac[6];
  float b[9];
};
__host__ __device__ __forceinline__ constexpr int s3i(int i, int j) {
  return i == 0 ? j : (i == 1 ? (j == 0 ? 1 : j + 2) : (j == 0 ? 2 : (j == 1 ? 4 : 5)));
}

__device__ __forceinline__ void rigid_sip(const float* body, float mscale, SIP& I) {
  SI s;
  rigid_si(body, mscale, s);
#pragma unroll
  for (int t = 0; t < 6; ++t) I.ac[t] = f2{s.a[t], s.c[t]};
#pragma unroll
  for (int i = 0; i < 9; ++i) I.b[i] = s.b[i];
}

__device__ __forceinline__ void sip_add(SIP& A, const SIP& B) {
#pragma unroll
  for (int t = 0; t < 6; ++t) A.ac[t] += B.ac[t];
#pragma unroll
  for (int i = 0; i < 9; ++i) A.b[i] += B.b[i];
}

// column ax of the 6 x 6 matrix as pairs: (A(i, ax), B^T(i, ax) = B(ax, i))
__device__ __forceinline__ f2 sip_col(const SIP& M, int ax, int i) { return f2{M.ac[s3i(i, ax)].x, M.b[ax * 3 + i]}; }

// y = M v for a v whose pair ax is zero (c_j of a joint about axis ax); v, y as pairs
__device__ __forceinline__ void sip_mul_sparse(const SIP& M, const f2* v, int ax, f2* o) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    f2 st = f2{0.0f, 0.0f};
    bool first = true;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if (j == ax) continue;
      st = first ? M.ac[s3i(i, j)] * v[j] : st + M.ac[s3i(i, j)] * v[j];
      first = false;
    }
    float s = st.x, t = st.y;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if (j == ax) continue;
      s = s + M.b[i * 3 + j] * v[j].y;
      t = t + M.b[j * 3 + i] * v[j].x;
    }
    o[i] = f2{s, t};
  }
}

// E v (rE) and E^T v (rET) on pairs: both halves rotate by the same joint rotation
__device__ __forceinline__ void rE2(int ax, float c, float s, const f2* v, f2* o) {
  if (ax == 0) {
    const f2 y = c * v[1] + s * v[2], z = c * v[2] - s * v[1];
    o[0] = v[0]; o[1] = y; o[2] = z;
  } else {
    const f2 x = c * v[0] - s * v[2], z = s * v[0] + c * v[2];
    o[0] = x; o[1] = v[1]; o[2] = z;
  }
}
__device__ __forceinline__ void rET2(int ax, float c, float s, const f2* v, f2* o) {
  if (ax == 0) {
    const f2 y = c * v[1] - s * v[2], z = s * v[1] + c * v[2];
    o[0] = v[0]; o[1] = y; o[2] = z;
  } else {
    const f2 x = c * v[0] + s * v[2], z = c * v[2] - s * v[0];
    o[0] = x; o[1] = v[1]; o[2] = z;
  }
}

// motion transform parent -> child on pairs: (w, v) -> (E w, E (v - r x w)), r with mask M
__device__ __forceinline__ void xm2(int ax, float c, float s, int M, const float* r, const f2* vin, f2* vout) {
  const int cm = cross_mask(M, 7);
  const float w[3] = {vin[0].x, vin[1].x, vin[2].x};
  f2 t[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) t[i] = f2{w[i], ((cm >> i) & 1) ? vin[i].y - cross_c(M, 7, i, r, w) : vin[i].y};
  rE2(ax, c, s, t, vout);
}

// force transform child -> parent on pairs: (n, f) -> (E^T n + r x E^T f, E^T f), r with mask M
__device__ __forceinline__ void xfT2(int ax, float c, float s, int M, const float* r, const f2* fin, f2* fout) {
  const int cm = cross_mask(M, 7);
  f2 nf[3];
  rET2(ax, c, s, fin, nf);
  const float f[3] = {nf[0].y, nf[1].y, nf[2].y};
#pragma unroll
  for (int i = 0; i < 3; ++i) fout[i] = f2{((cm >> i) & 1) ? nf[i].x + cross_c(M, 7, i, r, f) : nf[i].x, f[i]};
}

// X^T Ia X (xform_inertia) with the A and C blocks rotated together as pairs
__device__ __forceinline__ void xform_inertia2(int ax, float cq, float sq, int M, const float* r, const SIP& In,
                                               SIP& Out) {
  const float sp = ax == 0 ? sq : -sq;
  const float c2 = cq * cq - sp * sp, s2 = 2.0f * cq * sp;
  // rot_congruence_sym on (A, C) pairs
  const int f = ax, pI = ax == 0 ? 1 : 0, rI = 2;
  const f2 mff = In.ac[s3i(f, f)], mfp = In.ac[s3i(f, pI)], mfr = In.ac[s3i(f, rI)];
  const f2 mpp = In.ac[s3i(pI, pI)], mrr = In.ac[s3i(rI, rI)], mpr = In.ac[s3i(pI, rI)];
  const f2 h = 0.5f * (mpp + mrr), d = 0.5f * (mpp - mrr);
  const f2 qfp = cq * mfp - sp * mfr, qfr = sp * mfp + cq * mfr;
  const f2 qpp = h + d * c2 - mpr * s2, qrr = h - d * c2 + mpr * s2, qpr = d * s2 + mpr * c2;
  f2 Q[9];
  Q[f * 3 + f] = mff;
  Q[f * 3 + pI] = qfp; Q[pI * 3 + f] = qfp;
  Q[f * 3 + rI] = qfr; Q[rI * 3 + f] = qfr;
  Q[pI * 3 + pI] = qpp; Q[rI * 3 + rI] = qrr;
  Q[pI * 3 + rI] = qpr; Q[rI * 3 + pI] = qpr;
  float B[9], C[9];
  rot_congruence(ax, cq, sq, In.b, B);
#pragma unroll
  for (int i = 0; i < 9; ++i) C[i] = Q[i].y;
  // translation by r (xform_inertia): A'' = A' - BR^T - BR - RCR, B'' = B' + RC, C'' = C'
  const int mc = cross_mask(M, 7), mb = cross_mask(7, M);
  float RC[9], BR[9], RCR[9];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const float col[3] = {C[j], C[3 + j], C[6 + j]};
#pragma unroll
    for (int i = 0; i < 3; ++i) RC[3 * i + j] = ((mc >> i) & 1) ? cross_c(M, 7, i, r, col) : 0.0f;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      BR[3 * i + j] = ((mb >> j) & 1) ? cross_c(7, M, j, B + 3 * i, r) : 0.0f;
      RCR[3 * i + j] = ((mc >> i) & (mb >> j) & 1) ? cross_c(7, M, j, RC + 3 * i, r) : 0.0f;
    }
  const int II[6] = {0, 0, 0, 1, 1, 2}, JJ[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
  for (int t = 0; t < 6; ++t) {
    const int i = II[t], j = JJ[t];
    float v = Q[i * 3 + j].x;
    if ((mb >> i) & 1) v -= BR[j * 3 + i];
    if ((mb >> j) & 1) v -= BR[i * 3 + j];
    if ((mc >> i) & (mb >> j) & 1) v -= RCR[i * 3 + j];
    Out.ac[t] = f2{v, C[i * 3 + j]};
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) Out.b[3 * i + j] = ((mc >> i) & 1) ? B[3 * i + j] + RC[3 * i + j] : B[3 * i + j];
}

__device__ __forceinline__ float sip_get(const SIP& M, int i, int j) {
  if (i < 3 && j < 3) return M.ac[s3i(i, j)].x;
  if (i >= 3 && j >= 3) return M.ac[s3i(i - 3, j - 3)].y;
  if (i < 3) return M.b[i * 3 + (j - 3)];
  return M.b[j * 3 + (i - 3)];
}

// 6x6 SPD solve (Cholesky) of the packed inertia, identical instruction stream in every lane
__device__ __forceinline__ void solve6p(const SIP& M, const float* b, float* x) {
  float L[21];
#define LI(i, j) L[(i) * ((i) + 1) / 2 + (j)]
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j <= i; ++j) {
      float s = sip_get(M, i, j);
#pragma unroll
      for (int k = 0; k < j; ++k) s -= LI(i, k) * LI(j, k);
      if (i == j) LI(i, i) = frsq(fmaxf(s, 1e-30f));  // holds 1 / L_ii
      else LI(i, j) = s * LI(j, j);
    }
  float y[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    float s = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) s -= LI(i, k) * y[k];
    y[i] = s * LI(i, i);
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    float s = y[i];
#pragma unroll
    for (int k = i + 1; k < 6; ++k) s -= LI(k, i) * x[k];
    x[i] = s * LI(i, i);
  }
#undef LI
}

__device__ __forceinline__ void quat_to_R(const float* q, float* R) {
  float x = q[0], y = q[1], z = q[2], w = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - z * w); R[2] = 2 * (x * z + y * w);
  R[3] = 2 * (x * y + z * w); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - x * w);
  R[6] = 2 * (x * z - y * w); R[7] = 2 * (y * z + x * w); R[8] = 1 - 2 * (x * x + y * y);
}

// Terrain view of one env.  `patch` is an LDS copy of the PSZX x PSZY cells around
// the env's base at the start of the step, floor and ceiling interleaved, filled
// once per step by the whole block; the integrator's contact queries hit it and
// fall back to the HBM tile outside it (identical values: a pure cache).
// 20 rows (x) x 16 columns (y): the legs' bounding box spans up to 14 cells in x and 12 in y
// (p99 under N(0, 1) actions), the patch is placed on its centre, and the rows leave room for
// the motion during the step
#define PSZX 20
#define PSZY 16
static_assert(PSZY == 16 && PSZX % 2 == 0, "the LDS-DMA patch staging maps 2 rows of 16 cells to a wave");
struct Terr {
  const float* tile;  // (2, nx, ny) or nullptr
  int nx, ny;
  float hs;             // queries are relative to the env's terrain origin
  const float2* patch;  // LDS, PSZX x PSZY (floor, ceiling) or nullptr
  int pi0, pj0;
};

__device__ __forceinline__ float tile_at(const Terr& T, int layer, int i, int j) {
  i = min(max(i, 0), T.nx - 1);
  j = min(max(j, 0), T.ny - 1);
  return T.tile[((size_t)layer * T.nx + i) * T.ny + j];
}

struct CP {
  float k, d, kf, mu;
  float e, vb;  // restitution (the env's and the terrain's, averaged) and the bounce threshold
};

// ---- packed (v_pk_*_f32) contact: one wave issues a v_pk_fma_f32 (two FMAs) as fast as a
// v_fma_f32 (tools/probes/pk_rate.hip), so the floor and ceiling layers of a point are
// carried as the two halves of an f2 all the way from the mesh triangle to the force.
__device__ __forceinline__ f2 f2s(float v) { return f2{v, v}; }

// (floor, ceiling) at the four corners of cell (i, j): the LDS patch, or the tile outside it
// (the patch read unconditionally, the tile only in a wave with a lane outside the patch: as an if / else per lane
// the two paths were exec-mask branches every call)
__device__ __forceinline__ void cell_fetch(const Terr& T, int i, int j, f2& c00, f2& c10, f2& c01, f2& c11) {
  const unsigned li = (unsigned)(i - T.pi0), lj = (unsigned)(j - T.pj0);
  const bool in = (T.patch != nullptr) & (li < (unsigned)(PSZX - 1)) & (lj < (unsigned)(PSZY - 1));
  if (T.patch) {
    const float2* pp = T.patch + (in ? (int)(li * PSZY + lj) : 0);
    const float2 q00 = pp[0], q01 = pp[1], q10 = pp[PSZY], q11 = pp[PSZY + 1];
    c00 = f2{q00.x, q00.y}; c01 = f2{q01.x, q01.y}; c10 = f2{q10.x, q10.y}; c11 = f2{q11.x, q11.y};
  }
  if (__any(!in)) {
    if (!in) {
      c00 = f2{tile_at(T, 1, i, j), tile_at(T, 0, i, j)};
      c10 = f2{tile_at(T, 1, i + 1, j), tile_at(T, 0, i + 1, j)};
      c01 = f2{tile_at(T, 1, i, j + 1), tile_at(T, 0, i, j + 1)};
      c11 = f2{tile_at(T, 1, i + 1, j + 1), tile_at(T, 0, i + 1, j + 1)};
    }
  }
}

// (floor, ceiling) heights and gradients at world (x, y) in two halves, so that the corner reads are issued early and
// land while independent work runs: hq_fetch reads the cell's four (floor, ceiling) corners -- the LDS patch stores
// (floor, ceiling) per cell, i.e. already in f2 layout; the HBM tile outside it -- and hq_finish evaluates the
// triangle's plane.
struct HQ {
  f2 c00, c10, c01, c11;
  float a, b;
  bool up;  // the cell's upper triangle (a < b): (i, j), (i + 1, j + 1), (i, j + 1); else (i, j), (i + 1, j), (i + 1, j + 1)
};
__device__ __forceinline__ void hq_fetch(const Terr& T, float x, float y, HQ& q) {
  if (!T.tile) {
    q.c00 = q.c10 = q.c01 = q.c11 = f2{0.0f, 1e9f};
    q.a = q.b = 0.0f;
    q.up = false;
    return;
  }
  const float ihs = frcp(T.hs);
  const float u = fminf(fmaxf(x * ihs, -4.0f), (float)(T.nx + 4));
  const float v = fminf(fmaxf(y * ihs, -4.0f), (float)(T.ny + 4));
  const float fu = floorf(u), fv = floorf(v);
  q.a = u - fu;
  q.b = v - fv;
  q.up = q.a < q.b;
  cell_fetch(T, (int)fu, (int)fv, q.c00, q.c10, q.c01, q.c11);
}
// the cell and triangle of a capsule's deepest point (SEG_CELL, seg_deepest2): a = u - i, b = v - j on that triangle's
// plane, so at a mesh edge the normal is the one of the triangle the search chose, not whichever side floor() of a
// rounded coordinate lands on (which the f32 kernel and the f64 oracle would decide differently)
__device__ __forceinline__ void hq_fetch_cell(const Terr& T, float x, float y, int cell, HQ& q) {
  if (!T.tile) {
    q.c00 = q.c10 = q.c01 = q.c11 = f2{0.0f, 1e9f};
    q.a = q.b = 0.0f;
    q.up = false;
    return;
  }
  const float ihs = frcp(T.hs);
  const float u = fminf(fmaxf(x * ihs, -4.0f), (float)(T.nx + 4));
  const float v = fminf(fmaxf(y * ihs, -4.0f), (float)(T.ny + 4));
  const int i = (cell >> 16) - 16384, j = (cell & 0x7fff) - 16384;
  q.a = u - (float)i;
  q.b = v - (float)j;
  q.up = (cell >> 15) & 1;
  cell_fetch(T, i, j, q.c00, q.c10, q.c01, q.c11);
}
// height and gradient of (floor, ceiling) on the triangle.  Round 6: the surface is the heightfield's triangle mesh,
// as the reference collides with it (mesh_type 'trimesh'; tunnel.py:139-147 builds it with isaacgym terrain_utils.
// convert_heightfield_to_trimesh: every cell split along its (i, j) - (i + 1, j + 1) diagonal); oracle tri_query
__device__ __forceinline__ void hq_finish(const Terr& T, const HQ& q, f2& h, f2& gx, f2& gy) {
  const float ihs = frcp(T.hs);
  const f2 da = q.up ? q.c11 - q.c01 : q.c10 - q.c00, db = q.up ? q.c01 - q.c00 : q.c11 - q.c10;
  h = q.c00 + q.a * da + q.b * db;
  gx = da * ihs;
  gy = db * ihs;
}

// Restitution.  PhysX bounces a contact whose relative velocity exceeds the bounce threshold with the
// coefficient e (the average of the two shapes').  A penalty contact has no impact event to attach a velocity
// target to (no per-contact state), so e acts on the dissipation of the rebound: while a point separates
// faster than the threshold, the explicit part of the normal force gets + e (h k + d) vn, i.e. the fraction e
// of the linearly implicit contact's damping (the physical d and the h k of the implicit spring) is handed
// back; the added mass h (h k + d) n n^T stays, so the velocity update keeps a contraction factor
// (m + e c) / (m + c) <= 1 (c = h (h k + d)): no e in [0, 1] adds energy (tests/test_self_collision.py).
// e = 0 leaves the force bit for bit as before.
__device__ __forceinline__ f2 restitute(const CP& C, float h, f2 vn, f2 fn) {
  const float cr = (h * C.k + C.d) * C.e;
  return f2{(C.e > 0.0f & vn.x > C.vb) ? fn.x + cr * vn.x : fn.x, (C.e > 0.0f & vn.y > C.vb) ? fn.y + cr * vn.y : fn.y};
}

// The same contact, linearly implicit in the point velocity (the integrator's scheme: one 5 ms step
// per sim step, like PhysX's substeps = 1).  For an active layer the force at the end of the step,
// k (depth - h vn') - d vn' (normal) and -c_t vt' (regularised friction, c_t = min(kf, mu fn / |vt|)
// from the current state), with v' = v + h a_p, splits into an explicit force F and an added mass
//   Mp = h (h k + d) n n^T + h c_t (I - n n^T)
// on the point (world frame, summed over floor and ceiling; xx xy xz yy yz zz), which the caller
// puts into the link's articulated inertia, so the ABA accelerations include the contact response.
// oracle/go1_oracle.c sphere_contact_im is the f64 restatement.
__device__ __forceinline__ void sphere_contact_im(const Terr& T, const HQ& q, const CP& C, const float* p,
                                                  const float* pv, float r, float h, float* F, float* Mp) {
  f2 hh, gx, gy;
  hq_finish(T, q, hh, gx, gy);
  const f2 sg = f2{1.0f, -1.0f};
  const f2 dv = sg * (hh - p[2]) + r;  // floor: h + r - z, ceiling: z + r - h
  f2 nx = -sg * gx, ny = -sg * gy;
  f2 inv = nx * nx + ny * ny + 1.0f;
  inv = f2{frsq(inv.x), frsq(inv.y)};
  nx = nx * inv;
  ny = ny * inv;
  const f2 nz = sg * inv;
  const f2 depth = dv * inv;
  const f2 vn = pv[0] * nx + pv[1] * ny + pv[2] * nz;
  const f2 fn0 = C.k * depth - C.d * vn;          // activation: compressive at the current state
  const f2 fn = restitute(C, h, vn, fn0 - (h * C.k) * vn);  // k depth - (h k + d) vn [+ e (h k + d) vn]
  const f2 vtx = pv[0] - vn * nx, vty = pv[1] - vn * ny, vtz = pv[2] - vn * nz;
  const f2 vt2 = vtx * vtx + vty * vty + vtz * vtz;
  const f2 ivt = f2{frsq(fmaxf(vt2.x, 1e-18f)), frsq(fmaxf(vt2.y, 1e-18f))};
  const f2 vtn = vt2 * ivt;
  const f2 cm = C.mu * fn0;
  // c_t = min(kf, mu fn0 / |vt|); kf in the viscous limit |vt| -> 0
  const f2 ct = f2{(C.kf * vtn.x > cm.x & vtn.x > 1e-9f) ? cm.x * ivt.x : C.kf,
                   (C.kf * vtn.y > cm.y & vtn.y > 1e-9f) ? cm.y * ivt.y : C.kf};
  const bool ax = dv.x > 0.0f & fn0.x > 0.0f, ay = dv.y > 0.0f & fn0.y > 0.0f;
  const f2 fa = f2{ax ? fn.x : 0.0f, ay ? fn.y : 0.0f};
  const f2 sc = f2{ax ? ct.x : 0.0f, ay ? ct.y : 0.0f};
  const f2 Fx = fa * nx - sc * vtx, Fy = fa * ny - sc * vty, Fz = fa * nz - sc * vtz;
  F[0] = Fx.x + Fx.y;
  F[1] = Fy.x + Fy.y;
  F[2] = Fz.x + Fz.y;
  const float cn = h * (h * C.k + C.d);
  const f2 cd = h * sc, cnd = f2{ax ? cn : 0.0f, ay ? cn : 0.0f} - cd;  // (cn - cd) on active layers
  const f2 a = cnd * nx, b = cnd * ny, c = cnd * nz;
  const f2 mxx = a * nx + cd, mxy = a * ny, mxz = a * nz, myy = b * ny + cd, myz = b * nz, mzz = c * nz + cd;
  Mp[0] = mxx.x + mxx.y; Mp[1] = mxy.x + mxy.y; Mp[2] = mxz.x + mxz.y;
  Mp[3] = myy.x + myy.y; Mp[4] = myz.x + myz.y; Mp[5] = mzz.x + mzz.y;
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

// ---- capsules against the heightfield meshes (round 6; oracle/go1_oracle.c seg_deepest is the f64 restatement).  A
// capsule (segment A -> B, radius r) acts at the deepest point of its segment: the t in [0, 1] that maximises the
// vertical gap of either layer, floor h_f + r - z and ceiling z + r - h_c.  Both layers are triangle meshes over the
// grid (hq_finish), so along the segment the gaps are piecewise linear in t and their maximum lies at an end or where
// the segment's (x, y) projection crosses a mesh edge: a grid line u = k or v = k, or a cell diagonal u - v = k.  The
// candidates are exactly those (on an edge the height interpolates its two vertices): exact, and no serial walk --
// every candidate's reads are independent.  A half link of 0.1065 m crosses at most 3 lines of each grid direction
// and 4 diagonals at 0.05 m cells (go1_create rejects finer grids).  Each candidate carries the cell and triangle on
// the segment's incoming side of its edge; the contact takes that triangle's plane (hq_fetch_cell).  A candidate's
// key is its deeper layer's gap quantised to 1e-5 m, ties to the smaller t (the segment's first end; the link halves
// start at their outer ends, so a link lying flat is carried at both): this f32 search and the oracle's f64 one
// choose the same point.  On the plane: the lower end (ties: A).  The search runs once per control step; the chosen t
// is held for the control step's sim steps (phys_substep), as the trunk faces' vertices are.
#define SEG_QI 1.0e5f  // 1 / SEG_Q of the oracle
__device__ __forceinline__ int seg_quant(float g) { return (int)floorf(fminf(fmaxf(g, -1.0f), 1.0f) * SEG_QI); }
// cell (i, j in [-4, n + 4]) and triangle (up: the upper one) packed into a positive int
#define SEG_CELL(i, j, up) ((((i) + 16384) << 16) | ((up) ? 0x8000 : 0) | ((j) + 16384))
struct SegBest {
  int key;   // the best candidate's key: quantised gap (the deeper layer) x 4096 + the earlier t (4095 - 4095 t)
  float t;   // its t
  int cell;  // and its cell and triangle
};
__device__ __forceinline__ void seg_offer(SegBest& sb, f2 h, float z, float r, float t, int cell, bool valid) {
  const int q = seg_quant(fmaxf((h.x - z) + r, (z - h.y) + r));  // (the quantisation is monotone: = the max of both)
  const int key = q * 4096 + (4095 - (int)floorf(t * 4095.0f));
  const bool up = valid & (key > sb.key);  // an equal key (a vertex on several edges) keeps the first offer
  sb.key = up ? key : sb.key;
  sb.t = up ? t : sb.t;
  sb.cell = up ? cell : sb.cell;
}
// the (floor, ceiling) mesh vertices (vi, vj): the LDS patch in one batch of reads, then the HBM tile for the rare
// ones outside it (a wave-uniform branch), so the wave waits for the patch once per batch
template <int N>
__device__ __forceinline__ void verts_fetch(const Terr& T, const int* vi, const int* vj, f2* h) {
  unsigned out = T.patch ? 0u : (1u << N) - 1u;
  if (T.patch) {
#pragma unroll
    for (int n = 0; n < N; ++n) {
      // (unsigned: a negative offset is out of range too; outside the patch read cell 0, replaced below)
      const unsigned li = (unsigned)(vi[n] - T.pi0), lj = (unsigned)(vj[n] - T.pj0);
      const bool in = (li < (unsigned)PSZX) & (lj < (unsigned)PSZY);
      const float2 q = T.patch[in ? (int)(li * PSZY + lj) : 0];
      h[n] = f2{q.x, q.y};
      out |= in ? 0u : 1u << n;
    }
  }
  if (__any(out != 0u)) {
#pragma unroll
    for (int n = 0; n < N; ++n)
      if ((out >> n) & 1u) h[n] = f2{tile_at(T, 1, vi[n], vj[n]), tile_at(T, 0, vi[n], vj[n])};
  }
}
// deepest point of one segment (world ends A, B): t and SEG_CELL.  Two batches of candidates (the ends and the lines
// u = k; the lines v = k and the diagonals), each gathering its mesh vertices (verts_fetch) before comparing them
__device__ __forceinline__ float seg_deepest(const Terr& T, const float* A, const float* B, float r, int& cell) {
  if (!T.tile) {  // the plane: the lower end
    cell = SEG_CELL(0, 0, false);
    return seg_quant(r - B[2]) > seg_quant(r - A[2]) ? 1.0f : 0.0f;
  }
  const float ihs = frcp(T.hs);
  const float uA = fminf(fmaxf(A[0] * ihs, -4.0f), (float)(T.nx + 4)), vA = fminf(fmaxf(A[1] * ihs, -4.0f), (float)(T.ny + 4));
  const float uB = fminf(fmaxf(B[0] * ihs, -4.0f), (float)(T.nx + 4)), vB = fminf(fmaxf(B[1] * ihs, -4.0f), (float)(T.ny + 4));
  const float du = uB - uA, dv = vB - vA, dw = du - dv, dz = B[2] - A[2], zA = A[2];
  // an invalid candidate (beyond the segment's crossings) reads A's cell instead of an edge up to 4 cells off, which
  // could leave the LDS patch
  const int iA = (int)floorf(uA), jA = (int)floorf(vA);
  SegBest sb;
  sb.key = -2147483647 - 1;
  sb.t = 0.0f;
  sb.cell = SEG_CELL(0, 0, false);
  {  // the ends (vertices c00, c11 and c01 on the upper triangle / c10) and the grid lines u = k (the edge (k, j) -
     // (k, j + 1), entered from cell k - 1 (du > 0) or k)
    int vi[12], vj[12];
    float ca[5], cb[2], ct[3];
    int ccell[5];
    bool cup[2], cval[3];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const float u = e ? uB : uA, v = e ? vB : vA;
      const float fu = floorf(u), fv = floorf(v);
      const int i = (int)fu, j = (int)fv;
      ca[e] = u - fu;
      cb[e] = v - fv;
      cup[e] = ca[e] < cb[e];
      ccell[e] = SEG_CELL(i, j, cup[e]);
      vi[3 * e] = i; vj[3 * e] = j;
      vi[3 * e + 1] = i + 1; vj[3 * e + 1] = j + 1;
      vi[3 * e + 2] = cup[e] ? i : i + 1; vj[3 * e + 2] = cup[e] ? j + 1 : j;
    }
    const int k0 = (int)floorf(fminf(uA, uB)) + 1;
    const float hi = fmaxf(uA, uB), rdu = du != 0.0f ? frcp(du) : 0.0f;
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      const int k = k0 + m, n = 6 + 2 * m;
      const bool valid = (float)k < hi;
      const float t = valid ? ((float)k - uA) * rdu : 0.0f, v = vA + dv * t, fv = floorf(v), b = v - fv;
      const int j = (int)fv, i = du > 0.0f ? k - 1 : k;
      ct[m] = t; ca[2 + m] = b; cval[m] = valid;
      ccell[2 + m] = SEG_CELL(i, j, (float)(k - i) < b);
      vi[n] = valid ? k : iA; vj[n] = valid ? j : jA;
      vi[n + 1] = vi[n]; vj[n + 1] = vj[n] + 1;
    }
    f2 h[12];
    verts_fetch<12>(T, vi, vj, h);
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const f2 c00 = h[3 * e], c11 = h[3 * e + 1], cx = h[3 * e + 2];
      const f2 da = cup[e] ? c11 - cx : cx - c00, db = cup[e] ? cx - c00 : c11 - cx;
      seg_offer(sb, c00 + ca[e] * da + cb[e] * db, e ? B[2] : zA, r, (float)e, ccell[e], true);
    }
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      const f2 p0 = h[6 + 2 * m], p1 = h[7 + 2 * m];
      seg_offer(sb, p0 + ca[2 + m] * (p1 - p0), zA + dz * ct[m], r, ct[m], ccell[2 + m], cval[m]);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  {  // the grid lines v = k (the edge (i, k) - (i + 1, k), entered from cell k - 1 (dv > 0) or k) and the cell
     // diagonals u - v = k (the point (i + a, j + a) of cell (i, j), i - j = k, entered from the upper triangle (dw > 0:
     // u - v grows through k, a < b before) or the lower)
    int vi[14], vj[14];
    float ca[7], ct[7];
    int ccell[7];
    bool cval[7];
    {
      const int k0 = (int)floorf(fminf(vA, vB)) + 1;
      const float hi = fmaxf(vA, vB), rdv = dv != 0.0f ? frcp(dv) : 0.0f;
#pragma unroll
      for (int m = 0; m < 3; ++m) {
        const int k = k0 + m, n = 2 * m;
        const bool valid = (float)k < hi;
        const float t = valid ? ((float)k - vA) * rdv : 0.0f, u = uA + du * t, fu = floorf(u), a = u - fu;
        const int i = (int)fu, j = dv > 0.0f ? k - 1 : k;
        ct[m] = t; ca[m] = a; cval[m] = valid;
        ccell[m] = SEG_CELL(i, j, a < (float)(k - j));
        vi[n] = valid ? i : iA; vj[n] = valid ? k : jA;
        vi[n + 1] = vi[n] + 1; vj[n + 1] = vj[n];
      }
    }
    {
      const float wA = uA - vA, wB = uB - vB;
      const int k0 = (int)floorf(fminf(wA, wB)) + 1;
      const float hi = fmaxf(wA, wB), rdw = dw != 0.0f ? frcp(dw) : 0.0f;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int k = k0 + m, c = 3 + m, n = 2 * c;
        const bool valid = (float)k < hi;
        const float t = valid ? ((float)k - wA) * rdw : 0.0f, u = uA + du * t, fu = floorf(u), a = u - fu;
        const int i = (int)fu, j = i - k;
        ct[c] = t; ca[c] = a; cval[c] = valid;
        ccell[c] = SEG_CELL(i, j, dw > 0.0f);
        vi[n] = valid ? i : iA; vj[n] = valid ? j : jA;
        vi[n + 1] = vi[n] + 1; vj[n + 1] = vj[n] + 1;
      }
    }
    f2 h[14];
    verts_fetch<14>(T, vi, vj, h);
#pragma unroll
    for (int c = 0; c < 7; ++c) {
      const f2 p0 = h[2 * c], p1 = h[2 * c + 1];
      seg_offer(sb, p0 + ca[c] * (p1 - p0), zA + dz * ct[c], r, ct[c], ccell[c], cval[c]);
    }
  }
  cell = sb.cell;
  return sb.t;
}
// the lane's two segments (x, y halves of the contact pass)
__device__ __forceinline__ f2 seg_deepest2(const Terr& T, const f2* A, const f2* B, f2 r, int* cell) {
  const float a0[3] = {A[0].x, A[1].x, A[2].x}, b0[3] = {B[0].x, B[1].x, B[2].x};
  const float a1[3] = {A[0].y, A[1].y, A[2].y}, b1[3] = {B[0].y, B[1].y, B[2].y};
  const float tx = seg_deepest(T, a0, b0, r.x, cell[0]);
  __builtin_amdgcn_sched_barrier(0);  // one segment's vertex batch live at a time
  const float ty = seg_deepest(T, a1, b1, r.y, cell[1]);
  return f2{tx, ty};
}

__device__ __forceinline__ void point_force(const float* Rb, const float* lp, const float* F, float* fs) {
  float f[3], n[3];
  mat3T_vec(Rb, F, f);
  cross3(lp, f, n);
  fs[0] += n[0]; fs[1] += n[1]; fs[2] += n[2]; fs[3] += f[0]; fs[4] += f[1]; fs[5] += f[2];
}

// Physical state of one env as held by one lane of its quad.
// World position of this leg's foot body origin (rigid_body_state[:, feet, 0:3] after
// the last sim step), the kinematic chain of phys_substep without velocities.
__device__ void foot_world(const float* __restrict__ model, const float* root, const float* q, int leg, float* out) {
  float Rp[9], pp[3] = {root[0], root[1], root[2]};
  quat_to_R(root + 3, Rp);
  const float* origin = model + 13 * 10 + leg * 9;
  const float* foot = model + 13 * 10 + 4 * 9;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int ax = j == 0 ? 0 : 1;
    float rw[3], sn, cn;
    mat3_vec(Rp, origin + j * 3, rw);
    pp[0] += rw[0]; pp[1] += rw[1]; pp[2] += rw[2];
    pm_sincosf(q[j], &sn, &cn);
#pragma unroll
    for (int a = 0; a < 3; ++a) rE(ax, cn, sn, Rp + 3 * a, Rp + 3 * a);
  }
  float fw[3];
  mat3_vec(Rp, foot, fw);
  out[0] = pp[0] + fw[0]; out[1] = pp[1] + fw[1]; out[2] = pp[2] + fw[2];
}

// Centre (x, y) of the bounding box of the env's hips, knees and feet at the start of the
// step: the terrain patch is placed on it rather than on the base (16 x 16 cells around the
// base left ~6 % of the envs with a leg outside it, and one such lane sends its whole wave
// through the HBM fallback of every contact query).  Hardware sin / cos: only the placement
// of the patch depends on this, and the patch is a pure cache of the tile.
__device__ __forceinline__ float quad_min(float v) {
  v = fminf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, true)));
  return fminf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, true)));
}
__device__ __forceinline__ float quad_max(float v) {
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, true)));
  return fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, true)));
}
__device__ __forceinline__ void legs_bbox_centre(const float* pos, const float* quat, const float* q, int leg,
                                                 float* cx, float* cy) {
  const float sx = (leg & 2) ? -1.0f : 1.0f, sy = (leg & 1) ? -1.0f : 1.0f;
  float Rp[9], pp[3] = {pos[0], pos[1], pos[2]};
  quat_to_R(quat, Rp);
  float xmin = 1e30f, xmax = -1e30f, ymin = 1e30f, ymax = -1e30f;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    float o[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int i = 30 + 3 * j + k, sp = GO1_LEG_SIGN[i];
      o[k] = GO1_LEG_FL[i] * (sp == 0 ? 1.0f : (sp == 1 ? sx : (sp == 2 ? sy : sx * sy)));
    }
    float rw[3];
    mat3_vec(Rp, o, rw);
    pp[0] += rw[0]; pp[1] += rw[1]; pp[2] += rw[2];  // hip, thigh, calf (knee) origins
    if (j != 1) {
      xmin = fminf(xmin, pp[0]); xmax = fmaxf(xmax, pp[0]);
      ymin = fminf(ymin, pp[1]); ymax = fmaxf(ymax, pp[1]);
    }
    float sn, cn;
    __sincosf(q[j], &sn, &cn);
#pragma unroll
    for (int a = 0; a < 3; ++a) rE(j == 0 ? 0 : 1, cn, sn, Rp + 3 * a, Rp + 3 * a);
  }
  float fw[3];
  mat3_vec(Rp, GO1_MODEL_F32 + 13 * 10 + 4 * 9, fw);  // foot offset in the calf frame
  const float fx = pp[0] + fw[0], fy = pp[1] + fw[1];
  xmin = quad_min(fminf(xmin, fx)); xmax = quad_max(fmaxf(xmax, fx));
  ymin = quad_min(fminf(ymin, fy)); ymax = quad_max(fmaxf(ymax, fy));
  *cx = 0.5f * (xmin + xmax);
  *cy = 0.5f * (ymin + ymax);
}

// The config block through the constant address space: every uniform field read is a
// scalar (SMEM) load.  Through a generic pointer the compiler cannot prove that the
// kernel's stores leave the block unchanged, and emits vector loads, each a full memory
// round trip at its first use (inside the sub-step loop too).
typedef const __attribute__((address_space(4))) go1_config CCfg;

struct Phys {
  float pos[3], quat[4];  // base (replicated on the 16 lanes of the env)
  f2 wv[3];               // base angular and linear velocity (world) as (w_i, v_i) pairs
  float q[3], qd[3];                   // this lane's leg
};

// ---- the trunk box's faces against the heightfields (go1.urdf:53-58, the 0.3762 x 0.0935 x 0.114
// box; tunnel_fn.py:99-163, the ceiling's downward wedges).  The 8 box corners are contact points of the sub-step
// (above); a wedge apex or ridge that enters a face between its corners is a grid vertex of the heightfield
// inside the face's footprint (mesh triangles: a face's deepest point against them is a vertex or on the
// footprint's boundary).  Once per control step the env's 16 lanes scan the 10 x 10 vertices around the trunk
// (offsets -4 .. +5 on both axes: they hold the footprint's +-0.166 m at any yaw wherever the centre sits in its
// cell; 7 per lane, both layers in the halves: floor against the bottom face, ceiling against the top
// face) and keep, per face, the vertex inside the footprint nearest to (or deepest in) the face -- its signed
// depth, so a vertex that enters during the control step is already chosen -- compared quantised
// to 1e-5 m, ties to the lowest window position: a lexicographic maximum (associative: the same in any reduction
// order, and the oracle's).  Every sim step a penalty force acts at the two chosen vertices where they penetrate
// (face_force).  Scanning every sim step measured +3.7 k cycles per sim step per wave; the held choice is bounded
// by tests/test_held_contacts.py (held vs every sim step in the f64 oracle).
#define FACE_Q 1.0e-5f
#define FACE_W 10
__device__ __forceinline__ int face_key_max(int v) {  // max over the env's 16 lanes (quad, then the rows)
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, true));
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, true));
  auto a = __builtin_amdgcn_permlane16_swap((uint32_t)v, (uint32_t)v, false, false);
  v = max((int)a[0], (int)a[1]);
  auto b = __builtin_amdgcn_permlane32_swap((uint32_t)v, (uint32_t)v, false, false);
  return max((int)b[0], (int)b[1]);
}
#define FACE_SIGNED 0.1f  // signed depths from -0.1 m (a vertex farther from the face cannot reach it in a control step)
__device__ __forceinline__ void face_scan(const Terr& T, const float* R, const float* pos, const float* th, int sub16,
                                          int* sel) {
  const float ihs = frcp(T.hs);
  const int ci = (int)floorf(fminf(fmaxf(pos[0] * ihs, -16000.0f), 16000.0f));
  const int cj = (int)floorf(fminf(fmaxf(pos[1] * ihs, -16000.0f), 16000.0f));
  int key[2] = {-1, -1};
#pragma unroll
  for (int u = 0; u < (FACE_W * FACE_W + 15) / 16; ++u) {
    const int v = sub16 + 16 * u;
    const int i = ci + v % FACE_W - 4, j = cj + v / FACE_W - 4;
    const int li = i - T.pi0, lj = j - T.pj0;
    const bool inp = (v < FACE_W * FACE_W) & (li >= 0) & (li < PSZX) & (lj >= 0) & (lj < PSZY);
    const float2 hv = T.patch[min(max(li, 0), PSZX - 1) * PSZY + min(max(lj, 0), PSZY - 1)];
    const float dx = (float)i * T.hs - pos[0], dy = (float)j * T.hs - pos[1];
    const f2 dz = f2{hv.x, hv.y} - pos[2];
    const f2 cx = (R[0] * dx + R[3] * dy) + R[6] * dz, cy = (R[1] * dx + R[4] * dy) + R[7] * dz,
             cz = (R[2] * dx + R[5] * dy) + R[8] * dz;
    const f2 pen = f2{cz.x + th[2], th[2] - cz.y};  // floor vertex above the bottom face / ceiling below the top
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const bool in = inp & (fabsf(cx[hh]) <= th[0]) & (fabsf(cy[hh]) <= th[1]) & (pen[hh] > -FACE_SIGNED);
      const int q = (int)floorf(fminf(pen[hh] + FACE_SIGNED, 10.0f) * (1.0f / FACE_Q));  // signed depth, offset
      const int k = in ? (q << 7) | (127 - v) : -1;
      key[hh] = max(key[hh], k);
    }
  }
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const int k = face_key_max(key[hh]);
    const int v = 127 - (k & 127);
    const int i = ci + v % FACE_W - 4, j = cj + v / FACE_W - 4;
    sel[hh] = k < 0 ? -1 : ((i + 16384) << 16) | (j + 16384);
  }
}
// the penalty force of the two chosen vertices at the current pose (explicit: the trunk's 5 kg keep h sqrt(k / m)
// = 0.3 and h d / m = 0.08): normal k depth - d vn along the face normal (base frame +z on the bottom face, -z on
// the top), regularised Coulomb friction as the point contacts, nothing when the vertex left the footprint.
// Adds the base-frame wrench (angular, linear pairs) to w and the world force to Fw.
__device__ __forceinline__ void face_force(const Terr& T, const CP& C, const float* R, const float* pos, const float* vb,
                                           const float* th, const int* sel, f2* w, float* Fw) {
  f2 cx, cy, cz;
  bool ok[2];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const int i = (sel[hh] >> 16) - 16384, j = (sel[hh] & 0xffff) - 16384;
    const int li = i - T.pi0, lj = j - T.pj0;
    ok[hh] = sel[hh] >= 0 & li >= 0 & li < PSZX & lj >= 0 & lj < PSZY;
    const float2 hv = T.patch[min(max(li, 0), PSZX - 1) * PSZY + min(max(lj, 0), PSZY - 1)];
    const float dx = (float)i * T.hs - pos[0], dy = (float)j * T.hs - pos[1], dz = (hh == 0 ? hv.x : hv.y) - pos[2];
    cx[hh] = (R[0] * dx + R[3] * dy) + R[6] * dz;
    cy[hh] = (R[1] * dx + R[4] * dy) + R[7] * dz;
    cz[hh] = (R[2] * dx + R[5] * dy) + R[8] * dz;
  }
  const f2 pen = f2{cz.x + th[2], th[2] - cz.y};
  bool act[2];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) act[hh] = ok[hh] & (fabsf(cx[hh]) <= th[0]) & (fabsf(cy[hh]) <= th[1]) & (pen[hh] > 0.0f);
  if (!__any(act[0] || act[1])) return;
  const f2 nz = f2{1.0f, -1.0f};
  // the trunk's velocity at the vertex, base frame: v + w x c
  const f2 vx = vb[3] + (vb[1] * cz - vb[2] * cy), vy = vb[4] + (vb[2] * cx - vb[0] * cz), vz = vb[5] + (vb[0] * cy - vb[1] * cx);
  const f2 depth = f2{fminf(pen.x, 2.0f * th[2]), fminf(pen.y, 2.0f * th[2])};
  const f2 vn = vz * nz;
  const f2 fn = C.k * depth - C.d * vn;
  const f2 vt2 = vx * vx + vy * vy;
  const f2 ivt = f2{frsq(fmaxf(vt2.x, 1e-18f)), frsq(fmaxf(vt2.y, 1e-18f))};
  const f2 vtn = vt2 * ivt, cm = C.mu * fn;
  const f2 ct = f2{(C.kf * vtn.x > cm.x & vtn.x > 1e-9f) ? cm.x * ivt.x : C.kf,
                   (C.kf * vtn.y > cm.y & vtn.y > 1e-9f) ? cm.y * ivt.y : C.kf};
  const bool ax = act[0] & (fn.x > 0.0f), ay = act[1] & (fn.y > 0.0f);
  const f2 fa = f2{ax ? fn.x : 0.0f, ay ? fn.y : 0.0f}, sc = f2{ax ? ct.x : 0.0f, ay ? ct.y : 0.0f};
  const f2 Fx = -(sc * vx), Fy = -(sc * vy), Fz = fa * nz;
  const f2 mx = cy * Fz - cz * Fy, my = cz * Fx - cx * Fz, mz = cx * Fy - cy * Fx;
  w[0] += f2{mx.x + mx.y, Fx.x + Fx.y};
  w[1] += f2{my.x + my.y, Fy.x + Fy.y};
  w[2] += f2{mz.x + mz.y, Fz.x + Fz.y};
  const float F[3] = {Fx.x + Fx.y, Fy.x + Fy.y, Fz.x + Fz.y};
#pragma unroll
  for (int i = 0; i < 3; ++i) Fw[i] += R[3 * i] * F[0] + R[3 * i + 1] * F[1] + R[3 * i + 2] * F[2];
}

// sum over the 4 roles of a leg (the four 16-lane rows), bitwise identical on every lane
__device__ __forceinline__ float rsum(float v) { return rowsum4(v); }

// ---- self-collision (asset.self_collisions == 0, go1_crawling.py:44: Isaac Gym collides every pair of bodies no
// joint connects; oracle/go1_oracle.c phys_substep).  Round 6: the links as capsules over their full length
// (the sphere chains of rounds 3-5 had 46-55 mm holes).  Primitive 4 leg + k, owned by the lane of role
// k: 0 thigh capsule (thigh joint .. knee), 1 hip capsule, 2 calf capsule (knee .. foot), 3 foot sphere.  Pairs:
// every primitive of leg la against every primitive of leg lb (16 per leg pair); within a leg the links two joints
// apart (hip vs calf and foot, thigh vs foot); the thigh and calf capsules and the foot against the trunk box (the
// hip is the trunk's neighbour).  A pair acts at the closest points of its two segments as two spheres of the
// capsules' radii there (seg_closest), a capsule against the box at its point nearest the box (seg_box_t).
// Explicit penalty springs on the overlap, fn = ks pen - ds vn (compressive only), no friction, no added mass (the
// bodies sit in different ABA chains, or two joints apart).
// Broad phase in registers: each lane bounds its leg (thigh joint, knee, foot, hip-capsule ends, grown by their
// radii) by an AABB in the trunk frame, swaps the four legs' boxes over the quad (DPP) and tests the six leg pairs,
// the trunk box and the leg's own folded links; a wave whose envs have no candidate is done.  Otherwise, per env in
// LDS: the 16 primitives as (P0, r), (P1, 0), (V0, 0), (V1, 0) (segment ends and their velocities, world), and each
// lane sums the forces on its own primitive from its candidate partners (self_narrow).
#define SELF_ENV_FLOATS (16 * 16 + 4 + 32)
#define FACE_SEL_OFF (16 * 16)  // then the trunk faces' two vertices of the control step (face_scan)
#define SEG_T_OFF (16 * 16 + 4)  // then the capsules' deepest-point parameters of the control step, (x, y) per lane

// the lane's own primitive into this env's LDS scratch; rb: the radius of its bounding sphere about the segment's middle
// (half the segment plus r), for the narrow phase's first test
__device__ __forceinline__ void self_put(float* sc, int leg, int role, const float* P0, const float* P1, float r,
                                         float rb, const float* V0, const float* V1) {
  float4* Q = reinterpret_cast<float4*>(sc) + 4 * (4 * leg + role);
  Q[0] = make_float4(P0[0], P0[1], P0[2], r);
  Q[1] = make_float4(P1[0], P1[1], P1[2], rb);
  Q[2] = make_float4(V0[0], V0[1], V0[2], 0.0f);
  Q[3] = make_float4(V1[0], V1[1], V1[2], 0.0f);
}

// closest points of the segments P0 + s d1 and Q0 + t d2 (s, t in [0, 1]; a = |d1|^2, e = |d2|^2; a point has a
// or e = 0): Ericson's clamped construction, branch-free (oracle/go1_oracle.c seg_seg_closest), the lines' s formed
// without cancellation as (n . (d2 x r)) / (n . n), n = d1 x d2 (for nearly parallel links a e - b^2 cancels to a few
// ulps and would place the closest points anywhere along them)
__device__ __forceinline__ void seg_closest(const float* P0, const float* d1, const float* Q0, const float* d2,
                                            float& s, float& t) {
  const float r[3] = {P0[0] - Q0[0], P0[1] - Q0[1], P0[2] - Q0[2]};
  const float a = d1[0] * d1[0] + d1[1] * d1[1] + d1[2] * d1[2], e = d2[0] * d2[0] + d2[1] * d2[1] + d2[2] * d2[2];
  const float b = d1[0] * d2[0] + d1[1] * d2[1] + d1[2] * d2[2];
  const float c = d1[0] * r[0] + d1[1] * r[1] + d1[2] * r[2], f = d2[0] * r[0] + d2[1] * r[1] + d2[2] * r[2];
  float n[3], m[3];
  cross3(d1, d2, n);
  cross3(d2, r, m);
  const float den = n[0] * n[0] + n[1] * n[1] + n[2] * n[2], num = n[0] * m[0] + n[1] * m[1] + n[2] * m[2];
  const bool pa = a > 1e-12f, pe = e > 1e-12f;
  const float ia = pa ? frcp(a) : 0.0f, ie = pe ? frcp(e) : 0.0f;
  // every candidate computed, then selected (v_med3 clamps): as ternaries around the clamps the compiler had
  // made exec-mask branches of them, one wave paying each arm plus the hazard nops
  const float s0 = den > 1e-10f * a * e ? __builtin_amdgcn_fmed3f(num * frcp(den), 0.0f, 1.0f) : 0.0f;
  const float tt = (b * s0 + f) * ie;
  const float s_lo = __builtin_amdgcn_fmed3f(-c * ia, 0.0f, 1.0f), s_hi = __builtin_amdgcn_fmed3f((b - c) * ia, 0.0f, 1.0f);
  const float ss = tt < 0.0f ? s_lo : (tt > 1.0f ? s_hi : s0);
  const float t_pt = __builtin_amdgcn_fmed3f(f * ie, 0.0f, 1.0f);
  s = !pa ? 0.0f : (!pe ? s_lo : ss);
  t = !pe ? 0.0f : (!pa ? t_pt : __builtin_amdgcn_fmed3f(tt, 0.0f, 1.0f));
}

// the point of the segment P0 -> P1 (world) nearest the trunk box, deepest inside it: bisection on the sign of the
// derivative of the box's signed distance along the segment (convex), SEG_BISECT halvings (oracle/go1_oracle.c
// seg_box_t, which explains the sign); no square roots, and every midpoint an exact binary fraction
#define SEG_BISECT 20
__device__ __forceinline__ float seg_box_t(const float* P0, const float* P1, const float* R, const float* pos,
                                           const float* th) {
  float a0[3], d[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    a0[i] = R[i] * (P0[0] - pos[0]) + R[3 + i] * (P0[1] - pos[1]) + R[6 + i] * (P0[2] - pos[2]);
    d[i] = R[i] * (P1[0] - P0[0]) + R[3 + i] * (P1[1] - P0[1]) + R[6 + i] * (P1[2] - P0[2]);
  }
  float lo = 0.0f, hi = 1.0f;
#pragma unroll
  for (int it = 0; it < SEG_BISECT; ++it) {
    const float m = 0.5f * (lo + hi);
    float so = 0.0f, qmax = -1e30f, sin = 0.0f;
    bool out = false;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const float c = a0[i] + m * d[i], sd = c >= 0.0f ? d[i] : -d[i], q = fabsf(c) - th[i];
      so += q > 0.0f ? q * sd : 0.0f;
      out = out || q > 0.0f;
      sin = q > qmax ? sd : sin;
      qmax = fmaxf(qmax, q);
    }
    const float sl = out ? so : sin;
    lo = sl < 0.0f ? m : lo;
    hi = sl < 0.0f ? hi : m;
  }
  return 0.5f * (lo + hi);
}

// The force of a pair on one of its primitives: the pair is evaluated in its canonical order (A = the lower primitive
// index), spheres of the two radii at the closest points s (on A), t (on B); the force on A, or its negative on B
// (own_first false), and the own primitive's point (world).  A, B: (P0 r, P1, V0, V1) records in LDS, so the two
// lanes of a pair compute the same bits and apply exactly opposite forces.
__device__ __forceinline__ void self_pair_force(const float4* A, const float4* B, bool own_first, float ks, float ds,
                                                float* F, float* pown, bool& touch) {
  const float4 a0 = A[0], a1 = A[1], b0 = B[0], b1 = B[1];
  const float pa0[3] = {a0.x, a0.y, a0.z}, da[3] = {a1.x - a0.x, a1.y - a0.y, a1.z - a0.z};
  const float pb0[3] = {b0.x, b0.y, b0.z}, db[3] = {b1.x - b0.x, b1.y - b0.y, b1.z - b0.z};
  float s, t;
  seg_closest(pa0, da, pb0, db, s, t);
  const float pa[3] = {pa0[0] + s * da[0], pa0[1] + s * da[1], pa0[2] + s * da[2]};
  const float pb[3] = {pb0[0] + t * db[0], pb0[1] + t * db[1], pb0[2] + t * db[2]};
  const float d0 = pa[0] - pb[0], d1 = pa[1] - pb[1], d2 = pa[2] - pb[2];
  const float dd = d0 * d0 + d1 * d1 + d2 * d2, rs = a0.w + b0.w;
#pragma unroll
  for (int i = 0; i < 3; ++i) { pown[i] = own_first ? pa[i] : pb[i]; F[i] = 0.0f; }
  touch = dd < rs * rs;
  // the spring only where some lane of the wave has an overlap (most pairs the boxes let through do not touch; a
  // pair that does not has no force, so skipping it changes nothing)
  if (!__any(touch)) return;
  const float inv = dd > 1e-18f ? frsq(dd) : 0.0f;
  const float n0 = dd > 1e-18f ? d0 * inv : 0.0f, n1 = dd > 1e-18f ? d1 * inv : 0.0f, n2 = dd > 1e-18f ? d2 * inv : 1.0f;
  const float pen = rs - dd * inv;
  const float4 va0 = A[2], va1 = A[3], vb0 = B[2], vb1 = B[3];
  const float vr0 = (va0.x + s * (va1.x - va0.x)) - (vb0.x + t * (vb1.x - vb0.x));
  const float vr1 = (va0.y + s * (va1.y - va0.y)) - (vb0.y + t * (vb1.y - vb0.y));
  const float vr2 = (va0.z + s * (va1.z - va0.z)) - (vb0.z + t * (vb1.z - vb0.z));
  const float vn = vr0 * n0 + vr1 * n1 + vr2 * n2;
  float fn = ks * pen - ds * vn;
  fn = (touch & (fn > 0.0f)) ? fn : 0.0f;
  fn = own_first ? fn : -fn;
  F[0] = fn * n0; F[1] = fn * n1; F[2] = fn * n2;
}

// sphere A (centre, radius in w) against the trunk box (half extents th about the base origin): the force on A (world)
// added to F and the trunk's reaction wrench (base frame, (moment, force) about the base origin) added to wb
__device__ __forceinline__ void self_box_force(const float4 A, const float4 Av, const float* R, const float* pos,
                                               const float* vb, const float* th, float ks, float ds, float* F,
                                               float* wb) {
  const float w0 = A.x - pos[0], w1 = A.y - pos[1], w2 = A.z - pos[2];
  float c[3], q[3], d[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) c[i] = R[i] * w0 + R[3 + i] * w1 + R[6 + i] * w2;
#pragma unroll
  for (int i = 0; i < 3; ++i) { q[i] = fminf(fmaxf(c[i], -th[i]), th[i]); d[i] = c[i] - q[i]; }
  const float dd = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
  float nb[3], pen;
  if (dd > 0.0f) {
    const float inv = frsq(dd);
#pragma unroll
    for (int i = 0; i < 3; ++i) nb[i] = d[i] * inv;
    pen = A.w - dd * inv;
  } else {  // centre inside: out through the nearest face (lowest axis on ties), the depths compared quantised
    // to 0.1 mm (oracle BOX_Q): a segment's deepest point inside the box often has two faces equally near
    const float m0 = th[0] - fabsf(c[0]), m1 = th[1] - fabsf(c[1]), m2 = th[2] - fabsf(c[2]);
    const int q0 = (int)floorf(fminf(fmaxf(m0, -1.0f), 1.0f) * 1.0e4f), q1 = (int)floorf(fminf(fmaxf(m1, -1.0f), 1.0f) * 1.0e4f),
              q2 = (int)floorf(fminf(fmaxf(m2, -1.0f), 1.0f) * 1.0e4f);
    const int ax = ((q0 <= q1) & (q0 <= q2)) ? 0 : (q1 <= q2 ? 1 : 2);
    const float sg = c[ax] >= 0.0f ? 1.0f : -1.0f;
#pragma unroll
    for (int i = 0; i < 3; ++i) nb[i] = i == ax ? sg : 0.0f;
    q[ax] = sg * th[ax];
    pen = A.w + (ax == 0 ? m0 : (ax == 1 ? m1 : m2));
  }
  // the trunk's velocity at q (base frame v + w x q), relative normal velocity in the base frame
  const float vq0 = vb[3] + (vb[1] * q[2] - vb[2] * q[1]);
  const float vq1 = vb[4] + (vb[2] * q[0] - vb[0] * q[2]);
  const float vq2 = vb[5] + (vb[0] * q[1] - vb[1] * q[0]);
  float va[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) va[i] = R[i] * Av.x + R[3 + i] * Av.y + R[6 + i] * Av.z;
  const float vn = (va[0] - vq0) * nb[0] + (va[1] - vq1) * nb[1] + (va[2] - vq2) * nb[2];
  float fn = ks * pen - ds * vn;
  fn = ((dd < A.w * A.w) & (fn > 0.0f)) ? fn : 0.0f;
#pragma unroll
  for (int i = 0; i < 3; ++i) F[i] += fn * (R[3 * i] * nb[0] + R[3 * i + 1] * nb[1] + R[3 * i + 2] * nb[2]);
  const float f0 = -fn * nb[0], f1 = -fn * nb[1], f2v = -fn * nb[2];
  wb[0] += q[1] * f2v - q[2] * f1;
  wb[1] += q[2] * f0 - q[0] * f2v;
  wb[2] += q[0] * f1 - q[1] * f0;
  wb[3] += f0; wb[4] += f1; wb[5] += f2v;
}

template <int D>
__device__ __forceinline__ float quad_xor(float v) {  // the value of lane ^ D within the quad (DPP quad_perm)
  constexpr int c = D == 1 ? 0xB1 : (D == 2 ? 0x4E : 0x1B);
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), c, 0xF, 0xF, true));
}
__device__ __forceinline__ int quad_or(int v) {
  v |= __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, true);
  return v | __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, true);
}

// leg pairs lp: (0,1) = 0, (0,2) = 1, (0,3) = 2, (1,2) = 3, (1,3) = 4, (2,3) = 5

// Narrow phase (a wave whose broad phase found a candidate).  sc: this env's LDS scratch, the primitives already
// written (self_put).  Each lane sums the forces on its own primitive from its candidate partners: per candidate
// partner leg (a per-lane list walked with ctz: the loop runs as often as the lane with the most candidates needs),
// the leg's four primitives (the own leg's two-joints-apart ones for d = 0), each pair evaluated in its canonical
// order (the lower primitive index first), so the two lanes of a pair compute the same bits and apply exactly
// opposite forces, every sum in a fixed order.  Then the trunk box for a folded leg.  Output: the world force Fo on
// the own primitive and its moment Mo about the own body's origin pb; wb: the trunk reaction of the lane's box
// contact (base frame).
__device__ __forceinline__ void self_narrow(CCfg* __restrict__ cfg, float* sc, int leg, int role, int mask,
                                           const float* R, const float* pos, const float* vb, const float* th,
                                           const float* pb, float* Fo, float* Mo, float* wb) {
  const float ks = cfg->self_stiffness, ds = cfg->self_damping;
  const float4* Pr = reinterpret_cast<const float4*>(sc);
  const int io = 4 * leg + role;
  const int lp1 = (leg >> 1) ? 5 : 0, lp2 = (leg & 1) ? 4 : 1, lp3 = (leg == 0 || leg == 3) ? 2 : 3;
  // candidate partner legs, bit d: leg ^ d (d = 0: the own leg's links two joints apart, when folded)
  unsigned cand = ((mask >> (10 + leg)) & 1) | (((mask >> lp1) & 1) << 1) | (((mask >> lp2) & 1) << 2) |
                  (((mask >> lp3) & 1) << 3);
  // the own leg's partners of primitive `role`: thigh - foot, hip - calf / foot, calf - hip, foot - thigh / hip
  const unsigned keep_same = (0x32C8u >> (4 * role)) & 0xFu;  // role 0: 0x8, 1: 0xC, 2: 0x2, 3: 0x3
  auto acc = [&](const float* p, const float* F) {  // force F (world) on the own primitive at p
    const float p0 = p[0] - pb[0], p1 = p[1] - pb[1], p2 = p[2] - pb[2];
    Fo[0] += F[0]; Fo[1] += F[1]; Fo[2] += F[2];
    Mo[0] += p1 * F[2] - p2 * F[1];
    Mo[1] += p2 * F[0] - p0 * F[2];
    Mo[2] += p0 * F[1] - p1 * F[0];
  };
  // first the bounding boxes (the segment's ends grown by the radius, world axes) of the candidate legs' primitives,
  // all four partners' loads in one LDS round trip, into a per-lane work list (bit 4 d + m: primitive m of leg ^ d);
  // then the pairs of the list -- both loops run as often as the busiest lane needs
  unsigned work = 0u;
  {
    const float4 O0 = Pr[4 * io], O1 = Pr[4 * io + 1];
    const float olx = fminf(O0.x, O1.x) - O0.w, ohx = fmaxf(O0.x, O1.x) + O0.w;
    const float oly = fminf(O0.y, O1.y) - O0.w, ohy = fmaxf(O0.y, O1.y) + O0.w;
    const float olz = fminf(O0.z, O1.z) - O0.w, ohz = fmaxf(O0.z, O1.z) + O0.w;
#ifdef GO1_ABL_NO_TESTLOOP  // ablation build only: no partner tests (and so no pairs)
    cand = 0u;
#endif
#ifdef GO1_ABL_RT_NO_TESTLOOP  // ablation build only: the same, decided at run time (the code stays)
    cand = cfg->self_stiffness > 1e30f ? cand : 0u;
#endif
    while (__any(cand != 0u)) {
      const bool act = cand != 0u;
      const int d = act ? __builtin_ctz(cand) : 0;
      cand &= cand - 1u;
      const unsigned keep = !act ? 0u : (d == 0 ? keep_same : 0xFu);
      const float4* Q = Pr + 16 * (leg ^ d);
      float4 B0[4], B1[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) { B0[m] = Q[4 * m]; B1[m] = Q[4 * m + 1]; }
      __builtin_amdgcn_sched_barrier(0);
      unsigned bits = 0u;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const float r = B0[m].w;
        const bool ox = (fminf(B0[m].x, B1[m].x) - r <= ohx) & (olx <= fmaxf(B0[m].x, B1[m].x) + r);
        const bool oy = (fminf(B0[m].y, B1[m].y) - r <= ohy) & (oly <= fmaxf(B0[m].y, B1[m].y) + r);
        const bool oz = (fminf(B0[m].z, B1[m].z) - r <= ohz) & (olz <= fmaxf(B0[m].z, B1[m].z) + r);
        bits |= (ox & oy & oz) ? 1u << m : 0u;
      }
      work |= (bits & keep) << (4 * d);
    }
  }
  MARK(self_tests_done);
#ifdef GO1_ABL_NO_PAIRLOOP  // ablation build only: the pairs tested but never evaluated
  work = 0u;
#endif
#ifdef GO1_ABL_RT_NO_PAIRLOOP  // ablation build only: the same, decided at run time (the code stays)
  work = cfg->self_stiffness > 1e30f ? work : 0u;
#endif
  while (__any(work != 0u)) {
    const bool act = work != 0u;
    const int bit = act ? __builtin_ctz(work) : 0;
    work &= work - 1u;
    const int ip = 4 * (leg ^ (bit >> 2)) + (bit & 3);
    const bool first = io < ip;
    float F[3], p[3];
    bool touch;
    self_pair_force(Pr + 4 * min(io, ip), Pr + 4 * max(io, ip), first, ks, ds, F, p, touch);
    if (__any(act & touch)) {
      const float Fw[3] = {act ? F[0] : 0.0f, act ? F[1] : 0.0f, act ? F[2] : 0.0f};
      acc(p, Fw);
    }
  }
  MARK(self_pairs_done);
  // the trunk box, for a folded leg's thigh, calf and foot (the hip is the trunk's neighbour) whose segment's
  // trunk-frame AABB, grown by its radius, meets the box (the fold gate is coarse: most folded links are far from
  // the trunk, and a link that misses the grown box has no force -- skipping it changes nothing)
  const float4 O0 = Pr[4 * io], O1 = Pr[4 * io + 1];
#ifdef GO1_ABL_NO_BOXPHASE  // ablation build only: no capsule-box pairs
  bool on = false;
#else
  bool on = ((mask >> (6 + leg)) & 1) & (role != 1);
#endif
  {
    const float w0[3] = {O0.x - pos[0], O0.y - pos[1], O0.z - pos[2]}, w1[3] = {O1.x - pos[0], O1.y - pos[1], O1.z - pos[2]};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const float c0 = R[i] * w0[0] + R[3 + i] * w0[1] + R[6 + i] * w0[2];
      const float c1 = R[i] * w1[0] + R[3 + i] * w1[1] + R[6 + i] * w1[2];
      on = on & (fminf(c0, c1) - O0.w <= th[i]) & (fmaxf(c0, c1) + O0.w >= -th[i]);  // (&: && branches)
    }
  }
  if (__any(on)) {
    const float4 O2 = Pr[4 * io + 2], O3 = Pr[4 * io + 3];
    const float P0[3] = {O0.x, O0.y, O0.z}, P1[3] = {O1.x, O1.y, O1.z};
    const float u = role == 3 ? 0.0f : seg_box_t(P0, P1, R, pos, th);
    const float4 C = make_float4(O0.x + u * (O1.x - O0.x), O0.y + u * (O1.y - O0.y), O0.z + u * (O1.z - O0.z), O0.w);
    const float4 Cv = make_float4(O2.x + u * (O3.x - O2.x), O2.y + u * (O3.y - O2.y), O2.z + u * (O3.z - O2.z), 0.0f);
    float F[3] = {0.0f, 0.0f, 0.0f}, w6[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    self_box_force(C, Cv, R, pos, vb, th, ks, ds, F, w6);
#pragma unroll
    for (int i = 0; i < 6; ++i) wb[i] += on ? w6[i] : 0.0f;
    const float Fb[3] = {on ? F[0] : 0.0f, on ? F[1] : 0.0f, on ? F[2] : 0.0f};
    const float pc[3] = {C.x, C.y, C.z};
    acc(pc, Fb);
  }
  MARK(self_box_done);
}

// Broad phase, in registers, in the trunk frame (where the legs keep their places whatever the trunk's
// pose; world-axis boxes of a yawed trunk overlap every leg): bit lp of the result = leg pair lp's boxes overlap,
// bits 6 + leg and 10 + leg = the leg is folded past its joint band (its trunk-box and same-leg pairs are
// tested); the pair bits on the env's 16 lanes.  pth, pkn, pft: the thigh joint, knee and foot (world); hc0, hc1:
// the hip capsule's ends in the trunk frame; q: the leg's joints.
__device__ __forceinline__ int self_broad(int leg, const float* pth, const float* pkn, const float* pft, float rmax,
                                          const float* hc0, const float* hc1, float rhip,
                                          const float* R, const float* pos, const float* th, const float* q) {
  float b[3][3];  // the three points in the trunk frame, R^T (p - pos)
  const float* pts[3] = {pth, pkn, pft};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float w0 = pts[k][0] - pos[0], w1 = pts[k][1] - pos[1], w2 = pts[k][2] - pos[2];
#pragma unroll
    for (int i = 0; i < 3; ++i) b[k][i] = R[i] * w0 + R[3 + i] * w1 + R[6 + i] * w2;
  }
  // (bitwise &, |: short-circuit operators around the convergent DPP moves compile to exec-mask branches)
  bool o1 = true, o2 = true, o3 = true;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float clo = fminf(b[1][i], b[2][i]) - rmax, chi = fmaxf(b[1][i], b[2][i]) + rmax;  // knee .. foot
    const float tlo = fminf(b[0][i], clo), thi = fmaxf(b[0][i], chi);                       // + the thigh joint
    const float hlo = fminf(hc0[i], hc1[i]) - rhip, hhi = fmaxf(hc0[i], hc1[i]) + rhip;     // the hip capsule
    const float lo = fminf(tlo, hlo), hi = fmaxf(thi, hhi);
    const float lo1 = quad_xor<1>(lo), hi1 = quad_xor<1>(hi), lo2 = quad_xor<2>(lo), hi2 = quad_xor<2>(hi);
    const float lo3 = quad_xor<3>(lo), hi3 = quad_xor<3>(hi);
    o1 = o1 & (lo <= hi1) & (lo1 <= hi);
    o2 = o2 & (lo <= hi2) & (lo2 <= hi);
    o3 = o3 & (lo <= hi3) & (lo3 <= hi);
  }
  // the leg's own links two joints apart and the trunk box: out of reach while every joint of the leg is within
  // 0.1 rad of its URDF range (inside the band the capsules keep 8.6 mm same-leg and 14.8 mm box clearance;
  // tests/test_self_collision.py::test_fold_gate_is_sound), so only a leg outside that band goes to the narrow
  // phase for them (no branch here: the broad phase shares a basic block with the terrain contacts)
  const bool wild = (fabsf(q[0]) > 0.9029f) | (q[1] < -1.1472f) | (q[1] > 4.2888f) | (q[2] < -2.7966f) |
                    (q[2] > -0.8163f);
  const int fold = wild ? ((64 << leg) | (1024 << leg)) : 0;  // the narrow phase tests them exactly
  const int lp1 = (leg >> 1) ? 5 : 0;                         // (0,1) / (2,3)
  const int lp2 = (leg & 1) ? 4 : 1;                          // (0,2) / (1,3)
  const int lp3 = (leg == 0 || leg == 3) ? 2 : 3;             // (0,3) / (1,2)
  const int mask = (o1 ? 1 << lp1 : 0) | (o2 ? 1 << lp2 : 0) | (o3 ? 1 << lp3 : 0) | fold;
  return quad_or(mask);
}

// One integrator step of length h for the env of this lane.  Lane layout (16 per env): lane = 16 role + 4 env +
// leg.  The four roles of a leg compute the leg's kinematics and ABA passes redundantly (base quantities on all 16
// lanes), and split the leg's contact geometry two per lane (x, y halves of f2), each a capsule segment acting at
// its deepest point (seg_deepest2; a point is a degenerate segment):
//   role 0: thigh half at the thigh joint, thigh half at the knee   (body: thigh, thigh)
//   role 1: hip capsule, trunk corner 2 leg                          (body: hip, trunk)
//   role 2: calf half at the knee, calf half at the foot             (body: calf, calf)
//   role 3: foot sphere, trunk corner 2 leg + 1                      (body: calf, trunk)
// so each wave has four envs and the whole grid fills every SIMD.  The lane's self-collision primitive is its x
// half's link (thigh, hip, calf, foot).
// cf_raw: this lane's reported contact forces (x half with the own primitive's self-contact force, y half, the
// trunk's self-collision reaction of the lane's box contact and, on one lane, the trunk faces').
__device__ __forceinline__ void phys_substep(CCfg* __restrict__ cfg, const float* lds, Phys& S, const float* tau,
                                             float h, const float* g, float friction, float restitution,
                                             float payload, const Terr& T, int leg, int role, bool cf_out,
                                             float* cf_raw, float* self_sc, bool face_scan_now) {
#pragma clang fp contract(on)
  // Model constants are compile-time literals (go1_model_consts.h, checked against the
  // model block by go1_create): no LDS reads or waits for them inside the sub-step loop.
  // Per-leg floats are the FL values times the leg's mirror signs (loop-invariant products).
  (void)lds;
  const float* model = GO1_MODEL_F32;
  const float msx = (leg & 2) ? -1.0f : 1.0f, msy = (leg & 1) ? -1.0f : 1.0f, msxy = msx * msy;
  float LC[39];
#pragma unroll
  for (int i = 0; i < 39; ++i) {
    const int p = GO1_LEG_SIGN[i];
    LC[i] = p == 0 ? GO1_LEG_FL[i] : GO1_LEG_FL[i] * (p == 1 ? msx : (p == 2 ? msy : msxy));
  }
  MARK(phys_begin);
  const CP C = {cfg->contact_stiffness, cfg->contact_damping, cfg->friction_damping, friction,
                0.5f * (restitution + cfg->terrain_restitution), cfg->bounce_threshold};
  float R[9];
  quat_to_R(S.quat, R);
  f2 vbp[3];  // base-frame (angular, linear) velocity pairs: R^T on both halves at once
#pragma unroll
  for (int i = 0; i < 3; ++i) vbp[i] = R[i] * S.wv[0] + R[3 + i] * S.wv[1] + R[6 + i] * S.wv[2];
  const float vb[6] = {vbp[0].x, vbp[1].x, vbp[2].x, vbp[0].y, vbp[1].y, vbp[2].y};
  const float* th = model + 13 * 10 + 4 * 9 + 3 + 1;  // trunk half extents
#ifndef GO1_ABL_NO_FACES
  // the trunk faces' vertices of the control step (face_scan), chosen here where few values are live yet (wave-uniform
  // condition); one lane stores them for every sim step's face_force below (the same on the env's 16 lanes)
  if (T.patch && face_scan_now) {
    int sel[2];
    face_scan(T, R, S.pos, th, 4 * role + leg, sel);
    if (role == 0 && leg == 0) {
      int* fsel = reinterpret_cast<int*>(self_sc + FACE_SEL_OFF);
      fsel[0] = sel[0];
      fsel[1] = sel[1];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the env's other lanes read them (face_force)
  }
#endif
  // ---- this leg: kinematics, rigid bias forces and gravity (hip -> calf)
  const float* origin = LC + 30;
  const float* foot = model + 13 * 10 + 4 * 9;
  const float foot_r = foot[3];
  const float thigh_r = model[13 * 10 + 4 * 9 + 3 + 1 + 3];
  const float calf_r = model[13 * 10 + 4 * 9 + 3 + 1 + 3 + 1];
  const float hip_r = model[13 * 10 + 4 * 9 + 3 + 1 + 3 + 2];
  const float hip_y0 = model[13 * 10 + 4 * 9 + 3 + 1 + 3 + 3], hip_y1 = model[13 * 10 + 4 * 9 + 3 + 1 + 3 + 4];
  float cs[3][2];
  // the lane's two bodies (x, y halves of the contact pass), selected as the chain passes them: x half thigh (role
  // 0), hip (1), calf (2, 3); y half thigh (0), calf (2), trunk (odd rows)
  const bool even = (role & 1) == 0;
  f2 Rs[9], ps[3], vs[6];
#pragma unroll
  for (int i = 0; i < 9; ++i) Rs[i] = f2{0.0f, R[i]};
#pragma unroll
  for (int i = 0; i < 3; ++i) { ps[i] = f2{0.0f, S.pos[i]}; vs[i] = f2{0.0f, vb[i]}; vs[3 + i] = f2{0.0f, vb[3 + i]}; }
  float pth[3], pkn[3], pft[3];  // the thigh joint, the knee and the foot centre (world), for the broad phase
  f2 cjp[3][3], pAp[3][3];  // c_j and the articulated bias force as (angular, linear) pairs
  {
    // link frame: rows 0 and 1 of the rotation as pairs over the column (row0_k, row1_k)
    f2 R01[3], pp01 = f2{S.pos[0], S.pos[1]};
    float R2[3], pp2 = S.pos[2];
    f2 vp[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) { R01[k] = f2{R[k], R[3 + k]}; R2[k] = R[6 + k]; }
#pragma unroll
    for (int i = 0; i < 3; ++i) vp[i] = vbp[i];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int ax = j == 0 ? 0 : 1;
      const float* r = origin + j * 3;
      float sn, cn;
      hw_sincosf(S.q[j], &sn, &cn);
      cs[j][0] = cn; cs[j][1] = sn;
      f2 vj[3];
      xm2(ax, cn, sn, offset_mask(j), r, vp, vj);
      vj[ax].x += S.qd[j];
      // c_j = v_j x (S qd), S = unit axis ax: pair ax is exactly zero and never read
      {
        const float qdj = S.qd[j];
        const int p1 = (ax + 1) % 3, p2 = (ax + 2) % 3;  // (w x e_ax)_p1 = w_p2, (.)_p2 = -w_p1
        cjp[j][ax] = f2{0.0f, 0.0f};
        cjp[j][p1] = vj[p2] * qdj;
        cjp[j][p2] = -(vj[p1] * qdj);
      }
#pragma unroll
      for (int k = 0; k < 3; ++k)  // pp += Rp r over the components r may have
        if ((offset_mask(j) >> k) & 1) { pp01 += R01[k] * r[k]; pp2 += R2[k] * r[k]; }
      rE2(ax, cn, sn, R01, R01);
      rE(ax, cn, sn, R2, R2);
      // rigid bias force v x* I v about the link origin (gravity: a base acceleration, below)
      rigid_bias2(LC + 10 * j, vj, pAp[j]);
      const bool sx = j == 0 ? role == 1 : (j == 1 ? role == 0 : role >= 2);  // this link is the x half's
      const bool sy = j == 1 ? role == 0 : (j == 2 ? role == 2 : false);      // ... the y half's
      if (j > 0) {
        (j == 1 ? pth : pkn)[0] = pp01.x; (j == 1 ? pth : pkn)[1] = pp01.y; (j == 1 ? pth : pkn)[2] = pp2;
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float lr[3] = {R01[k].x, R01[k].y, R2[k]};  // column k of the link rotation
#pragma unroll
        for (int row = 0; row < 3; ++row) {
          Rs[3 * row + k].x = sx ? lr[row] : Rs[3 * row + k].x;
          Rs[3 * row + k].y = sy ? lr[row] : Rs[3 * row + k].y;
        }
      }
      const float pv[3] = {pp01.x, pp01.y, pp2};
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        ps[i].x = sx ? pv[i] : ps[i].x;
        ps[i].y = sy ? pv[i] : ps[i].y;
        vs[i].x = sx ? vj[i].x : vs[i].x;
        vs[i].y = sy ? vj[i].x : vs[i].y;
        vs[3 + i].x = sx ? vj[i].y : vs[3 + i].x;
        vs[3 + i].y = sy ? vj[i].y : vs[3 + i].y;
      }
      if (j == 2) {  // the foot centre (world), for the broad phase
        pft[0] = pp01.x + R01[0].x * foot[0] + R01[1].x * foot[1] + R01[2].x * foot[2];
        pft[1] = pp01.y + R01[0].y * foot[0] + R01[1].y * foot[1] + R01[2].y * foot[2];
        pft[2] = pp2 + R2[0] * foot[0] + R2[1] * foot[1] + R2[2] * foot[2];
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) vp[i] = vj[i];
    }
  }
  MARK(leg_kin_done);
  // ---- contacts: the lane's two segments (x, y halves) in the body frame of their link, their deepest points
  //      against the heightfields, the explicit force there and the added mass of the implicit contact
  // per lane: the body-frame wrench of the x half's link (thigh, hip or calf) and of the even rows' y half (the
  // same link), the trunk's share (odd rows' y halves, the box reactions)
  float fx[6], fy[6], fbase[6];
  f2 Fpt[3];          // world forces of the lane's two contact points
  float Fo[3] = {0.0f, 0.0f, 0.0f};  // the own primitive's self-contact force (world)
  float Fbs[3] = {0.0f, 0.0f, 0.0f};  // world reaction force on the trunk of the lane's self-collision box contact
  SIP cin[2];
#ifndef GO1_ABL_NO_CONTACT
  {
    f2 lpA[3], lpB[3], rr;
    {
      // segment ends in the link frame: halves walked from their outer ends (a link lying flat is carried at both)
      const float* kn = origin + 6;  // the knee: the calf joint's origin in the thigh frame
      const int cA = leg * 2, cB = leg * 2 + 1;  // this leg's trunk corners (roles 1, 3)
      const float crn[2][3] = {{(cA & 1) ? th[0] : -th[0], (cA & 2) ? th[1] : -th[1], (cA & 4) ? th[2] : -th[2]},
                               {(cB & 1) ? th[0] : -th[0], (cB & 2) ? th[1] : -th[1], (cB & 4) ? th[2] : -th[2]}};
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const float hyA = i == 1 ? msy * hip_y0 : 0.0f, hyB = i == 1 ? msy * hip_y1 : 0.0f;
        // (sel4: bit-test selects; equality chains on role compile to divergent branches)
        const float xa = sel4(role, 0.0f, hyA, 0.0f, foot[i]);
        const float xb = sel4(role, 0.5f * kn[i], hyB, 0.5f * foot[i], foot[i]);
        const float ya = sel4(role, kn[i], crn[0][i], foot[i], crn[1][i]);
        const float yb = sel4(role, 0.5f * kn[i], crn[0][i], 0.5f * foot[i], crn[1][i]);
        lpA[i] = f2{xa, ya};
        lpB[i] = f2{xb, yb};
      }
      rr = f2{sel4(role, thigh_r, hip_r, calf_r, foot_r), sel4(role, thigh_r, 0.0f, calf_r, 0.0f)};
    }
    // self-collision first (few values live yet): the broad phase, and the narrow phase in a wave with a candidate
    float wb[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f}, Mo[3] = {0.0f, 0.0f, 0.0f};
    MARK(self_begin);
#ifndef GO1_ABL_NO_SELF  // ablation build only: no self-collision
    const bool self_on = cfg->self_stiffness > 0.0f;
    int mask;
    {
      // the hip capsule's ends in the trunk frame: the hip joint + Rx(q) (0, y, 0)
      const f2 hy = msy * f2{hip_y0, hip_y1};
      const f2 hcy = origin[1] + cs[0][0] * hy, hcz = origin[2] + cs[0][1] * hy;
      const float hc0[3] = {origin[0], hcy.x, hcz.x}, hc1[3] = {origin[0], hcy.y, hcz.y};
      mask = self_broad(leg, pth, pkn, pft, fmaxf(foot_r, fmaxf(thigh_r, calf_r)), hc0, hc1, hip_r, R, S.pos, th,
                        S.q);
      mask = self_on ? mask : 0;
    }
#else
    const bool self_on = false;
    const int mask = 0;
#endif
    MARK(self_broad_done);
#ifdef GO1_ABL_NO_NARROW  // ablation build only: the broad phase runs, the narrow phase never does
    if (__any(mask != 0) && mask == 12345) {
#else
    if (__any(mask != 0)) {
#endif
      // the lane's own primitive (its x half's link): the whole segment, ends and their velocities (world)
      float P0[3], P1[3], V0[3], V1[3];
      {
        const float* kn = origin + 6;
        f2 e[3];  // (end 0, end 1) in the link frame
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const float hy0 = i == 1 ? msy * hip_y0 : 0.0f, hy1 = i == 1 ? msy * hip_y1 : 0.0f;
          e[i] = f2{sel4(role, 0.0f, hy0, 0.0f, foot[i]), sel4(role, kn[i], hy1, foot[i], foot[i])};
        }
        const float w[3] = {vs[0].x, vs[1].x, vs[2].x};
        const f2 wl[3] = {w[1] * e[2] - w[2] * e[1], w[2] * e[0] - w[0] * e[2], w[0] * e[1] - w[1] * e[0]};
        const f2 vlin[3] = {vs[3].x + wl[0], vs[4].x + wl[1], vs[5].x + wl[2]};
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const f2 p = ps[i].x + Rs[3 * i].x * e[0] + Rs[3 * i + 1].x * e[1] + Rs[3 * i + 2].x * e[2];
          const f2 v = Rs[3 * i].x * vlin[0] + Rs[3 * i + 1].x * vlin[1] + Rs[3 * i + 2].x * vlin[2];
          P0[i] = p.x; P1[i] = p.y; V0[i] = v.x; V1[i] = v.y;
        }
      }
      // bounding radius: half the link's segment (thigh, calf: half the knee / foot offset; hip: half the capsule's
      // segment; foot: a point) plus its radius
      const float half = sel4(role, 0.5f * fabsf(origin[8]), 0.5f * (hip_y1 - hip_y0), 0.5f * fabsf(foot[2]), 0.0f);
      self_put(self_sc, leg, role, P0, P1, rr.x, half + rr.x, V0, V1);
      // the block is this one wave (TPB 64): the other lanes' primitives are visible once the wave's own LDS
      // writes completed -- no s_barrier, and above all no vmcnt(0) drain of the terrain loads in flight
      static_assert(TPB == 64, "self-collision LDS exchange assumes one wave per block");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      MARK(self_put_done);
      const float pb[3] = {ps[0].x, ps[1].x, ps[2].x};
      self_narrow(cfg, self_sc, leg, role, mask, R, S.pos, vb, th, pb, Fo, Mo, wb);
      // the next sub-step's self_put must not overtake this one's partner reads of other lanes' records
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      MARK(self_narrow_done);
    }
    // world positions of the segment ends, the deepest point of each segment, its point kinematics
    f2 lp[3], pw[3], vw[3];
    HQ qa, qb;
    int cell[2];
    {
      f2 wA[3], wB[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        wA[i] = ps[i] + Rs[3 * i] * lpA[0] + Rs[3 * i + 1] * lpA[1] + Rs[3 * i + 2] * lpA[2];
        wB[i] = ps[i] + Rs[3 * i] * lpB[0] + Rs[3 * i + 1] * lpB[1] + Rs[3 * i + 2] * lpB[2];
      }
      MARK(seg_begin);
      // the search once per control step (wave-uniform), its t held in the env's LDS scratch for the other sim steps
      float2* held = reinterpret_cast<float2*>(self_sc + SEG_T_OFF) + (4 * role + leg);
      f2 ts;
      if (face_scan_now) {
#ifdef GO1_ABL_NO_WALK  // ablation build only: every segment at its first end
        ts = f2{0.0f, 0.0f} * (wA[0] + wB[0]);
        cell[0] = SEG_CELL((int)floorf(wA[0].x / T.hs), (int)floorf(wA[1].x / T.hs), false);
        cell[1] = SEG_CELL((int)floorf(wA[0].y / T.hs), (int)floorf(wA[1].y / T.hs), false);
#else
        ts = seg_deepest2(T, wA, wB, rr, cell);
#endif
        *held = make_float2(ts.x, ts.y);
      } else {
        const float2 hv = *held;
        ts = f2{hv.x, hv.y};
      }
      MARK(seg_done);
#pragma unroll
      for (int i = 0; i < 3; ++i) lp[i] = lpA[i] + ts * (lpB[i] - lpA[i]);
      // point kinematics: v = R (v_lin + w x lp), p = p_body + R lp
      const f2 wl[3] = {vs[1] * lp[2] - vs[2] * lp[1], vs[2] * lp[0] - vs[0] * lp[2], vs[0] * lp[1] - vs[1] * lp[0]};
      const f2 vlin[3] = {vs[3] + wl[0], vs[4] + wl[1], vs[5] + wl[2]};
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        pw[i] = ps[i] + Rs[3 * i] * lp[0] + Rs[3 * i + 1] * lp[1] + Rs[3 * i + 2] * lp[2];
        vw[i] = Rs[3 * i] * vlin[0] + Rs[3 * i + 1] * vlin[1] + Rs[3 * i + 2] * vlin[2];
      }
    }
    // the terrain contacts at the segments' deepest points: on the search step on the triangle the search chose, later
    // on the triangle under the point
    if (face_scan_now) {
      hq_fetch_cell(T, pw[0].x, pw[1].x, cell[0], qa);
      hq_fetch_cell(T, pw[0].y, pw[1].y, cell[1], qb);
    } else {
      hq_fetch(T, pw[0].x, pw[1].x, qa);
      hq_fetch(T, pw[0].y, pw[1].y, qb);
    }
    float Fa[3], Fb2[3], Ma[6], Mb[6];
    {
      const float pa[3] = {pw[0].x, pw[1].x, pw[2].x}, va[3] = {vw[0].x, vw[1].x, vw[2].x};
      const float pb[3] = {pw[0].y, pw[1].y, pw[2].y}, vb2[3] = {vw[0].y, vw[1].y, vw[2].y};
      sphere_contact_im(T, qa, C, pa, va, rr.x, h, Fa, Ma);
      sphere_contact_im(T, qb, C, pb, vb2, rr.y, h, Fb2, Mb);
    }
    if (self_on) {
#pragma unroll
      for (int i = 0; i < 3; ++i) Fbs[i] = R[3 * i] * wb[3] + R[3 * i + 1] * wb[4] + R[3 * i + 2] * wb[5];
    }
    const f2 F[3] = {f2{Fa[0], Fb2[0]}, f2{Fa[1], Fb2[1]}, f2{Fa[2], Fb2[2]}};
    // the ABA below solves for accelerations relative to free fall (gravity as a base
    // acceleration), so the added mass would respond to a - g: the force it sees is F - Mp g
    f2 Fd[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
      Fd[i] = F[i] - (f2{Ma[s3i(i, 0)], Mb[s3i(i, 0)]} * g[0] + f2{Ma[s3i(i, 1)], Mb[s3i(i, 1)]} * g[1] +
                      f2{Ma[s3i(i, 2)], Mb[s3i(i, 2)]} * g[2]);
    // body-frame force f = R^T Fd and moment lp x f; the own primitive's self-contact wrench (R^T Fo, R^T Mo) joins
    // the x half (its link)
    f2 f6[6];
#pragma unroll
    for (int j = 0; j < 3; ++j) f6[3 + j] = Rs[j] * Fd[0] + Rs[3 + j] * Fd[1] + Rs[6 + j] * Fd[2];
    f6[0] = lp[1] * f6[5] - lp[2] * f6[4];
    f6[1] = lp[2] * f6[3] - lp[0] * f6[5];
    f6[2] = lp[0] * f6[4] - lp[1] * f6[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      f6[j].x += Rs[j].x * Mo[0] + Rs[3 + j].x * Mo[1] + Rs[6 + j].x * Mo[2];
      f6[3 + j].x += Rs[j].x * Fo[0] + Rs[3 + j].x * Fo[1] + Rs[6 + j].x * Fo[2];
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      fx[i] = f6[i].x;
      fy[i] = even ? f6[i].y : 0.0f;
      fbase[i] = (even ? 0.0f : f6[i].y) + wb[i];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) Fpt[i] = F[i];
    // added masses into the body frame, M = Rs^T Mp Rs (both points as halves), then about the
    // body origin: A = S M S^T, B = S M, C = M, S = lp~ (S v = lp x v)
    const f2 Mw[6] = {f2{Ma[0], Mb[0]}, f2{Ma[1], Mb[1]}, f2{Ma[2], Mb[2]},
                      f2{Ma[3], Mb[3]}, f2{Ma[4], Mb[4]}, f2{Ma[5], Mb[5]}};
    f2 MR[9];  // Mp Rs (3 x 3, row-major)
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
        MR[3 * i + j] = Mw[s3i(i, 0)] * Rs[j] + Mw[s3i(i, 1)] * Rs[3 + j] + Mw[s3i(i, 2)] * Rs[6 + j];
    f2 M[9];  // Rs^T (Mp Rs), symmetric
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = i; j < 3; ++j) {
        M[3 * i + j] = Rs[i] * MR[j] + Rs[3 + i] * MR[3 + j] + Rs[6 + i] * MR[6 + j];
        M[3 * j + i] = M[3 * i + j];
      }
    f2 SM[9];  // lp~ M: row i = lp x (column of M) components
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      SM[j] = lp[1] * M[6 + j] - lp[2] * M[3 + j];
      SM[3 + j] = lp[2] * M[j] - lp[0] * M[6 + j];
      SM[6 + j] = lp[0] * M[3 + j] - lp[1] * M[j];
    }
    const int II[6] = {0, 0, 0, 1, 1, 2}, JJ[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const int i = II[k], j = JJ[k];
      const f2* r = SM + 3 * i;
      // (S M S^T)_ij = sum_l (SM)_il S_jl, S_j = (0, -lz, ly), (lz, 0, -lx), (-ly, lx, 0)
      const f2 a = j == 0 ? r[2] * lp[1] - r[1] * lp[2] : (j == 1 ? r[0] * lp[2] - r[2] * lp[0] : r[1] * lp[0] - r[0] * lp[1]);
      cin[0].ac[k][0] = a.x; cin[1].ac[k][0] = a.y;
      cin[0].ac[k][1] = M[3 * i + j].x; cin[1].ac[k][1] = M[3 * i + j].y;
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) { cin[0].b[i] = SM[i].x; cin[1].b[i] = SM[i].y; }
  }
#else  // ablation build only: no contacts
  (void)th; (void)foot_r; (void)thigh_r; (void)calf_r; (void)hip_r; (void)hip_y0; (void)hip_y1; (void)C; (void)T;
  (void)Rs; (void)ps; (void)vs; (void)pth; (void)pkn; (void)pft;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
#pragma unroll
    for (int t = 0; t < 6; ++t) cin[k].ac[t] = f2{0.0f, 0.0f};
#pragma unroll
    for (int i = 0; i < 9; ++i) cin[k].b[i] = 0.0f;
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) { fx[i] = 0.0f; fy[i] = 0.0f; fbase[i] = 0.0f; }
#pragma unroll
  for (int i = 0; i < 3; ++i) Fpt[i] = f2{0.0f, 0.0f};
#endif
  // the lane's contributions per body, summed over the leg's roles: thigh (rows 0-1: role 0's halves), calf (rows
  // 2-3: role 2's halves and role 3's foot) in one pair reduction; hip (role 1's x half) and the trunk (odd rows'
  // y halves, the box reactions) in a second
  SIP ci_th, ci_ca, ci_hp, ci_bs;
  {
    const bool hip_lane = role == 1;
    auto term = [&](int h, int k) -> float {  // value k of the lane's half h: the wrench (6), then the 21 inertia terms
      if (k < 6) return h == 0 ? fx[k] : fy[k];
      const int m = k - 6;
      return m < 12 ? cin[h].ac[m >> 1][m & 1] : cin[h].b[m - 12];
    };
    {  // thigh (rows 0-1) and calf (rows 2-3)
      float lg[6 + 21], th6[6 + 21], ca6[6 + 21];
#pragma unroll
      for (int k = 0; k < 27; ++k) lg[k] = (hip_lane ? 0.0f : term(0, k)) + (even ? term(1, k) : 0.0f);
      pairsum_rows_n<6 + 21>(lg, th6, ca6);
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        pAp[1][i] -= f2{th6[i], th6[3 + i]};
        pAp[2][i] -= f2{ca6[i], ca6[3 + i]};
      }
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        ci_th.ac[k] = f2{th6[6 + 2 * k], th6[6 + 2 * k + 1]};
        ci_ca.ac[k] = f2{ca6[6 + 2 * k], ca6[6 + 2 * k + 1]};
      }
#pragma unroll
      for (int i = 0; i < 9; ++i) { ci_th.b[i] = th6[18 + i]; ci_ca.b[i] = ca6[18 + i]; }
    }
    {  // the hip capsule (row 1's x half): the rows 0-1 sum of a value that only row 1 holds
      float hp[6 + 21], lo[6 + 21], hi[6 + 21];
#pragma unroll
      for (int k = 0; k < 27; ++k) hp[k] = hip_lane ? term(0, k) : 0.0f;
      pairsum_rows_n<6 + 21>(hp, lo, hi);
#pragma unroll
      for (int i = 0; i < 3; ++i) pAp[0][i] -= f2{lo[i], lo[3 + i]};
#pragma unroll
      for (int k = 0; k < 6; ++k) ci_hp.ac[k] = f2{lo[6 + 2 * k], lo[6 + 2 * k + 1]};
#pragma unroll
      for (int i = 0; i < 9; ++i) ci_hp.b[i] = lo[18 + i];
    }
    {  // the trunk: this leg's corners (odd rows' y halves) and the box reactions
      float bs[6 + 21];
#pragma unroll
      for (int k = 0; k < 27; ++k) bs[k] = k < 6 ? fbase[k] : (even ? 0.0f : term(1, k));
      rowsum4_n<6 + 21>(bs);
#pragma unroll
      for (int i = 0; i < 6; ++i) fbase[i] = bs[i];
#pragma unroll
      for (int k = 0; k < 6; ++k) ci_bs.ac[k] = f2{bs[6 + 2 * k], bs[6 + 2 * k + 1]};
#pragma unroll
      for (int i = 0; i < 9; ++i) ci_bs.b[i] = bs[18 + i];
    }
  }
  MARK(leg_kin_contacts_done);
  // ---- backward pass calf -> hip (articulated inertias with the contact added masses, bias
  //      forces with the explicit contact forces); the hip's inertia goes to the base
  f2 Up[3][3];  // U = column ax of the articulated inertia, (angular, linear) pairs
  float D[3], u[3];
  SIP Ip;
  f2 pp6[3];
  {
    SIP IA;
    rigid_sip(LC + 20, 1.0f, IA);
    sip_add(IA, ci_ca);
#pragma unroll
    for (int j = 2; j >= 0; --j) {
      const int ax = j == 0 ? 0 : 1;
      float t = tau[j];
      // joint-limit spring-damper, implicit in the joint: the torque at the end of the
      // sub-step, -k (q + h qd') - d qd' with qd' = qd + h qdd, moves (h d + h^2 k) qdd
      // into the joint inertia D (unconditionally stable for any k, d)
      const float lo = cfg->hard_limits[2 * j], hi = cfg->hard_limits[2 * j + 1];  // leg-uniform (go1_create)
      const bool lim_on = S.q[j] > hi || S.q[j] < lo;
      const float ex = S.q[j] > hi ? S.q[j] - hi : S.q[j] - lo;
      const float kl = cfg->limit_stiffness, dl = cfg->limit_damping;
      t -= lim_on ? kl * (ex + h * S.qd[j]) + dl * S.qd[j] : 0.0f;
#pragma unroll
      for (int i = 0; i < 3; ++i) Up[j][i] = sip_col(IA, ax, i);
      D[j] = IA.ac[s3i(ax, ax)].x + (lim_on ? h * dl + h * h * kl : 0.0f);
      u[j] = t - pAp[j][ax].x;
      const float invD = frcp(D[j]);
      D[j] = invD;  // the forward pass only needs 1 / D
      f2 V[3];  // U / D
#pragma unroll
      for (int i = 0; i < 3; ++i) V[i] = Up[j][i] * invD;
      SIP Ia;  // IA - U U^T / D: the A and C blocks as pairs, B scalar
      const int II[6] = {0, 0, 0, 1, 1, 2}, JJ[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
      for (int k = 0; k < 6; ++k) Ia.ac[k] = IA.ac[k] - Up[j][II[k]] * V[JJ[k]];
#pragma unroll
      for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) Ia.b[a * 3 + b] = IA.b[a * 3 + b] - Up[j][a].x * V[b].y;
      f2 Iac[3], pa[3], pt[3];
      sip_mul_sparse(Ia, cjp[j], ax, Iac);
      const float ud = u[j] * invD;
#pragma unroll
      for (int i = 0; i < 3; ++i) pa[i] = pAp[j][i] + Iac[i] + Up[j][i] * ud;
      SIP It;
      xform_inertia2(ax, cs[j][0], cs[j][1], offset_mask(j), origin + j * 3, Ia, It);
      xfT2(ax, cs[j][0], cs[j][1], offset_mask(j), origin + j * 3, pa, pt);
      if (j > 0) {
        rigid_sip(LC + 10 * (j - 1), 1.0f, IA);
        sip_add(IA, It);
        sip_add(IA, j == 2 ? ci_th : ci_hp);  // the thigh's / the hip capsule's contact added masses
#pragma unroll
        for (int i = 0; i < 3; ++i) pAp[j - 1][i] += pt[i];
      } else {
        Ip = It;
        sip_add(Ip, ci_bs);  // this leg's trunk corners: summed over the legs with the hips below
#pragma unroll
        for (int i = 0; i < 3; ++i) pp6[i] = pt[i];
      }
    }
  }
  MARK(backward_done);
  // ---- the trunk faces (face_scan / face_force): the vertices once per control step, the force every sim step
  f2 wface[3] = {f2{0.0f, 0.0f}, f2{0.0f, 0.0f}, f2{0.0f, 0.0f}};
  float Fface[3] = {0.0f, 0.0f, 0.0f};
#ifdef GO1_ABL_NO_FACES  // ablation build only: no trunk faces
  if (false) {
#else
  if (T.patch) {  // the tunnel; on the plane the corners are the faces' deepest points
#endif
    // the vertices chosen at the control step's first sim step (at the top of phys_substep) from the env's LDS scratch
    const int* fsel = reinterpret_cast<const int*>(self_sc + FACE_SEL_OFF);
    const int sel[2] = {fsel[0], fsel[1]};
    face_force(T, C, R, S.pos, vb, th, sel, wface, Fface);
  }
  MARK(faces_done);
  // ---- base: rigid inertia + quad sum of the four legs and the trunk corners
  const float* bb = model;
  const float mscale = (bb[0] + payload) * frcp(bb[0]);
  SIP I0;
  rigid_sip(bb, mscale, I0);
  f2 p0[3];
  float gb[3];
  rigid_bias2(bb, vbp, p0, mscale);
  mat3T_vec(R, g, gb);  // gravity in the base frame: added to the relative base acceleration below
#pragma unroll
  for (int k = 0; k < 6; ++k) Ip.ac[k] = f2{qsum(Ip.ac[k].x), qsum(Ip.ac[k].y)};
#pragma unroll
  for (int i = 0; i < 3; ++i) pp6[i] = f2{qsum(pp6[i].x - fbase[i]), qsum(pp6[i].y - fbase[3 + i])} - wface[i];
#pragma unroll
  for (int i = 0; i < 9; ++i) Ip.b[i] = qsum(Ip.b[i]);
  sip_add(I0, Ip);
  float rhs[6], a0[6];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    rhs[i] = -(p0[i].x + pp6[i].x);
    rhs[3 + i] = -(p0[i].y + pp6[i].y);
  }
#ifdef GO1_ABL_NO_BASESOLVE  // ablation build only: the base's 6x6 solve replaced by a diagonal scaling
#pragma unroll
  for (int i = 0; i < 6; ++i) a0[i] = rhs[i] * 0.05f;
  (void)I0;
#else
#ifdef GO1_ABL_NO_CHOL  // ablation build only: the Cholesky alone compiled out, its inputs kept live
  float tr = 0.0f;
#pragma unroll
  for (int k = 0; k < 6; ++k) tr += I0.ac[k].x + I0.ac[k].y;
#pragma unroll
  for (int k = 0; k < 9; ++k) tr += I0.b[k];
#pragma unroll
  for (int i = 0; i < 6; ++i) a0[i] = rhs[i] * tr * 1e-3f;
#else
  solve6p(I0, rhs, a0);
#endif
#endif
  MARK(base_solve_done);
  // ---- forward pass
  float qdd[3];
  {
    f2 ap[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) ap[i] = f2{a0[i], a0[3 + i]};
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int ax = j == 0 ? 0 : 1;
      f2 aj[3];
      xm2(ax, cs[j][0], cs[j][1], offset_mask(j), origin + j * 3, ap, aj);
#pragma unroll
      for (int i = 0; i < 3; ++i)
        if (i != ax) aj[i] += cjp[j][i];  // pair ax of c_j is zero
      const f2 ua = Up[j][0] * aj[0] + Up[j][1] * aj[1] + Up[j][2] * aj[2];
      qdd[j] = (u[j] - (ua.x + ua.y)) * D[j];
      aj[ax].x += qdd[j];
#pragma unroll
      for (int i = 0; i < 3; ++i) ap[i] = aj[i];
    }
  }
  MARK(forward_done);
  // ---- semi-implicit Euler (base identical in the quad)
  float wxv[3];
  cross3(vb, vb + 3, wxv);
  // a0 is relative to free fall: the base's linear acceleration is a0_lin + g; (angular, linear)
  // body-frame accelerations as pairs, rotated to the world and integrated together
  f2 ab[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) ab[i] = f2{a0[i], a0[3 + i] + gb[i] + wxv[i]};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    S.wv[i] += h * (R[3 * i] * ab[0] + R[3 * i + 1] * ab[1] + R[3 * i + 2] * ab[2]);
    S.pos[i] += h * S.wv[i].y;
  }
  {
    const float w[3] = {S.wv[0].x, S.wv[1].x, S.wv[2].x};
    const float wn2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    const float iwn = frsq(fmaxf(wn2, 1e-30f));
    const float wn = wn2 * iwn;
    const float thh = 0.5f * h * wn;
    float sth, cth;
    hw_sincosf(thh, &sth, &cth);
    const float sc = thh > 1e-12f ? sth * iwn : 0.5f * h;
    const float dq[4] = {w[0] * sc, w[1] * sc, w[2] * sc, cth};
    float* q = S.quat;
    float nq[4];
    nq[3] = dq[3] * q[3] - dq[0] * q[0] - dq[1] * q[1] - dq[2] * q[2];
    nq[0] = dq[3] * q[0] + dq[0] * q[3] + dq[1] * q[2] - dq[2] * q[1];
    nq[1] = dq[3] * q[1] - dq[0] * q[2] + dq[1] * q[3] + dq[2] * q[0];
    nq[2] = dq[3] * q[2] + dq[0] * q[1] - dq[1] * q[0] + dq[2] * q[3];
    const float inv = frsq(nq[0] * nq[0] + nq[1] * nq[1] + nq[2] * nq[2] + nq[3] * nq[3]);
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = nq[i] * inv;
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    S.qd[j] += h * qdd[j];
    S.q[j] += h * S.qd[j];
  }
  MARK(integrate_done);
  // this lane's contact forces of the sub-step (the last sub-step's survive the loop); summed
  // over the roles once, after the loop (cf_sum): no branch and no cross-lane work here
  (void)cf_out;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    cf_raw[i] = Fpt[i].x + Fo[i];
    cf_raw[3 + i] = Fpt[i].y;
    cf_raw[6 + i] = Fbs[i] + (role == 0 && leg == 0 ? Fface[i] : 0.0f);  // summed over the env's lanes (cf_sum)
  }
}

// reported contact forces from the last sub-step's per-lane values: thigh, calf, foot and hip of the lane's leg
// (role sums), the base (role and leg sums).  cf_raw: world forces of the lane's x half (with its primitive's
// self-contact force) and y half -- rows 0 (thigh, thigh), 1 (hip, corner), 2 (calf, calf), 3 (foot, corner) --
// then the trunk's self-collision reaction and faces
#define CF_RAW 9
__device__ __forceinline__ void cf_sum(const float* cf_raw, int role, float* cf_leg, float* cf_base, float* cf_hip) {
  float v[15];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float x = cf_raw[i], y = cf_raw[3 + i];
    v[i] = role == 0 ? x + y : 0.0f;                      // thigh
    v[3 + i] = role == 2 ? x + y : 0.0f;                  // calf
    v[6 + i] = role == 3 ? x : 0.0f;                      // foot
    v[9 + i] = role == 1 ? x : 0.0f;                      // hip
    v[12 + i] = ((role & 1) ? y : 0.0f) + cf_raw[6 + i];  // trunk corners, self-collision reactions, faces
  }
  rowsum4_n<15>(v);
#pragma unroll
  for (int i = 0; i < 9; ++i) cf_leg[i] = v[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    cf_base[i] = qsum(v[12 + i]);
    cf_hip[i] = v[9 + i];
  }
}

#pragma clang fp contract(off)

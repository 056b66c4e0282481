// go1_step.hip -- MI355X (gfx950) fused Go1 trajectory-tracking step + C ABI.
//
// One launch = one LeggedRobot.step() for every env
// (go1_gym/envs/base/legged_robot_trajectory_tracking.py:64-169):
//   4 x [actuator-net torques (:957-996, :1311-1320) -> native articulated-body
//        integrator (replaces gym.simulate / fetch_results / refresh, :82-88)]
//   -> post-physics: kinematics (:130-136), height scan (:1918-1970), target and
//      command logic (:774-932), terminations (:198-216), reward terms of both containers
//      (:320-355), reset_idx (:218-296), observations (:357-475), epilogue (:148-153).
//
// Decomposition: 16 lanes per env = 4 legs x 4 roles, lane = 16 role + 4 env + leg; a 64-lane
// wave carries 4 envs and a block is one wave (4096 envs -> 1024 waves, one per SIMD).  The four
// roles of a leg run that leg's kinematics and articulated-body passes redundantly (the 3-link
// chain is sequential) and split the parallel work: the leg's contact points, the actuator-net
// MFMA columns (a role is one row of the 16 x 4 B operand), the height-scan gathers and the
// stores.  Leg sums use DPP quad_perm, role sums v_permlane16/32_swap; both are butterflies, so
// every lane of an env holds bit-identical base quantities and solves the base 6 x 6 system.
// State is SoA row-major (n_envs, width) in HBM.  LDS holds the Go1 model block and per-joint
// config (ds_write after the prologue loads), the env's 20 x 16 (floor, ceiling) terrain patch
// (LDS-DMA, global_load_lds, at step start) and the per-env reward-term table.  See DESIGN.md 5.
// Numerics: the post-physics section is compiled with FP contraction OFF and
// uses the deterministic transcendentals of pmath.h, so it is bit-identical to
// the CPU oracle (oracle/go1_oracle.c) given the same physical state; the
// integrator uses FMA contraction and native sin/cos (f32, compared with the
// oracle's f64 integrator within a tolerance).
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
#define GO1_STAMP_SLOTS 160
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

// floor (layer 1) and ceiling (layer 0) heights and gradients at world (x, y), bilinear
__device__ __forceinline__ void height_query2(const Terr& T, float x, float y, float* hf, float* hc) {
  if (!T.tile) {
    hf[0] = 0.0f; hf[1] = 0.0f; hf[2] = 0.0f;
    hc[0] = 1e9f; hc[1] = 0.0f; hc[2] = 0.0f;
    return;
  }
  // bounded before the float -> int conversions (a diverged pose must not index memory)
  const float ihs = frcp(T.hs);
  const float u = fminf(fmaxf(x * ihs, -4.0f), (float)(T.nx + 4));
  const float v = fminf(fmaxf(y * ihs, -4.0f), (float)(T.ny + 4));
  const float fu = floorf(u), fv = floorf(v);
  const int i = (int)fu, j = (int)fv;
  const float a = u - fu, b = v - fv;
  float2 c00, c10, c01, c11;
  const int li = i - T.pi0, lj = j - T.pj0;
  if (T.patch && li >= 0 && li < PSZX - 1 && lj >= 0 && lj < PSZY - 1) {
    const float2* pp = T.patch + li * PSZY + lj;
    c00 = pp[0]; c01 = pp[1]; c10 = pp[PSZY]; c11 = pp[PSZY + 1];
  } else {
    c00 = make_float2(tile_at(T, 1, i, j), tile_at(T, 0, i, j));
    c10 = make_float2(tile_at(T, 1, i + 1, j), tile_at(T, 0, i + 1, j));
    c01 = make_float2(tile_at(T, 1, i, j + 1), tile_at(T, 0, i, j + 1));
    c11 = make_float2(tile_at(T, 1, i + 1, j + 1), tile_at(T, 0, i + 1, j + 1));
  }
  const float inv = ihs;
  hf[0] = (1 - a) * (1 - b) * c00.x + a * (1 - b) * c10.x + (1 - a) * b * c01.x + a * b * c11.x;
  hf[1] = ((1 - b) * (c10.x - c00.x) + b * (c11.x - c01.x)) * inv;
  hf[2] = ((1 - a) * (c01.x - c00.x) + a * (c11.x - c10.x)) * inv;
  hc[0] = (1 - a) * (1 - b) * c00.y + a * (1 - b) * c10.y + (1 - a) * b * c01.y + a * b * c11.y;
  hc[1] = ((1 - b) * (c10.y - c00.y) + b * (c11.y - c01.y)) * inv;
  hc[2] = ((1 - a) * (c01.y - c00.y) + a * (c11.y - c10.y)) * inv;
}

struct CP {
  float k, d, kf, mu;
};

// ---- packed (v_pk_*_f32) contact: one wave issues a v_pk_fma_f32 (two FMAs) as fast as a
// v_fma_f32 (tools/probes/pk_rate.hip), so the floor and ceiling layers of a point are
// carried as the two halves of an f2 all the way from the bilinear patch to the force.
__device__ __forceinline__ f2 f2s(float v) { return f2{v, v}; }

// (floor, ceiling) heights and gradients at world (x, y), bilinear, in two halves, so that the
// corner reads are issued early and land while independent work runs (the articulated-inertia
// chain of the sub-step): hq_fetch reads the four (floor, ceiling) corners -- the LDS patch stores
// (floor, ceiling) per cell, i.e. already in f2 layout; the HBM tile outside it -- and hq_finish
// interpolates.
struct HQ {
  f2 c00, c10, c01, c11;
  float a, b;
};
__device__ __forceinline__ void hq_fetch(const Terr& T, float x, float y, HQ& q) {
  if (!T.tile) {
    q.c00 = q.c10 = q.c01 = q.c11 = f2{0.0f, 1e9f};
    q.a = q.b = 0.0f;
    return;
  }
  const float ihs = frcp(T.hs);
  const float u = fminf(fmaxf(x * ihs, -4.0f), (float)(T.nx + 4));
  const float v = fminf(fmaxf(y * ihs, -4.0f), (float)(T.ny + 4));
  const float fu = floorf(u), fv = floorf(v);
  const int i = (int)fu, j = (int)fv;
  q.a = u - fu;
  q.b = v - fv;
#ifdef GO1_ABL_NO_FALLBACK  // ablation build only: every query from the (clamped) LDS patch
  const int li = min(max(i - T.pi0, 0), PSZX - 2), lj = min(max(j - T.pj0, 0), PSZY - 2);
#else
  const int li = i - T.pi0, lj = j - T.pj0;
#endif
  if (T.patch && li >= 0 && li < PSZX - 1 && lj >= 0 && lj < PSZY - 1) {
    const float2* pp = T.patch + li * PSZY + lj;
    const float2 q00 = pp[0], q01 = pp[1], q10 = pp[PSZY], q11 = pp[PSZY + 1];
    q.c00 = f2{q00.x, q00.y}; q.c01 = f2{q01.x, q01.y}; q.c10 = f2{q10.x, q10.y}; q.c11 = f2{q11.x, q11.y};
  } else {
    q.c00 = f2{tile_at(T, 1, i, j), tile_at(T, 0, i, j)};
    q.c10 = f2{tile_at(T, 1, i + 1, j), tile_at(T, 0, i + 1, j)};
    q.c01 = f2{tile_at(T, 1, i, j + 1), tile_at(T, 0, i, j + 1)};
    q.c11 = f2{tile_at(T, 1, i + 1, j + 1), tile_at(T, 0, i + 1, j + 1)};
  }
}
__device__ __forceinline__ void hq_finish(const Terr& T, const HQ& q, f2& h, f2& gx, f2& gy) {
  const float ihs = frcp(T.hs);
  const float a = q.a, b = q.b, a1 = 1.0f - a, b1 = 1.0f - b;
  h = (a1 * b1) * q.c00 + (a * b1) * q.c10 + (a1 * b) * q.c01 + (a * b) * q.c11;
  gx = (b1 * (q.c10 - q.c00) + b * (q.c11 - q.c01)) * ihs;
  gy = (a1 * (q.c01 - q.c00) + a * (q.c11 - q.c10)) * ihs;
}

// penalty contact of a sphere (centre p, velocity pv, radius r) with the floor (pushes up)
// and the ceiling (pushes down), both layers at once; F = floor + ceiling force
__device__ __forceinline__ void sphere_contact_pk(const Terr& T, const HQ& q, const CP& C, const float* p,
                                                  const float* pv, float r, float* F) {
  f2 h, gx, gy;
  hq_finish(T, q, h, gx, gy);
  const f2 sg = f2{1.0f, -1.0f};
  const f2 dv = sg * (h - p[2]) + r;  // floor: h + r - z, ceiling: z + r - h
  f2 nx = -sg * gx, ny = -sg * gy;
  f2 inv = nx * nx + ny * ny + 1.0f;
  inv = f2{frsq(inv.x), frsq(inv.y)};
  nx = nx * inv;
  ny = ny * inv;
  const f2 nz = sg * inv;
  const f2 depth = dv * inv;
  const f2 vn = pv[0] * nx + pv[1] * ny + pv[2] * nz;
  const f2 fn = C.k * depth - C.d * vn;
  const f2 vtx = pv[0] - vn * nx, vty = pv[1] - vn * ny, vtz = pv[2] - vn * nz;
  const f2 vt2 = vtx * vtx + vty * vty + vtz * vtz;
  const f2 ivt = f2{frsq(fmaxf(vt2.x, 1e-18f)), frsq(fmaxf(vt2.y, 1e-18f))};
  const f2 vtn = vt2 * ivt;
  const f2 cf = C.kf * vtn, cm = C.mu * fn;
  const f2 ft = f2{fminf(cf.x, cm.x), fminf(cf.y, cm.y)};
  const f2 fti = ft * ivt;
  // a layer acts only in penetration with a compressive normal force
  const bool ax = dv.x > 0.0f && fn.x > 0.0f, ay = dv.y > 0.0f && fn.y > 0.0f;
  const f2 fa = f2{ax ? fn.x : 0.0f, ay ? fn.y : 0.0f};
  const f2 sc = f2{(ax && vtn.x > 1e-9f) ? fti.x : 0.0f, (ay && vtn.y > 1e-9f) ? fti.y : 0.0f};
  const f2 Fx = fa * nx - sc * vtx, Fy = fa * ny - sc * vty, Fz = fa * nz - sc * vtz;
  F[0] = Fx.x + Fx.y;
  F[1] = Fy.x + Fy.y;
  F[2] = Fz.x + Fz.y;
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
  const f2 fn = fn0 - (h * C.k) * vn;              // k depth - (h k + d) vn
  const f2 vtx = pv[0] - vn * nx, vty = pv[1] - vn * ny, vtz = pv[2] - vn * nz;
  const f2 vt2 = vtx * vtx + vty * vty + vtz * vtz;
  const f2 ivt = f2{frsq(fmaxf(vt2.x, 1e-18f)), frsq(fmaxf(vt2.y, 1e-18f))};
  const f2 vtn = vt2 * ivt;
  const f2 cm = C.mu * fn0;
  // c_t = min(kf, mu fn0 / |vt|); kf in the viscous limit |vt| -> 0
  const f2 ct = f2{(C.kf * vtn.x > cm.x && vtn.x > 1e-9f) ? cm.x * ivt.x : C.kf,
                   (C.kf * vtn.y > cm.y && vtn.y > 1e-9f) ? cm.y * ivt.y : C.kf};
  const bool ax = dv.x > 0.0f && fn0.x > 0.0f, ay = dv.y > 0.0f && fn0.y > 0.0f;
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

__device__ __forceinline__ void sphere_contact(const Terr& T, const CP& C, const float* p, const float* pv, float r,
                                               float* F) {
  F[0] = F[1] = F[2] = 0.0f;
  float hq[2][3];
  height_query2(T, p[0], p[1], hq[1], hq[0]);
#pragma unroll
  for (int layer = 1; layer >= 0; --layer) {
    const float h = hq[layer][0], gx = hq[layer][1], gy = hq[layer][2];
    float n[3], dv;
    if (layer == 1) {
      dv = h + r - p[2];
      n[0] = -gx; n[1] = -gy; n[2] = 1.0f;
    } else {
      dv = p[2] + r - h;
      n[0] = gx; n[1] = gy; n[2] = -1.0f;
    }
    if (dv <= 0.0f) continue;
    const float inv = frsq(n[0] * n[0] + n[1] * n[1] + 1.0f);
    n[0] *= inv; n[1] *= inv; n[2] *= inv;
    const float depth = dv * inv;
    const float vn = pv[0] * n[0] + pv[1] * n[1] + pv[2] * n[2];
    const float fn = C.k * depth - C.d * vn;
    if (fn <= 0.0f) continue;
    const float vt[3] = {pv[0] - vn * n[0], pv[1] - vn * n[1], pv[2] - vn * n[2]};
    const float vt2 = vt[0] * vt[0] + vt[1] * vt[1] + vt[2] * vt[2];
    const float ivt = frsq(fmaxf(vt2, 1e-18f));
    const float vtn = vt2 * ivt;
    const float ft = fminf(C.kf * vtn, C.mu * fn);
    const float sc = vtn > 1e-9f ? ft * ivt : 0.0f;
    F[0] += fn * n[0] - sc * vt[0];
    F[1] += fn * n[1] - sc * vt[1];
    F[2] += fn * n[2] - sc * vt[2];
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

// sum over the 4 roles of a leg (the four 16-lane rows), bitwise identical on every lane
__device__ __forceinline__ float rsum(float v) { return rowsum4(v); }

// One integrator step of length h for the env of this lane.  Lane layout (16 per
// env): lane = 16 role + 4 env + leg.  The four roles of a leg compute the leg's
// kinematics and ABA passes redundantly (base quantities on all 16 lanes), and
// split the leg's 8 contact points [thigh x3, calf x2, foot, 2 trunk corners]
// two per lane, so each wave has four envs and the whole grid fills every SIMD.
// cf_out: this lane's reported contact forces (thigh, calf, foot of its leg; base).
// `lds` = the model block (GO1_MODEL_FLOATS) followed by the per-joint config arrays (LDS_*), staged
// in LDS once per block: the lane-dependent (per-leg) constants are re-read every sub-step
// because the physics keeps every VGPR busy, and LDS answers faster than the caches.
__device__ __forceinline__ void phys_substep(CCfg* __restrict__ cfg, const float* lds, Phys& S, const float* tau,
                                             float h, const float* g, float friction, float payload, const Terr& T,
                                             int leg, int role, bool cf_out, float* cf_raw) {
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
  const CP C = {cfg->contact_stiffness, cfg->contact_damping, cfg->friction_damping, friction};
  float R[9];
  quat_to_R(S.quat, R);
  f2 vbp[3];  // base-frame (angular, linear) velocity pairs: R^T on both halves at once
#pragma unroll
  for (int i = 0; i < 3; ++i) vbp[i] = R[i] * S.wv[0] + R[3 + i] * S.wv[1] + R[6 + i] * S.wv[2];
  const float vb[6] = {vbp[0].x, vbp[1].x, vbp[2].x, vbp[0].y, vbp[1].y, vbp[2].y};
  const float* th = model + 13 * 10 + 4 * 9 + 3 + 1;  // trunk half extents
  // ---- this leg: kinematics, rigid bias forces and gravity (hip -> calf)
  const float* origin = LC + 30;
  const float* foot = model + 13 * 10 + 4 * 9;
  const float foot_r = foot[3];
  const float thigh_r = model[13 * 10 + 4 * 9 + 3 + 1 + 3];
  const float calf_r = model[13 * 10 + 4 * 9 + 3 + 1 + 3 + 1];
  float cs[3][2];
  float Rl[2][9], pl[2][3], vl[2][6];  // thigh and calf frames for the contacts
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
      if (j > 0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) { Rl[j - 1][k] = R01[k].x; Rl[j - 1][3 + k] = R01[k].y; Rl[j - 1][6 + k] = R2[k]; }
        pl[j - 1][0] = pp01.x; pl[j - 1][1] = pp01.y; pl[j - 1][2] = pp2;
#pragma unroll
        for (int i = 0; i < 3; ++i) { vl[j - 1][i] = vj[i].x; vl[j - 1][3 + i] = vj[i].y; }
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) vp[i] = vj[i];
    }
  }
  MARK(leg_kin_done);
  // ---- contacts: points 2 role, 2 role + 1 of [thigh0, thigh1, thigh2, calf0, calf1, foot,
  //      corner 2 leg, corner 2 leg + 1] -- world position / velocity, terrain corners, the explicit
  //      force (body frame of the point's body) and the added mass of the implicit contact
  // per lane: the leg's (thigh | calf) share in the row pair of its body and the trunk corner's share
  float fleg[6] = {0, 0, 0, 0, 0, 0}, fbase[6] = {0, 0, 0, 0, 0, 0};
  f2 Fpt[3] = {f2{0.0f, 0.0f}, f2{0.0f, 0.0f}, f2{0.0f, 0.0f}};  // world forces of the lane's two points
  const bool even = (role & 1) == 0;
  // the contact inertias of this lane's points as one packed SIP per half (x, y = the two points):
  // [[S M S^T, S M], [M S^T, M]] with M = Rs^T Mp Rs in the body frame, S = lp~
  SIP cin[2];
#ifndef GO1_ABL_NO_CONTACT
  {
    // the lane's two points ride in the halves of f2 (v_pk) from the frame selection to
    // the body-frame force.  Points p: thigh 0-2, calf 3-4, foot 5 (on the calf), trunk corners
    // 6-7 (2 leg, 2 leg + 1).  Rows (roles): 0 (thigh0, thigh1), 1 (thigh2, corner 6),
    // 2 (calf0, calf1), 3 (foot, corner 7) -- x halves and the even rows' y halves belong to the
    // thigh on rows 0-1 and to the calf on rows 2-3 (one pair reduction, pairsum_rows_n), the odd
    // rows' y halves to the trunk
    f2 Rs[9], lp[3], rr, pw[3], vw[3];
    HQ qa, qb;
    {
      const bool lo_rows = role <= 1;  // x: thigh on rows 0-1, calf on rows 2-3; y: thigh, base, calf, base
      f2 ps[3], vs[6];
#pragma unroll
      for (int i = 0; i < 9; ++i)
        Rs[i] = f2{lo_rows ? Rl[0][i] : Rl[1][i], even ? (lo_rows ? Rl[0][i] : Rl[1][i]) : R[i]};
#pragma unroll
      for (int i = 0; i < 3; ++i) ps[i] = f2{lo_rows ? pl[0][i] : pl[1][i], even ? (lo_rows ? pl[0][i] : pl[1][i]) : S.pos[i]};
#pragma unroll
      for (int i = 0; i < 6; ++i) vs[i] = f2{lo_rows ? vl[0][i] : vl[1][i], even ? (lo_rows ? vl[0][i] : vl[1][i]) : vb[i]};
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int p = hh == 0 ? (role == 0 ? 0 : (role == 1 ? 2 : (role == 2 ? 3 : 5)))
                              : (role == 0 ? 1 : (role == 1 ? 6 : (role == 2 ? 4 : 7)));
        const bool on_thigh = p < 3, on_base = p >= 6;
        const int cx = leg * 2 + (p - 6);
        const float lz = -0.071f * (float)(on_thigh ? p + 1 : p - 2);
        lp[0][hh] = on_base ? ((cx & 1) ? th[0] : -th[0]) : (p == 5 ? foot[0] : 0.0f);
        lp[1][hh] = on_base ? ((cx & 2) ? th[1] : -th[1]) : (p == 5 ? foot[1] : 0.0f);
        lp[2][hh] = on_base ? ((cx & 4) ? th[2] : -th[2]) : (p == 5 ? foot[2] : lz);
        rr[hh] = on_base ? 0.0f : (on_thigh ? thigh_r : (p == 5 ? foot_r : calf_r));
      }
      // point kinematics: v = R (v_lin + w x lp), p = p_body + R lp
      const f2 wl[3] = {vs[1] * lp[2] - vs[2] * lp[1], vs[2] * lp[0] - vs[0] * lp[2], vs[0] * lp[1] - vs[1] * lp[0]};
      const f2 vlin[3] = {vs[3] + wl[0], vs[4] + wl[1], vs[5] + wl[2]};
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        pw[i] = ps[i] + Rs[3 * i] * lp[0] + Rs[3 * i + 1] * lp[1] + Rs[3 * i + 2] * lp[2];
        vw[i] = Rs[3 * i] * vlin[0] + Rs[3 * i + 1] * vlin[1] + Rs[3 * i + 2] * vlin[2];
      }
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
    const f2 F[3] = {f2{Fa[0], Fb2[0]}, f2{Fa[1], Fb2[1]}, f2{Fa[2], Fb2[2]}};
    // the ABA below solves for accelerations relative to free fall (gravity as a base
    // acceleration), so the added mass would respond to a - g: the force it sees is F - Mp g
    f2 Fd[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
      Fd[i] = F[i] - (f2{Ma[s3i(i, 0)], Mb[s3i(i, 0)]} * g[0] + f2{Ma[s3i(i, 1)], Mb[s3i(i, 1)]} * g[1] +
                      f2{Ma[s3i(i, 2)], Mb[s3i(i, 2)]} * g[2]);
    // body-frame force f = R^T Fd and moment lp x f
    f2 f6[6];
#pragma unroll
    for (int j = 0; j < 3; ++j) f6[3 + j] = Rs[j] * Fd[0] + Rs[3 + j] * Fd[1] + Rs[6 + j] * Fd[2];
    f6[0] = lp[1] * f6[5] - lp[2] * f6[4];
    f6[1] = lp[2] * f6[3] - lp[0] * f6[5];
    f6[2] = lp[0] * f6[4] - lp[1] * f6[3];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      fleg[i] = f6[i].x + (even ? f6[i].y : 0.0f);
      fbase[i] = even ? 0.0f : f6[i].y;
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
    // (S M) S^T: element (i, j) = (S M)_i . S_j row, S_j row = (lp x e)_j -> -(row i of SM) x lp
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
  (void)th; (void)foot_r; (void)thigh_r; (void)calf_r; (void)C; (void)T; (void)Rl; (void)pl; (void)vl;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
#pragma unroll
    for (int t = 0; t < 6; ++t) cin[k].ac[t] = f2{0.0f, 0.0f};
#pragma unroll
    for (int i = 0; i < 9; ++i) cin[k].b[i] = 0.0f;
  }
#endif
  // the lane's contributions per body (thigh, calf, base), then summed over the leg's roles
  SIP ci_th, ci_ca, ci_bs;
  {
    float lg[6 + 21], bs[6 + 21], th6[6 + 21], ca6[6 + 21];
#pragma unroll
    for (int i = 0; i < 6; ++i) { lg[i] = fleg[i]; bs[i] = fbase[i]; }
#pragma unroll
    for (int k = 0; k < 21; ++k) {
      const float x = k < 12 ? cin[0].ac[k >> 1][k & 1] : cin[0].b[k - 12];
      const float y = k < 12 ? cin[1].ac[k >> 1][k & 1] : cin[1].b[k - 12];
      lg[6 + k] = x + (even ? y : 0.0f);  // thigh on rows 0-1, calf on rows 2-3
      bs[6 + k] = even ? 0.0f : y;        // this leg's trunk corners
    }
    pairsum_rows_n<6 + 21>(lg, th6, ca6);
    rowsum4_n<6 + 21>(bs);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      pAp[1][i] -= f2{th6[i], th6[3 + i]};
      pAp[2][i] -= f2{ca6[i], ca6[3 + i]};
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) fbase[i] = bs[i];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      ci_th.ac[k] = f2{th6[6 + 2 * k], th6[6 + 2 * k + 1]};
      ci_ca.ac[k] = f2{ca6[6 + 2 * k], ca6[6 + 2 * k + 1]};
      ci_bs.ac[k] = f2{bs[6 + 2 * k], bs[6 + 2 * k + 1]};
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) { ci_th.b[i] = th6[18 + i]; ci_ca.b[i] = ca6[18 + i]; ci_bs.b[i] = bs[18 + i]; }
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
        if (j == 2) sip_add(IA, ci_th);  // the thigh's contact added masses
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
  for (int i = 0; i < 3; ++i) pp6[i] = f2{qsum(pp6[i].x - fbase[i]), qsum(pp6[i].y - fbase[3 + i])};
#pragma unroll
  for (int i = 0; i < 9; ++i) Ip.b[i] = qsum(Ip.b[i]);
  sip_add(I0, Ip);
  float rhs[6], a0[6];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    rhs[i] = -(p0[i].x + pp6[i].x);
    rhs[3 + i] = -(p0[i].y + pp6[i].y);
  }
  solve6p(I0, rhs, a0);
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
    cf_raw[i] = Fpt[i].x;
    cf_raw[3 + i] = Fpt[i].y;
  }
}

// reported contact forces from the last sub-step's per-lane values: thigh, calf, foot of
// the lane's leg (role sums) and the base (role and leg sums)
__device__ __forceinline__ void cf_sum(const float* cf_raw, int role, float* cf_leg, float* cf_base) {
  // cf_raw: world forces of the lane's two points (x, y); rows 0 (thigh, thigh), 1 (thigh, corner),
  // 2 (calf, calf), 3 (foot, corner)
  float v[12];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float x = cf_raw[i], y = cf_raw[3 + i];
    v[i] = role == 0 ? x + y : (role == 1 ? x : 0.0f);  // thigh
    v[3 + i] = role == 2 ? x + y : 0.0f;                 // calf
    v[6 + i] = role == 3 ? x : 0.0f;                     // foot
    v[9 + i] = (role & 1) ? y : 0.0f;                    // trunk corners
  }
  rowsum4_n<12>(v);
#pragma unroll
  for (int i = 0; i < 9; ++i) cf_leg[i] = v[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) cf_base[i] = qsum(v[9 + i]);
}

#pragma clang fp contract(off)

// =====================================================================
//                          the fused step kernel
// =====================================================================
struct KArgs {
  go1_state st;
  go1_terrain ter;
  go1_step_args a;
  // extras["time_outs"] rebinding (:289-291) without a launch of its own: flag words
  // [3] ("some env reset in step k" for k mod 3); this step sets flags[cur], applies the
  // previous step's rebinding for its own envs in the prologue (prev_time_out != NULL),
  // and clears flags[nxt] for the next step.
  int32_t* flags;
  int cur, prv, nxt;
  const uint8_t* prev_time_out;
  uint8_t* prev_extras;
  // global reward bucketing (go1_config.indefinite_slots != 0): per-env scaled slot rewards
  // (n_envs, GO1_MAX_TERMS) and this step's bank of their f64 sums over envs
  float* bucket_r;
  double* bucket_sum;
};

// Waypoint w of the trajectory a reset draws (trajectory_function.py), torch's f32 op order.
// Trajectory uniforms follow the obs-noise slots: slot GO1_U_NOISE + num_obs + k.
__device__ void traj_waypoint(CCfg* __restrict__ c, const Rng& rng, const float* root, int w, float* o) {
  const int ub = GO1_U_NOISE + c->num_obs;
  if (c->traj_kind == 1) {
    // _traj_fn_random_target (:70-93): num_targets = traj_length / num_interp + 1 poses per channel, drawn
    // x, y, z, yaw, pitch, roll; pose 0 := 0; waypoint (s, j) = pose s + (j + 1) (pose s+1 - pose s) / ni
    const int ni = c->traj_interp, nt = c->traj_length / ni + 1, sg = w / ni, j = w % ni;
    const float rng_of[6] = {c->traj_x_range, c->traj_y_range, c->traj_z_range, c->traj_yaw_range,
                             c->traj_pitch_range, c->traj_roll_range};
    const int out_of[6] = {0, 1, 2, 5, 4, 3};  // draw channel -> [x y z roll pitch yaw]
#pragma unroll
    for (int ch = 0; ch < 6; ++ch) {
      const float r = rng_of[ch];
      const float a = sg == 0 ? 0.0f : rng(ub + ch * nt + sg) * 2.0f * r - r;
      const float b = rng(ub + ch * nt + sg + 1) * 2.0f * r - r;
      const float delta = (b - a) / (float)ni;
      o[out_of[ch]] = a + (float)(j + 1) * delta;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) o[i] = o[i] + root[i];
  } else if (c->traj_kind == 2) {
    // _traj_fn_random_goal (:28-41): one pose, broadcast to every waypoint
    o[0] = (rng(ub) - 0.5f) * c->traj_x_range + c->traj_x_mean;
    o[0] = o[0] + root[0];
    o[1] = (rng(ub + 1) - 0.5f) * c->traj_y_range + c->traj_y_mean;
    o[1] = o[1] + root[1];
    o[2] = 0.0f + c->traj_base_z;
    o[3] = 0.0f;
    o[4] = 0.0f;
    o[5] = rng(ub + 2) * 2.0f * c->traj_yaw_range - c->traj_yaw_range;
  } else {
    // _traj_fn_fixed_target (:14-26): waypoint w at (w + 1) x (base_x, base_y) from the base
    const float k = (float)(w + 1);
    o[0] = k * c->traj_base_x + root[0];
    o[1] = k * c->traj_base_y + root[1];
    o[2] = c->traj_base_z;
    o[3] = c->traj_roll;
    o[4] = c->traj_pitch;
    o[5] = c->traj_yaw;
  }
}

// reset_idx for one env, computed redundantly by the lanes of the env (:218-296).  `u(slot)` is
// the reset's uniform of slots 0 .. GO1_RESET_SLOTS - 1 (the step kernel draws their Philox
// blocks once per env, one block per lane, and passes them through LDS); `rng` serves the
// trajectory draws beyond them.  `eo` = env_origins[e] (loaded ahead by the caller).
#define GO1_RESET_SLOTS 36
template <class U>
__device__ void reset_env(CCfg* __restrict__ c, const U& u, const Rng& rng, const float* eo, int leg,
                          const float* ddp, float* root, float* q, float* qd, float* strength, float* offset,
                          float* traj) {
  float s = u(0) * c->strength_range + c->strength_lo;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int d = leg * 3 + j;
    strength[j] = s;
    offset[j] = u(1 + d) * c->offset_range + c->offset_lo;
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int d = leg * 3 + j;
    float f = c->reset_dof_range * u(13 + d) + c->reset_dof_lo;
    q[j] = ddp[d] * f;
    qd[j] = 0.0f;
  }
#pragma unroll
  for (int i = 0; i < 13; ++i) root[i] = c->base_init_state[i];
  root[0] = root[0] + eo[0];
  root[1] = root[1] + eo[1];
  root[2] = root[2] + eo[2];
  if (c->custom_origins) {
    root[0] = root[0] + (c->x_init_range2 * u(25) + c->x_init_lo);
    root[1] = root[1] + (c->y_init_range2 * u(26) + c->y_init_lo);
    root[0] = root[0] + c->x_init_offset;
    root[1] = root[1] + c->y_init_offset;
  }
  float yaw = c->yaw_range2 * u(27) + c->yaw_lo;
  float thh = yaw / 2.0f, sth, cth;
  pm_sincosf(thh, &sth, &cth);
  float qv[4] = {0.0f * sth, 0.0f * sth, 1.0f * sth, cth};
  float qn = sqrtf(fmaf(qv[3], qv[3], fmaf(qv[2], qv[2], fmaf(qv[1], qv[1], qv[0] * qv[0]))));
  if (qn < 1e-9f) qn = 1e-9f;
#pragma unroll
  for (int i = 0; i < 4; ++i) root[3 + i] = qv[i] / qn;
#pragma unroll
  for (int i = 0; i < 6; ++i) root[7 + i] = c->reset_vel_range * u(28 + i) + c->reset_vel_lo;
  traj_waypoint(c, rng, root, 0, traj);
}
static_assert(28 + 6 <= GO1_RESET_SLOTS, "reset_env's uniform slots");

// every waypoint w = first, first + stride, ... of the env's new trajectory (_resample_trajectory :949-955)
__device__ void write_trajectory(CCfg* __restrict__ c, const Rng& rng, const float* root, float* __restrict__ dst,
                                 int first, int stride) {
  for (int w = first; w < c->traj_length; w += stride) {
    float wp[6];
    traj_waypoint(c, rng, root, w, wp);
#pragma unroll
    for (int i = 0; i < 6; ++i) dst[w * 6 + i] = wp[i];
  }
}

// CI(field): an integer config field, a compile-time constant in the specialised instantiation
// (go1_spec.h, the README configuration; go1_create selects it when every field matches)
#define CI(f) (SPEC ? (decltype(c->f))(GO1_SPEC_##f) : c->f)
template <bool INJ, int KPTS, bool SPEC>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(1, 1))) void go1_step_kernel(
    const go1_config* __restrict__ c_gen, KArgs K) {
  CCfg* __restrict__ c = (CCfg*)c_gen;
  const go1_state& st = K.st;
  const go1_step_args& A = K.a;
  const int n = c->n_envs;
  const int leg = threadIdx.x & 3;
  const int lane = threadIdx.x & 63, lq = lane >> 4;
  // lane = 16 role + 4 env + leg: the four roles of an (env, leg) form one column of
  // the 16 x 4 MFMA B operand, so the actuator-net inputs and outputs never move
  const int role = lane >> 4, el = (lane >> 2) & 3, sub16 = 4 * role + leg;
  const bool owner = role == 0;  // the lane of a leg that stores its per-leg outputs
  const int e = blockIdx.x * SEPB + el;  // n % 16 == 0 (go1_create): every wave is full
  (void)n;
#ifdef GO1_STAMPS
  s_go1_stamp_k = 0;
#endif
  MARK(kernel_begin);
#ifdef GO1_ABL_EMPTY  // ablation build only: launch and wave dispatch alone
  if (c->n_envs > 0) return;
#endif
  MlpFrag F;
  mlp_load(c_gen->actuator, lane, F);  // lane-indexed: generic pointer
  const Rng rng = {A.uniforms, A.rng_seed, A.rng_step, e, e + c->env_id_offset, CI(u_per_env)};
  // the previous step's extras["time_outs"] rebinding, for this wave's envs (flags of the
  // previous launch are complete now), and the flag the next launch will set is cleared
  // (loaded with the state, applied after the prologue's single wait: no round trip of its own)
  const bool rebind = K.prev_time_out != nullptr;
  int rebind_flag = rebind ? K.flags[K.prv] : 0;
  const uint8_t rebind_val = rebind ? K.prev_time_out[e] : 0;
  if (blockIdx.x == 0 && lane == 0) K.flags[K.nxt] = 0;
  const size_t d0 = (size_t)e * NDOF + leg * 3;
  // stored lag (go1_state.lag): the scaled actions of the last K = GO1_LAG_STEPS(decimation) steps,
  // oldest first; the README configuration (decimation 4) keeps K = 2 in the specialised kernel
  const int dec = c->decimation;
  constexpr int KMAX = SPEC ? 2 : GO1_LAG_SLOTS;
  const int KL = SPEC ? 2 : GO1_LAG_STEPS(dec);
  const float* lag_in = st.lag + (size_t)e * 12 * KL + leg * 3;

  // ---------------- load
  float act[3], q[3], qd[3], eh[2][3], vh[2][3], strength[3], offset[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    act[j] = clampf(A.actions[d0 + j], -CI(clip_actions), CI(clip_actions));
    q[j] = st.dof_pos[d0 + j];
    qd[j] = st.dof_vel[d0 + j];
    strength[j] = st.motor_strength[d0 + j];
    offset[j] = st.motor_offset[d0 + j];
    eh[0][j] = st.pos_err_hist[(size_t)e * 24 + leg * 3 + j];
    eh[1][j] = st.pos_err_hist[(size_t)e * 24 + 12 + leg * 3 + j];
    vh[0][j] = st.vel_hist[(size_t)e * 24 + leg * 3 + j];
    vh[1][j] = st.vel_hist[(size_t)e * 24 + 12 + leg * 3 + j];
  }
  // per-joint constants and the stored lag entries the sub-steps read: loaded here so that no
  // sub-step waits on a memory round trip
  float dflt[3], tlim[3], lag_pre[KMAX][3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    dflt[j] = c->default_dof_pos[leg * 3 + j];
    tlim[j] = c->torque_limits[leg * 3 + j];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) lag_pre[k][j] = k < KL ? lag_in[k * 12 + j] : 0.0f;
  }
  const float friction = st.friction[e], payload = st.payload[e];
  // the env origin a reset needs, with the prologue loads (no memory round trip in the reset path)
  const float eo_pre[3] = {K.ter.env_origins[(size_t)e * 3], K.ter.env_origins[(size_t)e * 3 + 1],
                           K.ter.env_origins[(size_t)e * 3 + 2]};
  const float cam_pitch = st.base_rotation[(size_t)e * 3 + 1];  // previous step's pitch (:1939)
  // ---- the post-physics state inputs ride with the prologue loads (one wait for all of
  // them); they are held across the sub-step loop (AGPRs), so after the physics only the
  // height-scan gathers make a memory round trip
  const int ep_in = st.episode_length[e];
  const int idx_in = st.curr_pose_index[e];
  const int coll_in = st.collision_count[e];
  const float restitution = st.restitution[e];
  const int TL = CI(traj_length), NT = CI(n_terms), NS = NT + 3;
  float traj_in[6], ldv[3], la[3];
  {
    // the current waypoint trajectories[e, curr_pose_index[e]] (:850-853); traj_length 1 needs no index
    const float* trj = st.trajectory + (size_t)e * 6 * TL;
    if (TL != 1) trj += 6 * min(max(idx_in, 0), TL - 1);
#pragma unroll
    for (int i = 0; i < 6; ++i) traj_in[i] = trj[i];
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    ldv[j] = st.last_dof_vel[d0 + j];
    la[j] = st.last_actions[d0 + j];
  }
  // reward slot k (Cfg.reward_scales order) belongs to the env's lane sub16 == k: its term id,
  // scale and episode sum; lanes 0..2 also carry total, total_pos, total_neg
  const int my_id = sub16 < NT ? c_gen->term_ids[sub16] : GO1_T_NONE;
  const float my_scale = A.reward_scales[sub16];
  float my_sum = sub16 < NT ? st.episode_sums[(size_t)e * NS + sub16] : 0.0f;
  float my_tot = sub16 < 3 ? st.episode_sums[(size_t)e * NS + NT + sub16] : 0.0f;
  Phys P;
  if (!INJ) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      P.pos[i] = st.root[(size_t)e * 13 + i];
      P.wv[i] = f2{st.root[(size_t)e * 13 + 10 + i], st.root[(size_t)e * 13 + 7 + i]};
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) P.quat[i] = st.root[(size_t)e * 13 + 3 + i];
  }
  Terr T = {nullptr, CI(hf_nx), CI(hf_ny), CI(horizontal_scale), nullptr, 0, 0};
  __shared__ float2 s_patch[SEPB][PSZX * PSZY];
  __shared__ float s_phys[(LDS_FLOATS + 63) / 64 * 64];
  // Block = one wave, so LDS needs no barrier here (a wave's LDS operations execute in
  // order).  The model block and the terrain patches are staged with LDS-DMA
  // (global_load_lds: no VGPR round trip, no __syncthreads fence draining the state loads);
  // nothing reads them before the first sub-step's physics, so the first actuator-net
  // evaluation runs while they land (the compiler waits vmcnt before the first ds_read).
  int tix = 0;  // the env's terrain tile and origin, loaded with the state
  float org_x = 0.0f, org_y = 0.0f;
  if (CI(terrain_kind) == 1) {
    tix = K.ter.env_tile[e];
    org_x = K.ter.env_terrain_origin[(size_t)e * 3];
    org_y = K.ter.env_terrain_origin[(size_t)e * 3 + 1];
  }
  // every ordinary load of the prologue is waited for here, once: a use of an ordinary load
  // result while LDS-DMA is in flight would make the compiler wait vmcnt(0) for the DMA too.
  // The model block goes through VGPRs (ds_write after this wait): LDS written by DMA makes
  // the compiler wait vmcnt(0) before every later ds_read of it, which would serialise the
  // post-physics gathers behind the height-grid reads.
  {
    float mv[(LDS_FLOATS + 63) / 64];
#pragma unroll
    for (int k = 0; k < (LDS_FLOATS + 63) / 64; ++k) {
      const int i = 64 * k + lane;
      mv[k] = i < GO1_MODEL_FLOATS ? c_gen->model[i] : c_gen->default_dof_pos[min(i, LDS_FLOATS - 1) - GO1_MODEL_FLOATS];
    }
    MARK(pro_loads_issued);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    MARK(pro_loads_landed);
#pragma unroll
    for (int k = 0; k < (LDS_FLOATS + 63) / 64; ++k) s_phys[64 * k + lane] = mv[k];  // padded to 64
  }
  if (CI(terrain_kind) == 1) {
    T.tile = K.ter.tiles + (size_t)tix * 2 * CI(hf_nx) * CI(hf_ny);
    if (!INJ) {
      // The integrator runs relative to the env's terrain origin: world x, y
      // reach ~100 m, where an f32 ulp is 7.6e-6 m, and on a terrain step the contact forces
      // depend on x with a gain of ~1e3 s^-1 (k x height gradient), so world-frame contact points
      // put ~1e-2 relative errors into the next dof velocities.  root - origin is exact in f32
      // (both are multiples of the origin's ulp, |difference| < |root|); the world position is
      // rebuilt once after the last sub-step.
      P.pos[0] -= org_x;
      P.pos[1] -= org_y;
      // patch centred on the legs' bounding box at the start of the step
      float bx, by;
      legs_bbox_centre(P.pos, P.quat, q, leg, &bx, &by);
      MARK(pro_bbox_done);
      T.pi0 = (int)floorf(fminf(fmaxf(bx / T.hs, -64.0f), (float)(CI(hf_nx) + 64))) - PSZX / 2;
      T.pj0 = (int)floorf(fminf(fmaxf(by / T.hs, -64.0f), (float)(CI(hf_ny) + 64))) - PSZY / 2;
      T.patch = &s_patch[el][0];
      const int nx = CI(hf_nx), ny = CI(hf_ny);
      // 4 x PSZX / 2 LDS-DMA dword loads per wave: load k of env el2 fills s_patch[el2]
      // dwords 64 k .. 64 k + 63, i.e. cells 32 k + lane / 2 (rows 2 k, 2 k + 1 of PSZY = 16
      // columns), floor (lane even) or ceiling (lane odd).
      // The env's tile and patch corner come from its lane 4 el (wave-uniform readlane).
      const int cj = (lane >> 1) & 15, ci_l = lane >> 5;
      const size_t layer_off = (lane & 1) ? 0 : (size_t)nx;  // floor = layer 1, ceiling = layer 0
#pragma unroll
      for (int el2 = 0; el2 < SEPB; ++el2) {
        const int tix_s = __builtin_amdgcn_readlane(tix, 4 * el2);
        const int pi_s = __builtin_amdgcn_readlane(T.pi0, 4 * el2);
        const int pj_s = __builtin_amdgcn_readlane(T.pj0, 4 * el2);
        const float* tl = K.ter.tiles + (size_t)tix_s * 2 * nx * ny;
        const int gj = min(max(pj_s + cj, 0), ny - 1);
#pragma unroll
        for (int k = 0; k < PSZX / 2; ++k) {
          const int gi = min(max(pi_s + 2 * k + ci_l, 0), nx - 1);
          __builtin_amdgcn_global_load_lds(tl + (layer_off + gi) * ny + gj, (float*)&s_patch[el2][0] + 64 * k, 4, 0, 0);
        }
      }
    }
  }
  MARK(pro_dma_issued);
  asm volatile("" : "+v"(rebind_flag));  // kept in a VGPR: a scalar branch on it would wait early
  if (rebind && sub16 == 0 && rebind_flag) K.prev_extras[e] = rebind_val;
  float scaled[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    scaled[j] = act[j] * CI(action_scale);
    if (j == 0) scaled[j] = scaled[j] * CI(hip_scale_reduction);
  }

  // ---------------- decimation loop (:82-88)
  // The lag ring is pushed once per sim sub-step with the same scaled action
  // (:973), so sub-step s reads the slot s+1 of the incoming ring and the ring
  // leaves the step as [old4, old5, old6, scaled x 4].
  float torque[3], tgt[3];
  float cf_raw[6] = {0, 0, 0, 0, 0, 0}, cf_leg[9], cf_base[3];
  for (int sub = 0; sub < dec; ++sub) {
    // _compute_torques (:957-996)
    {
      // inputs of this lane's three joints ...
      // the ring's oldest slot after this sub-step's push (:973-974) is old slot sub + 1, i.e. the
      // scaled action of `back` steps ago (stored entry KL - back), or this step's for back = 0
      const int m = 6 - sub;
      const int back = m <= 0 ? 0 : (m + dec - 1) / dec;  // wave-uniform: scalar selects below
      float xin[3][6];
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        float lg = scaled[j];
#pragma unroll
        for (int k = 0; k < KMAX; ++k) lg = back == KL - k ? lag_pre[k][j] : lg;
        tgt[j] = lg + dflt[j];
        const float err = q[j] - tgt[j] + offset[j];
        xin[j][0] = err; xin[j][1] = eh[0][j]; xin[j][2] = eh[1][j];
        xin[j][3] = qd[j]; xin[j][4] = vh[0][j]; xin[j][5] = vh[1][j];
      }
      // ... -> 3 MFMA groups per wave: group j holds joint j of the 16 (env, leg) items
      // of the wave in column 4 env + leg; row (= role) q supplies inputs q and 4 + q of
      // its own leg and receives the item's torque in place.
      MARK(mlp_begin);
      float tq[3] = {0.0f, 0.0f, 0.0f};
      float b0[3], b1v[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const float* y = xin[j];
        b0[j] = sel4(lq, y[0], y[1], y[2], y[3]);
        b1v[j] = sel4(lq, y[4], y[5], 0.0f, 0.0f);
      }
#ifdef GO1_ABL_NO_MLP
#pragma unroll
      for (int j = 0; j < 3; ++j) tq[j] = 0.0f * (b0[j] + b1v[j]);  // ablation build only: no actuator net
#else
      mlp_group3(F, b0, b1v, tq);
#endif
#ifdef GO1_ABL_NO_MLP
#pragma unroll
      for (int j = 0; j < 3; ++j) tq[j] += -20.0f * xin[j][0] - 0.5f * xin[j][3];  // PD stand-in
#endif
      MARK(mlp_done);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        eh[1][j] = eh[0][j];
        eh[0][j] = xin[j][0];
        vh[1][j] = vh[0][j];
        vh[0][j] = qd[j];
        const float t = tq[j] * strength[j];
        const float lim = tlim[j];
        torque[j] = clampf(t, -lim, lim);
      }
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
#ifndef GO1_ABL_NO_PHYS
      for (int k = 0; k < c->n_internal; ++k) {
        const bool last = (sub == dec - 1) && (k == c->n_internal - 1);
        phys_substep(c, s_phys, P, torque, h, A.sim_gravity, friction, payload, T, leg, role, last, cf_raw);
      }
#else
      P.qd[0] += 1e-4f * torque[0]; P.qd[1] += 1e-4f * torque[1]; P.qd[2] += 1e-4f * torque[2];
#endif
#pragma unroll
      for (int j = 0; j < 3; ++j) { q[j] = P.q[j]; qd[j] = P.qd[j]; }
    }
    if (A.dbg_torques && owner) {
#pragma unroll
      for (int j = 0; j < 3; ++j) A.dbg_torques[((size_t)sub * n + e) * NDOF + leg * 3 + j] = torque[j];
    }
  }
  cf_sum(cf_raw, role, cf_leg, cf_base);
  float root[13];
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
      root[i] = P.pos[i]; root[7 + i] = P.wv[i].y; root[10 + i] = P.wv[i].x;
    }
    root[0] = P.pos[0] + org_x;
    root[1] = P.pos[1] + org_y;
#pragma unroll
    for (int i = 0; i < 4; ++i) root[3 + i] = P.quat[i];
  }
  // height scan (:1918-1965) samples at the post-physics, pre-reset pose: the gathers are
  // issued here and consumed by the height observations at the end
  const bool hplane = CI(terrain_kind) == 0;
  const float scan_x = root[0], scan_y = root[1];
  // camera_pitch_angle (:1934-1939): the previous step's pitch, or 0 with rotate_camera
  const float cam_p = CI(rotate_camera) ? 0.0f : cam_pitch;
  float camx = 0.0f, camy = 0.0f;
  if (!hplane) {
    const float cos_p = pm_cosf(cam_p);
    camx = CI(camera_offset_x) * cos_p;
    camy = 0.0f * cos_p;
  }
  auto sample = [&](int i, int j, float& h0, float& h1) {
    if (hplane) { h0 = 1.0f; h1 = 0.0f; return; }
    float px = s_phys[LDS_GX + i] + scan_x;
    float py = s_phys[LDS_GY + j] + scan_y;
    if (CI(camera_zero)) { px = px + camx; py = py + camy; }
    px = px - org_x;
    py = py - org_y;
    // .long() truncation then clip (:1948-1952); the float is bounded first so that a
    // non-finite pose cannot turn the conversion into undefined behaviour
    const float fx = fminf(fmaxf(px / CI(horizontal_scale), -1.0f), (float)CI(hf_nx));
    const float fy = fminf(fmaxf(py / CI(horizontal_scale), -1.0f), (float)CI(hf_ny));
    int ix = (int)fx, iy = (int)fy;
    ix = ix < 0 ? 0 : (ix > CI(hf_nx) - 2 ? CI(hf_nx) - 2 : ix);
    iy = iy < 0 ? 0 : (iy > CI(hf_ny) - 2 ? CI(hf_ny) - 2 : iy);
    h0 = T.tile[(size_t)ix * CI(hf_ny) + iy];
    h1 = T.tile[((size_t)CI(hf_nx) + ix) * CI(hf_ny) + iy];
  };
  const int x_start = CI(measure_front_half) ? GO1_GRID_X / 2 + 1 : 0;
  const int n_pts = (GO1_GRID_X - x_start) * GO1_GRID_Y;
  // the env's 16 lanes take points sub16 + 16 k (KPTS = 7 for the 110 front-half points, 15 for all 231)
  float hv[KPTS][2];
#ifdef GO1_ABL_NO_SCAN  // ablation build only: no height-scan gathers
  const bool scan = false;
#else
  const bool scan = CI(observe_heights) != 0;
#endif
#pragma unroll
  for (int k = 0; k < KPTS; ++k) {
    const int p = min(sub16 + 16 * k, n_pts - 1);
    hv[k][0] = hv[k][1] = 0.0f;
    if (scan) sample(x_start + p / GO1_GRID_Y, p % GO1_GRID_Y, hv[k][0], hv[k][1]);
  }

  if (A.contact_forces && owner) {
    float* o = A.contact_forces + (size_t)e * NB * 3;
    if (leg == 0) { o[0] = cf_base[0]; o[1] = cf_base[1]; o[2] = cf_base[2]; }
    float* ol = o + (1 + leg * 4) * 3;
    ol[0] = 0.0f; ol[1] = 0.0f; ol[2] = 0.0f;  // hip: no contact geometry in the native model
#pragma unroll
    for (int i = 0; i < 9; ++i) ol[3 + i] = cf_leg[i];
  }

  MARK(post_begin);
  // ================= post_physics_step (:114-169), contraction off =================
  const int ep = ep_in + 1;
  float blv[3], bav[3], pg[3], rpy[3], rel_lin[3], rel_rot[3];
  auto post_kin = [&](const float* tr) {
    const float qb[4] = {root[3], root[4], root[5], root[6]};
    quat_rotate_inverse_f(qb, root + 7, blv);
    quat_rotate_inverse_f(qb, root + 10, bav);
    quat_rotate_inverse_f(qb, A.gravity_vec, pg);
    // _plan_target_pose / _compute_relative_target_pose (:850-932)
    const float rel_in[3] = {tr[0] - root[0], tr[1] - root[1], tr[2] - root[2]};
    quat_apply_yaw_inverse_f(qb, rel_in, rel_lin);
    quat_to_rpy_f(qb, rpy);
#pragma unroll
    for (int i = 0; i < 3; ++i) rel_rot[i] = wrap_to_pi_f(tr[3 + i] - rpy[i]);
  };
  post_kin(traj_in);
  float cmd[2] = {rel_lin[0], rel_lin[1]};

  MARK(post_kin_done);
  // DR every rand_interval (:822-824)
  const bool dr_step = ep % CI(rand_interval) == 0;
  if (dr_step) {
    const float sv = rng(34) * CI(strength_range) + CI(strength_lo);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      strength[j] = sv;
      offset[j] = rng(35 + leg * 3 + j) * CI(offset_range) + CI(offset_lo);
    }
  }
  const float rel_norm = norm2_f(rel_lin[0], rel_lin[1]);
  const bool switched = rel_norm < CI(switch_dist);
  // waypoint switch, capped at the last waypoint (:836-844)
  int idx = idx_in;
  if (switched) { idx += 1; if (idx > TL - 1) idx = TL - 1; }
  const bool reached = switched && idx == TL - 1;
  // collision count (:848): this lane's thigh + calf, base on lane 0
  float coll_l = (norm3_f(cf_leg[0], cf_leg[1], cf_leg[2]) > 0.1f ? 1.0f : 0.0f) +
                 (norm3_f(cf_leg[3], cf_leg[4], cf_leg[5]) > 0.1f ? 1.0f : 0.0f);
  if (leg == 0 && norm3_f(cf_base[0], cf_base[1], cf_base[2]) > 0.1f) coll_l += 1.0f;
  const float coll = qsum(coll_l);

  // check_termination (:198-216)
  const bool time_out = (float)ep > CI(max_episode_length);
  bool reset = time_out, diverged = false;
  if (CI(use_terminal_body_height) && root[2] < CI(terminal_body_height)) reset = true;
  if (CI(terminate_end_of_trajectory) && reached && (float)ep > CI(t_reach)) reset = true;  // (:211-213)
  if (CI(use_terminal_body_rotation) && pg[2] > 0.0f) reset = true;                        // (:215-216)
  if (!INJ) {
    // native-integrator divergence guard (no reference counterpart: PhysX does not
    // return non-finite states): an env whose state is not finite, or beyond
    // GO1_DIVERGED in any component, is reset, and nothing of its diverged state reaches
    // an output (zero reward, post-reset observations, see below)
    bool finite = true;
#pragma unroll
    for (int i = 0; i < 13; ++i) finite = finite && fabsf(root[i]) < GO1_DIVERGED;
#pragma unroll
    for (int j = 0; j < 3; ++j) finite = finite && fabsf(q[j]) < GO1_DIVERGED && fabsf(qd[j]) < GO1_DIVERGED;
    diverged = qsum(finite ? 0.0f : 1.0f) != 0.0f;
    if (diverged) reset = true;
    if (diverged && sub16 == 0 && A.diverged_count) atomicAdd((unsigned long long*)A.diverged_count, 1ull);
  }

  MARK(termination_done);
  // ---- compute_reward (:320-355): the container's functions (reward_crawling.py,
  // trajectory_tracking_reward.py) for the terms with a nonzero scale.  Every lane of an env
  // holds the same term values; the env's lane sub16 == 0 files them in an LDS row by term id,
  // and the reward is then summed in slot (reward_scales) order.  One wave per block: the
  // wave's LDS operations complete in order, no barrier.
  __shared__ float s_terms[SEPB][GO1_T_COUNT];
  const uint32_t tm = CI(term_mask);
#define PUT(id, v)                          \
  do {                                      \
    const float v_ = (v);                   \
    if (sub16 == 0) s_terms[el][(id)] = v_; \
  } while (0)
  const float vxy2 = sq_f(blv[0]) + sq_f(blv[1]);
  const float vmag = norm2_f(blv[0], blv[1]);
  const float mag = rel_norm;
  // the target velocity towards the waypoint (reward_crawling.py:83-87, trajectory_tracking_reward.py:79-85)
  float tx = rel_lin[0] / (mag + 1e-6f) * CI(target_lin_vel);
  float ty = rel_lin[1] / (mag + 1e-6f) * CI(target_lin_vel);
  {
    const float gate = mag > CI(lin_reaching_criterion) ? 1.0f : 0.0f;
    tx = tx * gate;
    ty = ty * gate;
  }
  const float le = sq_f(tx - blv[0]) + sq_f(ty - blv[1]);
  {
    float x[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) x[j] = sq_f(torque[j]);
    PUT(GO1_T_TORQUES, qsum((x[0] + x[1]) + x[2]));
#pragma unroll
    for (int j = 0; j < 3; ++j) x[j] = sq_f((ldv[j] - qd[j]) / CI(dt));
    PUT(GO1_T_DOF_ACC, qsum((x[0] + x[1]) + x[2]));
#pragma unroll
    for (int j = 0; j < 3; ++j) x[j] = sq_f(la[j] - act[j]);
    PUT(GO1_T_ACTION_RATE, qsum((x[0] + x[1]) + x[2]));
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int d = leg * 3 + j;
      const float lo = q[j] - s_phys[LDS_DPL + 2 * d];
      const float hi = q[j] - s_phys[LDS_DPL + 2 * d + 1];
      const float o = -(lo < 0.0f ? lo : 0.0f);
      x[j] = o + (hi > 0.0f ? hi : 0.0f);
    }
    PUT(GO1_T_DOF_POS_LIMITS, qsum((x[0] + x[1]) + x[2]));
  }
  PUT(GO1_T_COLLISION, coll);
  PUT(GO1_T_BASE_HEIGHT, sq_f(root[2] - CI(base_height_target)));
  PUT(GO1_T_ANG_VEL_XY, sq_f(bav[0]) + sq_f(bav[1]));
  PUT(GO1_T_ORIENTATION, sq_f(pg[0]) + sq_f(pg[1]));
  PUT(GO1_T_LARGE_VEL, vxy2 * (vmag > 0.5f ? 1.0f : 0.0f));  // reward_crawling.py:53-56
  PUT(GO1_T_LIN_VEL_Z, sq_f(blv[2]));
  PUT(GO1_T_REACHING_Z, sq_f(rel_lin[2]));
  PUT(GO1_T_REACHING_ROLL, sq_f(rel_rot[0]));
  PUT(GO1_T_REACHING_PITCH, sq_f(rel_rot[1]));
  PUT(GO1_T_REACHING_YAW_ABS, sq_f(rel_rot[2]));
  PUT(GO1_T_SURVIVE, 1.0f);
  {
    const float rch = reached ? 1.0f : 0.0f, after = (float)ep > CI(t_reach) ? 1.0f : 0.0f;
    PUT(GO1_T_REACH_GOAL, rch);
    PUT(GO1_T_REACH_GOAL_T, rch * (float)ep);
    PUT(GO1_T_REACH_GOAL_TR, rch * after);
    PUT(GO1_T_LINEAR_VEL, norm3_f(blv[0], blv[1], blv[2]) > 0.7f ? 1.0f : 0.0f);
    PUT(GO1_T_STALLING, -((vmag < CI(small_vel_threshold) && mag > CI(large_dist_threshold)) ? 1.0f : 0.0f));
    // e2e (reward_crawling.py:61-77)
    const float r_e2e = expf(-vxy2 / CI(tracking_sigma_lin)) * (mag < CI(switch_dist) ? 1.0f : 0.0f) * after;
    const float r_end = (mag < CI(switch_dist) ? 1.0f : 0.0f) * CI(max_episode_length);
    PUT(GO1_T_E2E, CI(terminate_end_of_trajectory) ? r_end : r_e2e);
  }
  {  // exploration_lin (reward_crawling.py:79-108) / reaching_linear_vel
    const int form = CI(lin_vel_form);
    float r = expf(-le / CI(tracking_sigma_lin));
    r = form == 1 ? fabsf(tx - blv[0]) + fabsf(ty - blv[1]) : r;
    r = form == 2 ? le : r;
    if (form == 3) {
      const float rx = tx / CI(target_lin_vel) * blv[0] / (vmag + 1e-6f);
      const float ry = ty / CI(target_lin_vel) * blv[1] / (vmag + 1e-6f);
      r = rx + ry;
      r = r * (vmag > CI(small_vel_threshold) ? 1.0f : 0.0f);
      r = r + expf(-(vmag * vmag) / CI(tracking_sigma_lin)) * (mag < CI(lin_reaching_criterion) ? 1.0f : 0.0f);
    }
    PUT(GO1_T_EXPLORATION_LIN, r);
  }
  {  // exploration_yaw (reward_crawling.py:110-120) / reaching_yaw
    float ta = rel_rot[2];
    const float m = fabsf(ta);
    ta = ta / (m + 1e-6f) * CI(target_ang_vel);
    ta = ta * (m > CI(ang_reaching_criterion) ? 1.0f : 0.0f);
    PUT(GO1_T_EXPLORATION_YAW, expf(-sq_f(ta - bav[2]) / CI(tracking_sigma_ang)));
  }
  // the rest of TrajectoryTrackingRewards, only when one of them is scaled
  constexpr uint32_t TT_HEAVY = (1u << GO1_T_DOF_VEL) | (1u << GO1_T_DOF_POS) | (1u << GO1_T_TASK) |
                                (1u << GO1_T_TASK_OLD) | (1u << GO1_T_EXPLORATION);
  if (tm & TT_HEAVY) {
    float x[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) x[j] = sq_f(qd[j]);
    PUT(GO1_T_DOF_VEL, qsum((x[0] + x[1]) + x[2]));  // trajectory_tracking_reward.py:21-23
#pragma unroll
    for (int j = 0; j < 3; ++j) x[j] = sq_f(q[j] - s_phys[LDS_DDP + leg * 3 + j]);
    PUT(GO1_T_DOF_POS, qsum((x[0] + x[1]) + x[2]));  // :31-33
    // task (:74-89)
    PUT(GO1_T_TASK, expf(-le / CI(tracking_sigma_lin)) * (mag < CI(large_dist_threshold) ? 1.0f : 0.0f));
    {  // task_old (:51-55)
      float r = 0.5f / (0.5f + mag) / CI(t_reach);
      PUT(GO1_T_TASK_OLD, r * ((float)ep > CI(t_reach) ? 1.0f : 0.0f));
    }
    {  // exploration (:91-99)
      float r = blv[0] * rel_lin[0] + blv[1] * rel_lin[1];
      r = r / (mag + 1e-6f);
      r = r / (vmag + 1e-6f);
      PUT(GO1_T_EXPLORATION, r * (vmag > CI(small_vel_threshold) ? 1.0f : 0.0f));
    }
  }
  // feet_air_time (trajectory_tracking_reward.py:126-137) mutates last_contacts / feet_air_time
  float air_new = 0.0f, lc_new = 0.0f;
  if ((tm >> GO1_T_FEET_AIR_TIME) & 1u) {
    float air = st.feet_air_time[(size_t)e * 4 + leg];
    const float lc = st.last_contacts[(size_t)e * 4 + leg];
    const bool contact = cf_leg[8] > 1.0f;  // foot z force
    const bool filt = contact || lc != 0.0f;
    lc_new = contact ? 1.0f : 0.0f;
    const bool first = air > 0.0f && filt;
    air = air + CI(dt);
    const float r = (air - 0.5f) * (first ? 1.0f : 0.0f);
    air_new = air * (filt ? 0.0f : 1.0f);
    PUT(GO1_T_FEET_AIR_TIME, qsum(r));
  }
#undef PUT
  // slot order: rew_buf += term * scale (:326-340).  Lane k forms slot k's scaled reward and
  // updates its episode sum; every lane then adds the slots up in order from LDS.  pos / neg bucket
  // by the sign of the sum over envs, which for a sign-definite term is the sign of its scale.
  __shared__ float s_r[SEPB][GO1_MAX_TERMS];
  const bool global_buckets = CI(indefinite_slots) != 0;
  const bool live = (CI(live_slots) >> sub16) & 1u;
  {
    float t = live ? s_terms[el][my_id] : 0.0f;
    if (diverged) t = 0.0f;
    if (A.dbg_terms && sub16 < NT) A.dbg_terms[(size_t)e * GO1_MAX_TERMS + sub16] = t;
    const float r = t * my_scale;
    s_r[el][sub16] = r;
    if (live) my_sum = my_sum + r;
    if (global_buckets && live) {
      K.bucket_r[(size_t)e * GO1_MAX_TERMS + sub16] = r;
      atomicAdd(K.bucket_sum + sub16, (double)r);
    }
  }
  // sign of each slot's scale, as a slot bitmask (every env of the wave has the same scales):
  // slot k of env 0 is lane 16 (k >> 2) + (k & 3)
  const uint64_t nonneg = __ballot(my_scale >= 0.0f);
  const uint32_t posm = (uint32_t)((nonneg & 0xFull) | ((nonneg >> 12) & 0xF0ull) | ((nonneg >> 24) & 0xF00ull) |
                                   ((nonneg >> 36) & 0xF000ull));
  const uint32_t livem = CI(live_slots);
  float rew = 0.0f, pos = 0.0f, neg = 0.0f;
  {
    float rr[GO1_MAX_TERMS];
#pragma unroll
    for (int k = 0; k < GO1_MAX_TERMS; ++k) rr[k] = s_r[el][k];
#pragma unroll
    for (int k = 0; k < GO1_MAX_TERMS; ++k) {
      if ((livem >> k) & 1u) {
        rew = rew + rr[k];
        if ((posm >> k) & 1u) pos = pos + rr[k]; else neg = neg + rr[k];
      }
    }
  }
  if (CI(reward_mode) == 1) rew = rew < 0.0f ? 0.0f : rew;            // only_positive_rewards (:341-342)
  else if (CI(reward_mode) == 2) rew = pos * expf(neg / CI(sigma_rew_neg));  // ji22 style (:343-344)
  // episode sums total / total_pos / total_neg (:346-348); with global buckets the bucket launch
  // adds total_pos / total_neg (and the ji22 reward)
  if (sub16 == 0 && !(global_buckets && CI(reward_mode) == 2)) my_tot = my_tot + rew;
  if (!global_buckets) {
    if (sub16 == 1) my_tot = my_tot + pos;
    if (sub16 == 2) my_tot = my_tot + neg;
  }

  MARK(rewards_done);
  // ---- reset_idx (:218-296); the height scan below still samples at the pre-reset pose
  float traj_new[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) traj_new[i] = traj_in[i];
  const int LOGW = NT + 6;
  const bool compact = A.episode_log_count != nullptr;
  if (A.episode_log && !compact && owner && leg == 0 && !reset) A.episode_log[(size_t)e * LOGW + NS] = 0.0f;
  // compact log: the wave's reset envs append their rows (LOGW + 2 wide: + step tag, env id)
  // at one atomic per wave; the host orders the rows by (tag, env) as the reference logs them
  int log_row = -1;
  if (compact) {
    const uint64_t rmask = __ballot(reset && owner && leg == 0);  // lane 4 el: env el's role 0, leg 0
    if (rmask != 0ull) {
      int base = 0;
      if (lane == 0) base = atomicAdd(A.episode_log_count, __popcll(rmask));
      base = __shfl(base, 0);
      log_row = base + __popcll(rmask & ((1ull << (4 * el)) - 1ull));
      if (log_row >= A.episode_log_cap) log_row = -1;  // dropped; the count keeps it (the host reports overflow)
    }
  }
  if (reset && A.episode_log && (!compact || log_row >= 0)) {
    // reset_idx logging (:256-271): pre-reset sums, episode length, reached, goal distance
    float* lg = compact ? A.episode_log + (size_t)log_row * (LOGW + 2) : A.episode_log + (size_t)e * LOGW;
    if (compact && sub16 == 0) {
      lg[LOGW] = (float)A.episode_log_tag;
      lg[LOGW + 1] = (float)e;
    }
    if (sub16 < NT) lg[sub16] = my_sum;
    if (sub16 < 3) lg[NT + sub16] = my_tot;
    if (sub16 == 0) {
      lg[NS] = (float)ep;
      lg[NS + 1] = reached ? 1.0f : 0.0f;
      lg[NS + 2] = diverged ? 0.0f : norm3_f(rel_lin[0], rel_lin[1], rel_lin[2]);
    }
  }
  if (reset) {
#ifndef GO1_ABL_NO_RESET  // ablation build only: resets keep the state
    {
      // the reset's uniforms (slots 0 .. 35 = Philox blocks 0 .. 8): lane sub16 < 9 of the env
      // draws block sub16 (one evaluation per lane instead of one per draw), the env's lanes read
      // them back from LDS (one wave per block: its LDS operations complete in order)
      __shared__ float s_ru[SEPB][GO1_RESET_SLOTS];
      if (sub16 < GO1_RESET_SLOTS / 4) {
        float uq[4];
        rng.quad(sub16, uq);
#pragma unroll
        for (int k = 0; k < 4; ++k) s_ru[el][4 * sub16 + k] = uq[k];
      }
      const float* ru = s_ru[el];
      auto u = [ru](int slot) { return ru[slot]; };
      reset_env(c, u, rng, eo_pre, leg, s_phys + LDS_DDP, root, q, qd, strength, offset, traj_new);
    }
    write_trajectory(c, rng, root, st.trajectory + (size_t)e * 6 * TL, sub16, 16);
#endif
    idx = 0;
    my_sum = 0.0f;
    my_tot = 0.0f;
    air_new = 0.0f;  // feet_air_time[env_ids] = 0 (:248); last_contacts is kept
    cmd[0] = 0.0f;  // commands is a view of local_relative_linear, zeroed by reset_idx (:252, :802)
    cmd[1] = 0.0f;
    // a diverged env observes (and stores as its pitch) its post-reset pose instead, and its
    // actuator-net history (pos_err / vel of the last sub-steps, never reset by reset_idx) is
    // cleared: it holds the diverged state, which would otherwise drive the next step's torques
    if (diverged) {
      post_kin(traj_new);
#pragma unroll
      for (int j = 0; j < 3; ++j) eh[0][j] = eh[1][j] = vh[0][j] = vh[1][j] = 0.0f;
    }
  }
  const int coll_count = reset ? 0 : coll_in + (int)coll;

  MARK(reset_done);
  // ---- compute_observations (:357-475)
  const int NO = CI(num_obs);
  float* o = A.obs + (size_t)e * NO;
  float* oh = A.obs_history ? A.obs_history + (size_t)e * NO : nullptr;  // optional second copy
  const float clip = CI(clip_obs);
  // noise uniforms rng(47 + i) (:472-473): every lane draws exactly two Philox blocks, the
  // same two-block code path in all lanes (the per-value calls of the two store branches
  // ran five Philox evaluations per wave, one after the other): role r < 3 needs slots
  // 52 + d (dof pos) and 64 + d (dof vel), role 3 slots 47, 48, 49 (gravity)
  const int dn = leg * 3 + (role < 3 ? role : 0);
  float uA[4], uB[4];
  {
    const int sa = role < 3 ? 52 + dn : 44, sb = role < 3 ? 64 + dn : 48;
    if (CI(add_noise)) {
      rng.quad(sa >> 2, uA);
      rng.quad(sb >> 2, uB);
    }
  }
  auto put = [&](int i, float v, float nv, float u, bool noisy) {
    if (noisy && CI(add_noise)) v = v + (2.0f * u - 1.0f) * nv;
    v = clampf(v, -clip, clip);
    o[i] = v;
    if (oh) oh[i] = v;
  };
  // role r < 3 writes joint r of its leg; role 3 of leg 0 writes gravity and commands, role 3
  // of leg 1 the episode progress (timestep_in_obs, :375-377: post-reset episode length)
  if (role == 3 && leg == 0) {
    put(0, pg[0], CI(noise_gravity), uA[3], true);
    put(1, pg[1], CI(noise_gravity), uB[0], true);
    put(2, pg[2], CI(noise_gravity), uB[1], true);
    put(3, cmd[0] * 1.0f, 0.0f, 0.0f, false);
    put(4, cmd[1] * 1.0f, 0.0f, 0.0f, false);
  }
  if (CI(timestep_in_obs) && role == 3 && leg == 1)
    put(41, (float)(reset ? 0 : ep) / CI(max_episode_length), 0.0f, 0.0f, false);
  if (role < 3) {
    const int j = role, d = dn;
    const float qj = sel3(j, q), qdj = sel3(j, qd), aj = sel3(j, act);
    const float un = sel4((52 + d) & 3, uA[0], uA[1], uA[2], uA[3]);
    const float uv = sel4((64 + d) & 3, uB[0], uB[1], uB[2], uB[3]);
    put(5 + d, (qj - s_phys[LDS_DDP + d]) * CI(obs_scale_dof_pos), CI(noise_dof_pos), un, true);
    put(17 + d, qdj * CI(obs_scale_dof_vel), CI(noise_dof_vel), uv, true);
    put(29 + d, aj, 0.0f, 0.0f, false);
  }
  MARK(obs_props_done);
  // height observations (:395-411) from the samples gathered after the physics
  if (scan) {
    const int o_h = 41 + CI(timestep_in_obs);
    const float zroot = root[2];  // post-reset (:401)
    const float cam_z = pm_sinf(cam_p) * CI(camera_offset_norm);
#pragma unroll
    for (int k = 0; k < KPTS; ++k) {
      const int p = sub16 + 16 * k;
      if (p < n_pts) {
#pragma unroll
        for (int layer = 0; layer < 2; ++layer) {
          float hh = hv[k][layer];
          if (CI(camera_zero)) {
            hh = hh - zroot;
            hh = hh - cam_z;
            hh = clampf(hh, -0.3f, 0.3f);
          } else {
            hh = clampf(hh, 0.0f, CI(ceiling_height));
            hh = hh / CI(ceiling_height);
            hh = hh - 0.5f;
          }
          const float v = clampf(hh * CI(obs_scale_heights), -clip, clip);
          o[o_h + layer * n_pts + p] = v;
          if (oh) oh[o_h + layer * n_pts + p] = v;
        }
      }
    }
  }
  MARK(heights_done);
  if (A.dbg_heights) {
    float* od = A.dbg_heights + (size_t)e * 2 * GO1_GRID_X * GO1_GRID_Y;
    for (int p = sub16; p < GO1_GRID_X * GO1_GRID_Y; p += 16) {
      float h0, h1;
      sample(p / GO1_GRID_Y, p % GO1_GRID_Y, h0, h1);
      od[p] = h0;
      od[GO1_GRID_X * GO1_GRID_Y + p] = h1;
    }
  }
  if (sub16 == 0) {
    float* pv = A.priv + (size_t)e * GO1_NUM_PRIV;
    pv[0] = clampf((friction - CI(priv_friction_shift)) * CI(priv_friction_scale), -clip, clip);
    pv[1] = clampf((restitution - CI(priv_rest_shift)) * CI(priv_rest_scale), -clip, clip);
  }

  MARK(priv_done);
  if (A.aux) {
    // TrajectoryTrackingEnv.step extras (trajectory_tracking/__init__.py:25-41), post-reset state
    float* ax = A.aux + (size_t)e * GO1_AUX;
    if (role == 2 && leg == 0) {
#pragma unroll
      for (int i = 0; i < 3; ++i) { ax[i] = blv[i]; ax[3 + i] = bav[i]; }
      ax[6] = cmd[0];
      ax[7] = cmd[1];
    }
    if (role == 1) {
      float fp[3];
      foot_world(c_gen->model, root, q, leg, fp);
#pragma unroll
      for (int i = 0; i < 3; ++i) ax[8 + leg * 3 + i] = fp[i];
    }
    if (owner)
#pragma unroll
      for (int i = 0; i < 3; ++i) ax[20 + leg * 3 + i] = diverged ? 0.0f : torque[i];
  }

  MARK(aux_done);
  // ---------------- write back (epilogue :148-153): role r < 3 stores joint r of its
  // leg, role 3 of leg 0 stores the env-level state
#ifdef GO1_ABL_NO_STORE  // ablation build only: no state write-back
  if (false) {
#else
  if (role < 3) {
#endif
    const int j = role;
    auto pick = [&](const float* v3) { return sel3(j, v3); };
    const size_t dj = d0 + j;
    st.dof_pos[dj] = pick(q);
    st.dof_vel[dj] = pick(qd);
    st.last_actions[dj] = pick(act);
    st.last_dof_vel[dj] = pick(qd);
    if (reset || dr_step) {  // changed only by a reset or the DR re-randomisation (:822-824)
      st.motor_strength[dj] = pick(strength);
      st.motor_offset[dj] = pick(offset);
    }
    st.joint_pos_target[dj] = pick(tgt);
    // stored lag shifts by one step: entries 1 .. KL - 1 (from the prologue's registers: a reload
    // would put an L2 round trip at every wave's end), then this step's scaled action
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
      if (k < KL) st.lag[(size_t)e * 12 * KL + k * 12 + leg * 3 + j] =
          reset ? 0.0f : (k == KL - 1 ? pick(scaled) : pick(lag_pre[k + 1 < KMAX ? k + 1 : k]));
    st.pos_err_hist[(size_t)e * 24 + leg * 3 + j] = pick(eh[0]);
    st.pos_err_hist[(size_t)e * 24 + 12 + leg * 3 + j] = pick(eh[1]);
    st.vel_hist[(size_t)e * 24 + leg * 3 + j] = pick(vh[0]);
    st.vel_hist[(size_t)e * 24 + 12 + leg * 3 + j] = pick(vh[1]);
  }
  if (role == 3 && (tm >> GO1_T_FEET_AIR_TIME) & 1u) {
    st.feet_air_time[(size_t)e * 4 + leg] = air_new;
    st.last_contacts[(size_t)e * 4 + leg] = lc_new;
  }
  if (role == 3 && leg == 0) {
#pragma unroll
    for (int i = 0; i < 13; ++i) st.root[(size_t)e * 13 + i] = root[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) st.base_rotation[(size_t)e * 3 + i] = rpy[i];
    st.episode_length[e] = reset ? 0 : ep;
    st.curr_pose_index[e] = idx;
    st.collision_count[e] = coll_count;
    A.rew[e] = rew;
    A.reset[e] = reset;
    A.time_out[e] = time_out;
    if (A.dbg_commands) { A.dbg_commands[e * 2] = cmd[0]; A.dbg_commands[e * 2 + 1] = cmd[1]; }
    if (A.dbg_reached) A.dbg_reached[e] = reached;
  }
  if (sub16 < NT) st.episode_sums[(size_t)e * NS + sub16] = my_sum;
  if (sub16 < 3) st.episode_sums[(size_t)e * NS + NT + sub16] = my_tot;
  // one atomic per wave when any env of the wave reset (extras["time_outs"] rebinding, :289-291)
  if (__ballot(reset && leg == 0) != 0ull && (threadIdx.x & 63) == 0) atomicOr(K.flags + K.cur, 1);
  MARK(kernel_end);
}

// extras["time_outs"] = time_out of the last step, if any env reset in it (go1_sync_time_outs:
// the rebinding of that step, applied on demand; idempotent).
__global__ void go1_finalize_kernel(int n, const int32_t* __restrict__ flag, const uint8_t* __restrict__ time_out,
                                    uint8_t* __restrict__ extras) {
  int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n && *flag) extras[e] = time_out[e];
}

// reset_idx (:218-296) of masked envs, or of a list of env ids (ids != nullptr: slot k of the
// list -> env ids[k]; out-of-range ids skipped)
__global__ __launch_bounds__(TPB) void go1_reset_kernel(const go1_config* __restrict__ c_gen, go1_state st,
                                                        go1_terrain ter, const uint8_t* __restrict__ mask,
                                                        const int32_t* __restrict__ ids, int n_ids,
                                                        const float* __restrict__ U, uint64_t seed, uint64_t step) {
  CCfg* __restrict__ c = (CCfg*)c_gen;
  const int leg = threadIdx.x & 3;
  const int slot = blockIdx.x * EPB + (threadIdx.x >> 2);
  int e;
  if (ids) {
    if (slot >= n_ids) return;
    e = ids[slot];
    if (e < 0 || e >= c->n_envs) return;
  } else {
    e = slot;
    if (e >= c->n_envs || !mask[e]) return;
  }
  const Rng rng = {U, seed, step, e, e + c->env_id_offset, c->u_per_env};
  float root[13], q[3], qd[3], strength[3], offset[3], traj[6];
  const float eo[3] = {ter.env_origins[(size_t)e * 3], ter.env_origins[(size_t)e * 3 + 1],
                       ter.env_origins[(size_t)e * 3 + 2]};
  reset_env(c, rng, rng, eo, leg, c_gen->default_dof_pos, root, q, qd, strength, offset, traj);
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
    for (int k = 0; k < GO1_LAG_STEPS(c->decimation); ++k)
      st.lag[(size_t)e * 12 * GO1_LAG_STEPS(c->decimation) + k * 12 + leg * 3 + j] = 0.0f;
  }
  write_trajectory(c, rng, root, st.trajectory + (size_t)e * 6 * c->traj_length, leg, 4);
  st.feet_air_time[(size_t)e * 4 + leg] = 0.0f;  // (:248)
  const int ns = c->n_terms + 3;
  for (int k = leg; k < ns; k += 4) st.episode_sums[(size_t)e * ns + k] = 0.0f;
  if (leg == 0) {
#pragma unroll
    for (int i = 0; i < 13; ++i) st.root[(size_t)e * 13 + i] = root[i];
    st.episode_length[e] = 0;
    st.curr_pose_index[e] = 0;
    st.collision_count[e] = 0;
  }
  (void)traj;
}

// Global pos / neg bucketing (:330-336) when some reward slot has no fixed sign: the step kernel
// recorded every env's scaled slot rewards and their sums over envs (f64); here each env's
// rew_buf_pos / rew_buf_neg are rebuilt in slot order with the reference's bucket test on the sum's
// sign, added to total_pos / total_neg (the state's episode sums, or the episode-log row of an env
// the step reset), and the ji22-style reward is formed (:343-344).
__global__ void go1_bucket_kernel(const go1_config* __restrict__ c, go1_state st, const float* __restrict__ r_all,
                                  const double* __restrict__ bsum, double* __restrict__ bsum_next,
                                  const uint8_t* __restrict__ reset, float* __restrict__ rew,
                                  float* __restrict__ episode_log) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int nt = c->n_terms, ns = nt + 3;
  if (blockIdx.x == 0 && threadIdx.x < GO1_MAX_TERMS) bsum_next[threadIdx.x] = 0.0;
  if (e >= c->n_envs) return;
  float pos = 0.0f, neg = 0.0f;
  for (int k = 0; k < nt; ++k) {
    if (c->term_ids[k] == GO1_T_NONE) continue;
    const float r = r_all[(size_t)e * GO1_MAX_TERMS + k];
    const double S = bsum[k];
    if (S >= 0.0) pos = pos + r;
    else if (S <= 0.0) neg = neg + r;
  }
  float* t = (reset[e] && episode_log) ? episode_log + (size_t)e * (nt + 6) + nt
                                       : (reset[e] ? nullptr : st.episode_sums + (size_t)e * ns + nt);
  if (c->reward_mode == 2) {
    const float rw = pos * expf(neg / c->sigma_rew_neg);
    rew[e] = rw;
    if (t) t[0] = t[0] + rw;
  }
  if (t) {
    t[1] = t[1] + pos;
    t[2] = t[2] + neg;
  }
}

__global__ __launch_bounds__(64) void go1_actuator_kernel(const go1_config* __restrict__ c,
                                                         const float* __restrict__ x, float* __restrict__ out,
                                                         int n) {
  const int lane = threadIdx.x & 63, q = lane >> 4;
  MlpFrag F;
  mlp_load(c->actuator, lane, F);
  const int n_groups = (n + 15) / 16;
  for (int g = blockIdx.x; g < n_groups; g += gridDim.x) {  // uniform per wave: all lanes stay active
    const int row = g * 16 + (lane & 15);
    const float* r = x + (size_t)min(row, n - 1) * 6;
    const float b0 = r[q];
    const float b1v = q < 2 ? r[4 + q] : 0.0f;
    const float t = mlp_group(F, b0, b1v);
    if (q == 0 && row < n) out[row] = t;
  }
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
  int32_t* d_flags = nullptr;  // 3 "some env reset in step k" words (k mod 3)
  float* d_bucket_r = nullptr;    // global reward bucketing scratch (indefinite_slots != 0)
  double* d_bucket_sum = nullptr; // 2 banks x GO1_MAX_TERMS
  uint64_t count = 0;          // go1_step calls so far
  bool spec = false;           // every GO1_SPEC_FIELDS value matches: the specialised kernel runs
  const uint8_t* prev_time_out = nullptr;
  uint8_t* prev_extras = nullptr;
};

static thread_local std::string g_err;

// the specialised kernel's values must match bit for bit (-0.0 and 0.0 are different constants)
template <class T>
static bool spec_eq(T a, T b) { return memcmp(&a, &b, sizeof(T)) == 0; }
static bool spec_match(const go1_config& c) {
  bool m = true;
#define GO1_SPEC_CHECK(f, v) m = m && spec_eq(c.f, (decltype(c.f))(v));
  GO1_SPEC_FIELDS(GO1_SPEC_CHECK)
#undef GO1_SPEC_CHECK
  // the specialised kernel keeps GO1_LAG_STEPS(4) = 2 stored lag entries in registers (the sub-step
  // loop itself stays run-time)
  return m && c.decimation == 4;
}

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
// the library's other translation units (go1_terrain.hip) report through the same message
int go1_internal_fail(int code, const std::string& msg) { return fail(code, msg); }

#define HIP_TRY(x)                                                                      \
  do {                                                                                  \
    hipError_t _e = (x);                                                                \
    if (_e != hipSuccess) return fail(GO1_E_HIP, std::string(#x ": ") + hipGetErrorString(_e)); \
  } while (0)

extern "C" {
#ifdef GO1_STAMPS
int go1_debug_stamps(void* host, size_t bytes) {
  if (bytes > sizeof(g_go1_stamps)) bytes = sizeof(g_go1_stamps);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_go1_stamps), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
#endif

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
  if (cfg->n_envs % EPB != 0)
    return fail(GO1_E_ARG, "go1_create: n_envs must be a multiple of 16 (one wave = 16 envs x 4 legs)");
  if (cfg->n_terms < 0 || cfg->n_terms > GO1_MAX_TERMS) return fail(GO1_E_ARG, "go1_create: n_terms");
  for (int k = 0; k < cfg->n_terms; ++k)
    if (cfg->term_ids[k] != GO1_T_NONE && (cfg->term_ids[k] < 0 || cfg->term_ids[k] >= GO1_T_COUNT))
      return fail(GO1_E_ARG, "go1_create: bad term id");
  if (cfg->traj_length < 1 || cfg->traj_length > GO1_MAX_TRAJ || cfg->traj_kind < 0 || cfg->traj_kind > 2 ||
      (cfg->traj_kind == 1 && (cfg->traj_interp < 1 || cfg->traj_length % cfg->traj_interp != 0)))
    return fail(GO1_E_ARG, "go1_create: trajectory shape");
  {
    const int n_pts = (cfg->measure_front_half ? GO1_GRID_X - (GO1_GRID_X / 2 + 1) : GO1_GRID_X) * GO1_GRID_Y;
    const int width = 41 + (cfg->timestep_in_obs ? 1 : 0) + (cfg->observe_heights ? 2 * n_pts : 0);
    if (cfg->num_obs != width) return fail(GO1_E_ARG, "go1_create: num_obs does not match the observation layout");
    const int traj_u = cfg->traj_kind == 1 ? 6 * (cfg->traj_length / cfg->traj_interp + 1)
                                           : (cfg->traj_kind == 2 ? 3 : 0);
    if (cfg->u_per_env != GO1_U_NOISE + width + traj_u) return fail(GO1_E_ARG, "go1_create: u_per_env");
  }
  for (int leg = 0; leg < 4; ++leg)  // joint offsets must have the sparsity the kernel exploits
    for (int j = 0; j < 3; ++j)
      for (int k = 0; k < 3; ++k)
        if (!((offset_mask(j) >> k) & 1) && cfg->model[13 * 10 + leg * 9 + j * 3 + k] != 0.0f)
          return fail(GO1_E_ARG, "go1_create: joint offsets must be hip (x, y, 0), thigh (0, y, 0), calf (0, 0, z)");
  // the integrator's model constants are compiled in (go1_model_consts.h): the block must match
  if (memcmp(cfg->model, GO1_MODEL_F32, sizeof(GO1_MODEL_F32)) != 0)
    return fail(GO1_E_ARG, "go1_create: model block differs from the compiled Go1 model "
                           "(regenerate csrc/go1_model_consts.h with tools/gen_model_consts.py)");
  for (int leg = 1; leg < 4; ++leg)  // the integrator reads leg 0's joint limits for every leg
    for (int k = 0; k < 6; ++k)
      if (cfg->hard_limits[leg * 6 + k] != cfg->hard_limits[k])
        return fail(GO1_E_ARG, "go1_create: hard joint limits must be the same for every leg");
  go1_handle* h = new (std::nothrow) go1_handle();
  if (!h) return fail(GO1_E_ARG, "go1_create: out of host memory");
  h->cfg = *cfg;
  h->spec = spec_match(*cfg);
  hipError_t e1 = hipMalloc(&h->d_cfg, sizeof(go1_config));
  hipError_t e2 = hipMalloc(&h->d_flags, 3 * sizeof(int32_t));
  if (e1 != hipSuccess || e2 != hipSuccess) {
    if (h->d_cfg) (void)hipFree(h->d_cfg);
    if (h->d_flags) (void)hipFree(h->d_flags);
    delete h;
    return fail(GO1_E_HIP, "go1_create: hipMalloc failed");
  }
  HIP_TRY(hipMemcpy(h->d_cfg, cfg, sizeof(go1_config), hipMemcpyHostToDevice));
  HIP_TRY(hipMemset(h->d_flags, 0, 3 * sizeof(int32_t)));
  if (cfg->indefinite_slots) {
    HIP_TRY(hipMalloc(&h->d_bucket_r, (size_t)cfg->n_envs * GO1_MAX_TERMS * sizeof(float)));
    HIP_TRY(hipMalloc(&h->d_bucket_sum, 2 * GO1_MAX_TERMS * sizeof(double)));
    HIP_TRY(hipMemset(h->d_bucket_r, 0, (size_t)cfg->n_envs * GO1_MAX_TERMS * sizeof(float)));
    HIP_TRY(hipMemset(h->d_bucket_sum, 0, 2 * GO1_MAX_TERMS * sizeof(double)));
  }
  *out = h;
  return GO1_OK;
}

int go1_bind(go1_handle* h, const go1_state* s, const go1_plane* planes) {
  if (!h || !s || !planes) return fail(GO1_E_ARG, "go1_bind: null argument (state and plane descriptors required)");
  const void* p[] = {s->root, s->dof_pos, s->dof_vel, s->last_actions, s->last_dof_vel, s->lag, s->pos_err_hist,
                     s->vel_hist, s->motor_strength, s->motor_offset, s->friction, s->restitution, s->payload,
                     s->episode_length, s->curr_pose_index, s->trajectory, s->base_rotation, s->collision_count,
                     s->episode_sums, s->joint_pos_target, s->feet_air_time, s->last_contacts};
  static_assert(sizeof(p) / sizeof(p[0]) == GO1_STATE_PLANES, "go1_state planes");
  static const char* names[GO1_STATE_PLANES] = {
      "root", "dof_pos", "dof_vel", "last_actions", "last_dof_vel", "lag", "pos_err_hist", "vel_hist",
      "motor_strength", "motor_offset", "friction", "restitution", "payload", "episode_length",
      "curr_pose_index", "trajectory", "base_rotation", "collision_count", "episode_sums", "joint_pos_target",
      "feet_air_time", "last_contacts"};
  const int64_t width[GO1_STATE_PLANES] = {13, 12, 12, 12, 12, 12 * GO1_LAG_STEPS(h->cfg.decimation), 24, 24, 12,
                                           12, 1, 1, 1, 1, 1,
                                           6 * (int64_t)h->cfg.traj_length, 3, 1, h->cfg.n_terms + 3, 12, 4, 4};
  for (int i = 0; i < GO1_STATE_PLANES; ++i) {
    const go1_plane& d = planes[i];
    const int dt = (i == 13 || i == 14 || i == 17) ? GO1_DTYPE_I32 : GO1_DTYPE_F32;
    if (!p[i]) return fail(GO1_E_ARG, std::string("go1_bind: state plane ") + names[i] + " is null");
    if (d.rows != h->cfg.n_envs || d.cols != width[i] || d.dtype != dt)
      return fail(GO1_E_ARG, std::string("go1_bind: state plane ") + names[i] + " must be (" +
                                 std::to_string(h->cfg.n_envs) + ", " + std::to_string(width[i]) + ") " +
                                 (dt == GO1_DTYPE_I32 ? "int32" : "float32"));
    if (d.col_stride != 1 || (d.rows > 1 && d.row_stride != d.cols))
      return fail(GO1_E_ARG, std::string("go1_bind: state plane ") + names[i] +
                                 " is not dense row-major (strides " + std::to_string(d.row_stride) + ", " +
                                 std::to_string(d.col_stride) + "): pass a contiguous tensor");
  }
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
  KArgs K;
  K.st = h->st;
  K.ter = h->ter;
  K.a = *a;
  K.flags = h->d_flags;
  K.cur = (int)(h->count % 3);
  K.prv = (int)((h->count + 2) % 3);
  K.nxt = (int)((h->count + 1) % 3);
  K.prev_time_out = h->prev_time_out;
  K.prev_extras = h->prev_extras;
  const int bank = (int)(h->count & 1);
  K.bucket_r = h->d_bucket_r;
  K.bucket_sum = h->d_bucket_sum ? h->d_bucket_sum + bank * GO1_MAX_TERMS : nullptr;
  dim3 grid(n / SEPB), block(TPB);
  const bool full = !h->cfg.measure_front_half;  // 231 scanned points: 15 per lane instead of 7
  if (a->episode_log_count && (!a->episode_log || a->episode_log_cap < 0 || h->cfg.indefinite_slots))
    return fail(GO1_E_ARG, "go1_step: a compact episode log needs episode_log, a capacity >= 0 and no indefinite "
                           "reward slots (their bucket pass rewrites rows by env)");
  // The optional event pair is attached to the kernel's own dispatch (hipExtLaunchKernelGGL: the
  // events take the dispatch packet's start / end timestamps, as a profiler's kernel trace does),
  // so ev_end - ev_begin is the kernel's duration without the queue work of separate event records.
  hipEvent_t e0 = (hipEvent_t)a->ev_begin, e1 = (hipEvent_t)a->ev_end;
  auto go = [&](auto kern) {
    if (e0 || e1) hipExtLaunchKernelGGL(kern, grid, block, 0, s, e0, e1, 0, h->d_cfg, K);
    else hipLaunchKernelGGL(kern, grid, block, 0, s, h->d_cfg, K);
  };
  if (inj) {  // parity mode: the README configuration replays through the specialised kernel too
    if (full) go(go1_step_kernel<true, 15, false>);
    else if (h->spec) go(go1_step_kernel<true, 7, true>);
    else go(go1_step_kernel<true, 7, false>);
  } else if (h->spec) {  // the README configuration (go1_spec.h): measure_front_half, 7 points per lane
    go(go1_step_kernel<false, 7, true>);
  } else {
    if (full) go(go1_step_kernel<false, 15, false>);
    else go(go1_step_kernel<false, 7, false>);
  }
  HIP_TRY(hipGetLastError());
  if (h->cfg.indefinite_slots) {
    hipLaunchKernelGGL(go1_bucket_kernel, dim3((n + 255) / 256), dim3(256), 0, s, h->d_cfg, h->st, h->d_bucket_r,
                       h->d_bucket_sum + bank * GO1_MAX_TERMS, h->d_bucket_sum + (bank ^ 1) * GO1_MAX_TERMS,
                       a->reset, a->rew, a->episode_log);
    HIP_TRY(hipGetLastError());
  }
h->prev_time_out = a->time_out;
  h->prev_extras = a->extras_time_outs;
  h->count++;
  return GO1_OK;
}

int go1_specialize(go1_handle* h, int enable) {
  if (!h) return fail(GO1_E_ARG, "go1_specialize: null handle");
  if (enable && !spec_match(h->cfg)) return fail(GO1_E_ARG, "go1_specialize: the config differs from the specialised one (go1_spec.h)");
  h->spec = enable != 0;
  return GO1_OK;
}

int go1_is_specialized(go1_handle* h) { return h && h->spec ? 1 : 0; }

int go1_sync_time_outs(go1_handle* h, void* stream) {
  if (!h) return fail(GO1_E_ARG, "go1_sync_time_outs: null handle");
  if (!h->prev_time_out) return GO1_OK;  // no step yet
  const int n = h->cfg.n_envs;
  hipLaunchKernelGGL(go1_finalize_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, n,
                     h->d_flags + (h->count + 2) % 3, h->prev_time_out, h->prev_extras);
  HIP_TRY(hipGetLastError());
  return GO1_OK;
}

int go1_time_outs_pending(go1_handle* h, int64_t out[3]) {
  if (!h || !out) return fail(GO1_E_ARG, "go1_time_outs_pending: null argument");
  out[0] = out[1] = out[2] = 0;
  if (!h->prev_time_out) return GO1_OK;  // no step yet: extras_time_outs is current
  out[0] = (int64_t)(uintptr_t)(h->d_flags + (h->count + 2) % 3);
  out[1] = (int64_t)(uintptr_t)h->prev_time_out;
  out[2] = (int64_t)(uintptr_t)h->prev_extras;
  return GO1_OK;
}

int go1_reset_envs(go1_handle* h, const uint8_t* mask, const float* uniforms, uint64_t rng_seed, uint64_t rng_step,
                   void* stream) {
  if (!h || !mask) return fail(GO1_E_ARG, "go1_reset_envs: null argument");
  if (!h->bound || !h->has_terrain) return fail(GO1_E_STATE, "go1_reset_envs: bind state and terrain first");
  const int n = h->cfg.n_envs;
  hipLaunchKernelGGL(go1_reset_kernel, dim3((n + EPB - 1) / EPB), dim3(TPB), 0, (hipStream_t)stream, h->d_cfg,
                     h->st, h->ter, mask, nullptr, 0, uniforms, rng_seed, rng_step);
  HIP_TRY(hipGetLastError());
  return GO1_OK;
}

int go1_reset_idx(go1_handle* h, const int32_t* ids, int32_t n_ids, const float* uniforms, uint64_t rng_seed,
                  uint64_t rng_step, void* stream) {
  if (!h || (!ids && n_ids > 0) || n_ids < 0) return fail(GO1_E_ARG, "go1_reset_idx: bad argument");
  if (!h->bound || !h->has_terrain) return fail(GO1_E_STATE, "go1_reset_idx: bind state and terrain first");
  if (n_ids == 0) return GO1_OK;  // reset_idx returns early on an empty list (:220-221)
  hipLaunchKernelGGL(go1_reset_kernel, dim3((n_ids + EPB - 1) / EPB), dim3(TPB), 0, (hipStream_t)stream, h->d_cfg,
                     h->st, h->ter, nullptr, ids, n_ids, uniforms, rng_seed, rng_step);
  HIP_TRY(hipGetLastError());
  return GO1_OK;
}

int go1_actuator_net(go1_handle* h, const float* x, float* out, int32_t n_rows, void* stream) {
  if (!h || !x || !out || n_rows < 0) return fail(GO1_E_ARG, "go1_actuator_net: bad argument");
  if (n_rows == 0) return GO1_OK;
  const int groups = (n_rows + 15) / 16;
  hipLaunchKernelGGL(go1_actuator_kernel, dim3(groups < 4096 ? groups : 4096), dim3(64), 0, (hipStream_t)stream,
                     h->d_cfg, x, out, n_rows);
  HIP_TRY(hipGetLastError());
  return GO1_OK;
}

int go1_destroy(go1_handle* h) {
  if (!h) return GO1_OK;
  if (h->d_cfg) (void)hipFree(h->d_cfg);
  if (h->d_flags) (void)hipFree(h->d_flags);
  if (h->d_bucket_r) (void)hipFree(h->d_bucket_r);
  if (h->d_bucket_sum) (void)hipFree(h->d_bucket_sum);
  delete h;
  return GO1_OK;
}

}  // extern "C"

/*
 * go1_oracle.c -- CPU ORACLE of the Go1 trajectory-tracking step.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or the timed CPU baseline) -- never as the thing measured or shipped.
 *
 * It restates, in plain C, the reference algorithm of
 *   go1_gym/envs/base/legged_robot_trajectory_tracking.py  (cited :line below)
 *   go1_gym/envs/rewards/reward_crawling.py               (RewardsCrawling)
 *   go1_gym/envs/trajectories/trajectory_function.py      (_traj_fn_fixed_target)
 *   go1_gym/utils/math_utils.py                            (quat_apply_yaw_inverse, wrap_to_pi, ...)
 *   isaacgym.torch_utils (absent; published formulas restated)
 * with every f32 operation in the order torch evaluates it, so that integer /
 * boolean outputs (height-scan indices, termination and reset masks) are
 * bit-exact.  Parity pinned by the tests/golden npz fixtures, generated from the
 * reference's own code (tests/golden/make_golden.py).
 *
 * The rigid-body dynamics (PhysX in the reference, a closed binary that is not
 * available) is replaced by this build's own floating-base articulated-body
 * algorithm + heightfield contact, restated here in f64 as the oracle for the
 * f32 HIP integrator.  Physics parity with PhysX is UNPINNED.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).
 */
#include <math.h>
#include <limits.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/go1_mi355x.h"
#include "portable_math.h"

/* Working precision of the native integrator restatement: double for the oracle
 * (libgo1_oracle.so), float for the like-for-like CPU timing baseline
 * (libgo1_oracle_f32.so, -DGO1O_REAL=float -fsingle-precision-constant; <tgmath.h>
 * makes sqrt/sin/cos/floor/fmin/fmax follow the argument type).  The post-physics
 * code is f32 in both builds (explicit sqrtf/expf/... calls). */
#ifndef GO1O_REAL
#define GO1O_REAL double
#endif
typedef GO1O_REAL real;
#include <tgmath.h>
#undef I /* <complex.h> (via <tgmath.h>) defines I; the model uses it as a field name */

#define NDOF 12
#define NB 17
#define PI_F 3.14159265358979323846f
#define TWO_PI_F ((float)(2.0 * 3.14159265358979323846))

/* ------------------------------------------------------------------ Philox */
/* Philox4x32-10 (Salmon et al., SC'11).  counter = (env, slot/4, step lo, step hi),
 * key = seed.  u = (x >> 8) * 2^-24 in [0, 1). */
static void philox4x32(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0;
    uint32_t h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
    uint32_t n0 = h1 ^ c[1] ^ k0, n2 = h0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = l1; c[2] = n2; c[3] = l0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}

float go1o_uniform(uint64_t seed, uint64_t step, uint32_t env, uint32_t slot) {
  uint32_t c[4] = {env, slot >> 2, (uint32_t)step, (uint32_t)(step >> 32)};
  philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  return (float)(c[slot & 3] >> 8) * (1.0f / 16777216.0f);
}

/* parity mode: caller uniforms of local env e; otherwise Philox keyed by the GLOBAL env id */
static float draw(const go1_config* c, const go1_step_args* a, const float* U, int e, int slot) {
  if (U) return U[(size_t)e * c->u_per_env + slot];
  return go1o_uniform(a->rng_seed, a->rng_step, (uint32_t)(e + c->env_id_offset), (uint32_t)slot);
}

/* ------------------------------------------------------------ actuator net */
/* eval_actuator_network (:1311-1320): Linear(6,32) softsign Linear(32,32) softsign
 * Linear(32,1).  The accumulation ORDER is the one the HIP kernel's f32 MFMA
 * tiles produce (v_mfma_f32_16x16x4_f32 is a k-ordered fmaf chain), so the two
 * are bit-identical; torch's own order is unspecified (tests use a tolerance):
 *   layer 1, unit u : acc = b1[u]; k = 0..7 ascending (inputs padded 6 -> 8 with zeros)
 *   layer 2, unit v : acc = b2[v]; k = 16 m + 4 q + r for m in 0..1, r in 0..3, q in 0..3
 *   layer 3         : p_q = fma chain over u = 16 m + 4 q + r (m, r ascending) from 0;
 *                     out = ((p0 + p1) + (p2 + p3)) + b3
 */
float go1o_actuator_eval(const float* W, const float x[6]) {
  const float *w1 = W, *b1 = W + 192, *w2 = W + 224, *b2 = W + 1248, *w3 = W + 1280, *b3 = W + 1312;
  float xp[8] = {x[0], x[1], x[2], x[3], x[4], x[5], 0.0f, 0.0f};
  float h1[32], h2[32];
  for (int u = 0; u < 32; ++u) {
    float acc = b1[u];
    for (int k = 0; k < 8; ++k) acc = fmaf(k < 6 ? w1[u * 6 + k] : 0.0f, xp[k], acc);
    h1[u] = acc / (fabsf(acc) + 1.0f);
  }
  for (int v = 0; v < 32; ++v) {
    float acc = b2[v];
    for (int m = 0; m < 2; ++m)
      for (int r = 0; r < 4; ++r)
        for (int q = 0; q < 4; ++q) {
          int k = 16 * m + 4 * q + r;
          acc = fmaf(w2[v * 32 + k], h1[k], acc);
        }
    h2[v] = acc / (fabsf(acc) + 1.0f);
  }
  float p[4];
  for (int q = 0; q < 4; ++q) {
    float a = 0.0f;
    for (int m = 0; m < 2; ++m)
      for (int r = 0; r < 4; ++r) {
        int u = 16 * m + 4 * q + r;
        a = fmaf(w3[u], h2[u], a);
      }
    p[q] = a;
  }
  return ((p[0] + p[1]) + (p[2] + p[3])) + b3[0];
}

void go1o_actuator_batch(const float* W, const float* x, float* out, int n) {
#pragma omp parallel for schedule(static)
  for (int i = 0; i < n; ++i) out[i] = go1o_actuator_eval(W, x + (size_t)i * 6);
}

/* ------------------------------------------------------- torch-order quats */
/* isaacgym.torch_utils.quat_rotate_inverse, q = (x, y, z, w) */
static void quat_rotate_inverse_f(const float* q, const float* v, float* out) {
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

/* math_utils.quat_apply_yaw_inverse: zero x,y of q, normalize, rotate inverse */
static void quat_apply_yaw_inverse_f(const float* q, const float* v, float* out) {
  float qy[4] = {0.0f, 0.0f, q[2], q[3]};
  float n2 = fmaf(qy[3], qy[3], fmaf(qy[2], qy[2], fmaf(qy[1], qy[1], qy[0] * qy[0])));
  float n = sqrtf(n2);
  if (n < 1e-9f) n = 1e-9f;
  for (int i = 0; i < 4; ++i) qy[i] = qy[i] / n;
  quat_rotate_inverse_f(qy, v, out);
}

/* torch.remainder for f32 divisor b > 0 */
static float remainder_f(float a, float b) {
  float m = fmodf(a, b);
  if (m != 0.0f && ((b < 0.0f) != (m < 0.0f))) m += b;
  return m;
}

/* math_utils.wrap_to_pi (in place, :20-24) */
static float wrap_to_pi_f(float a) {
  a = remainder_f(a, TWO_PI_F);
  if (a > PI_F) a = a - TWO_PI_F;
  return a;
}

/* quaternion_to_roll_pitch_yaw = wrap_to_pi(get_euler_xyz(q)) (math_utils.py:42-48) */
static void quat_to_rpy_f(const float* q, float* rpy) {
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

static float norm2_f(float x, float y) { return sqrtf(fmaf(y, y, x * x)); }
static float norm3_f(float x, float y, float z) { return sqrtf(fmaf(z, z, fmaf(y, y, x * x))); }
static float sq_f(float x) { return x * x; }

/* sum over the 12 dofs in the grouping the HIP kernel uses (one leg per lane:
 * ((x0+x1)+x2) per leg, then (leg0+leg1)+(leg2+leg3)).  torch's own CPU order
 * is not specified; the parity tests use a float tolerance against it. */
static float sum12_legs(const float* x) {
  float s[4];
  for (int l = 0; l < 4; ++l) s[l] = (x[3 * l] + x[3 * l + 1]) + x[3 * l + 2];
  return (s[0] + s[1]) + (s[2] + s[3]);
}

/* ====================================================================== */
/*                      native physics, f64 restatement                    */
/* ====================================================================== */
typedef struct { real m[6][6]; } M6;

typedef struct {
  real mass, com[3], I[3][3]; /* inertia about COM */
} Body;

typedef struct {
  Body base;
  Body leg[4][3];
  real origin[4][3][3]; /* joint origins in parent frame */
  real foot[3], foot_r, trunk_half[3], thigh_r, calf_r;
  real hip_r, hip_y[2]; /* hip capsule: radius, segment ends on the hip link's y axis (FL; mirrored by side) */
} Model;

static void load_model(const go1_config* c, Model* M) {
  const float* p = c->model;
  int k = 0;
  Body* bodies[13];
  bodies[0] = &M->base;
  for (int l = 0; l < 4; ++l)
    for (int j = 0; j < 3; ++j) bodies[1 + l * 3 + j] = &M->leg[l][j];
  for (int b = 0; b < 13; ++b) {
    Body* B = bodies[b];
    B->mass = p[k++];
    for (int i = 0; i < 3; ++i) B->com[i] = p[k++];
    real xx = p[k++], xy = p[k++], xz = p[k++], yy = p[k++], yz = p[k++], zz = p[k++];
    B->I[0][0] = xx; B->I[0][1] = xy; B->I[0][2] = xz;
    B->I[1][0] = xy; B->I[1][1] = yy; B->I[1][2] = yz;
    B->I[2][0] = xz; B->I[2][1] = yz; B->I[2][2] = zz;
  }
  for (int l = 0; l < 4; ++l)
    for (int j = 0; j < 3; ++j)
      for (int i = 0; i < 3; ++i) M->origin[l][j][i] = p[k++];
  for (int i = 0; i < 3; ++i) M->foot[i] = p[k++];
  M->foot_r = p[k++];
  for (int i = 0; i < 3; ++i) M->trunk_half[i] = p[k++];
  M->thigh_r = p[k++];
  M->calf_r = p[k++];
  M->hip_r = p[k++];
  M->hip_y[0] = p[k++];
  M->hip_y[1] = p[k++];
}

static void cross3(const real* a, const real* b, real* o) {
  real x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
  o[0] = x; o[1] = y; o[2] = z;
}

/* rigid spatial inertia about the body frame origin: [[Ic + m(c.c 1 - c c^T), m c~], [m c~^T, m 1]] */
static void rigid_inertia(const Body* B, real mass_scale, M6* I) {
  real m = B->mass * mass_scale;
  const real* c = B->com;
  real cc = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
  memset(I, 0, sizeof(*I));
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) I->m[i][j] = B->I[i][j] * mass_scale + m * ((i == j ? cc : 0.0) - c[i] * c[j]);
  real cx[3][3] = {{0, -c[2], c[1]}, {c[2], 0, -c[0]}, {-c[1], c[0], 0}};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      I->m[i][3 + j] = m * cx[i][j];
      I->m[3 + j][i] = m * cx[i][j];
    }
  for (int i = 0; i < 3; ++i) I->m[3 + i][3 + i] = m;
}

static void m6_vec(const M6* A, const real* v, real* o) {
  for (int i = 0; i < 6; ++i) {
    real s = 0;
    for (int j = 0; j < 6; ++j) s += A->m[i][j] * v[j];
    o[i] = s;
  }
}

/* spatial force cross product v x* f, v = (w, v), f = (n, f) */
static void crf(const real* v, const real* f, real* o) {
  real a[3], b[3], c[3];
  cross3(v, f, a);
  cross3(v + 3, f + 3, b);
  cross3(v, f + 3, c);
  for (int i = 0; i < 3; ++i) { o[i] = a[i] + b[i]; o[3 + i] = c[i]; }
}

/* rotation matrix E (parent->child coords) of a revolute joint about unit axis ax by q:
 * E = Rot(ax, q)^T */
static void joint_E(int ax, real q, real E[3][3]) {
  real c = cos(q), s = sin(q);
  memset(E, 0, sizeof(real) * 9);
  if (ax == 0) {
    E[0][0] = 1; E[1][1] = c; E[1][2] = s; E[2][1] = -s; E[2][2] = c;
  } else {
    E[1][1] = 1; E[0][0] = c; E[0][2] = -s; E[2][0] = s; E[2][2] = c;
  }
}

/* motion transform parent -> child: (w, v) -> (E w, E (v - r x w)) */
static void xform_motion(real E[3][3], const real* r, const real* vin, real* vout) {
  real rw[3], t[3];
  cross3(r, vin, rw);
  for (int i = 0; i < 3; ++i) t[i] = vin[3 + i] - rw[i];
  for (int i = 0; i < 3; ++i) {
    vout[i] = E[i][0] * vin[0] + E[i][1] * vin[1] + E[i][2] * vin[2];
    vout[3 + i] = E[i][0] * t[0] + E[i][1] * t[1] + E[i][2] * t[2];
  }
}

/* force transform child -> parent: (n, f) -> (E^T n + r x E^T f, E^T f) */
static void xform_force_T(real E[3][3], const real* r, const real* fin, real* fout) {
  real n[3], f[3], rf[3];
  for (int i = 0; i < 3; ++i) {
    n[i] = E[0][i] * fin[0] + E[1][i] * fin[1] + E[2][i] * fin[2];
    f[i] = E[0][i] * fin[3] + E[1][i] * fin[4] + E[2][i] * fin[5];
  }
  cross3(r, f, rf);
  for (int i = 0; i < 3; ++i) { fout[i] = n[i] + rf[i]; fout[3 + i] = f[i]; }
}

/* X^T A X for X = motion transform (E, r) */
static void xform_inertia_T(real E[3][3], const real* r, const M6* A, M6* out) {
  /* build X explicitly: X = [[E, 0], [-E r~, E]] */
  real X[6][6];
  memset(X, 0, sizeof(X));
  real rx[3][3] = {{0, -r[2], r[1]}, {r[2], 0, -r[0]}, {-r[1], r[0], 0}};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      X[i][j] = E[i][j];
      X[3 + i][3 + j] = E[i][j];
      real s = 0;
      for (int k = 0; k < 3; ++k) s += E[i][k] * rx[k][j];
      X[3 + i][j] = -s;
    }
  real T[6][6];
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j < 6; ++j) {
      real s = 0;
      for (int k = 0; k < 6; ++k) s += A->m[i][k] * X[k][j];
      T[i][j] = s;
    }
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j < 6; ++j) {
      real s = 0;
      for (int k = 0; k < 6; ++k) s += X[k][i] * T[k][j];
      out->m[i][j] = s;
    }
}

/* solve SPD 6x6 A x = b (Cholesky) */
static void solve6(const M6* A, const real* b, real* x) {
  real L[6][6] = {{0}};
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j <= i; ++j) {
      real s = A->m[i][j];
      for (int k = 0; k < j; ++k) s -= L[i][k] * L[j][k];
      if (i == j) L[i][i] = sqrt(s > (real)1e-30 ? s : (real)1e-30);
      else L[i][j] = s / L[j][j];
    }
  real y[6];
  for (int i = 0; i < 6; ++i) {
    real s = b[i];
    for (int k = 0; k < i; ++k) s -= L[i][k] * y[k];
    y[i] = s / L[i][i];
  }
  for (int i = 5; i >= 0; --i) {
    real s = y[i];
    for (int k = i + 1; k < 6; ++k) s -= L[k][i] * x[k];
    x[i] = s / L[i][i];
  }
}

static void quat_to_R(const real* q, real R[3][3]) {
  real x = q[0], y = q[1], z = q[2], w = q[3];
  R[0][0] = 1 - 2 * (y * y + z * z); R[0][1] = 2 * (x * y - z * w); R[0][2] = 2 * (x * z + y * w);
  R[1][0] = 2 * (x * y + z * w); R[1][1] = 1 - 2 * (x * x + z * z); R[1][2] = 2 * (y * z - x * w);
  R[2][0] = 2 * (x * z - y * w); R[2][1] = 2 * (y * z + x * w); R[2][2] = 1 - 2 * (x * x + y * y);
}

/* ---- terrain queries (tile layer 0 ceiling, 1 floor).  Round 6: the surface is the heightfield's triangle mesh, as
 * the reference collides with it (mesh_type 'trimesh', legged_robot_trajectory_tracking.py:1450-1480; tunnel.py:139-147
 * builds it with isaacgym terrain_utils.convert_heightfield_to_trimesh): every cell (i, j) split along its
 * (i, j) - (i + 1, j + 1) diagonal into the triangles (i, j), (i + 1, j), (i + 1, j + 1) ("lower", a >= b) and (i, j),
 * (i + 1, j + 1), (i, j + 1) ("upper"), a = u - i, b = v - j.  (convert_heightfield_to_trimesh's slope threshold,
 * which moves vertices sideways under steep steps, is not modelled: the surface stays on the grid.)  Rounds 1-5 used the
 * bilinear patch; a triangle surface is piecewise linear along any segment, which makes a capsule's deepest point a
 * finite candidate set (seg_deepest). */
typedef struct {
  const float* tile; /* (2, nx, ny) or NULL for plane */
  int nx, ny;
  real ox, oy, hs;
} TerrainView;

static real tile_at(const TerrainView* T, int layer, int i, int j) {
  if (i < 0) i = 0;
  if (i > T->nx - 1) i = T->nx - 1;
  if (j < 0) j = 0;
  if (j > T->ny - 1) j = T->ny - 1;
  return (real)T->tile[((size_t)layer * T->nx + i) * T->ny + j];
}

/* height and gradient of layer at world (x, y) on triangle `up` (0 lower, 1 upper) of cell (ci, cj): the cell and
 * triangle a capsule's deepest-point search found the point on (seg_deepest), so that at an edge of the mesh (a ridge,
 * a spike's apex) the normal is the one of the triangle chosen there, not whichever side floor() of a rounded
 * coordinate lands on; tri_locate gives them for a point query */
static void tri_query(const TerrainView* T, int layer, real x, real y, int ci, int cj, int up, real* h, real* gx,
                      real* gy) {
  if (!T->tile) {
    *h = layer == 1 ? 0.0 : 1e9;
    *gx = *gy = 0.0;
    return;
  }
  real u = fmin(fmax((x - T->ox) / T->hs, -4.0), T->nx + 4.0), v = fmin(fmax((y - T->oy) / T->hs, -4.0), T->ny + 4.0);
  real a = u - ci, b = v - cj;
  real h00 = tile_at(T, layer, ci, cj), h10 = tile_at(T, layer, ci + 1, cj);
  real h01 = tile_at(T, layer, ci, cj + 1), h11 = tile_at(T, layer, ci + 1, cj + 1);
  real da = up ? h11 - h01 : h10 - h00, db = up ? h01 - h00 : h11 - h10;
  *h = h00 + a * da + b * db;
  *gx = da / T->hs;
  *gy = db / T->hs;
}
static void tri_locate(const TerrainView* T, real x, real y, int* cell) {
  real u = fmin(fmax((x - T->ox) / T->hs, -4.0), T->nx + 4.0), v = fmin(fmax((y - T->oy) / T->hs, -4.0), T->ny + 4.0);
  real fu = floor(u), fv = floor(v);
  cell[0] = (int)fu;
  cell[1] = (int)fv;
  cell[2] = (u - fu) < (v - fv);
}
/* height and gradient of layer at world (x, y): the triangle under the point */
static void height_query(const TerrainView* T, int layer, real x, real y, real* h, real* gx, real* gy) {
  int cell[3] = {0, 0, 0};
  if (T->tile) tri_locate(T, x, y, cell);
  tri_query(T, layer, x, y, cell[0], cell[1], cell[2], h, gx, gy);
}

typedef struct {
  real k, d, kf, mu;
  real e, vb; /* restitution (env and terrain averaged, PhysX's default combine) and the bounce threshold */
} ContactParams;

/* The integrator's contact scheme (go1_step.hip sphere_contact_im): contact forces linearly
 * implicit in the point velocity, so the integrator stays stable at one 5 ms step per sim step
 * (go1o_set_implicit_contact(0) restores the explicit penalty forces of round 1 for
 * tools/implicit_contact_study.py).  For an active layer with depth d0 and normal velocity vn, the normal force at the
 * end of the step, k (d0 - h vn') - d vn' with vn' = vn + h n.a_p, splits into an explicit part
 * k d0 - (h k + d) vn and an added mass h (h k + d) n n^T on the point; the regularised friction
 * -c_t vt' (c_t = min(kf, mu fn / |vt|) from the current state) adds h c_t (I - n n^T).  The added
 * masses enter the links' articulated inertias (point_inertia), so the ABA solves for the
 * accelerations that already include the contact response. */
static int g_implicit_contact = 1;
void go1o_set_implicit_contact(int on) { g_implicit_contact = on; }

/* penalty contact of a sphere (centre p, velocity pv, radius r) against floor and
 * ceiling; returns world force F (and, implicit option, adds the point's added mass to Mp) */
static void sphere_contact_im_cell(const TerrainView* T, const ContactParams* C, const real* p, const real* pv, real r,
                                   real* F, real h, real Mp[3][3], const int* cell) {
  F[0] = F[1] = F[2] = 0.0;
  for (int layer = 1; layer >= 0; --layer) {
    real hh, gx, gy;
    if (cell) tri_query(T, layer, p[0], p[1], cell[0], cell[1], cell[2], &hh, &gx, &gy);
    else height_query(T, layer, p[0], p[1], &hh, &gx, &gy);
    real n[3], dv;
    if (layer == 1) {
      dv = hh + r - p[2];
      n[0] = -gx; n[1] = -gy; n[2] = 1.0;
    } else {
      dv = p[2] + r - hh;
      n[0] = gx; n[1] = gy; n[2] = -1.0;
    }
    if (dv <= 0.0) continue;
    real inv = 1.0 / sqrt(n[0] * n[0] + n[1] * n[1] + 1.0);
    for (int i = 0; i < 3; ++i) n[i] *= inv;
    real depth = dv * inv;
    real vn = pv[0] * n[0] + pv[1] * n[1] + pv[2] * n[2];
    real fn0 = C->k * depth - C->d * vn;
    if (fn0 <= 0.0) continue;
    real fn = C->k * depth - (h * C->k + C->d) * vn;
    /* restitution: separating faster than the bounce threshold, the fraction e of the contact's damping
       (h k + d) is handed back (go1_device.h restitute) */
    if (C->e > 0.0 && vn > C->vb) fn += C->e * (h * C->k + C->d) * vn;
    real vt[3] = {pv[0] - vn * n[0], pv[1] - vn * n[1], pv[2] - vn * n[2]};
    real vtn = sqrt(vt[0] * vt[0] + vt[1] * vt[1] + vt[2] * vt[2]);
    real ct = C->kf;
    if (vtn > 1e-9 && C->mu * fn0 < ct * vtn) ct = C->mu * fn0 / vtn;
    real cn = h * (h * C->k + C->d), cd = h * ct;
    for (int i = 0; i < 3; ++i) {
      F[i] += fn * n[i] - ct * vt[i];
      for (int j = 0; j < 3; ++j) Mp[i][j] += (cn - cd) * n[i] * n[j] + (i == j ? cd : 0.0);
    }
  }
}
static void sphere_contact_im(const TerrainView* T, const ContactParams* C, const real* p, const real* pv, real r,
                              real* F, real h, real Mp[3][3]) {
  sphere_contact_im_cell(T, C, p, pv, r, F, h, Mp, NULL);
}

/* the added mass Mp (world, at local point lp of a link with rotation Rb) as a spatial inertia
 * about the link origin: [[lp~ M lp~^T, lp~ M], [M lp~^T, M]], M = Rb^T Mp Rb */
static void point_inertia(real Rb[3][3], const real* lp, real Mp[3][3], M6* I) {
  real M[3][3], S[3][3], SM[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      real a = 0;
      for (int k = 0; k < 3; ++k)
        for (int l = 0; l < 3; ++l) a += Rb[k][i] * Mp[k][l] * Rb[l][j];
      M[i][j] = a;
    }
  S[0][0] = 0; S[0][1] = -lp[2]; S[0][2] = lp[1];
  S[1][0] = lp[2]; S[1][1] = 0; S[1][2] = -lp[0];
  S[2][0] = -lp[1]; S[2][1] = lp[0]; S[2][2] = 0;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      real a = 0;
      for (int k = 0; k < 3; ++k) a += S[i][k] * M[k][j];
      SM[i][j] = a;
    }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      real a = 0;
      for (int k = 0; k < 3; ++k) a += SM[i][k] * S[j][k];  /* (S M) S^T */
      I->m[i][j] += a;
      I->m[i][3 + j] += SM[i][j];
      I->m[3 + j][i] += SM[i][j];
      I->m[3 + i][3 + j] += M[i][j];
    }
}

/* penalty contact of a sphere (centre p, velocity pv, radius r) against floor and
 * ceiling; returns world force F */
static void sphere_contact(const TerrainView* T, const ContactParams* C, const real* p, const real* pv, real r,
                           real* F) {
  F[0] = F[1] = F[2] = 0.0;
  for (int layer = 1; layer >= 0; --layer) {
    real h, gx, gy;
    height_query(T, layer, p[0], p[1], &h, &gx, &gy);
    real n[3], dv;
    if (layer == 1) { /* floor, normal up */
      dv = h + r - p[2];
      n[0] = -gx; n[1] = -gy; n[2] = 1.0;
    } else {
      dv = p[2] + r - h;
      n[0] = gx; n[1] = gy; n[2] = -1.0;
    }
    if (dv <= 0.0) continue;
    real inv = 1.0 / sqrt(n[0] * n[0] + n[1] * n[1] + 1.0);
    for (int i = 0; i < 3; ++i) n[i] *= inv;
    real depth = dv * inv;
    real vn = pv[0] * n[0] + pv[1] * n[1] + pv[2] * n[2];
    real fn = C->k * depth - C->d * vn;
    if (fn <= 0.0) continue;
    real vt[3] = {pv[0] - vn * n[0], pv[1] - vn * n[1], pv[2] - vn * n[2]};
    real vtn = sqrt(vt[0] * vt[0] + vt[1] * vt[1] + vt[2] * vt[2]);
    real ft = C->kf * vtn, fmax = C->mu * fn;
    if (ft > fmax) ft = fmax;
    real s = vtn > 1e-9 ? ft / vtn : 0.0;
    for (int i = 0; i < 3; ++i) F[i] += fn * n[i] - s * vt[i];
  }
}

/* Collision geometry per leg (round 6: capsules over the links' full length, no sphere chains), in the frame of
 * their link:
 *   hip  : capsule, segment (0, +-hip_y[0], 0) .. (0, +-hip_y[1], 0), radius hip_r (go1.urdf:106-111 as a capsule per
 *          replace_cylinder_with_capsule; the sign is the leg's side)
 *   thigh: capsule, segment (0,0,0) .. the knee (the calf joint's origin, (0,0,-0.213)), radius thigh_r (the
 *          0.213 x 0.0245 x 0.034 box of go1.urdf:148-153 as the capsule of its narrow half width)
 *   calf : capsule, segment (0,0,0) .. the foot offset (0,0,-0.213), radius calf_r (go1.urdf:176-181)
 *   foot : sphere at the foot offset (calf frame), radius foot_r (go1.urdf:201-205)
 * Trunk: the 8 corners of the collision box (radius 0) and its faces (face_scan).
 * Against the heightfields every capsule acts at the deepest point of its segment (seg_deepest): the hip capsule
 * at one point, the thigh and calf at one point per half (each half walked from its outer end, so a link lying
 * flat is carried at both ends). */

/* The deepest point of the segment A -> B (world) of a capsule of radius r against the floor and ceiling meshes
 * (go1_device.h seg_deepest2 is the f32 restatement): the t in [0, 1] that maximises the vertical gap of either layer,
 * floor h_f(x, y) + r - z and ceiling z + r - h_c(x, y).  Both meshes are triangles over the grid (tri_query), so
 * along the segment the gaps are piecewise linear in t and their maximum lies at an end or where the segment's (x, y)
 * projection crosses a mesh edge: a grid line u = k, v = k or a cell diagonal u - v = k.  The candidates are exactly
 * those (on an edge the height is the interpolation of its two vertices), so the search is exact and needs no
 * walk; each candidate carries the cell and triangle on the segment's incoming side of the edge, whose plane the
 * contact then uses.  A candidate's key is its deeper layer's gap quantised to SEG_Q, ties to the smaller t (the
 * segment's first end: the halves of the thigh and calf start at their outer ends, so a link lying flat is carried at
 * both), so the f32 kernel and this f64 restatement choose the same point.  On the plane the lower end (ties: A).
 * phys_substep searches once per control step and holds t for the control step's other sim steps (the kernel's
 * cadence, as for the trunk faces). */
#define SEG_Q 1.0e-5
static long seg_quant(real g) { return (long)floor(fmin(fmax(g, -1.0), 1.0) / SEG_Q); }
typedef struct {
  long key; /* the best candidate's key: quantised gap (the deeper layer) x 4096 + the earlier t (4095 - 4095 t) */
  real t;
  int c[3];
} SegBest;
static void seg_offer(SegBest* sb, const real* h, real z, real r, real t, int ci, int cj, int up) {
  long qf = seg_quant((h[0] - z) + r), qc = seg_quant((z - h[1]) + r);
  long key = (qf > qc ? qf : qc) * 4096 + (4095 - (long)floor(t * 4095.0));
  if (key > sb->key) { /* an equal key (a vertex on several edges) keeps the first offer */
    sb->key = key;
    sb->t = t;
    sb->c[0] = ci; sb->c[1] = cj; sb->c[2] = up;
  }
}
static real seg_deepest(const TerrainView* T, const real* A, const real* B, real r, int* cell) {
  cell[0] = cell[1] = cell[2] = 0;
  if (!T->tile) return seg_quant(r - B[2]) > seg_quant(r - A[2]) ? 1.0 : 0.0;
  real uA = fmin(fmax((A[0] - T->ox) / T->hs, -4.0), T->nx + 4.0), vA = fmin(fmax((A[1] - T->oy) / T->hs, -4.0), T->ny + 4.0);
  real uB = fmin(fmax((B[0] - T->ox) / T->hs, -4.0), T->nx + 4.0), vB = fmin(fmax((B[1] - T->oy) / T->hs, -4.0), T->ny + 4.0);
  real du = uB - uA, dv = vB - vA, dw = du - dv, dz = B[2] - A[2];
  SegBest sb = {LONG_MIN, 0.0, {0, 0, 0}};
  real h[2];
  /* the ends */
  for (int e = 0; e < 2; ++e) {
    const real* P = e ? B : A;
    int c[3];
    real gx, gy;
    tri_locate(T, P[0], P[1], c);
    tri_query(T, 1, P[0], P[1], c[0], c[1], c[2], &h[0], &gx, &gy);
    tri_query(T, 0, P[0], P[1], c[0], c[1], c[2], &h[1], &gx, &gy);
    seg_offer(&sb, h, P[2], r, (real)e, c[0], c[1], c[2]);
  }
  /* grid lines u = k */
  for (int k = (int)floor(fmin(uA, uB)) + 1; k < fmax(uA, uB); ++k) {
    real t = (k - uA) / du, v = vA + dv * t;
    int j = (int)floor(v), i = du > 0.0 ? k - 1 : k;
    real b = v - j;
    for (int L = 0; L < 2; ++L) {
      int layer = L == 0 ? 1 : 0;
      h[L] = tile_at(T, layer, k, j) + b * (tile_at(T, layer, k, j + 1) - tile_at(T, layer, k, j));
    }
    seg_offer(&sb, h, A[2] + dz * t, r, t, i, j, (real)(k - i) < b);
  }
  /* grid lines v = k */
  for (int k = (int)floor(fmin(vA, vB)) + 1; k < fmax(vA, vB); ++k) {
    real t = (k - vA) / dv, u = uA + du * t;
    int i = (int)floor(u), j = dv > 0.0 ? k - 1 : k;
    real a = u - i;
    for (int L = 0; L < 2; ++L) {
      int layer = L == 0 ? 1 : 0;
      h[L] = tile_at(T, layer, i, k) + a * (tile_at(T, layer, i + 1, k) - tile_at(T, layer, i, k));
    }
    seg_offer(&sb, h, A[2] + dz * t, r, t, i, j, a < (real)(k - j));
  }
  /* cell diagonals u - v = k (the point (i + a, j + a) of cell (i, j), i - j = k) */
  real wA = uA - vA, wB = uB - vB;
  for (int k = (int)floor(fmin(wA, wB)) + 1; k < fmax(wA, wB); ++k) {
    real t = (k - wA) / dw, u = uA + du * t;
    int i = (int)floor(u), j = i - k;
    real a = u - i;
    for (int L = 0; L < 2; ++L) {
      int layer = L == 0 ? 1 : 0;
      h[L] = tile_at(T, layer, i, j) + a * (tile_at(T, layer, i + 1, j + 1) - tile_at(T, layer, i, j));
    }
    seg_offer(&sb, h, A[2] + dz * t, r, t, i, j, dw > 0.0); /* incoming: u - v < k, i.e. a < b: upper */
  }
  for (int m = 0; m < 3; ++m) cell[m] = sb.c[m];
  return sb.t;
}

/* closest points of the segments P0 -> P1 and Q0 -> Q1: parameters s (on P) and t (on Q) in [0, 1] (Ericson,
 * Real-Time Collision Detection 5.1.9; a degenerate segment (a point) has s = 0 or t = 0).  The unclamped s of the two
 * lines, (b f - c e) / (a e - b^2), is formed without cancellation as (n . (d2 x r)) / (n . n), n = d1 x d2 (Lagrange's
 * identity): for nearly parallel links a e - b^2 cancels to a few f32 ulps, and the f32 kernel would otherwise
 * place the closest points anywhere along them. */
static void seg_seg_closest(const real* P0, const real* P1, const real* Q0, const real* Q1, real* s_out, real* t_out) {
  real d1[3], d2[3], r[3], n[3], m[3];
  for (int i = 0; i < 3; ++i) { d1[i] = P1[i] - P0[i]; d2[i] = Q1[i] - Q0[i]; r[i] = P0[i] - Q0[i]; }
  real a = d1[0] * d1[0] + d1[1] * d1[1] + d1[2] * d1[2], e = d2[0] * d2[0] + d2[1] * d2[1] + d2[2] * d2[2];
  real f = d2[0] * r[0] + d2[1] * r[1] + d2[2] * r[2];
  real s = 0.0, t = 0.0;
  if (a <= 1e-12 && e <= 1e-12) {
    s = t = 0.0;
  } else if (a <= 1e-12) {
    t = fmin(fmax(f / e, 0.0), 1.0);
  } else {
    real c = d1[0] * r[0] + d1[1] * r[1] + d1[2] * r[2];
    if (e <= 1e-12) {
      s = fmin(fmax(-c / a, 0.0), 1.0);
    } else {
      real b = d1[0] * d2[0] + d1[1] * d2[1] + d1[2] * d2[2];
      cross3(d1, d2, n);
      cross3(d2, r, m);
      real den = n[0] * n[0] + n[1] * n[1] + n[2] * n[2], num = n[0] * m[0] + n[1] * m[1] + n[2] * m[2];
      s = den > 1e-10 * a * e ? fmin(fmax(num / den, 0.0), 1.0) : 0.0;
      t = (b * s + f) / e;
      if (t < 0.0) { t = 0.0; s = fmin(fmax(-c / a, 0.0), 1.0); }
      else if (t > 1.0) { t = 1.0; s = fmin(fmax((b - c) / a, 0.0), 1.0); }
    }
  }
  *s_out = s;
  *t_out = t;
}

/* exposed for tests/test_capsules.py: the deepest point of a segment against one (2, nx, ny) tile at the origin,
 * and the closest points of two segments */
double go1o_seg_deepest(const float* tile, int nx, int ny, double hs, const double* A, const double* B, double r) {
  TerrainView T = {tile, nx, ny, 0.0, 0.0, (real)hs};
  real a[3] = {A[0], A[1], A[2]}, b[3] = {B[0], B[1], B[2]};
  int cell[3];
  return (double)seg_deepest(&T, a, b, (real)r, cell);
}
void go1o_seg_closest(const double* P0, const double* P1, const double* Q0, const double* Q1, double* st) {
  real p0[3], p1[3], q0[3], q1[3], s, t;
  for (int i = 0; i < 3; ++i) { p0[i] = P0[i]; p1[i] = P1[i]; q0[i] = Q0[i]; q1[i] = Q1[i]; }
  seg_seg_closest(p0, p1, q0, q1, &s, &t);
  st[0] = s;
  st[1] = t;
}

/* the point of the segment P0 -> P1 (world) nearest the trunk box (deepest inside it).  The box's signed distance is
 * convex, so along the segment it is a convex function of t; its minimum is found by bisection on the sign of the
 * derivative (SEG_BISECT halvings, 2^-20 of the segment ~ 0.2 um on a 0.213 m link; every midpoint an exact binary
 * fraction in f32 and f64 alike).  Outside the box the distance |q+| (q_i = |c_i| - th_i) has the derivative's sign
 * of sum_i q+_i sgn(c_i) d_i; inside, max_i q_i has sgn(c_k) d_k for the deepest axis k (the lowest on ties).  Round
 * 6's first cut ran a golden-section search on the distance itself (32 evaluations with a square root each), the
 * slowest waves' largest section.  go1_device.h seg_box_t is the f32 restatement. */
#define SEG_BISECT 20
#define BOX_Q 1.0e-4
static long box_quant(real d) { return (long)floor(fmin(fmax(d, -1.0), 1.0) / BOX_Q); }
static real seg_box_t(const real* P0, const real* P1, real R[3][3], const real* pos, const real* th) {
  real a0[3], d[3];
  for (int i = 0; i < 3; ++i) {
    a0[i] = R[0][i] * (P0[0] - pos[0]) + R[1][i] * (P0[1] - pos[1]) + R[2][i] * (P0[2] - pos[2]);
    d[i] = R[0][i] * (P1[0] - P0[0]) + R[1][i] * (P1[1] - P0[1]) + R[2][i] * (P1[2] - P0[2]);
  }
  real lo = 0.0, hi = 1.0;
  for (int it = 0; it < SEG_BISECT; ++it) {
    const real m = 0.5 * (lo + hi);
    real so = 0.0, qmax = -1e30, sin = 0.0;
    int out = 0;
    for (int i = 0; i < 3; ++i) {
      const real c = a0[i] + m * d[i], sg = c >= 0.0 ? 1.0 : -1.0, q = fabs(c) - th[i];
      if (q > 0.0) { so += q * sg * d[i]; out = 1; }
      if (q > qmax) { qmax = q; sin = sg * d[i]; }
    }
    const real sl = out ? so : sin;
    if (sl < 0.0) lo = m; else hi = m;
  }
  return 0.5 * (lo + hi);
}

typedef struct {
  real pos[3], quat[4], v[3], w[3];
  real q[NDOF], qd[NDOF];
  int face[2]; /* the trunk faces' contact vertices of the control step (face_scan), -1: none */
  real seg_t[4][5]; /* per leg the capsules' deepest points of the control step (seg_deepest): hip, thigh x2, calf x2 */
} PhysState;

/* world pose/velocity of a point given body pose (Rb, pb) and body spatial velocity
 * (w, v) in body coords at body origin */
static void point_kin(real Rb[3][3], const real* pb, const real* vb, const real* lp, real* pw, real* vw) {
  real wl[3], vl[3];
  cross3(vb, lp, wl);
  for (int i = 0; i < 3; ++i) vl[i] = vb[3 + i] + wl[i];
  for (int i = 0; i < 3; ++i) {
    pw[i] = pb[i] + Rb[i][0] * lp[0] + Rb[i][1] * lp[1] + Rb[i][2] * lp[2];
    vw[i] = Rb[i][0] * vl[0] + Rb[i][1] * vl[1] + Rb[i][2] * vl[2];
  }
}

/* world force F at local point lp -> body-coords spatial force (n, f) at origin */
static void point_force(real Rb[3][3], const real* lp, const real* F, real* fs) {
  real f[3];
  for (int i = 0; i < 3; ++i) f[i] = Rb[0][i] * F[0] + Rb[1][i] * F[1] + Rb[2][i] * F[2];
  real n[3];
  cross3(lp, f, n);
  for (int i = 0; i < 3; ++i) { fs[i] += n[i]; fs[3 + i] += f[i]; }
}

/* Self-collision (asset.self_collisions == 0, go1_crawling.py:44: Isaac Gym collides every pair of bodies that
 * no joint connects; go1_device.h self_narrow): the primitives 4 leg + k of the legs (k: 0 thigh capsule, 1 hip
 * capsule, 2 calf capsule, 3 foot sphere; the collision geometry above); pairs: every primitive of leg la against
 * every primitive of leg lb (la < lb, 16 per leg pair), within a leg the links two joints apart (hip capsule vs calf
 * capsule and foot, thigh capsule vs foot: SELF_SAME_A / _B), and the thigh / calf capsules and the foot against
 * the trunk box (half extents trunk_half about the base origin; the hip is the trunk's neighbour).  A pair acts at
 * the closest points of its two segments (seg_seg_closest) as two spheres of the capsules' radii there; a capsule
 * against the box at its point nearest the box (seg_box_t).  Explicit penalty springs fn = ks pen - ds vn on the
 * overlap, compressive only, no friction; the force on the primitive of the lower index is computed, the other
 * gets its negative at its own closest point, the trunk the box pairs' reaction. */
#define SELF_NSAME 3
static const int SELF_SAME_A[SELF_NSAME] = {1, 1, 0};
static const int SELF_SAME_B[SELF_NSAME] = {2, 3, 3};
static void self_sphere_force(const real* pa, const real* va, real ra, const real* pb, const real* vb, real rb,
                              real ks, real ds, real* F) {
  real d[3] = {pa[0] - pb[0], pa[1] - pb[1], pa[2] - pb[2]};
  real dd = d[0] * d[0] + d[1] * d[1] + d[2] * d[2], rs = ra + rb;
  F[0] = F[1] = F[2] = 0.0;
  if (!(dd < rs * rs)) return;
  real dist = sqrt(dd), n[3] = {0.0, 0.0, 1.0};
  if (dd > 1e-18) for (int i = 0; i < 3; ++i) n[i] = d[i] / dist;
  else dist = 0.0;
  real vn = (va[0] - vb[0]) * n[0] + (va[1] - vb[1]) * n[1] + (va[2] - vb[2]) * n[2];
  real fn = ks * (rs - dist) - ds * vn;
  if (fn <= 0.0) return;
  for (int i = 0; i < 3; ++i) F[i] = fn * n[i];
}

/* sphere (world pa, va, radius r) against the trunk box: force on the sphere (world) and the trunk's
 * reaction wrench (base frame, (moment, force) about the base origin) added to wb */
static void self_box_force(const real* pa, const real* va, real r, real R[3][3], const real* pos, const real* vbase,
                           const real* th, real ks, real ds, real* F, real* wb) {
  real c[3], q[3], d[3], nb[3], pen;
  F[0] = F[1] = F[2] = 0.0;
  for (int i = 0; i < 3; ++i) c[i] = R[0][i] * (pa[0] - pos[0]) + R[1][i] * (pa[1] - pos[1]) + R[2][i] * (pa[2] - pos[2]);
  for (int i = 0; i < 3; ++i) { q[i] = fmin(fmax(c[i], -th[i]), th[i]); d[i] = c[i] - q[i]; }
  real dd = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
  if (!(dd < r * r)) return;
  if (dd > 0.0) {
    real dist = sqrt(dd);
    for (int i = 0; i < 3; ++i) nb[i] = d[i] / dist;
    pen = r - dist;
  } else { /* centre inside: out through the nearest face, lowest axis on ties -- compared quantised to BOX_Q: the
            * deepest point of a segment inside the box is often where two faces are equally near, and there the f32
            * kernel and this f64 restatement must choose the same face */
    real m[3];
    long mq[3];
    for (int i = 0; i < 3; ++i) { m[i] = th[i] - fabs(c[i]); mq[i] = box_quant(m[i]); }
    int ax = (mq[0] <= mq[1] && mq[0] <= mq[2]) ? 0 : (mq[1] <= mq[2] ? 1 : 2);
    real sg = c[ax] >= 0.0 ? 1.0 : -1.0;
    for (int i = 0; i < 3; ++i) nb[i] = i == ax ? sg : 0.0;
    q[ax] = sg * th[ax];
    pen = r + m[ax];
  }
  real vq[3], w[3] = {vbase[0], vbase[1], vbase[2]}, wq[3];
  cross3(w, q, wq);
  for (int i = 0; i < 3; ++i) vq[i] = vbase[3 + i] + wq[i];
  real vab[3];
  for (int i = 0; i < 3; ++i) vab[i] = R[0][i] * va[0] + R[1][i] * va[1] + R[2][i] * va[2];
  real vn = (vab[0] - vq[0]) * nb[0] + (vab[1] - vq[1]) * nb[1] + (vab[2] - vq[2]) * nb[2];
  real fn = ks * pen - ds * vn;
  if (fn <= 0.0) return;
  for (int i = 0; i < 3; ++i) F[i] = fn * (R[i][0] * nb[0] + R[i][1] * nb[1] + R[i][2] * nb[2]);
  real fb[3] = {-fn * nb[0], -fn * nb[1], -fn * nb[2]}, tq[3];
  cross3(q, fb, tq);
  for (int i = 0; i < 3; ++i) { wb[i] += tq[i]; wb[3 + i] += fb[i]; }
}

/* The trunk box's faces against the heightfields (go1_device.h face_scan / face_force; go1.urdf:53-58,
 * tunnel_fn.py:99-163): once per control step, per face the grid vertex inside its footprint nearest to (or deepest
 * in) the face -- the floor against the bottom face, the ceiling against the top -- among the 10 x 10 vertices around
 * the trunk centre (offsets -4 .. +5 on both axes: they cover the footprint's +-0.166 m at any yaw, whatever the
 * centre's position in its cell), signed depths from -FACE_SIGNED compared quantised to 1e-5 m, ties to the lowest
 * window position; every sim step an explicit penalty force at the two vertices where they penetrate, along the face
 * normal (k depth - d vn, depth capped at the box height) with the regularised Coulomb friction of the point
 * contacts.  The GPU scans its LDS terrain patch (which holds the trunk's footprint), this restatement the tile
 * (both clamp at the tile's edges). */
#define FACE_Q 1.0e-5
#define FACE_W 10
#define FACE_SIGNED 0.1
static void face_scan(const TerrainView* T, real R[3][3], const real* pos, const real* th, int* sel) {
  /* (positions relative to the tile's origin (ox, oy): zero in the step, which integrates in terrain coordinates) */
  const real px = pos[0] - T->ox, py = pos[1] - T->oy;
  int ci = (int)floor(fmin(fmax(px / T->hs, -16000.0), 16000.0)), cj = (int)floor(fmin(fmax(py / T->hs, -16000.0), 16000.0));
  for (int hh = 0; hh < 2; ++hh) {
    int best = -1;
    for (int v = 0; v < FACE_W * FACE_W; ++v) {
      int i = ci + v % FACE_W - 4, j = cj + v / FACE_W - 4;
      real d[3] = {i * T->hs - px, j * T->hs - py, tile_at(T, hh == 0 ? 1 : 0, i, j) - pos[2]}, c[3];
      for (int k = 0; k < 3; ++k) c[k] = R[0][k] * d[0] + R[1][k] * d[1] + R[2][k] * d[2];
      real pen = hh == 0 ? c[2] + th[2] : th[2] - c[2];
      if (!(fabs(c[0]) <= th[0] && fabs(c[1]) <= th[1] && pen > -FACE_SIGNED)) continue;
      int q = (int)floor(fmin(pen + FACE_SIGNED, 10.0) / FACE_Q);
      int key = (q << 7) | (127 - v);
      if (key > best) best = key;
    }
    if (best < 0) { sel[hh] = -1; continue; }
    int v = 127 - (best & 127);
    int i = ci + v % FACE_W - 4, j = cj + v / FACE_W - 4;
    sel[hh] = ((i + 16384) << 16) | (j + 16384);
  }
}
/* adds the base-frame wrench (moment about the base origin, force) to wb and the world force to Fw */
static void face_force(const TerrainView* T, const ContactParams* C, real R[3][3], const real* pos, const real* vb,
                       const real* th, const int* sel, real* wb, real* Fw) {
  for (int hh = 0; hh < 2; ++hh) {
    if (sel[hh] < 0) continue;
    int i = (sel[hh] >> 16) - 16384, j = (sel[hh] & 0xffff) - 16384;
    real d[3] = {i * T->hs - (pos[0] - T->ox), j * T->hs - (pos[1] - T->oy), tile_at(T, hh == 0 ? 1 : 0, i, j) - pos[2]},
         c[3];
    for (int k = 0; k < 3; ++k) c[k] = R[0][k] * d[0] + R[1][k] * d[1] + R[2][k] * d[2];
    real pen = hh == 0 ? c[2] + th[2] : th[2] - c[2];
    if (!(fabs(c[0]) <= th[0] && fabs(c[1]) <= th[1] && pen > 0.0)) continue;
    real nz = hh == 0 ? 1.0 : -1.0;
    real v[3] = {vb[3] + (vb[1] * c[2] - vb[2] * c[1]), vb[4] + (vb[2] * c[0] - vb[0] * c[2]),
                 vb[5] + (vb[0] * c[1] - vb[1] * c[0])};
    real depth = fmin(pen, 2.0 * th[2]), vn = v[2] * nz;
    real fn = C->k * depth - C->d * vn;
    if (!(fn > 0.0)) continue;
    real vt = sqrt(v[0] * v[0] + v[1] * v[1]);
    real ct = (C->kf * vt > C->mu * fn && vt > 1e-9) ? C->mu * fn / vt : C->kf;
    real F[3] = {-ct * v[0], -ct * v[1], fn * nz}, m[3];
    cross3(c, F, m);
    for (int k = 0; k < 3; ++k) { wb[k] += m[k]; wb[3 + k] += F[k]; }
    for (int k = 0; k < 3; ++k) Fw[k] += R[k][0] * F[0] + R[k][1] * F[1] + R[k][2] * F[2];
  }
}

/* One integrator step of length h with torques tau.  Writes net contact forces
 * per reported body (17 x 3, world) into cf (may be NULL). */
/* tests/test_held_contacts.py: make a held choice every sim step (bit 0: the trunk faces' vertices, bit 1: the
 * capsules' deepest points), to measure what holding them for a control step changes */
static int g_rescan_every_step = 0;
void go1o_set_rescan_every_step(int mask) { g_rescan_every_step = mask; }
static void phys_substep(const Model* M, const go1_config* cfg, PhysState* S, const real* tau, real h,
                         const real* g, real friction, real restitution, real payload, const TerrainView* T,
                         real* cf, int scan_now) {
  const int face_scan_now = scan_now || (g_rescan_every_step & 1);
  const int seg_scan_now = scan_now || (g_rescan_every_step & 2);
  ContactParams C = {cfg->contact_stiffness, cfg->contact_damping, cfg->friction_damping, friction,
                     0.5 * (restitution + (real)cfg->terrain_restitution), cfg->bounce_threshold};
  real R[3][3];
  quat_to_R(S->quat, R);
  real vb[6]; /* base spatial velocity, body coords */
  for (int i = 0; i < 3; ++i) {
    vb[i] = R[0][i] * S->w[0] + R[1][i] * S->w[1] + R[2][i] * S->w[2];
    vb[3 + i] = R[0][i] * S->v[0] + R[1][i] * S->v[1] + R[2][i] * S->v[2];
  }
  real gb[3];
  for (int i = 0; i < 3; ++i) gb[i] = R[0][i] * g[0] + R[1][i] * g[1] + R[2][i] * g[2];
  if (cf) memset(cf, 0, sizeof(real) * NB * 3);

  /* base rigid inertia (payload added to the trunk, inertia scaled by mass ratio) */
  real mscale = (M->base.mass + payload) / M->base.mass;
  M6 IA0;
  rigid_inertia(&M->base, mscale, &IA0);
  real pA0[6], hmom[6];
  m6_vec(&IA0, vb, hmom);
  crf(vb, hmom, pA0);
  {
    real fext[6] = {0}, fg[3], cg[3];
    real m = M->base.mass * mscale;
    for (int i = 0; i < 3; ++i) fg[i] = m * gb[i];
    cross3(M->base.com, fg, cg);
    for (int i = 0; i < 3; ++i) { fext[i] += cg[i]; fext[3 + i] += fg[i]; }
    for (int cx = 0; cx < 8; ++cx) {
      real lp[3] = {(cx & 1) ? M->trunk_half[0] : -M->trunk_half[0], (cx & 2) ? M->trunk_half[1] : -M->trunk_half[1],
                      (cx & 4) ? M->trunk_half[2] : -M->trunk_half[2]};
      real pw[3], vw[3], F[3];
      point_kin(R, S->pos, vb, lp, pw, vw);
      if (g_implicit_contact) {
        real Mp[3][3] = {{0}};
        sphere_contact_im(T, &C, pw, vw, 0.0, F, h, Mp);
        point_inertia(R, lp, Mp, &IA0);
      } else {
        sphere_contact(T, &C, pw, vw, 0.0, F);
      }
      point_force(R, lp, F, fext);
      if (cf) for (int i = 0; i < 3; ++i) cf[i] += F[i];
    }
    for (int i = 0; i < 6; ++i) pA0[i] -= fext[i];
  }

  /* per-leg quantities kept for the forward pass */
  real E[4][3][3][3], vj[4][3][6], cj[4][3][6], U[4][3][6], D[4][3], u[4][3];
  real Rw_all[4][3][3][3], pw_all[4][3][3];
  for (int l = 0; l < 4; ++l) {
    real Rp[3][3], pp[3], vp[6];
    memcpy(Rp, R, sizeof(Rp));
    memcpy(pp, S->pos, sizeof(pp));
    memcpy(vp, vb, sizeof(vp));
    real (*Rw)[3][3] = Rw_all[l], (*pw_)[3] = pw_all[l];
    for (int j = 0; j < 3; ++j) {
      int ax = j == 0 ? 0 : 1, dof = l * 3 + j;
      const real* r = M->origin[l][j];
      joint_E(ax, S->q[dof], E[l][j]);
      xform_motion(E[l][j], r, vp, vj[l][j]);
      vj[l][j][ax] += S->qd[dof];
      /* c = v x (S qd) */
      real sq[3] = {0, 0, 0};
      sq[ax] = S->qd[dof];
      cross3(vj[l][j], sq, cj[l][j]);
      cross3(vj[l][j] + 3, sq, cj[l][j] + 3);
      /* world pose of the link */
      real rw[3];
      for (int i = 0; i < 3; ++i) rw[i] = Rp[i][0] * r[0] + Rp[i][1] * r[1] + Rp[i][2] * r[2];
      for (int i = 0; i < 3; ++i) {
        pw_[j][i] = pp[i] + rw[i];
        for (int k = 0; k < 3; ++k)
          Rw[j][i][k] = Rp[i][0] * E[l][j][k][0] + Rp[i][1] * E[l][j][k][1] + Rp[i][2] * E[l][j][k][2];
      }
      memcpy(Rp, Rw[j], sizeof(Rp));
      memcpy(pp, pw_[j], sizeof(pp));
      memcpy(vp, vj[l][j], sizeof(vp));
    }
  }
  /* self-collision: body-frame wrenches on the legs' links (wsl[l][j], j = hip, thigh, calf), reported forces per
   * body (cfs, the cf layout) and the trunk's reaction wrench */
  real wsl[4][3][6], cfs[NB][3], wself[6] = {0, 0, 0, 0, 0, 0};
  memset(wsl, 0, sizeof(wsl));
  memset(cfs, 0, sizeof(cfs));
  if (cfg->self_stiffness > 0.0f) {
    /* primitive 4 l + k: link j, segment ends lp0 -> lp1 in the link frame, world ends P0 / P1, their velocities */
    real SP[16][2][3], SV[16][2][3], SL[16][2][3], SR[16];
    int SJ[16], SB[16];
    for (int l = 0; l < 4; ++l)
      for (int k = 0; k < 4; ++k) {
        int j = k == 0 ? 1 : (k == 1 ? 0 : 2), p = 4 * l + k;
        real lp[2][3] = {{0, 0, 0}, {0, 0, 0}};
        const real sy = (l & 1) ? -1.0 : 1.0;
        if (k == 0) { for (int i = 0; i < 3; ++i) lp[1][i] = M->origin[l][2][i]; }        /* thigh: joint .. knee */
        else if (k == 1) { lp[0][1] = sy * M->hip_y[0]; lp[1][1] = sy * M->hip_y[1]; }    /* hip capsule */
        else if (k == 2) { for (int i = 0; i < 3; ++i) lp[1][i] = M->foot[i]; }          /* calf: knee .. foot */
        else { for (int i = 0; i < 3; ++i) lp[0][i] = lp[1][i] = M->foot[i]; }            /* foot sphere */
        for (int e = 0; e < 2; ++e) {
          for (int i = 0; i < 3; ++i) SL[p][e][i] = lp[e][i];
          point_kin(Rw_all[l][j], pw_all[l][j], vj[l][j], lp[e], SP[p][e], SV[p][e]);
        }
        SR[p] = k == 0 ? M->thigh_r : (k == 1 ? M->hip_r : (k == 2 ? M->calf_r : M->foot_r));
        SJ[p] = j;
        SB[p] = k == 3 ? 1 + l * 4 + 3 : 1 + l * 4 + j; /* reported body (the foot its own) */
      }
    const real ks = cfg->self_stiffness, ds = cfg->self_damping;
    /* force F (world) on primitive p at segment parameter s: its link's wrench and its body's reported force */
#define SELF_APPLY(p, sp, F)                                                                              \
  do {                                                                                                    \
    int l_ = (p) / 4;                                                                                     \
    real lpp[3];                                                                                          \
    for (int i_ = 0; i_ < 3; ++i_) lpp[i_] = SL[p][0][i_] + (sp) * (SL[p][1][i_] - SL[p][0][i_]);         \
    point_force(Rw_all[l_][SJ[p]], lpp, (F), wsl[l_][SJ[p]]);                                              \
    for (int i_ = 0; i_ < 3; ++i_) cfs[SB[p]][i_] += (F)[i_];                                             \
  } while (0)
    /* a pair (ia < ib): spheres of the two radii at the segments' closest points */
#define SELF_PAIR(ia, ib)                                                                                 \
  do {                                                                                                    \
    real s_, t_, pa_[3], va_[3], pb_[3], vb_[3], F_[3], G_[3];                                            \
    seg_seg_closest(SP[ia][0], SP[ia][1], SP[ib][0], SP[ib][1], &s_, &t_);                                \
    for (int i_ = 0; i_ < 3; ++i_) {                                                                      \
      pa_[i_] = SP[ia][0][i_] + s_ * (SP[ia][1][i_] - SP[ia][0][i_]);                                     \
      va_[i_] = SV[ia][0][i_] + s_ * (SV[ia][1][i_] - SV[ia][0][i_]);                                     \
      pb_[i_] = SP[ib][0][i_] + t_ * (SP[ib][1][i_] - SP[ib][0][i_]);                                     \
      vb_[i_] = SV[ib][0][i_] + t_ * (SV[ib][1][i_] - SV[ib][0][i_]);                                     \
    }                                                                                                     \
    self_sphere_force(pa_, va_, SR[ia], pb_, vb_, SR[ib], ks, ds, F_);                                    \
    for (int i_ = 0; i_ < 3; ++i_) G_[i_] = -F_[i_];                                                      \
    SELF_APPLY(ia, s_, F_);                                                                               \
    SELF_APPLY(ib, t_, G_);                                                                               \
  } while (0)
    /* every primitive pair of two different legs */
    for (int la = 0; la < 4; ++la)
      for (int lb = la + 1; lb < 4; ++lb)
        for (int a = 0; a < 4; ++a)
          for (int b = 0; b < 4; ++b) SELF_PAIR(la * 4 + a, lb * 4 + b);
    /* the non-adjacent links of one leg: hip capsule vs calf capsule / foot, thigh capsule vs foot */
    for (int l = 0; l < 4; ++l)
      for (int p2 = 0; p2 < SELF_NSAME; ++p2) SELF_PAIR(l * 4 + SELF_SAME_A[p2], l * 4 + SELF_SAME_B[p2]);
    /* the thigh / calf capsules and the foot against the trunk box (the hip is the trunk's neighbour) */
    for (int l = 0; l < 4; ++l)
      for (int k = 0; k < 4; ++k) {
        if (k == 1) continue;
        int p = 4 * l + k;
        real t = k == 3 ? 0.0 : seg_box_t(SP[p][0], SP[p][1], R, S->pos, M->trunk_half);
        real pc[3], vc[3], F[3], wb[6] = {0, 0, 0, 0, 0, 0};
        for (int i = 0; i < 3; ++i) {
          pc[i] = SP[p][0][i] + t * (SP[p][1][i] - SP[p][0][i]);
          vc[i] = SV[p][0][i] + t * (SV[p][1][i] - SV[p][0][i]);
        }
        self_box_force(pc, vc, SR[p], R, S->pos, vb, M->trunk_half, ks, ds, F, wb);
        for (int i = 0; i < 6; ++i) wself[i] += wb[i];
        SELF_APPLY(p, t, F);
        /* the trunk's reported contact force includes the reaction (world frame) */
        for (int i = 0; i < 3; ++i) cfs[0][i] += R[i][0] * wb[3] + R[i][1] * wb[4] + R[i][2] * wb[5];
      }
#undef SELF_PAIR
#undef SELF_APPLY
    for (int i = 0; i < 6; ++i) pA0[i] -= wself[i];
    if (cf) for (int b2 = 0; b2 < NB; ++b2) for (int i = 0; i < 3; ++i) cf[b2 * 3 + i] += cfs[b2][i];
  }
  for (int l = 0; l < 4; ++l) {
    M6 IA[3];
    real pA[3][6];
    real (*Rw)[3][3] = Rw_all[l], (*pw_)[3] = pw_all[l];
    /* rigid inertias, bias forces, gravity and contact */
    for (int j = 0; j < 3; ++j) {
      const Body* B = &M->leg[l][j];
      rigid_inertia(B, 1.0, &IA[j]);
      real hm[6];
      m6_vec(&IA[j], vj[l][j], hm);
      crf(vj[l][j], hm, pA[j]);
      real gl[3], fext[6] = {0}, fg[3], cg[3];
      for (int i = 0; i < 3; ++i) gl[i] = Rw[j][0][i] * g[0] + Rw[j][1][i] * g[1] + Rw[j][2][i] * g[2];
      for (int i = 0; i < 3; ++i) fg[i] = B->mass * gl[i];
      cross3(B->com, fg, cg);
      for (int i = 0; i < 3; ++i) { fext[i] += cg[i] + wsl[l][j][i]; fext[3 + i] += fg[i] + wsl[l][j][3 + i]; }
      int body_idx = 1 + l * 4 + j; /* hip, thigh, calf */
      /* the link's heightfield contacts: per capsule (half) its deepest point (seg_deepest), the foot sphere */
      real segs[3][2][3], rads[3];
      int nseg = 0, foot_seg = -1;
      const real sy = (l & 1) ? -1.0 : 1.0;
      memset(segs, 0, sizeof(segs));
      if (j == 0) { /* hip capsule: one point */
        segs[0][0][1] = sy * M->hip_y[0]; segs[0][1][1] = sy * M->hip_y[1];
        rads[0] = M->hip_r;
        nseg = 1;
      } else { /* thigh / calf: the halves, each from its outer end to the middle */
        const real* end = j == 1 ? M->origin[l][2] : M->foot;
        for (int i = 0; i < 3; ++i) {
          segs[0][1][i] = 0.5 * end[i];
          segs[1][0][i] = end[i];
          segs[1][1][i] = 0.5 * end[i];
        }
        rads[0] = rads[1] = j == 1 ? M->thigh_r : M->calf_r;
        nseg = 2;
        if (j == 2) { /* the foot sphere */
          for (int i = 0; i < 3; ++i) segs[2][0][i] = segs[2][1][i] = M->foot[i];
          rads[2] = M->foot_r;
          foot_seg = 2;
          nseg = 3;
        }
      }
      for (int p = 0; p < nseg; ++p) {
        real wA[3], wB[3], vA_[3], vB_[3], lp[3], pw[3], vw[3], F[3];
        point_kin(Rw[j], pw_[j], vj[l][j], segs[p][0], wA, vA_);
        point_kin(Rw[j], pw_[j], vj[l][j], segs[p][1], wB, vB_);
        int cell[3];
        const int slot = j == 0 ? 0 : 2 * j - 1 + p; /* hip; thigh 1, 2; calf 3, 4 */
        real t = 0.0;
        if (p != foot_seg) {
          if (seg_scan_now) S->seg_t[l][slot] = seg_deepest(T, wA, wB, rads[p], cell);
          t = S->seg_t[l][slot];
        }
        for (int i = 0; i < 3; ++i) lp[i] = segs[p][0][i] + t * (segs[p][1][i] - segs[p][0][i]);
        point_kin(Rw[j], pw_[j], vj[l][j], lp, pw, vw);
        if (g_implicit_contact) {
          real Mp[3][3] = {{0}};
          sphere_contact_im_cell(T, &C, pw, vw, rads[p], F, h, Mp, T->tile && seg_scan_now && p != foot_seg ? cell : NULL);
          point_inertia(Rw[j], lp, Mp, &IA[j]);
        } else {
          sphere_contact(T, &C, pw, vw, rads[p], F);
        }
        point_force(Rw[j], lp, F, fext);
        int bi = p == foot_seg ? body_idx + 1 : body_idx; /* foot body reported separately */
        if (cf) for (int i = 0; i < 3; ++i) cf[bi * 3 + i] += F[i];
      }
      for (int i = 0; i < 6; ++i) pA[j][i] -= fext[i];
    }
    /* backward pass calf -> hip */
    for (int j = 2; j >= 0; --j) {
      int ax = j == 0 ? 0 : 1, dof = l * 3 + j;
      real t = tau[dof];
      /* native joint-limit spring-damper at the URDF limits */
      /* implicit in the joint: the torque at the end of the sub-step, -k (q + h qd') - d qd'
         with qd' = qd + h qdd, moves (h d + h^2 k) qdd to the joint inertia D */
      real lo = cfg->hard_limits[dof * 2], hi = cfg->hard_limits[dof * 2 + 1], Dimp = 0.0;
      if (S->q[dof] > hi || S->q[dof] < lo) {
        real ex = S->q[dof] > hi ? S->q[dof] - hi : S->q[dof] - lo;
        t -= cfg->limit_stiffness * (ex + h * S->qd[dof]) + cfg->limit_damping * S->qd[dof];
        Dimp = h * cfg->limit_damping + h * h * cfg->limit_stiffness;
      }
      for (int i = 0; i < 6; ++i) U[l][j][i] = IA[j].m[i][ax];
      D[l][j] = IA[j].m[ax][ax] + Dimp;
      u[l][j] = t - pA[j][ax];
      M6 Ia;
      real pa[6], Iac[6];
      for (int a = 0; a < 6; ++a)
        for (int b = 0; b < 6; ++b) Ia.m[a][b] = IA[j].m[a][b] - U[l][j][a] * U[l][j][b] / D[l][j];
      m6_vec(&Ia, cj[l][j], Iac);
      for (int i = 0; i < 6; ++i) pa[i] = pA[j][i] + Iac[i] + U[l][j][i] * u[l][j] / D[l][j];
      M6 Ip;
      real pp2[6];
      xform_inertia_T(E[l][j], M->origin[l][j], &Ia, &Ip);
      xform_force_T(E[l][j], M->origin[l][j], pa, pp2);
      if (j > 0) {
        for (int a = 0; a < 6; ++a) for (int b = 0; b < 6; ++b) IA[j - 1].m[a][b] += Ip.m[a][b];
        for (int i = 0; i < 6; ++i) pA[j - 1][i] += pp2[i];
      } else {
        for (int a = 0; a < 6; ++a) for (int b = 0; b < 6; ++b) IA0.m[a][b] += Ip.m[a][b];
        for (int i = 0; i < 6; ++i) pA0[i] += pp2[i];
      }
    }
  }
  /* the trunk faces: vertices once per control step, the force every sim step (the tunnel only) */
  if (T->tile) {
    real wf[6] = {0, 0, 0, 0, 0, 0}, Ff[3] = {0, 0, 0};
    if (face_scan_now) face_scan(T, R, S->pos, M->trunk_half, S->face);
    face_force(T, &C, R, S->pos, vb, M->trunk_half, S->face, wf, Ff);
    for (int i = 0; i < 6; ++i) pA0[i] -= wf[i];
    if (cf) for (int i = 0; i < 3; ++i) cf[i] += Ff[i];
  }
  /* base acceleration */
  real a0[6], mp[6];
  for (int i = 0; i < 6; ++i) mp[i] = -pA0[i];
  solve6(&IA0, mp, a0);
  real qdd[NDOF];
  for (int l = 0; l < 4; ++l) {
    real ap[6];
    memcpy(ap, a0, sizeof(ap));
    for (int j = 0; j < 3; ++j) {
      int ax = j == 0 ? 0 : 1, dof = l * 3 + j;
      real aj[6];
      xform_motion(E[l][j], M->origin[l][j], ap, aj);
      for (int i = 0; i < 6; ++i) aj[i] += cj[l][j][i];
      real Ua = 0;
      for (int i = 0; i < 6; ++i) Ua += U[l][j][i] * aj[i];
      qdd[dof] = (u[l][j] - Ua) / D[l][j];
      aj[ax] += qdd[dof];
      memcpy(ap, aj, sizeof(ap));
    }
  }
  /* semi-implicit Euler: classical accelerations of the base in world coords */
  real wv[3], alin_b[3], aw[3], al[3];
  cross3(vb, vb + 3, wv);
  for (int i = 0; i < 3; ++i) alin_b[i] = a0[3 + i] + wv[i];
  for (int i = 0; i < 3; ++i) {
    aw[i] = R[i][0] * a0[0] + R[i][1] * a0[1] + R[i][2] * a0[2];
    al[i] = R[i][0] * alin_b[0] + R[i][1] * alin_b[1] + R[i][2] * alin_b[2];
  }
  for (int i = 0; i < 3; ++i) {
    S->w[i] += h * aw[i];
    S->v[i] += h * al[i];
    S->pos[i] += h * S->v[i];
  }
  {
    /* q <- exp(h w / 2) (x) q, world-frame angular velocity */
    real th = 0.5 * h * sqrt(S->w[0] * S->w[0] + S->w[1] * S->w[1] + S->w[2] * S->w[2]);
    real sc = th > 1e-12 ? sin(th) / (th / (0.5 * h)) : 0.5 * h;
    real dq[4] = {S->w[0] * sc, S->w[1] * sc, S->w[2] * sc, cos(th)};
    real* q = S->quat;
    real nq[4];
    nq[3] = dq[3] * q[3] - dq[0] * q[0] - dq[1] * q[1] - dq[2] * q[2];
    nq[0] = dq[3] * q[0] + dq[0] * q[3] + dq[1] * q[2] - dq[2] * q[1];
    nq[1] = dq[3] * q[1] - dq[0] * q[2] + dq[1] * q[3] + dq[2] * q[0];
    nq[2] = dq[3] * q[2] + dq[0] * q[1] - dq[1] * q[0] + dq[2] * q[3];
    real n = sqrt(nq[0] * nq[0] + nq[1] * nq[1] + nq[2] * nq[2] + nq[3] * nq[3]);
    for (int i = 0; i < 4; ++i) q[i] = nq[i] / n;
  }
  for (int d = 0; d < NDOF; ++d) {
    S->qd[d] += h * qdd[d];
    S->q[d] += h * S->qd[d];
  }
}

/* Mechanical energy of a state (physics invariant tests): the kinetic energy of the 13 rigid bodies plus
 * their potential energy in the gravity field g (world), with the integrator's kinematics and inertias. */
double go1o_energy(const go1_config* cfg, const double* pos, const double* quat, const double* v, const double* w,
                   const double* q, const double* qd, const double* g, double payload) {
  Model M;
  load_model(cfg, &M);
  real R[3][3], qt[4] = {quat[0], quat[1], quat[2], quat[3]};
  quat_to_R(qt, R);
  real vb[6];
  for (int i = 0; i < 3; ++i) {
    vb[i] = R[0][i] * w[0] + R[1][i] * w[1] + R[2][i] * w[2];
    vb[3 + i] = R[0][i] * v[0] + R[1][i] * v[1] + R[2][i] * v[2];
  }
  real mscale = (M.base.mass + payload) / M.base.mass, e = 0.0;
  M6 I;
  real hm[6];
  rigid_inertia(&M.base, mscale, &I);
  m6_vec(&I, vb, hm);
  for (int i = 0; i < 6; ++i) e += 0.5 * vb[i] * hm[i];
  for (int i = 0; i < 3; ++i) {
    real ci = pos[i] + R[i][0] * M.base.com[0] + R[i][1] * M.base.com[1] + R[i][2] * M.base.com[2];
    e -= M.base.mass * mscale * g[i] * ci;
  }
  for (int l = 0; l < 4; ++l) {
    real Rp[3][3], pp[3], vp[6];
    memcpy(Rp, R, sizeof(Rp));
    for (int i = 0; i < 3; ++i) pp[i] = pos[i];
    memcpy(vp, vb, sizeof(vp));
    for (int j = 0; j < 3; ++j) {
      int ax = j == 0 ? 0 : 1, dof = l * 3 + j;
      const real* r = M.origin[l][j];
      real E[3][3], vj[6], Rw[3][3], pw[3];
      joint_E(ax, q[dof], E);
      xform_motion(E, r, vp, vj);
      vj[ax] += qd[dof];
      for (int i = 0; i < 3; ++i) {
        pw[i] = pp[i] + Rp[i][0] * r[0] + Rp[i][1] * r[1] + Rp[i][2] * r[2];
        for (int k = 0; k < 3; ++k) Rw[i][k] = Rp[i][0] * E[k][0] + Rp[i][1] * E[k][1] + Rp[i][2] * E[k][2];
      }
      const Body* B = &M.leg[l][j];
      rigid_inertia(B, 1.0, &I);
      m6_vec(&I, vj, hm);
      for (int i = 0; i < 6; ++i) e += 0.5 * vj[i] * hm[i];
      for (int i = 0; i < 3; ++i) {
        real ci = pw[i] + Rw[i][0] * B->com[0] + Rw[i][1] * B->com[1] + Rw[i][2] * B->com[2];
        e -= B->mass * g[i] * ci;
      }
      memcpy(Rp, Rw, sizeof(Rp));
      memcpy(pp, pw, sizeof(pp));
      memcpy(vp, vj, sizeof(vp));
    }
  }
  return (double)e;
}

/* exposed for the physics invariant tests: run n substeps of length h on a
 * state given as doubles; tiles may be NULL (plane) */
void go1o_physics(const go1_config* cfg, double* pos, double* quat, double* v, double* w, double* q, double* qd,
                  const double* tau, int n_sub, double h, const double* g, double friction, double restitution,
                  double payload,
                  const float* tile, double ox, double oy, double* cf_out) {
  Model M;
  load_model(cfg, &M);
  PhysState S;
  real tr[NDOF], gr[3], cfr[NB * 3];
  for (int i = 0; i < 3; ++i) { S.pos[i] = pos[i]; S.v[i] = v[i]; S.w[i] = w[i]; gr[i] = g[i]; }
  for (int i = 0; i < 4; ++i) S.quat[i] = quat[i];
  for (int d = 0; d < NDOF; ++d) { S.q[d] = q[d]; S.qd[d] = qd[d]; tr[d] = tau[d]; }
  TerrainView T = {tile, cfg->hf_nx, cfg->hf_ny, ox, oy, cfg->horizontal_scale};
  /* the trunk-face vertices chosen once per control step (decimation x n_internal sim steps), as the kernel does */
  const int scan = cfg->decimation * cfg->n_internal > 0 ? cfg->decimation * cfg->n_internal : 1;
  for (int i = 0; i < n_sub; ++i)
    phys_substep(&M, cfg, &S, tr, (real)h, gr, (real)friction, (real)restitution, (real)payload, &T, cfr, i % scan == 0);
  for (int i = 0; i < 3; ++i) { pos[i] = S.pos[i]; v[i] = S.v[i]; w[i] = S.w[i]; }
  for (int i = 0; i < 4; ++i) quat[i] = S.quat[i];
  for (int d = 0; d < NDOF; ++d) { q[d] = S.q[d]; qd[d] = S.qd[d]; }
  if (cf_out)
    for (int i = 0; i < NB * 3; ++i) cf_out[i] = cfr[i];
}

/* ====================================================================== */
/*                              the step                                   */
/* ====================================================================== */
/* `lag` is the reference's 7-slot ring (lag_buffer, slot 0 oldest), expanded from the stored form by
 * step_env (lag_expand) and stored back after the physics (lag_store) */
static void compute_torques(const go1_config* c, const go1_state* st, int e, const float* act, float* torque,
                            float* lag) {
  float* eh = st->pos_err_hist + (size_t)e * 24;
  float* vh = st->vel_hist + (size_t)e * 24;
  const float* dp = st->dof_pos + (size_t)e * NDOF;
  const float* dv = st->dof_vel + (size_t)e * NDOF;
  /* actions_scaled (:969-970); lag push (:973-974) */
  float scaled[NDOF];
  for (int d = 0; d < NDOF; ++d) {
    scaled[d] = act[d] * c->action_scale;
    if (d % 3 == 0) scaled[d] = scaled[d] * c->hip_scale_reduction;
  }
  memmove(lag, lag + NDOF, sizeof(float) * NDOF * (GO1_LAG_SLOTS - 1));
  memcpy(lag + NDOF * (GO1_LAG_SLOTS - 1), scaled, sizeof(scaled));
  for (int d = 0; d < NDOF; ++d) {
    float tgt = lag[d] + c->default_dof_pos[d];
    st->joint_pos_target[(size_t)e * NDOF + d] = tgt;
    float err = dp[d] - tgt + st->motor_offset[(size_t)e * NDOF + d];
    float x[6] = {err, eh[d], eh[NDOF + d], dv[d], vh[d], vh[NDOF + d]};
    float t = go1o_actuator_eval(c->actuator, x);
    eh[NDOF + d] = eh[d];
    eh[d] = err;
    vh[NDOF + d] = vh[d];
    vh[d] = dv[d];
    t = t * st->motor_strength[(size_t)e * NDOF + d];
    float lim = c->torque_limits[d];
    torque[d] = t < -lim ? -lim : (t > lim ? lim : t);
  }
}

/* _reset_idx for one env (:218-296): DR, dofs, root, trajectory, buffers */
static void reset_env(const go1_config* c, const go1_state* st, const go1_terrain* ter, int e, const go1_step_args* a,
                      const float* U) {
  /* _randomize_dof_props (:744-754) */
  float us = draw(c, a, U, e, 0);
  float s = us * c->strength_range + c->strength_lo;
  for (int d = 0; d < NDOF; ++d) {
    st->motor_strength[(size_t)e * NDOF + d] = s;
    float uo = draw(c, a, U, e, 1 + d);
    st->motor_offset[(size_t)e * NDOF + d] = uo * c->offset_range + c->offset_lo;
  }
  /* _reset_dofs (:998-1008) */
  for (int d = 0; d < NDOF; ++d) {
    float u = draw(c, a, U, e, 13 + d);
    float f = c->reset_dof_range * u + c->reset_dof_lo;
    st->dof_pos[(size_t)e * NDOF + d] = c->default_dof_pos[d] * f;
    st->dof_vel[(size_t)e * NDOF + d] = 0.0f;
  }
  /* _reset_root_states (:1015-1052) */
  float* r = st->root + (size_t)e * 13;
  for (int i = 0; i < 13; ++i) r[i] = c->base_init_state[i];
  const float* eo = ter->env_origins + (size_t)e * 3;
  r[0] = r[0] + eo[0];
  r[1] = r[1] + eo[1];
  r[2] = r[2] + eo[2];
  if (c->custom_origins) {
    float ux = draw(c, a, U, e, 25), uy = draw(c, a, U, e, 26);
    r[0] = r[0] + (c->x_init_range2 * ux + c->x_init_lo);
    r[1] = r[1] + (c->y_init_range2 * uy + c->y_init_lo);
    r[0] = r[0] + c->x_init_offset;
    r[1] = r[1] + c->y_init_offset;
  }
  float yaw = c->yaw_range2 * draw(c, a, U, e, 27) + c->yaw_lo;
  /* quat_from_angle_axis(yaw, z) then quat_unit */
  float th = yaw / 2.0f;
  float sth, cth;
  pm_sincosf(th, &sth, &cth);
  float qv[4] = {0.0f * sth, 0.0f * sth, 1.0f * sth, cth};
  float qn = sqrtf(fmaf(qv[3], qv[3], fmaf(qv[2], qv[2], fmaf(qv[1], qv[1], qv[0] * qv[0]))));
  if (qn < 1e-9f) qn = 1e-9f;
  for (int i = 0; i < 4; ++i) r[3 + i] = qv[i] / qn;
  for (int i = 0; i < 6; ++i) r[7 + i] = c->reset_vel_range * draw(c, a, U, e, 28 + i) + c->reset_vel_lo;
  /* _resample_trajectory (:949-955) */
  st->curr_pose_index[e] = 0;
  float* tr = st->trajectory + (size_t)e * 6 * c->traj_length;
  const int ub = GO1_U_NOISE + c->num_obs; /* trajectory draws follow the obs-noise slots */
  if (c->traj_kind == 1) {
    /* _traj_fn_random_target (trajectory_function.py:70-93): traj_length / num_interp + 1 poses per
     * channel drawn x, y, z, yaw, pitch, roll (torch.rand * 2 * range - range); pose 0 := 0;
     * waypoint (s, j) = pose s + (j + 1) * (pose s+1 - pose s) / num_interp; then + base xyz */
    const int ni = c->traj_interp, nt = c->traj_length / ni + 1;
    const float rg[6] = {c->traj_x_range, c->traj_y_range, c->traj_z_range, c->traj_yaw_range,
                         c->traj_pitch_range, c->traj_roll_range};
    const int col[6] = {0, 1, 2, 5, 4, 3};
    float pose[6][GO1_MAX_TRAJ + 1];
    for (int ch = 0; ch < 6; ++ch)
      for (int t = 0; t < nt; ++t)
        pose[ch][t] = t == 0 ? 0.0f : draw(c, a, U, e, ub + ch * nt + t) * 2.0f * rg[ch] - rg[ch];
    for (int sg = 0; sg + 1 < nt; ++sg)
      for (int j = 0; j < ni; ++j)
        for (int ch = 0; ch < 6; ++ch) {
          float delta = (pose[ch][sg + 1] - pose[ch][sg]) / (float)ni;
          tr[(sg * ni + j) * 6 + col[ch]] = pose[ch][sg] + (float)(j + 1) * delta;
        }
    for (int w = 0; w < c->traj_length; ++w)
      for (int i = 0; i < 3; ++i) tr[w * 6 + i] = tr[w * 6 + i] + r[i];
  } else if (c->traj_kind == 2) {
    /* _traj_fn_random_goal (trajectory_function.py:28-41): one pose broadcast to every waypoint */
    float x = (draw(c, a, U, e, ub) - 0.5f) * c->traj_x_range + c->traj_x_mean;
    x = x + r[0];
    float y = (draw(c, a, U, e, ub + 1) - 0.5f) * c->traj_y_range + c->traj_y_mean;
    y = y + r[1];
    float yaw = draw(c, a, U, e, ub + 2) * 2.0f * c->traj_yaw_range - c->traj_yaw_range;
    for (int w = 0; w < c->traj_length; ++w) {
      float* o = tr + w * 6;
      o[0] = x; o[1] = y; o[2] = 0.0f + c->traj_base_z; o[3] = 0.0f; o[4] = 0.0f; o[5] = yaw;
    }
  } else {
    /* _traj_fn_fixed_target (trajectory_function.py:14-26): arange(1, T+1) * base_x + base x */
    for (int w = 0; w < c->traj_length; ++w) {
      float* o = tr + w * 6;
      float k = (float)(w + 1);
      o[0] = k * c->traj_base_x + r[0];
      o[1] = k * c->traj_base_y + r[1];
      o[2] = c->traj_base_z;
      o[3] = c->traj_roll;
      o[4] = c->traj_pitch;
      o[5] = c->traj_yaw;
    }
  }
  /* buffers (:246-254, :262, :273, :295-296) */
  for (int d = 0; d < NDOF; ++d) {
    st->last_actions[(size_t)e * NDOF + d] = 0.0f;
    st->last_dof_vel[(size_t)e * NDOF + d] = 0.0f;
  }
  st->episode_length[e] = 0;
  const int ns = c->n_terms + 3;
  for (int k = 0; k < ns; ++k) st->episode_sums[(size_t)e * ns + k] = 0.0f;
  for (int l = 0; l < 4; ++l) st->feet_air_time[(size_t)e * 4 + l] = 0.0f; /* (:248) */
  st->collision_count[e] = 0;
  const int K = GO1_LAG_STEPS(c->decimation);
  for (int i = 0; i < 12 * K; ++i) st->lag[(size_t)e * 12 * K + i] = 0.0f;
}

/* go1_state.lag (the scaled actions of the last K = GO1_LAG_STEPS(decimation) steps, oldest first) <->
 * the reference's ring of GO1_LAG_SLOTS per-sim-step pushes (:973-974): slot 6 - j is entry
 * K - 1 - floor(j / decimation) */
static void lag_expand(const go1_config* c, const float* stored, float* ring) {
  const int K = GO1_LAG_STEPS(c->decimation);
  for (int s = 0; s < GO1_LAG_SLOTS; ++s)
    memcpy(ring + s * NDOF, stored + (K - 1 - (GO1_LAG_SLOTS - 1 - s) / c->decimation) * NDOF, NDOF * sizeof(float));
}
static void lag_store(const go1_config* c, const float* ring, float* stored) {
  const int K = GO1_LAG_STEPS(c->decimation);
  for (int k = 0; k < K; ++k)
    memcpy(stored + k * NDOF, ring + (GO1_LAG_SLOTS - 1 - (K - 1 - k) * c->decimation) * NDOF, NDOF * sizeof(float));
}

int go1o_reset_envs(const go1_config* c, const go1_state* st, const go1_terrain* ter, const uint8_t* mask,
                    const float* U, uint64_t seed, uint64_t step) {
  go1_step_args a;
  memset(&a, 0, sizeof(a));
  a.rng_seed = seed;
  a.rng_step = step;
  for (int e = 0; e < c->n_envs; ++e)
    if (mask[e]) reset_env(c, st, ter, e, &a, U);
  return 0;
}

/* World position of leg l's foot body origin (rigid_body_state[:, feet, 0:3]) */
static void foot_world(const Model* M, const float* root, const float* dp, int l, float* out) {
  real qd4[4] = {root[3], root[4], root[5], root[6]};
  real R[3][3], Rp[3][3], pp[3] = {root[0], root[1], root[2]};
  quat_to_R(qd4, R);
  memcpy(Rp, R, sizeof(Rp));
  for (int j = 0; j < 3; ++j) {
    real E[3][3], Rw[3][3];
    const real* r = M->origin[l][j];
    for (int i = 0; i < 3; ++i) pp[i] += Rp[i][0] * r[0] + Rp[i][1] * r[1] + Rp[i][2] * r[2];
    joint_E(j == 0 ? 0 : 1, dp[l * 3 + j], E);
    for (int i = 0; i < 3; ++i)
      for (int k = 0; k < 3; ++k) Rw[i][k] = Rp[i][0] * E[k][0] + Rp[i][1] * E[k][1] + Rp[i][2] * E[k][2];
    memcpy(Rp, Rw, sizeof(Rp));
  }
  for (int i = 0; i < 3; ++i)
    out[i] = (float)(pp[i] + Rp[i][0] * M->foot[0] + Rp[i][1] * M->foot[1] + Rp[i][2] * M->foot[2]);
}

/* Full step for env e.  Returns nothing; writes outputs. */
#define GO1_DIVERGED 1.0e4f /* |state component| treated as a diverged integrator (HIP kernel) */

/* base velocities, projected gravity, relative target pose and rpy of a root state
 * (:119-136, _compute_relative_target_pose :922-932) */
static void post_kin(const float* root, const float* gravity_vec, const float* tr, float* blv, float* bav, float* pg,
                     float* rel_lin, float* rpy, float* rel_rot) {
  float q[4] = {root[3], root[4], root[5], root[6]};
  quat_rotate_inverse_f(q, root + 7, blv);
  quat_rotate_inverse_f(q, root + 10, bav);
  quat_rotate_inverse_f(q, gravity_vec, pg);
  float rel_in[3] = {tr[0] - root[0], tr[1] - root[1], tr[2] - root[2]};
  quat_apply_yaw_inverse_f(q, rel_in, rel_lin);
  quat_to_rpy_f(q, rpy);
  for (int i = 0; i < 3; ++i) rel_rot[i] = wrap_to_pi_f(tr[3 + i] - rpy[i]);
}

static void step_env(const go1_config* c, const Model* M, const go1_state* st, const go1_terrain* ter,
                     const go1_step_args* a, int e, float* r_slots) {
  const int n = c->n_envs;
  const float* U = a->uniforms;
  float act[NDOF];
  for (int d = 0; d < NDOF; ++d) {
    float x = a->actions[(size_t)e * NDOF + d];
    act[d] = x < -c->clip_actions ? -c->clip_actions : (x > c->clip_actions ? c->clip_actions : x);
  }
  float* root = st->root + (size_t)e * 13;
  float* dp = st->dof_pos + (size_t)e * NDOF;
  float* dv = st->dof_vel + (size_t)e * NDOF;
  float torque[NDOF];
  float cf[NB * 3];
  memset(cf, 0, sizeof(cf));
  const float* tile = NULL;
  real ox = 0, oy = 0;
  if (c->terrain_kind == 1) {
    tile = ter->tiles + (size_t)ter->env_tile[e] * 2 * c->hf_nx * c->hf_ny;
    ox = ter->env_terrain_origin[(size_t)e * 3];
    oy = ter->env_terrain_origin[(size_t)e * 3 + 1];
  }
  float ring[GO1_LAG_SLOTS * NDOF];
  float* lag_st = st->lag + (size_t)e * 12 * GO1_LAG_STEPS(c->decimation);
  lag_expand(c, lag_st, ring);
  PhysState S;
  if (!a->inj_dof) {
    for (int i = 0; i < 3; ++i) {
      S.pos[i] = root[i]; S.v[i] = root[7 + i]; S.w[i] = root[10 + i];
    }
    /* the integrator works relative to the env's terrain origin: world x, y reach ~100 m, where an f32
     * ulp is 7.6e-6 m, and the contact forces on a terrain step depend on x with ~1e3 s^-1 gain
     * (k * height gradient); root - origin is exact in f32 (Sterbenz) and keeps ~1e-7 m resolution */
    S.pos[0] = (real)root[0] - ox;
    S.pos[1] = (real)root[1] - oy;
    for (int i = 0; i < 4; ++i) S.quat[i] = root[3 + i];
    for (int d = 0; d < NDOF; ++d) { S.q[d] = dp[d]; S.qd[d] = dv[d]; }
  }
  for (int sub = 0; sub < c->decimation; ++sub) {
    compute_torques(c, st, e, act, torque, ring);
    if (a->dbg_torques)
      for (int d = 0; d < NDOF; ++d) a->dbg_torques[((size_t)sub * n + e) * NDOF + d] = torque[d];
    if (a->inj_dof) {
      const float* id = a->inj_dof + ((size_t)sub * n + e) * NDOF * 2;
      for (int d = 0; d < NDOF; ++d) { dp[d] = id[2 * d]; dv[d] = id[2 * d + 1]; }
    } else {
      real tau[NDOF], g[3] = {a->sim_gravity[0], a->sim_gravity[1], a->sim_gravity[2]};
      real cfd[NB * 3];
      for (int d = 0; d < NDOF; ++d) tau[d] = torque[d];
      TerrainView T = {tile, c->hf_nx, c->hf_ny, 0, 0, c->horizontal_scale};
      real h = (real)c->sim_dt / c->n_internal;
      for (int k = 0; k < c->n_internal; ++k)
        phys_substep(M, c, &S, tau, h, g, st->friction[e], st->restitution[e], st->payload[e], &T, cfd,
                     sub == 0 && k == 0);
      for (int d = 0; d < NDOF; ++d) { dp[d] = (float)S.q[d]; dv[d] = (float)S.qd[d]; }
      for (int i = 0; i < NB * 3; ++i) cf[i] = (float)cfd[i];
    }
  }
  lag_store(c, ring, lag_st);
  if (a->inj_dof) {
    for (int i = 0; i < 13; ++i) root[i] = a->inj_root[(size_t)e * 13 + i];
    for (int i = 0; i < NB * 3; ++i) cf[i] = a->inj_contact[(size_t)e * NB * 3 + i];
  } else {
    for (int i = 0; i < 3; ++i) {
      root[i] = (float)S.pos[i]; root[7 + i] = (float)S.v[i]; root[10 + i] = (float)S.w[i];
    }
    root[0] = (float)(S.pos[0] + ox);
    root[1] = (float)(S.pos[1] + oy);
    for (int i = 0; i < 4; ++i) root[3 + i] = (float)S.quat[i];
  }
  if (a->contact_forces)
    for (int i = 0; i < NB * 3; ++i) a->contact_forces[(size_t)e * NB * 3 + i] = cf[i];

  /* ---------------- post_physics_step (:114-169) */
  int ep = st->episode_length[e] + 1;
  st->episode_length[e] = ep;
  const int TL = c->traj_length, NT = c->n_terms, NS = NT + 3;
  int idx = st->curr_pose_index[e];
  /* the current waypoint trajectories[e, curr_pose_index[e]] (:850-853) */
  const float* traj_cur = st->trajectory + (size_t)e * 6 * TL + 6 * (idx < 0 ? 0 : (idx > TL - 1 ? TL - 1 : idx));
  float blv[3], bav[3], pg[3], rel_lin[3], rpy[3], rel_rot[3];
  post_kin(root, a->gravity_vec, traj_cur, blv, bav, pg, rel_lin, rpy, rel_rot);

  /* _get_heights (:1918-1965), camera pitch = previous step's base_rotation, or 0 with
   * rotate_camera (:1934-1939) */
  float* brot = st->base_rotation + (size_t)e * 3;
  float cam_pitch = c->rotate_camera ? 0.0f : brot[1];
  float heights[2][GO1_GRID_X][GO1_GRID_Y];
  if (c->terrain_kind == 1) {
    const float* eto = ter->env_terrain_origin + (size_t)e * 3;
    float cos_p = pm_cosf(cam_pitch);
    float camx = c->camera_offset_x * cos_p;
    float camy = 0.0f * cos_p;
    for (int i = 0; i < GO1_GRID_X; ++i)
      for (int j = 0; j < GO1_GRID_Y; ++j) {
        float px = c->height_grid_x[i] + root[0];
        float py = c->height_grid_y[j] + root[1];
        if (c->camera_zero) { px = px + camx; py = py + camy; }
        px = px - eto[0];
        py = py - eto[1];
        float fx = fminf(fmaxf(px / c->horizontal_scale, -1.0f), (float)c->hf_nx);
        float fy = fminf(fmaxf(py / c->horizontal_scale, -1.0f), (float)c->hf_ny);
        long ix = (long)fx;
        long iy = (long)fy;
        if (ix < 0) ix = 0;
        if (ix > c->hf_nx - 2) ix = c->hf_nx - 2;
        if (iy < 0) iy = 0;
        if (iy > c->hf_ny - 2) iy = c->hf_ny - 2;
        for (int layer = 0; layer < 2; ++layer)
          heights[layer][i][j] = tile[((size_t)layer * c->hf_nx + ix) * c->hf_ny + iy];
      }
  } else {
    for (int i = 0; i < GO1_GRID_X; ++i)
      for (int j = 0; j < GO1_GRID_Y; ++j) { heights[0][i][j] = 1.0f; heights[1][i][j] = 0.0f; }
  }
  if (a->dbg_heights) memcpy(a->dbg_heights + (size_t)e * 2 * GO1_GRID_X * GO1_GRID_Y, heights, sizeof(heights));

  for (int i = 0; i < 3; ++i) brot[i] = rpy[i];
  float cmd[2] = {rel_lin[0], rel_lin[1]}; /* command_type "xy" (:801-802) */

  /* DR every rand_interval (:822-824) */
  if (ep % c->rand_interval == 0) {
    float us = draw(c, a, U, e, 34);
    float s = us * c->strength_range + c->strength_lo;
    for (int d = 0; d < NDOF; ++d) {
      st->motor_strength[(size_t)e * NDOF + d] = s;
      st->motor_offset[(size_t)e * NDOF + d] = draw(c, a, U, e, 35 + d) * c->offset_range + c->offset_lo;
    }
  }
  /* switch / reached (:836-844): advance on reach, capped at the last waypoint */
  float rel_norm = norm2_f(rel_lin[0], rel_lin[1]);
  int switched = rel_norm < c->switch_dist;
  if (switched) { idx += 1; if (idx > TL - 1) idx = TL - 1; }
  st->curr_pose_index[e] = idx;
  int reached = switched && idx == TL - 1;
  if (a->dbg_reached) a->dbg_reached[e] = (uint8_t)reached;
  /* collision_count (:848): thigh x4, calf x4, base */
  static const int PEN[9] = {2, 6, 10, 14, 3, 7, 11, 15, 0};
  float coll = 0.0f;
  for (int k = 0; k < 9; ++k) {
    const float* f = cf + PEN[k] * 3;
    if (norm3_f(f[0], f[1], f[2]) > 0.1f) coll += 1.0f;
  }
  st->collision_count[e] += (int)coll;

  /* check_termination (:198-216) */
  int time_out = (float)ep > c->max_episode_length;
  int reset = time_out, diverged = 0;
  if (c->use_terminal_body_height && root[2] < c->terminal_body_height) reset = 1;
  if (c->terminate_end_of_trajectory && reached && (float)ep > c->t_reach) reset = 1; /* (:211-213) */
  if (c->use_terminal_body_rotation && pg[2] > 0.0f) reset = 1;                        /* (:215-216) */
  if (!a->inj_dof) { /* native-integrator divergence guard (see the HIP kernel) */
    int finite = 1;
    for (int i = 0; i < 13; ++i) finite = finite && fabsf(root[i]) < GO1_DIVERGED;
    for (int d = 0; d < NDOF; ++d) finite = finite && fabsf(dp[d]) < GO1_DIVERGED && fabsf(dv[d]) < GO1_DIVERGED;
    diverged = !finite;
    if (diverged) reset = 1;
    if (diverged && a->diverged_count) {
#pragma omp atomic
      a->diverged_count[0] += 1;
    }
  }

  /* compute_reward (:320-355): the container's reward functions for the nonzero-scaled terms
   * (reward_crawling.py, trajectory_tracking_reward.py), by go1_term id */
  float tv[GO1_T_COUNT];
  memset(tv, 0, sizeof(tv));
  {
    float x[NDOF];
    const float* ldv = st->last_dof_vel + (size_t)e * NDOF;
    const float* la = st->last_actions + (size_t)e * NDOF;
    for (int d = 0; d < NDOF; ++d) x[d] = sq_f(torque[d]);
    tv[GO1_T_TORQUES] = sum12_legs(x);
    for (int d = 0; d < NDOF; ++d) x[d] = sq_f((ldv[d] - dv[d]) / c->dt);
    tv[GO1_T_DOF_ACC] = sum12_legs(x);
    tv[GO1_T_COLLISION] = coll;
    for (int d = 0; d < NDOF; ++d) x[d] = sq_f(la[d] - act[d]);
    tv[GO1_T_ACTION_RATE] = sum12_legs(x);
    for (int d = 0; d < NDOF; ++d) {
      float lo = dp[d] - c->dof_pos_limits[2 * d];
      float hi = dp[d] - c->dof_pos_limits[2 * d + 1];
      float o = -(lo < 0.0f ? lo : 0.0f);
      x[d] = o + (hi > 0.0f ? hi : 0.0f);
    }
    tv[GO1_T_DOF_POS_LIMITS] = sum12_legs(x);
    for (int d = 0; d < NDOF; ++d) x[d] = sq_f(dv[d]);
    tv[GO1_T_DOF_VEL] = sum12_legs(x); /* trajectory_tracking_reward.py:21-23 */
    for (int d = 0; d < NDOF; ++d) x[d] = sq_f(dp[d] - c->default_dof_pos[d]);
    tv[GO1_T_DOF_POS] = sum12_legs(x); /* :31-33 */
  }
  tv[GO1_T_BASE_HEIGHT] = sq_f(root[2] - c->base_height_target);
  tv[GO1_T_ANG_VEL_XY] = sq_f(bav[0]) + sq_f(bav[1]);
  tv[GO1_T_ORIENTATION] = sq_f(pg[0]) + sq_f(pg[1]);
  float vxy2 = sq_f(blv[0]) + sq_f(blv[1]);
  float vmag = norm2_f(blv[0], blv[1]);
  tv[GO1_T_LARGE_VEL] = vxy2 * (vmag > 0.5f ? 1.0f : 0.0f); /* reward_crawling.py:53-56 */
  tv[GO1_T_LIN_VEL_Z] = sq_f(blv[2]);
  tv[GO1_T_REACHING_Z] = sq_f(rel_lin[2]);
  tv[GO1_T_REACHING_ROLL] = sq_f(rel_rot[0]);
  tv[GO1_T_REACHING_PITCH] = sq_f(rel_rot[1]);
  tv[GO1_T_REACHING_YAW_ABS] = sq_f(rel_rot[2]);
  tv[GO1_T_SURVIVE] = 1.0f;
  tv[GO1_T_REACH_GOAL] = reached ? 1.0f : 0.0f;
  tv[GO1_T_REACH_GOAL_T] = (reached ? 1.0f : 0.0f) * (float)ep;
  tv[GO1_T_REACH_GOAL_TR] = (reached ? 1.0f : 0.0f) * ((float)ep > c->t_reach ? 1.0f : 0.0f);
  tv[GO1_T_LINEAR_VEL] = norm3_f(blv[0], blv[1], blv[2]) > 0.7f ? 1.0f : 0.0f;
  {
    float mag = rel_norm;
    /* e2e (reward_crawling.py:61-77) */
    if (c->terminate_end_of_trajectory) {
      tv[GO1_T_E2E] = (mag < c->switch_dist ? 1.0f : 0.0f) * c->max_episode_length;
    } else {
      float r_e2e = expf(-vxy2 / c->tracking_sigma_lin);
      tv[GO1_T_E2E] = r_e2e * (mag < c->switch_dist ? 1.0f : 0.0f) * ((float)ep > c->t_reach ? 1.0f : 0.0f);
    }
    /* target velocity towards the waypoint (reward_crawling.py:83-87) */
    float tx = rel_lin[0] / (mag + 1e-6f) * c->target_lin_vel;
    float ty = rel_lin[1] / (mag + 1e-6f) * c->target_lin_vel;
    float gate = mag > c->lin_reaching_criterion ? 1.0f : 0.0f;
    tx = tx * gate;
    ty = ty * gate;
    float le = sq_f(tx - blv[0]) + sq_f(ty - blv[1]);
    /* exploration_lin (reward_crawling.py:79-108) / reaching_linear_vel */
    if (c->lin_vel_form == 1) {
      tv[GO1_T_EXPLORATION_LIN] = fabsf(tx - blv[0]) + fabsf(ty - blv[1]);
    } else if (c->lin_vel_form == 2) {
      tv[GO1_T_EXPLORATION_LIN] = le;
    } else if (c->lin_vel_form == 3) {
      float rx = tx / c->target_lin_vel * blv[0] / (vmag + 1e-6f);
      float ry = ty / c->target_lin_vel * blv[1] / (vmag + 1e-6f);
      float r = rx + ry;
      r = r * (vmag > c->small_vel_threshold ? 1.0f : 0.0f);
      r = r + expf(-(vmag * vmag) / c->tracking_sigma_lin) * (mag < c->lin_reaching_criterion ? 1.0f : 0.0f);
      tv[GO1_T_EXPLORATION_LIN] = r;
    } else {
      tv[GO1_T_EXPLORATION_LIN] = expf(-le / c->tracking_sigma_lin);
    }
    /* task (trajectory_tracking_reward.py:74-89), task_old (:51-55) */
    tv[GO1_T_TASK] = expf(-le / c->tracking_sigma_lin) * (mag < c->large_dist_threshold ? 1.0f : 0.0f);
    {
      float r = 0.5f / (0.5f + mag) / c->t_reach;
      tv[GO1_T_TASK_OLD] = r * ((float)ep > c->t_reach ? 1.0f : 0.0f);
    }
    /* exploration (:91-99) */
    {
      float r = blv[0] * rel_lin[0] + blv[1] * rel_lin[1];
      r = r / (mag + 1e-6f);
      r = r / (vmag + 1e-6f);
      tv[GO1_T_EXPLORATION] = r * (vmag > c->small_vel_threshold ? 1.0f : 0.0f);
    }
    /* stalling (:105-108) */
    tv[GO1_T_STALLING] = -((vmag < c->small_vel_threshold && mag > c->large_dist_threshold) ? 1.0f : 0.0f);
  }
  {
    /* exploration_yaw (reward_crawling.py:110-120) / reaching_yaw */
    float ta = rel_rot[2];
    float m = fabsf(ta);
    ta = ta / (m + 1e-6f) * c->target_ang_vel;
    ta = ta * (m > c->ang_reaching_criterion ? 1.0f : 0.0f);
    float ae = sq_f(ta - bav[2]);
    tv[GO1_T_EXPLORATION_YAW] = expf(-ae / c->tracking_sigma_ang);
  }
  if (c->term_mask & (1u << GO1_T_FEET_AIR_TIME)) {
    /* feet_air_time (trajectory_tracking_reward.py:126-137): mutates last_contacts / feet_air_time */
    float* air = st->feet_air_time + (size_t)e * 4;
    float* lc = st->last_contacts + (size_t)e * 4;
    float rl[4];
    for (int l = 0; l < 4; ++l) {
      int contact = cf[(4 + 4 * l) * 3 + 2] > 1.0f;
      int filt = contact || lc[l] != 0.0f;
      lc[l] = contact ? 1.0f : 0.0f;
      int first = air[l] > 0.0f && filt;
      air[l] = air[l] + c->dt;
      rl[l] = (air[l] - 0.5f) * (first ? 1.0f : 0.0f);
      air[l] = air[l] * (filt ? 0.0f : 1.0f);
    }
    tv[GO1_T_FEET_AIR_TIME] = (rl[0] + rl[1]) + (rl[2] + rl[3]); /* the HIP kernel's quad-sum order */
  }
  if (diverged) /* nothing of a diverged state reaches an output */
    memset(tv, 0, sizeof(tv));
  /* slot order (reward_scales order); pos / neg by the sign of the scale for sign-definite terms,
   * by the sign of the sum over envs (second pass, go1o_step) when some slot is indefinite */
  float rew = 0.0f, pos = 0.0f, neg = 0.0f;
  float* sums = st->episode_sums + (size_t)e * NS;
  for (int k = 0; k < NT; ++k) {
    int id = c->term_ids[k];
    float t = id == GO1_T_NONE ? 0.0f : tv[id];
    if (a->dbg_terms) a->dbg_terms[(size_t)e * GO1_MAX_TERMS + k] = t;
    if (id == GO1_T_NONE) continue;
    float r = t * a->reward_scales[k];
    rew = rew + r;
    if (a->reward_scales[k] >= 0.0f) pos = pos + r; else neg = neg + r;
    sums[k] = sums[k] + r;
    if (r_slots) r_slots[(size_t)e * GO1_MAX_TERMS + k] = r;
  }
  if (c->reward_mode == 1) rew = rew < 0.0f ? 0.0f : rew;                /* (:341-342) */
  else if (c->reward_mode == 2) rew = pos * expf(neg / c->sigma_rew_neg); /* (:343-344) */
  if (!c->indefinite_slots) {
    sums[NT] = sums[NT] + rew;
    sums[NT + 1] = sums[NT + 1] + pos;
    sums[NT + 2] = sums[NT + 2] + neg;
  } else if (c->reward_mode != 2) {
    sums[NT] = sums[NT] + rew;
  }

  /* reset_idx (:218-296) for this env.  self.commands is a VIEW of
   * local_relative_linear[:, :2] (:802), which reset_idx zeroes in place (:252),
   * so a reset env observes a zero command this step. */
  const int LOGW = NT + 6;
  if (a->episode_log && !reset) a->episode_log[(size_t)e * LOGW + NS] = 0.0f;
  if (reset && a->episode_log) { /* reset_idx logging (:256-271) */
    float* lg = a->episode_log + (size_t)e * LOGW;
    for (int k2 = 0; k2 < NS; ++k2) lg[k2] = sums[k2];
    lg[NS] = (float)ep;
    lg[NS + 1] = reached ? 1.0f : 0.0f;
    lg[NS + 2] = diverged ? 0.0f : norm3_f(rel_lin[0], rel_lin[1], rel_lin[2]);
  }
  if (reset) {
    reset_env(c, st, ter, e, a, U);
    cmd[0] = 0.0f;
    cmd[1] = 0.0f;
    if (diverged) { /* a diverged env observes (and stores as its pitch) its post-reset pose, and its
                       actuator-net history (never reset by reset_idx) is cleared (see the HIP kernel) */
      post_kin(root, a->gravity_vec, st->trajectory + (size_t)e * 6 * TL, blv, bav, pg, rel_lin, rpy, rel_rot);
      for (int i = 0; i < 3; ++i) brot[i] = rpy[i];
      for (int i = 0; i < 2 * NDOF; ++i) {
        st->pos_err_hist[(size_t)e * 2 * NDOF + i] = 0.0f;
        st->vel_hist[(size_t)e * 2 * NDOF + i] = 0.0f;
      }
    }
  }
  if (a->dbg_commands) { a->dbg_commands[e * 2] = cmd[0]; a->dbg_commands[e * 2 + 1] = cmd[1]; }

  /* compute_observations (:357-475) -- post-reset dof/root/episode length, pre-reset gravity/cmd/heights */
  const int NO = c->num_obs;
  float* o = a->obs + (size_t)e * NO;
  o[0] = pg[0]; o[1] = pg[1]; o[2] = pg[2];
  o[3] = cmd[0] * 1.0f; o[4] = cmd[1] * 1.0f;
  for (int d = 0; d < NDOF; ++d) {
    o[5 + d] = (dp[d] - c->default_dof_pos[d]) * c->obs_scale_dof_pos;
    o[17 + d] = dv[d] * c->obs_scale_dof_vel;
    o[29 + d] = act[d];
  }
  int k = 41;
  if (c->timestep_in_obs) o[k++] = (float)st->episode_length[e] / c->max_episode_length; /* (:375-377) */
  if (c->observe_heights) {
    int x_start = c->measure_front_half ? GO1_GRID_X / 2 + 1 : 0;
    float zroot = root[2];
    float cam_z = pm_sinf(cam_pitch) * c->camera_offset_norm;
    for (int layer = 0; layer < 2; ++layer)
      for (int i = x_start; i < GO1_GRID_X; ++i)
        for (int j = 0; j < GO1_GRID_Y; ++j) {
          float h = heights[layer][i][j];
          if (c->camera_zero) {
            h = h - zroot;
            h = h - cam_z;
            h = h < -0.3f ? -0.3f : (h > 0.3f ? 0.3f : h);
          } else {
            h = h < 0.0f ? 0.0f : (h > c->ceiling_height ? c->ceiling_height : h);
            h = h / c->ceiling_height;
            h = h - 0.5f;
          }
          o[k++] = h * c->obs_scale_heights;
        }
  }
  if (c->add_noise) {
    for (int i = 0; i < NO; ++i) {
      float nv = 0.0f;
      if (i < 3) nv = c->noise_gravity;
      else if (i >= 5 && i < 17) nv = c->noise_dof_pos;
      else if (i >= 17 && i < 29) nv = c->noise_dof_vel;
      float u = draw(c, a, U, e, GO1_U_NOISE + i);
      o[i] = o[i] + (2.0f * u - 1.0f) * nv;
    }
  }
  for (int i = 0; i < NO; ++i) {
    float v = o[i];
    o[i] = v < -c->clip_obs ? -c->clip_obs : (v > c->clip_obs ? c->clip_obs : v);
  }
  float* pv = a->priv + (size_t)e * GO1_NUM_PRIV;
  pv[0] = (st->friction[e] - c->priv_friction_shift) * c->priv_friction_scale;
  pv[1] = (st->restitution[e] - c->priv_rest_shift) * c->priv_rest_scale;
  for (int i = 0; i < 2; ++i) pv[i] = pv[i] < -c->clip_obs ? -c->clip_obs : (pv[i] > c->clip_obs ? c->clip_obs : pv[i]);

  if (a->aux) { /* TrajectoryTrackingEnv.step extras (trajectory_tracking/__init__.py:25-41) */
    float* ax = a->aux + (size_t)e * GO1_AUX;
    for (int i = 0; i < 3; ++i) { ax[i] = blv[i]; ax[3 + i] = bav[i]; }
    ax[6] = cmd[0];
    ax[7] = cmd[1];
    for (int l = 0; l < 4; ++l) foot_world(M, root, dp, l, ax + 8 + 3 * l);
    for (int d = 0; d < NDOF; ++d) ax[20 + d] = diverged ? 0.0f : torque[d];
  }

  /* epilogue (:148-153) */
  for (int d = 0; d < NDOF; ++d) {
    st->last_actions[(size_t)e * NDOF + d] = act[d];
    st->last_dof_vel[(size_t)e * NDOF + d] = dv[d];
  }
  a->rew[e] = rew;
  a->reset[e] = (uint8_t)reset;
  a->time_out[e] = (uint8_t)time_out;
}

int go1o_step(const go1_config* c, const go1_state* st, const go1_terrain* ter, const go1_step_args* a) {
  Model M;
  load_model(c, &M);
  int any = 0;
  const int n = c->n_envs;
  float* r_slots = c->indefinite_slots ? (float*)calloc((size_t)n * GO1_MAX_TERMS, sizeof(float)) : NULL;
#pragma omp parallel for schedule(static) reduction(| : any)
  for (int e = 0; e < n; ++e) {
    step_env(c, &M, st, ter, a, e, r_slots);
    any |= a->reset[e];
  }
  if (r_slots) {
    /* global pos / neg buckets (:330-336): sign of the sum of each slot over all envs */
    const int NT = c->n_terms, NS = NT + 3;
    double S[GO1_MAX_TERMS];
    for (int k = 0; k < NT; ++k) {
      S[k] = 0.0;
      for (int e = 0; e < n; ++e) S[k] += r_slots[(size_t)e * GO1_MAX_TERMS + k];
    }
    for (int e = 0; e < n; ++e) {
      float pos = 0.0f, neg = 0.0f;
      for (int k = 0; k < NT; ++k) {
        if (c->term_ids[k] == GO1_T_NONE) continue;
        float r = r_slots[(size_t)e * GO1_MAX_TERMS + k];
        if (S[k] >= 0.0) pos = pos + r;
        else if (S[k] <= 0.0) neg = neg + r;
      }
      float* t = a->reset[e] ? (a->episode_log ? a->episode_log + (size_t)e * (NT + 6) + NT : NULL)
                             : st->episode_sums + (size_t)e * NS + NT;
      if (c->reward_mode == 2) {
        float rw = pos * expf(neg / c->sigma_rew_neg);
        a->rew[e] = rw;
        if (t) t[0] = t[0] + rw;
      }
      if (t) {
        t[1] = t[1] + pos;
        t[2] = t[2] + neg;
      }
    }
    free(r_slots);
  }
  if (a->extras_time_outs && any)
    for (int e = 0; e < n; ++e) a->extras_time_outs[e] = a->time_out[e];
  return 0;
}

int go1o_abi_version(void) { return GO1_ABI_VERSION; }

/* test export (tests/test_oracle_contact.py): the spatial inertia of an added point mass */
void go1o_point_inertia(const double* Rb9, const double* lp9, const double* Mp9, double* out36) {
  real Rb[3][3], Mp[3][3], lp[3] = {(real)lp9[0], (real)lp9[1], (real)lp9[2]};
  M6 I;
  memset(&I, 0, sizeof(I));
  for (int i = 0; i < 9; ++i) { Rb[i / 3][i % 3] = (real)Rb9[i]; Mp[i / 3][i % 3] = (real)Mp9[i]; }
  point_inertia(Rb, lp, Mp, &I);
  for (int i = 0; i < 36; ++i) out36[i] = I.m[i / 6][i % 6];
}

// go1_velocity.hip -- MI355X (gfx950) fused Go1 velocity-tracking step + C ABI (include/go1_velocity.h).
//
// One go1_vel_step = one VelocityTrackingEasyEnv.step + HistoryWrapper.step
// (go1_gym/envs/base/legged_robot_velocity_tracking.py, bare :N below) in two launches:
//   go1_vel_step_kernel: 4 x [actuator-net torques (:925-964) -> the native articulated-body integrator
//     of go1_device.h (phys_substep, plane terrain)] -> post-physics (:108-154): kinematics, the gait
//     clock (_step_contact_targets :844-923), DR (:714-717), terminations (:156-166), the CoRL reward
//     terms and command sums (:281-318, go1_gym/envs/rewards/corl_rewards.py), reset_idx's state part
//     (:168-257), observations (:320-509), the epilogue (:144-149) and the appended obs_history row.
//   go1_vel_curriculum_kernel: workgroups 0 .. nblk - 1 run _resample_commands (:728-842) for the envs the
//     step reset (RewardThresholdCurriculum.update, Curriculum.sample: go1_gym/envs/base/curriculum.py) and
//     patch their observed commands, then the interval resample of the next step ahead of time, the per-env
//     draws split over the workgroups; the other workgroups shift the history (obs_history[:, 70:] -> the
//     new buffer) when the sliding window rewinds.
// Lane layout of the step kernel as in go1_step.hip: 16 lanes per env = 4 legs x 4 roles, four envs per
// one-wave block.  Post-physics arithmetic is f32 with contraction off in torch's operation order, the
// transcendentals of the gait clock and the rewards via f64 (correctly rounded f32 but for rare double
// roundings), so the results match oracle/vel_oracle.py to the ulp of numpy's own exp / sin / erf.
#include "go1_device.h"
#include "../../include/go1_velocity.h"

#include <algorithm>
#include <cstdlib>
#include <vector>

typedef const __attribute__((address_space(4))) go1_vel_config VCfg;
#define VLAG 2  // GO1_LAG_STEPS(decimation) for decimation 4..6 (go1_vel_create checks it)
#define SQRT2_F 1.41421353816986083984f  // (float)math.sqrt(2)
#define CAT_PRONK 0
#define CAT_TROT 1
#define CAT_PACE 2
#define CAT_BOUND 3

// ---------------------------------------------------------------- f64 draws (curriculum RandomState)
struct RngD {
  const double* U;  // parity mode (n_envs, GO1_VEL_D_PER_ENV) or nullptr
  uint64_t seed, step;
  int e, gid;
  __device__ double operator()(int slot) const {
    if (U) return U[(size_t)e * GO1_VEL_D_PER_ENV + slot];
    // numpy's random_sample from two 32-bit words: (a >> 5, b >> 6) -> 53 bits
    uint32_t c[4] = {(uint32_t)gid, 0x40000000u | ((uint32_t)slot >> 1), (uint32_t)step, (uint32_t)(step >> 32)};
    philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint32_t a = c[2 * (slot & 1)] >> 5, b = c[2 * (slot & 1) + 1] >> 6;
    return ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
  }
};

// ---------------------------------------------------------------- f32 helpers (torch order)
__device__ __forceinline__ float sin_rn(float x) { return (float)sin((double)x); }
__device__ __forceinline__ float cos_rn(float x) { return (float)cos((double)x); }
__device__ __forceinline__ float exp_rn(float x) { return (float)exp((double)x); }
__device__ __forceinline__ float erf_rn(float x) { return (float)erf((double)x); }
// torch.distributions.Normal(0, kappa).cdf: 0.5 (1 + erf((x - 0) (1 / kappa) / sqrt(2)))
__device__ __forceinline__ float normal_cdf(float x, float inv_kappa) {
  return 0.5f * (1.0f + erf_rn((x - 0.0f) * inv_kappa / SQRT2_F));
}
__device__ __forceinline__ float norm4_f(float a, float b, float c, float d) {
  return sqrtf(fmaf(d, d, fmaf(c, c, fmaf(b, b, a * a))));
}
// isaacgym.torch_utils.quat_apply: b + w t + xyz x t, t = 2 (xyz x b)
__device__ __forceinline__ void quat_apply_f(const float* a, const float* b, float* o) {
  float t[3] = {(a[1] * b[2] - a[2] * b[1]) * 2.0f, (a[2] * b[0] - a[0] * b[2]) * 2.0f,
                (a[0] * b[1] - a[1] * b[0]) * 2.0f};
  float c[3] = {a[1] * t[2] - a[2] * t[1], a[2] * t[0] - a[0] * t[2], a[0] * t[1] - a[1] * t[0]};
#pragma unroll
  for (int i = 0; i < 3; ++i) o[i] = (b[i] + a[3] * t[i]) + c[i];
}
__device__ __forceinline__ void normalize4_f(float* q) {
  float n = norm4_f(q[0], q[1], q[2], q[3]);
  if (n < 1e-9f) n = 1e-9f;
#pragma unroll
  for (int i = 0; i < 4; ++i) q[i] = q[i] / n;
}
// quat_from_angle_axis for a unit coordinate axis (then quat_unit)
__device__ __forceinline__ void quat_from_axis_f(float angle, int axis, float* q) {
  const float th = angle / 2.0f, s = sin_rn(th), c = cos_rn(th);
#pragma unroll
  for (int i = 0; i < 3; ++i) q[i] = (i == axis ? 1.0f : 0.0f) * s;
  q[3] = c;
  normalize4_f(q);
}
// isaacgym.torch_utils.quat_mul (the factored product)
__device__ __forceinline__ void quat_mul_f(const float* a, const float* b, float* o) {
  const float x1 = a[0], y1 = a[1], z1 = a[2], w1 = a[3], x2 = b[0], y2 = b[1], z2 = b[2], w2 = b[3];
  const float ww = (z1 + x1) * (x2 + y2), yy = (w1 - y1) * (w2 + z2), zz = (w1 + y1) * (w2 - z2);
  const float xx = ww + yy + zz;
  const float qq = 0.5f * (xx + (z1 - x1) * (x2 - y2));
  o[3] = qq - ww + (z1 - y1) * (y2 - z2);
  o[0] = qq - xx + (x1 + w1) * (x2 + w2);
  o[1] = qq - yy + (w1 - x1) * (y2 + z2);
  o[2] = qq - zz + (z1 + y1) * (w2 - x2);
}
// the value of leg I's lane of this lane's quad (the legs of an (env, role)), DPP quad_perm broadcast
template <int I>
__device__ __forceinline__ float quad_at(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), I * 0x55, 0xF, 0xF, true));
}
// (((0 + t0) + t1) + t2) + t3: the reference's `reward = 0; for i: reward += t_i` over the four feet
__device__ __forceinline__ float quad_seq_sum(float v) {
  return (((0.0f + quad_at<0>(v)) + quad_at<1>(v)) + quad_at<2>(v)) + quad_at<3>(v);
}
// obs column without noise (noise_vec 0): v + (2u - 1) * 0 changes only a -0.0 (to +0.0 for u >= 0.5)
__device__ __forceinline__ float noise_free(float v, bool add_noise, const Rng& rng, int slot) {
  if (add_noise && v == 0.0f && signbit(v)) {
    if (rng(slot) >= 0.5f) v = 0.0f;
  }
  return v;
}

// World position and velocity of this leg's foot body origin (rigid_body_state[:, feet, 0:3 / 7:10])
// from the base state and the leg's joints: motion transforms down the chain (xm), then the foot
// offset in the calf frame (point_kin).
__device__ void foot_state(const float* root, const float* q, const float* qd, int leg, float* fp, float* fv) {
  const float sx = (leg & 2) ? -1.0f : 1.0f, sy = (leg & 1) ? -1.0f : 1.0f;
  float Rp[9], pp[3] = {root[0], root[1], root[2]}, vb[6];
  quat_to_R(root + 3, Rp);
  mat3T_vec(Rp, root + 10, vb);
  mat3T_vec(Rp, root + 7, vb + 3);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    float o[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int i = 30 + 3 * j + k, sp = GO1_LEG_SIGN[i];
      o[k] = GO1_LEG_FL[i] * (sp == 0 ? 1.0f : (sp == 1 ? sx : (sp == 2 ? sy : sx * sy)));
    }
    const int ax = j == 0 ? 0 : 1;
    float sn, cn, vj[6], rw[3];
    pm_sincosf(q[j], &sn, &cn);
    xm(ax, cn, sn, offset_mask(j), o, vb, vj);
    vj[ax] += qd[j];
    mat3_vec(Rp, o, rw);
    pp[0] += rw[0]; pp[1] += rw[1]; pp[2] += rw[2];
#pragma unroll
    for (int a = 0; a < 3; ++a) rE(ax, cn, sn, Rp + 3 * a, Rp + 3 * a);
#pragma unroll
    for (int i = 0; i < 6; ++i) vb[i] = vj[i];
  }
  point_kin(Rp, pp, vb, GO1_MODEL_F32 + 13 * 10 + 4 * 9, fp, fv);
}

// reset_idx's state part for one env, on the lane of leg `leg` (:168-257 after _resample_commands):
// _randomize_dof_props (:663-683), _reset_dofs (:966-981), _reset_root_states (:983-1019, plane: no
// custom origins).  u(slot): the env's f32 uniforms.
template <class U>
__device__ void vel_reset_env(VCfg* v, const U& u, const float* eo, int leg, float* root, float* q, float* qd,
                              float* strength, float* offset) {
  const float s = u(GO1_VEL_U_RESET_DR) * v->strength_range + v->strength_lo;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int d = leg * 3 + j;
    strength[j] = s;
    offset[j] = u(GO1_VEL_U_RESET_DR + 1 + d) * v->offset_range + v->offset_lo;
    q[j] = v->default_dof_pos[d] * (v->reset_dof_range * u(GO1_VEL_U_RESET_DOF + d) + v->reset_dof_lo);
    qd[j] = 0.0f;
  }
#pragma unroll
  for (int i = 0; i < 13; ++i) root[i] = v->base_init_state[i];
  root[0] = root[0] + eo[0];
  root[1] = root[1] + eo[1];
  root[2] = root[2] + eo[2];
  const float yaw = v->yaw_range * u(GO1_VEL_U_RESET_YAW) + v->yaw_lo;
  quat_from_axis_f(yaw, 2, root + 3);
#pragma unroll
  for (int i = 0; i < 6; ++i) root[7 + i] = v->reset_vel_range * u(GO1_VEL_U_RESET_VEL + i) + v->reset_vel_lo;
}

// =====================================================================
//                          the fused step kernel
// =====================================================================
struct VArgs {
  go1_vel_state st;
  go1_vel_step_args a;
  const float* env_origins;
  int hist_w;      // obs_history row width (70 x history_len)
  int64_t hist_ld; // obs_history_out row stride (floats)
  // the curriculum launch's selection lists (CkRec, B = this step's resets, A = the next step's interval
  // resample, n_envs each) and their counts (B low, A high word); czero: the other slot's counts, cleared here
  // (the launch that read them has completed, stream order)
  int4* clist;
  unsigned long long* ccnt;
  unsigned long long* czero;
  int doA;
};

template <bool INJ>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(1, 1))) void go1_vel_step_kernel(
    const go1_config* __restrict__ c_gen, const go1_vel_config* __restrict__ v_gen, VArgs K) {
  CCfg* __restrict__ c = (CCfg*)c_gen;
  VCfg* __restrict__ v = (VCfg*)v_gen;
  const go1_vel_state& st = K.st;
  const go1_vel_step_args& A = K.a;
  const int lane = threadIdx.x & 63, leg = lane & 3, lq = lane >> 4;
  const int role = lane >> 4, el = (lane >> 2) & 3, sub16 = 4 * role + leg;
  const bool owner = role == 0;
  const int e = blockIdx.x * SEPB + el;  // n % 16 == 0 (go1_vel_create)
  MlpFrag F;
  mlp_load(c_gen->actuator, lane, F);
  __shared__ float s_mlp[MLP_PARK_FLOATS * 64];  // the fragments across the sub-step loop (mlp_park)
  mlp_park(F, s_mlp, lane);
  const Rng rng = {A.uniforms, A.rng_seed, A.rng_step, e, e + c->env_id_offset, GO1_VEL_U_PER_ENV};
  const size_t d0 = (size_t)e * NDOF + leg * 3;
  const int dec = c->decimation;
  const float* lag_in = st.lag + (size_t)e * 12 * VLAG + leg * 3;
  const int NT = v->n_terms;

  // ---------------- load
  float act[3], q[3], qd[3], eh[2][3], vh[2][3], strength[3], offset[3], dflt[3], tlim[3], lag_pre[VLAG][3];
  float ldv[3], la[3], lla[3], ljpt[3], lljpt[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    act[j] = clampf(A.actions[d0 + j], -c->clip_actions, c->clip_actions);
    q[j] = st.dof_pos[d0 + j];
    qd[j] = st.dof_vel[d0 + j];
    strength[j] = st.motor_strength[d0 + j];
    offset[j] = st.motor_offset[d0 + j];
    eh[0][j] = st.pos_err_hist[(size_t)e * 24 + leg * 3 + j];
    eh[1][j] = st.pos_err_hist[(size_t)e * 24 + 12 + leg * 3 + j];
    vh[0][j] = st.vel_hist[(size_t)e * 24 + leg * 3 + j];
    vh[1][j] = st.vel_hist[(size_t)e * 24 + 12 + leg * 3 + j];
    dflt[j] = c->default_dof_pos[leg * 3 + j];
    tlim[j] = c->torque_limits[leg * 3 + j];
#pragma unroll
    for (int k = 0; k < VLAG; ++k) lag_pre[k][j] = lag_in[k * 12 + j];
    ldv[j] = st.last_dof_vel[d0 + j];
    la[j] = st.last_actions[d0 + j];
    lla[j] = st.last_last_actions[d0 + j];
    ljpt[j] = st.last_joint_pos_target[d0 + j];
    lljpt[j] = st.last_last_joint_pos_target[d0 + j];
  }
  const float friction = st.friction[e], payload = st.payload[e], restitution = st.restitution[e];
  __shared__ __attribute__((aligned(16))) float s_self[SEPB][SELF_ENV_FLOATS];  // self-collision scratch
  const float eo_pre[3] = {K.env_origins[(size_t)e * 3], K.env_origins[(size_t)e * 3 + 1],
                           K.env_origins[(size_t)e * 3 + 2]};
  const int ep_in = st.episode_length[e];
  const float gait_in = st.gait_indices[e];
  const float lc_in = st.last_contacts[(size_t)e * 4 + leg];
  // the curriculum's record of the env (category and bin before the resample), with the prologue loads
  const int cat_in = st.command_categories[e], bin_in = st.command_bins[e];
  // reward slots: lane sub16 holds slots sub16 and 16 + sub16 (command sums: NT + 5 of them, episode sums
  // NT + 1: the terms, then "total")
  const int NC = NT + GO1_VEL_SUM_EXTRA, NE = NT + 1;
  float cs[2], es[2];
  float my_scale[2];
  int my_id[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = sub16 + 16 * h;
    cs[h] = k < NC ? st.command_sums[(size_t)e * NC + k] : 0.0f;
    es[h] = k < NE ? st.episode_sums[(size_t)e * NE + k] : 0.0f;
    my_scale[h] = k < NT ? A.reward_scales[k] : 0.0f;
    my_id[h] = k < NT ? v_gen->term_ids[k] : -1;
  }
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
  const Terr T = {nullptr, 0, 0, 1.0f, nullptr, 0, 0};  // the plane: floor z = 0, no ceiling
  float scaled[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    scaled[j] = act[j] * c->action_scale;
    if (j == 0) scaled[j] = scaled[j] * c->hip_scale_reduction;
  }

  // ---------------- decimation loop (:76-82): lag ring pushed per sim step (:940-942)
  float torque[3], tgt[3];
  float cf_raw[CF_RAW] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, cf_leg[9], cf_base[3], cf_hip[3];
  for (int sub = 0; sub < dec; ++sub) {
    {
      const int m = 6 - sub;
      const int back = m <= 0 ? 0 : (m + dec - 1) / dec;
      float xin[3][6];
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        float lg = scaled[j];
#pragma unroll
        for (int k = 0; k < VLAG; ++k) lg = back == VLAG - k ? lag_pre[k][j] : lg;
        tgt[j] = lg + dflt[j];
        const float err = q[j] - tgt[j] + offset[j];
        xin[j][0] = err; xin[j][1] = eh[0][j]; xin[j][2] = eh[1][j];
        xin[j][3] = qd[j]; xin[j][4] = vh[0][j]; xin[j][5] = vh[1][j];
      }
      float tq[3] = {0.0f, 0.0f, 0.0f}, b0[3], b1v[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const float* y = xin[j];
        b0[j] = sel4(lq, y[0], y[1], y[2], y[3]);
        b1v[j] = sel4(lq, y[4], y[5], 0.0f, 0.0f);
      }
      {
        MlpFrag Fs;
        mlp_unpark(Fs, s_mlp, lane);
        mlp_group3(Fs, b0, b1v, tq);
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        eh[1][j] = eh[0][j];
        eh[0][j] = xin[j][0];
        vh[1][j] = vh[0][j];
        vh[0][j] = qd[j];
        torque[j] = clampf(tq[j] * strength[j], -tlim[j], tlim[j]);
      }
    }
    if (INJ) {
      const float* id = A.inj_dof + ((size_t)sub * c->n_envs + e) * NDOF * 2;
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
        const bool last = (sub == dec - 1) && (k == c->n_internal - 1);
        phys_substep(c, nullptr, P, torque, h, A.sim_gravity, friction, restitution, payload, T, leg, role, last,
                     cf_raw, s_self[el], sub == 0 && k == 0);
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) { q[j] = P.q[j]; qd[j] = P.qd[j]; }
    }
    if (A.dbg_torques && owner) {
#pragma unroll
      for (int j = 0; j < 3; ++j) A.dbg_torques[((size_t)sub * c->n_envs + e) * NDOF + leg * 3 + j] = torque[j];
    }
  }
  // the commands are first read by the post-physics (the gait clock): loaded here, not with the prologue, so
  // that they do not occupy 15 registers through the sub-steps (the self-collision narrow phase needs them)
  float cmd[GO1_VEL_NUM_COMMANDS];
#pragma unroll
  for (int k = 0; k < GO1_VEL_NUM_COMMANDS; ++k) cmd[k] = st.commands[(size_t)e * GO1_VEL_NUM_COMMANDS + k];
  float root[13], fp[3], fv[3];
  if (INJ) {
#pragma unroll
    for (int i = 0; i < 13; ++i) root[i] = A.inj_root[(size_t)e * 13 + i];
    const float* ic = A.inj_contact + (size_t)e * NB * 3;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      cf_base[i] = ic[i];
      cf_hip[i] = ic[(1 + leg * 4) * 3 + i];
    }
#pragma unroll
    for (int b = 0; b < 3; ++b)
#pragma unroll
      for (int i = 0; i < 3; ++i) cf_leg[b * 3 + i] = ic[(2 + leg * 4 + b) * 3 + i];
    const float* ft = A.inj_feet + ((size_t)e * 4 + leg) * 6;
#pragma unroll
    for (int i = 0; i < 3; ++i) { fp[i] = ft[i]; fv[i] = ft[3 + i]; }
  } else {
    cf_sum(cf_raw, role, cf_leg, cf_base, cf_hip);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      root[i] = P.pos[i]; root[7 + i] = P.wv[i].y; root[10 + i] = P.wv[i].x;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) root[3 + i] = P.quat[i];
    foot_state(root, q, qd, leg, fp, fv);
  }
  if (A.contact_forces && owner) {
    float* o = A.contact_forces + (size_t)e * NB * 3;
    if (leg == 0) { o[0] = cf_base[0]; o[1] = cf_base[1]; o[2] = cf_base[2]; }
    float* ol = o + (1 + leg * 4) * 3;
    ol[0] = cf_hip[0]; ol[1] = cf_hip[1]; ol[2] = cf_hip[2];
#pragma unroll
    for (int i = 0; i < 9; ++i) ol[3 + i] = cf_leg[i];
  }

  // ================= post_physics_step (:108-154), contraction off =================
  const int ep = ep_in + 1;
  float blv[3], bav[3], pg[3];
  {
    const float qb[4] = {root[3], root[4], root[5], root[6]};
    quat_rotate_inverse_f(qb, root + 7, blv);
    quat_rotate_inverse_f(qb, root + 10, bav);
    quat_rotate_inverse_f(qb, A.gravity_vec, pg);
  }
  // ---- _step_contact_targets (:844-923): this lane's foot
  const float gait = remainder_f(gait_in + v->dt * cmd[4], 1.0f);
  float fi_raw;
  {
    const float ph = cmd[5], off = cmd[6], bnd = cmd[7];
    const float f0 = ((gait + ph) + off) + bnd, f1 = gait + off, f2_ = gait + bnd, f3 = gait + ph;
    fi_raw = sel4(leg, f0, f1, f2_, f3);  // (bit-test selects: an equality chain on leg compiles to a switch)
  }
  const float foot_idx = remainder_f(fi_raw, 1.0f);  // self.foot_indices
  float fiw = fi_raw;
  {
    const float dur = cmd[8], r = remainder_f(fi_raw, 1.0f);
    if (r < dur) fiw = r * (0.5f / dur);
    else if (r > dur) fiw = 0.5f + (r - dur) * (0.5f / (1.0f - dur));
  }
  const float clock = sin_rn(TWO_PI_F * fiw);
  float desired;
  {
    const float ik = 1.0f / v->kappa_gait_probs, r = remainder_f(fiw, 1.0f);
    desired = normal_cdf(r, ik) * (1.0f - normal_cdf(r - 0.5f, ik)) +
              normal_cdf(r - 1.0f, ik) * (1.0f - normal_cdf((r - 0.5f) - 1.0f, ik));
  }
  if (A.dbg_gait && owner) {
    float* g = A.dbg_gait + (size_t)e * 12;
    g[leg] = foot_idx;
    g[4 + leg] = clock;
    g[8 + leg] = desired;
  }
  // ---- DR every rand_interval (:714-717)
  // slots 2 .. 14 = Philox blocks 0 .. 3: lane sub16 < 4 of the env draws block sub16 into LDS and the
  // env's lanes read their slots back (one evaluation per lane instead of four in a row; one wave per
  // block: its LDS operations complete in order)
  __shared__ float s_u[SEPB][48];
  const bool dr_step = ep % v->rand_interval == 0;
  if (dr_step) {
    if (sub16 < 4) {
      float uq[4];
      rng.quad(sub16, uq);
#pragma unroll
      for (int k = 0; k < 4; ++k) s_u[el][4 * sub16 + k] = uq[k];
    }
    const float sv = s_u[el][GO1_VEL_U_DR] * v->strength_range + v->strength_lo;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      strength[j] = sv;
      offset[j] = s_u[el][GO1_VEL_U_DR + 1 + leg * 3 + j] * v->offset_range + v->offset_lo;
    }
  }
  // ---- check_termination (:156-166): base contact, time-out, body height (measured_heights = 0 on a plane)
  const bool time_out = (float)ep > v->max_episode_length;
  bool reset = norm3_f(cf_base[0], cf_base[1], cf_base[2]) > 1.0f || time_out;
  if (v->use_terminal_body_height && root[2] < v->terminal_body_height) reset = true;
  bool diverged = false;
  if (!INJ) {  // native-integrator divergence guard (go1_step.hip): the env is reset, its rewards zeroed
    bool finite = true;
#pragma unroll
    for (int i = 0; i < 13; ++i) finite = finite & (fabsf(root[i]) < GO1_DIVERGED);
#pragma unroll
    for (int j = 0; j < 3; ++j) finite = finite & (fabsf(q[j]) < GO1_DIVERGED) & (fabsf(qd[j]) < GO1_DIVERGED);
    diverged = qsum(finite ? 0.0f : 1.0f) != 0.0f;
    if (diverged) reset = true;
  }

  // ---- compute_reward (:281-318): CoRLRewards terms filed by id in an LDS row per env
  __shared__ float s_terms[SEPB][GO1_VT_COUNT];
#define PUT(id, val)                           \
  do {                                         \
    const float v_ = (val);                    \
    if (sub16 == 0) s_terms[el][(id)] = v_;    \
  } while (0)
  auto sum12 = [](const float* x) { return qsum((x[0] + x[1]) + x[2]); };
  {
    const float d0_ = cmd[0] - blv[0], d1_ = cmd[1] - blv[1];
    PUT(GO1_VT_TRACKING_LIN_VEL, exp_rn(-(d0_ * d0_ + d1_ * d1_) / v->tracking_sigma));
    const float dz = cmd[2] - bav[2];
    PUT(GO1_VT_TRACKING_ANG_VEL, exp_rn(-(dz * dz) / v->tracking_sigma_yaw));
  }
  PUT(GO1_VT_LIN_VEL_Z, blv[2] * blv[2]);
  PUT(GO1_VT_ANG_VEL_XY, bav[0] * bav[0] + bav[1] * bav[1]);
  PUT(GO1_VT_ORIENTATION, pg[0] * pg[0] + pg[1] * pg[1]);
  {
    float x[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) x[j] = torque[j] * torque[j];
    PUT(GO1_VT_TORQUES, sum12(x));
#pragma unroll
    for (int j = 0; j < 3; ++j) x[j] = qd[j] * qd[j];
    PUT(GO1_VT_DOF_VEL, sum12(x));
#pragma unroll
    for (int j = 0; j < 3; ++j) { const float a = (ldv[j] - qd[j]) / v->dt; x[j] = a * a; }
    PUT(GO1_VT_DOF_ACC, sum12(x));
#pragma unroll
    for (int j = 0; j < 3; ++j) { const float a = la[j] - act[j]; x[j] = a * a; }
    PUT(GO1_VT_ACTION_RATE, sum12(x));
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int d = leg * 3 + j;
      const float lo = fminf(q[j] - v->dof_pos_limits[2 * d], 0.0f);
      const float hi = fmaxf(q[j] - v->dof_pos_limits[2 * d + 1], 0.0f);
      x[j] = -lo + hi;
    }
    PUT(GO1_VT_DOF_POS_LIMITS, sum12(x));
#pragma unroll
    for (int j = 0; j < 3; ++j) { const float a = q[j] - v->default_dof_pos[leg * 3 + j]; x[j] = a * a; }
    PUT(GO1_VT_DOF_POS, sum12(x));
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float a = tgt[j] - ljpt[j];
      x[j] = (a * a) * (la[j] != 0.0f ? 1.0f : 0.0f);
    }
    PUT(GO1_VT_ACTION_SMOOTHNESS_1, sum12(x));
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float a = tgt[j] - 2.0f * ljpt[j] + lljpt[j];
      x[j] = ((a * a) * (la[j] != 0.0f ? 1.0f : 0.0f)) * (lla[j] != 0.0f ? 1.0f : 0.0f);
    }
    PUT(GO1_VT_ACTION_SMOOTHNESS_2, sum12(x));
  }
  {  // collision on thighs and calves (penalize_contacts_on): integer counts, exact in any order
    const float th = norm3_f(cf_leg[0], cf_leg[1], cf_leg[2]) > 0.1f ? 1.0f : 0.0f;
    const float ca = norm3_f(cf_leg[3], cf_leg[4], cf_leg[5]) > 0.1f ? 1.0f : 0.0f;
    PUT(GO1_VT_COLLISION, qsum(th) + qsum(ca));
  }
  {
    const float d = root[2] - (cmd[3] + v->base_height_target);
    PUT(GO1_VT_JUMP, -(d * d));
  }
  {
    const float ff = norm3_f(cf_leg[6], cf_leg[7], cf_leg[8]);
    const float tf = -(1.0f - desired) * (1.0f - exp_rn(-1.0f * (ff * ff) / v->gait_force_sigma));
    PUT(GO1_VT_TRACKING_CONTACTS_SHAPED_FORCE, quad_seq_sum(tf) / 4.0f);
    const float vv = norm3_f(fv[0], fv[1], fv[2]);
    const float tv = -(desired * (1.0f - exp_rn(-1.0f * (vv * vv) / v->gait_vel_sigma)));
    PUT(GO1_VT_TRACKING_CONTACTS_SHAPED_VEL, quad_seq_sum(tv) / 4.0f);
  }
  // feet_slip (corl:107-113) updates last_contacts when it is evaluated
  const bool slip_live = [&] {
    bool l = false;
    for (int k = 0; k < NT; ++k) l = l || v->term_ids[k] == GO1_VT_FEET_SLIP;
    return l;
  }();
  const bool contact = cf_leg[8] > 1.0f;
  {
    const bool filt = contact || lc_in != 0.0f;
    const float sp = norm2_f(fv[0], fv[1]);
    PUT(GO1_VT_FEET_SLIP, qsum((filt ? 1.0f : 0.0f) * (sp * sp)));
  }
  {  // feet_clearance_cmd_linear (corl:130-135)
    const float phs = 1.0f - fabsf(1.0f - clampf(foot_idx * 2.0f - 1.0f, 0.0f, 1.0f) * 2.0f);
    const float th = cmd[9] * phs + 0.02f;
    const float d = th - fp[2];
    PUT(GO1_VT_FEET_CLEARANCE_CMD_LINEAR, qsum((d * d) * (1.0f - desired)));
  }
  {  // orientation_control (corl:181-193)
    float qr[4], qp[4], dq[4], dpg[3];
    quat_from_axis_f(-cmd[11], 0, qr);
    quat_from_axis_f(-cmd[10], 1, qp);
    quat_mul_f(qr, qp, dq);
    quat_rotate_inverse_f(dq, A.gravity_vec_after, dpg);
    const float a = pg[0] - dpg[0], b = pg[1] - dpg[1];
    PUT(GO1_VT_ORIENTATION_CONTROL, a * a + b * b);
  }
  {  // raibert_heuristic (corl:195-237)
    const float rel[3] = {fp[0] - root[0], fp[1] - root[1], fp[2] - root[2]};
    float qy[4] = {0.0f, 0.0f, -root[5], root[6]};  // quat_apply_yaw(quat_conjugate(base_quat), .)
    normalize4_f(qy);
    float fb[3];
    quat_apply_f(qy, rel, fb);
    const float w = cmd[12], ln = cmd[13];
    const float ys = (leg & 1) ? -w / 2.0f : w / 2.0f;
    const float xs = (leg & 2) ? -ln / 2.0f : ln / 2.0f;
    const float phs = fabsf(1.0f - foot_idx * 2.0f) * 1.0f - 0.5f;
    const float freq = cmd[4];
    const float y_vel = cmd[2] * ln / 2.0f;
    float yo = phs * y_vel * (0.5f / freq);
    if (leg >= 2) yo = yo * -1.0f;
    const float xo = phs * cmd[0] * (0.5f / freq);
    const float ex = fabsf((xs + xo) - fb[0]), ey = fabsf((ys + yo) - fb[1]);
    PUT(GO1_VT_RAIBERT_HEURISTIC, qsum(ex * ex + ey * ey));
  }
#undef PUT
  // slot order (:289-301): rew += term * scale; pos / neg by the slot's fixed sign; episode and
  // command sums per slot lane
  __shared__ float s_r[SEPB][GO1_VEL_MAX_TERMS];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = sub16 + 16 * h;
    if (k < NT) {
      float t = s_terms[el][my_id[h]];
      if (diverged) t = 0.0f;
      if (A.dbg_terms) A.dbg_terms[(size_t)e * GO1_VEL_MAX_TERMS + k] = t;
      const float r = t * my_scale[h];
      s_r[el][k] = r;
      es[h] = es[h] + r;
      const bool shaped = my_id[h] == GO1_VT_TRACKING_CONTACTS_SHAPED_FORCE ||
                          my_id[h] == GO1_VT_TRACKING_CONTACTS_SHAPED_VEL;
      cs[h] = cs[h] + (shaped ? my_scale[h] + r : r);
    }
  }
  float rew = 0.0f, pos = 0.0f, neg = 0.0f;
  {
    const uint32_t np = v->nonpos_slots;
    for (int k = 0; k < NT; ++k) {
      const float r = s_r[el][k];
      rew = rew + r;
      if ((np >> k) & 1u) neg = neg + r; else pos = pos + r;
    }
  }
  if (v->reward_mode == 1) rew = rew < 0.0f ? 0.0f : rew;
  else if (v->reward_mode == 2) rew = pos * exp_rn(neg / v->sigma_rew_neg);
  if (diverged) rew = 0.0f;
  // episode_sums["total"] (:306) and the command-sum extras (:314-318)
  {
    const float rx = blv[0] - cmd[0], rz = bav[2] - cmd[2];
    const float extra[GO1_VEL_SUM_EXTRA] = {blv[0], bav[2], rx * rx, rz * rz, 1.0f};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = sub16 + 16 * h;
      if (k == NT) es[h] = es[h] + rew;
      if (k >= NT && k < NC && !diverged) cs[h] = cs[h] + extra[min(max(k - NT, 0), GO1_VEL_SUM_EXTRA - 1)];
    }
  }

  // ---- reset_idx (:168-257) state part; the commands are resampled by the curriculum launch
  float lla_out[3], la_obs[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) { la_obs[j] = la[j]; }
  float gait_out = gait;
  if (A.episode_log_count) {
    const uint64_t rmask = __ballot(reset && owner && leg == 0);
    if (rmask != 0ull) {
      int base = 0;
      if (lane == 0) base = atomicAdd(A.episode_log_count, __popcll(rmask));
      base = __shfl(base, 0);
      const int row = base + __popcll(rmask & ((1ull << (4 * el)) - 1ull));
      if (reset && A.episode_log_cap > 0) {  // a ring: the newest rows overwrite the oldest
        float* lg = A.episode_log + (size_t)((uint32_t)row % (uint32_t)A.episode_log_cap) * (NE + 2);
#pragma unroll
        for (int h = 0; h < 2; ++h)
          if (sub16 + 16 * h < NE) lg[sub16 + 16 * h] = es[h];
        if (sub16 == 0) { lg[NE] = __int_as_float(A.episode_log_tag); lg[NE + 1] = (float)e; }
      }
    }
  }
  if (reset) {
    __shared__ float s_ru[SEPB][48];
    // the reset's uniforms (slots 12 .. 59 = Philox blocks 3 .. 14): lane sub16 < 12 draws block 3 + sub16
    if (sub16 < 12) {
      float uq[4];
      rng.quad(3 + sub16, uq);
#pragma unroll
      for (int k = 0; k < 4; ++k) s_ru[el][4 * sub16 + k] = uq[k];
    }
    const float* ru = s_ru[el];
    auto u = [ru](int slot) { return ru[slot - 12]; };
    vel_reset_env(v, u, eo_pre, leg, root, q, qd, strength, offset);
#pragma unroll
    for (int j = 0; j < 3; ++j) la_obs[j] = 0.0f;
    gait_out = 0.0f;
#pragma unroll
    for (int h = 0; h < 2; ++h) es[h] = 0.0f;
    if (diverged) {  // observe the post-reset pose; clear the actuator-net history of the diverged state
      const float qb[4] = {root[3], root[4], root[5], root[6]};
      quat_rotate_inverse_f(qb, A.gravity_vec, pg);
#pragma unroll
      for (int j = 0; j < 3; ++j) eh[0][j] = eh[1][j] = vh[0][j] = vh[1][j] = 0.0f;
    }
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) lla_out[j] = la_obs[j];  // epilogue: last_last_actions <- last_actions

  // ---- compute_observations (:320-509): role r < 3 writes joint r's four columns, role 3 leg l the
  // gravity component l (l < 3), commands l, l + 4, l + 8, l + 12 and the clock of foot l
  float* o = A.obs + (size_t)e * GO1_VEL_NUM_OBS;
  float* oh = A.obs_history_out ? A.obs_history_out + (size_t)e * K.hist_ld + (K.hist_w - GO1_VEL_NUM_OBS) : nullptr;
  const float clip = v->clip_obs;
  const bool noisy = v->add_noise != 0;
  auto put = [&](int i, float val) {
    val = clampf(val, -clip, clip);
    o[i] = val;
    if (oh) oh[i] = val;
  };
  auto noise = [&](float val, int i, float u) { return noisy ? val + (2.0f * u - 1.0f) * v->noise_vec[i] : val; };
  // the noisy columns' uniforms (gravity 0 .. 2, dof pos 18 .. 29, dof vel 30 .. 41: slots 47 .. 88 =
  // Philox blocks 11 .. 22): lane sub16 < 12 draws block 11 + sub16 into LDS
  float uq = 0.0f, uv = 0.0f, ugr = 0.0f;
  if (noisy) {
    if (sub16 < 12) {
      float u4[4];
      rng.quad(11 + sub16, u4);
#pragma unroll
      for (int k = 0; k < 4; ++k) s_u[el][4 * sub16 + k] = u4[k];
    }
    const int d = leg * 3 + (role < 3 ? role : 0);
    uq = s_u[el][GO1_VEL_U_NOISE + 18 + d - 44];
    uv = s_u[el][GO1_VEL_U_NOISE + 30 + d - 44];
    ugr = s_u[el][GO1_VEL_U_NOISE + (leg < 3 ? leg : 0) - 44];
  }
  static_assert(GO1_VEL_U_NOISE == 47 && GO1_VEL_U_DR + 13 <= 16, "the shared noise / DR Philox blocks");
  if (role < 3) {
    const int j = role, d = leg * 3 + j;
    const float qj = sel3(j, q), qdj = sel3(j, qd), aj = sel3(j, act), lj = sel3(j, la_obs);
    put(18 + d, noise((qj - v->default_dof_pos[d]) * v->obs_scale_dof_pos, 18 + d, uq));
    put(30 + d, noise(qdj * v->obs_scale_dof_vel, 30 + d, uv));
    put(42 + d, noise_free(aj, noisy, rng, GO1_VEL_U_NOISE + 42 + d));
    put(54 + d, noise_free(lj, noisy, rng, GO1_VEL_U_NOISE + 54 + d));
  } else {
    if (leg < 3) {
      const float g = sel3(leg, pg);
      put(leg, noise(g, leg, ugr));
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int k = leg + 4 * m;
      if (k < GO1_VEL_NUM_COMMANDS) {
        const float ck = sel4(leg, cmd[4 * m], cmd[4 * m + 1], cmd[4 * m + 2], cmd[4 * m + 3 < 15 ? 4 * m + 3 : 14]);
        put(3 + k, noise_free(ck * v->cmd_scale[k], noisy, rng, GO1_VEL_U_NOISE + 3 + k));
      }
    }
    put(66 + leg, noise_free(clock, noisy, rng, GO1_VEL_U_NOISE + 66 + leg));
  }
  if (sub16 == 0) {
    float* pv = A.priv + (size_t)e * 2;
    pv[0] = clampf((friction - v->priv_friction_shift) * v->priv_friction_scale, -clip, clip);
    pv[1] = clampf((restitution - v->priv_rest_shift) * v->priv_rest_scale, -clip, clip);
  }
  if (A.aux) {
    float* ax = A.aux + (size_t)e * GO1_VEL_AUX;
    if (role == 3 && leg == 0) {
#pragma unroll
      for (int i = 0; i < 3; ++i) { ax[i] = blv[i]; ax[3 + i] = bav[i]; }
    }
    if (role == 1) {
#pragma unroll
      for (int i = 0; i < 3; ++i) ax[6 + leg * 3 + i] = fp[i];
    }
    if (owner) {
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        ax[18 + leg * 3 + i] = torque[i];
        ax[30 + leg * 3 + i] = tgt[i];
      }
    }
  }

  // ---- the curriculum launch's selection lists.  A record per selected env: (env, category, bin, success)
  // -- RewardThresholdCurriculum.update's inputs (:736-757, curriculum.py:135-154) over this step's command
  // sums -- so the curriculum's workgroups never read the command state they rewrite (a late
  // workgroup counting after another one's sampling).  B: this step's resets (:168 -> :182); A: the next
  // step's interval resample, (episode_length + 1) % resample_interval == 0 (:702-704).  One 64-bit atomic per
  // wave with a selected env; the lists are in atomic order (the curriculum's results do not depend on it).
  if (K.clist) {
    bool fail = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k < v->n_task) {
        const int slot = v->task_slot[k];
#pragma unroll
        for (int h = 0; h < 2; ++h)
          if (sub16 + 16 * h == slot && !(cs[h] / v->curriculum_ep_len > v->task_threshold[k])) fail = true;
      }
    }
    const uint64_t fails = __ballot(fail);
    const bool ok = ((fails >> (4 * el)) & 0x000F000F000F000Full) == 0ull;
    const bool lead = lane == 4 * el;  // role 0, leg 0 of the env
    const int ep_out = reset ? 0 : ep;
    const bool selB = lead && reset, selA = lead && K.doA && (ep_out + 1) % v->resample_interval == 0;
    const uint64_t mB = __ballot(selB), mA = __ballot(selA);
    if ((mB | mA) != 0ull) {
      unsigned long long base = 0ull;
      if (lane == 0)
        base = atomicAdd(K.ccnt, (unsigned long long)__popcll(mB) | ((unsigned long long)__popcll(mA) << 32));
      const uint32_t bB = (uint32_t)__shfl((int)(uint32_t)base, 0), bA = (uint32_t)__shfl((int)(uint32_t)(base >> 32), 0);
      const uint64_t below = (1ull << lane) - 1ull;
      const int4 rec = make_int4(e, cat_in, bin_in, ok ? 1 : 0);
      if (selB) K.clist[bB + __popcll(mB & below)] = rec;
      if (selA) K.clist[(size_t)c->n_envs + bA + __popcll(mA & below)] = rec;
    }
    if (blockIdx.x == 0 && lane == 0) *K.czero = 0ull;
  }

  // ---------------- write back (epilogue :144-149)
  if (role < 3) {
    const int j = role;
    const size_t dj = d0 + j;
    st.dof_pos[dj] = sel3(j, q);
    st.dof_vel[dj] = sel3(j, qd);
    st.last_dof_vel[dj] = sel3(j, qd);
    st.last_actions[dj] = sel3(j, act);
    st.last_last_actions[dj] = sel3(j, lla_out);
    st.last_last_joint_pos_target[dj] = sel3(j, ljpt);
    st.last_joint_pos_target[dj] = sel3(j, tgt);
    if (reset || dr_step) {
      st.motor_strength[dj] = sel3(j, strength);
      st.motor_offset[dj] = sel3(j, offset);
    }
#pragma unroll
    for (int k = 0; k < VLAG; ++k)
      st.lag[(size_t)e * 12 * VLAG + k * 12 + leg * 3 + j] =
          reset ? 0.0f : (k == VLAG - 1 ? sel3(j, scaled) : sel3(j, lag_pre[k + 1 < VLAG ? k + 1 : k]));
    st.pos_err_hist[(size_t)e * 24 + leg * 3 + j] = sel3(j, eh[0]);
    st.pos_err_hist[(size_t)e * 24 + 12 + leg * 3 + j] = sel3(j, eh[1]);
    st.vel_hist[(size_t)e * 24 + leg * 3 + j] = sel3(j, vh[0]);
    st.vel_hist[(size_t)e * 24 + 12 + leg * 3 + j] = sel3(j, vh[1]);
  }
  if (role == 3 && slip_live) st.last_contacts[(size_t)e * 4 + leg] = contact ? 1.0f : 0.0f;
  if (role == 3 && leg == 0) {
#pragma unroll
    for (int i = 0; i < 13; ++i) st.root[(size_t)e * 13 + i] = root[i];
    st.episode_length[e] = reset ? 0 : ep;
    st.gait_indices[e] = gait_out;
    A.rew[e] = rew;
    A.reset[e] = reset;
    A.time_out[e] = time_out;
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = sub16 + 16 * h;
    if (k < NC) st.command_sums[(size_t)e * NC + k] = cs[h];
    if (k < NE) st.episode_sums[(size_t)e * NE + k] = es[h];
  }
}

// explicit reset_idx(ids) state part (4 lanes per env, one per leg)
__global__ __launch_bounds__(TPB) void go1_vel_reset_kernel(const go1_vel_config* __restrict__ v_gen,
                                                            go1_vel_state st, const float* __restrict__ env_origins,
                                                            const int32_t* __restrict__ ids, int n_ids, int n_envs,
                                                            const float* __restrict__ U, uint64_t seed, uint64_t step,
                                                            int env_id_offset, float* episode_log,
                                                            int32_t* episode_log_count, int episode_log_cap,
                                                            int episode_log_tag) {
  VCfg* __restrict__ v = (VCfg*)v_gen;
  const int leg = threadIdx.x & 3;
  const int slot = blockIdx.x * EPB + (threadIdx.x >> 2);
  if (slot >= n_ids) return;
  const int e = ids[slot];
  if (e < 0 || e >= n_envs) return;
  const Rng rng = {U, seed, step, e, e + env_id_offset, GO1_VEL_U_PER_ENV};
  const int NE = v->n_terms + 1;
  if (leg == 0) {  // the episode log (:199-205) reads the sums, then reset_idx clears them
    if (episode_log_count) {
      const int row = atomicAdd(episode_log_count, 1);
      if (episode_log_cap > 0) {
        float* lg = episode_log + (size_t)((uint32_t)row % (uint32_t)episode_log_cap) * (NE + 2);
        for (int k = 0; k < NE; ++k) lg[k] = st.episode_sums[(size_t)e * NE + k];
        lg[NE] = __int_as_float(episode_log_tag);
        lg[NE + 1] = (float)e;
      }
    }
    for (int k = 0; k < NE; ++k) st.episode_sums[(size_t)e * NE + k] = 0.0f;
  }
  float root[13], q[3], qd[3], strength[3], offset[3];
  const float eo[3] = {env_origins[(size_t)e * 3], env_origins[(size_t)e * 3 + 1], env_origins[(size_t)e * 3 + 2]};
  vel_reset_env(v, rng, eo, leg, root, q, qd, strength, offset);
  const size_t d0 = (size_t)e * NDOF + leg * 3;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    st.dof_pos[d0 + j] = q[j];
    st.dof_vel[d0 + j] = qd[j];
    st.motor_strength[d0 + j] = strength[j];
    st.motor_offset[d0 + j] = offset[j];
    st.last_actions[d0 + j] = 0.0f;
    st.last_last_actions[d0 + j] = 0.0f;
    st.last_dof_vel[d0 + j] = 0.0f;
#pragma unroll
    for (int k = 0; k < VLAG; ++k) st.lag[(size_t)e * 12 * VLAG + k * 12 + leg * 3 + j] = 0.0f;
  }
  if (leg == 0) {
#pragma unroll
    for (int i = 0; i < 13; ++i) st.root[(size_t)e * 13 + i] = root[i];
    st.episode_length[e] = 0;
    st.gait_indices[e] = 0.0f;
  }
}

__global__ void go1_vel_mask_kernel(const int32_t* __restrict__ ids, int n_ids, int n, uint8_t* __restrict__ m) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_ids && ids[i] >= 0 && ids[i] < n) m[ids[i]] = 1;
}

// =====================================================================
//        command curriculum (_resample_commands) + history shift
// =====================================================================
#define CK_THREADS 1024
#ifdef GO1_VEL_STAMPS  // diagnostic build only (tools/vel_stamps.py): per section of block 0, cycle sums
// [phase B / A][section] and the number of phases that ran with selected envs
__device__ unsigned long long g_vstamps[2][16];
#define VSTAMP(ph, k, t0)                                                            \
  do {                                                                              \
    if (threadIdx.x == 0 && blockIdx.x == 0) {                                      \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();                    \
      atomicAdd(&g_vstamps[ph][k], t_ - t0);                                        \
      t0 = t_;                                                                      \
    }                                                                               \
  } while (0)
#else
#define VSTAMP(ph, k, t0)
#endif
#define CK_PRE 1024  // list records prefetched into LDS per phase (one per thread); the rest read from memory
static_assert(CK_PRE <= CK_THREADS, "the prologue fills one prefetched record per thread (S.rec[ph][tid], tid < CK_THREADS)");
// the curriculum's record of a selected env: (env, command category, command bin, success of every task over the
// episode's command sums) -- written by the step kernel (or go1_vel_list_kernel) before the launch
typedef int4 CkRec;
struct CArgs {
  // the prologue's inputs lead (a launch that preloads the first kernel-argument dwords into registers has them
  // without a load)
  int n_envs, nb, R;    // nb, R: v->n_bins, v->resample_interval (no load of the config block in the prologue)
  int doA;              // A kind below: the next step's interval resample
  const uint8_t* maskB; // B kind below: reset_idx's envs
  const int32_t* episode_length;  // st.episode_length
  double* cdf;          // (GO1_VEL_N_CATEGORIES, n_bins): numpy's normalised cdf of each curriculum
  int32_t* cdf_ok;      // [GO1_VEL_N_CATEGORIES]: cdf current for the weights
  const CkRec* list;    // the selection lists: B at [0, n_envs), A at [n_envs, 2 n_envs)
  const unsigned long long* cnt;  // their lengths: B low word, A high word
  go1_vel_state st;
  const double* grid;   // (GO1_VEL_N_KEYS, n_bins)
  const int32_t* adj_ptr;  // neighbourhood table (CSR): cells adjacent to bin b are adj_idx[adj_ptr[b] ..]
  const int32_t* adj_idx;
  int env_id_offset;
  int nblk;             // curriculum workgroups (blocks 0 .. nblk - 1; the rest shift the history)
  int* done;            // their completion count (zero between launches)
  uint64_t seed;
  // B kind: the envs of maskB (reset_idx's resample)
  const float* UB;
  const double* UDB;
  uint64_t stepB;
  // A kind: envs with (episode_length + 1) % resample_interval == 0 (the next step's interval resample)
  const float* UA;
  const double* UDA;
  uint64_t stepA;
  // with B: extras["time_outs"] = time_out if some env was selected (:251-252), and the obs / obs_history
  // command columns of the resampled envs
  const uint8_t* time_out;
  uint8_t* extras_time_outs;
  float* obs;
  float* hist_out;
  const float* hist_in;
  int64_t ld_in, ld_out;  // row strides (floats)
  int hist_w;
  int hist_aligned;  // hist_w and both strides % 4 == 0, both buffers 16-byte aligned: 16-byte chunks
  uint32_t delay;    // test knob (GO1_VEL_CK_DELAY, 0 in use): workgroups 1.. wait this many s_memtime ticks before
                     // their success counts, so workgroup 0 samples (writes the command state) first
};

// numpy's pairwise summation (np.add.reduce of a contiguous f64 array), PW_BLOCKSIZE 128
template <int D>
__device__ double np_pairwise_sum(const double* a, int n) {
  if (D == 0 || n <= 128) {
    if (n < 8) {
      double r = 0.0;
      for (int i = 0; i < n; ++i) r += a[i];
      return r;
    }
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  int n2 = n / 2;
  n2 -= n2 % 8;
  return np_pairwise_sum<(D > 0 ? D - 1 : 0)>(a, n2) + np_pairwise_sum<(D > 0 ? D - 1 : 0)>(a + n2, n - n2);
}

__device__ __forceinline__ float remainder1(float a) { return remainder_f(a, 1.0f); }

// LDS of a curriculum workgroup (one allocation for the launch)
struct CkShared {
  int hist[GO1_VEL_N_CATEGORIES * GO1_VEL_MAX_BINS];  // success count per (category, bin)
  double p[GO1_VEL_N_CATEGORIES * GO1_VEL_MAX_BINS];  // per category: the cdf the sampling searches
  double w[GO1_VEL_N_CATEGORIES * GO1_VEL_MAX_BINS];  // the curriculum weights (committed by the last workgroup)
  int list[GO1_VEL_N_CATEGORIES * GO1_VEL_MAX_BINS];  // distinct (category, bin) success pairs
  int inc[GO1_VEL_N_CATEGORIES * GO1_VEL_MAX_BINS];   // +0.2 steps per weight cell
  CkRec rec[2][CK_PRE];                               // the first CK_PRE records of the B and the A list
  int cnt[4];                                         // |list B|, |list A|, |pairs|, last-workgroup flag
  int dirty[GO1_VEL_N_CATEGORIES];                    // weights changed in this phase
  int pvalid[GO1_VEL_N_CATEGORIES];                   // p holds the cdf of the current weights
  int rec_[GO1_VEL_N_CATEGORIES];                     // p recomputed in this launch (the cache to commit)
  int wchg;                                           // some weight changed in this launch
  int wloaded;                                        // w holds the weights (loaded on first need)
};

// Workgroup barrier for LDS hand-offs: every exchange between the curriculum's sections goes through LDS, and
// __syncthreads also waits out every global access in flight -- the sampling's command / observation stores
// and the rebinding's writes, ~2 k cycles at each phase end for nothing (nothing in the launch reads them back).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// the weights into LDS, once per launch, when a phase first needs them (called by the whole workgroup)
__device__ void ensure_weights(VCfg* v, const CArgs& K, CkShared& S) {
  if (S.wloaded) return;
  const int nb = K.nb;
  for (int i = threadIdx.x; i < GO1_VEL_N_CATEGORIES * nb; i += CK_THREADS) {
    const int c = i / nb;
    S.w[(size_t)c * GO1_VEL_MAX_BINS + (i - c * nb)] = K.st.curriculum_weights[i];
  }
  lds_barrier();
  if (threadIdx.x == 0) S.wloaded = 1;
  lds_barrier();
}

// The curriculum runs on K.nblk workgroups.  Everything _resample_commands computes for the batch as a whole --
// the selections, the success counts, the weight update and the cdf -- is computed by every workgroup from the
// same inputs (identical results, no cross-workgroup hand-off); the per-env work (the draws, the commands, the
// observation patch) is split: the env at position i of a phase's ascending list belongs to workgroup
// i % nblk.  The last workgroup to finish commits the weights and the cdf cache.  An env selected by both
// phases is written by phase A only (its phase-B commands reach this step's observation; the state the
// reference's second resample overwrites is never written twice by two workgroups), and phase A's success
// check for it recomputes the category and bin phase B drew (a pure function of its draws and phase B's cdf).
__device__ __forceinline__ bool selectedB(const CArgs& K, int e) { return K.maskB && K.maskB[e] != 0; }
__device__ __forceinline__ bool selectedA(const CArgs& K, int e, int R) {
  return K.doA && (K.st.episode_length[e] + 1) % R == 0;
}

// The launch is latency-bound: a handful of envs per phase behind a chain of barrier-separated sections, and
// a barrier waits out every memory access in flight.  So each section issues all the memory reads it can at
// once: the prologue loads the list lengths, the first CK_PRE records of both lists (at clamped positions,
// before their lengths are known) and the cached cdfs in one round trip; a phase then costs the success counts
// (LDS only), the weight update (when some env succeeded), the cdf of changed weights, and the sampling
// (commands and grid cells together).
// The prologue's inputs come as the launch's leading scalar arguments (the same values as the CArgs fields):
// with kernel-argument preloading they arrive in registers with the wave.
__device__ __forceinline__ void resample_prologue(VCfg* v, const CArgs& K, CkShared& S, int pn, int pnb,
                                                  const unsigned long long* pcnt, const CkRec* plist,
                                                  const double* pcdf, const int32_t* pcdf_ok) {
  const int tid = threadIdx.x, n = pn, nb = pnb;
#ifdef GO1_VEL_STAMPS
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
  const int lane = tid & 63, wv = tid >> 6;
  const unsigned long long cc = *pcnt;
  const CkRec rB = plist[min(tid, n - 1)], rA = plist[(size_t)n + min(tid, n - 1)];
  for (int i = tid; i < GO1_VEL_N_CATEGORIES * nb; i += CK_THREADS) S.hist[i] = 0;
  if (tid < GO1_VEL_N_CATEGORIES) { S.dirty[tid] = 0; S.rec_[tid] = 0; }
  if (tid == 0) { S.wchg = 0; S.wloaded = 0; S.cnt[2] = 0; S.cnt[3] = 0; }
  // the cached cdfs (wave c), whether or not a phase will need them
  double t[GO1_VEL_MAX_BINS / 64];
  int ok = 0;
  if (wv < GO1_VEL_N_CATEGORIES) {  // the weights are loaded only when a phase needs them (ensure_weights)
    const int c = wv & 3;
    const double* g = pcdf + (size_t)c * nb;
    ok = pcdf_ok[c];
    // unconditional loads (index clamped): a load under a condition makes hipcc wait for it right away
#pragma unroll
    for (int i = 0; i < GO1_VEL_MAX_BINS / 64; ++i) t[i] = g[min(lane + 64 * i, nb - 1)];
  }
  const int nB = (int)(uint32_t)cc, nA = (int)(uint32_t)(cc >> 32);
  if (tid == 0) { S.cnt[0] = nB; S.cnt[1] = nA; }
  if (tid < nB) S.rec[0][tid] = rB;
  if (tid < nA) S.rec[1][tid] = rA;
  if (wv < GO1_VEL_N_CATEGORIES) {
    const int c = wv & 3;
    double* dst = S.p + (size_t)c * GO1_VEL_MAX_BINS;
#pragma unroll
    for (int i = 0; i < GO1_VEL_MAX_BINS / 64; ++i)
      if (lane + 64 * i < nb) dst[lane + 64 * i] = t[i];
    if (lane == 0) S.pvalid[c] = ok;
  }
  lds_barrier();
  VSTAMP(0, 10, t0);
}

// record i of a phase's list (ph 0: B, 1: A)
__device__ __forceinline__ CkRec ck_rec(const CArgs& K, const CkShared& S, int ph, int i) {
  return i < CK_PRE ? S.rec[ph][i] : K.list[(size_t)ph * K.n_envs + i];
}

// searchsorted(cdf, u, side='right') clipped to the last bin (numpy's choice)
__device__ __forceinline__ int cdf_search(const double* cdf, int nb, double u) {
  int lo = 0, hi = nb;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (cdf[mid] <= u) lo = mid + 1; else hi = mid;
  }
  return min(lo, nb - 1);
}

// the category draw of a resample: category c when 0.25 c <= u < 0.25 (c + 1) (as f32), -1 otherwise
__device__ __forceinline__ int draw_category(float uc) {
  int cat = -1;
  for (int c = 0; c < GO1_VEL_N_CATEGORIES; ++c)
    if ((float)(0.25 * c) <= uc && uc < (float)(0.25 * (c + 1))) cat = c;
  return cat;
}

// One resample (_resample_commands :728-842) of kind B (mask) or A (interval), by the whole workgroup.
__device__ void resample_phase(VCfg* v, const CArgs& K, bool kindB, CkShared& S) {
  const int tid = threadIdx.x, n = K.n_envs, nb = K.nb, R = K.R;
  const int blk = blockIdx.x, nblk = K.nblk;
  const go1_vel_state& st = K.st;
  const float* U = kindB ? K.UB : K.UA;
  const double* UD = kindB ? K.UDB : K.UDA;
  const uint64_t step = kindB ? K.stepB : K.stepA;
  const int ucat = kindB ? GO1_VEL_U_CAT_B : GO1_VEL_U_CAT_A;
  const int dch = kindB ? GO1_VEL_D_CHOICE_B : GO1_VEL_D_CHOICE_A;
  const int NC = v->n_terms + GO1_VEL_SUM_EXTRA;
  const int ph = kindB ? 0 : 1;
#ifdef GO1_VEL_STAMPS
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
  const int count = S.cnt[ph];
  VSTAMP(ph, 0, t0);
  if (count == 0) return;  // len(env_ids) == 0 (:730): nothing, not even the time-out rebinding
  VSTAMP(ph, 15, t0);
  if (K.delay && blk > 0) {  // test knob only (tests/test_gpu_velocity.py)
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t1 < (unsigned long long)K.delay) __builtin_amdgcn_s_sleep(16);
  }
  // ---- RewardThresholdCurriculum.update per old category (:736-757, curriculum.py:135-154): success
  // counts per (category, bin), and the list of the (category, bin) pairs that have any.  The inputs come
  // from the records (the state at the end of the step), never from the command state the sampling rewrites.
  for (int i = tid; i < count; i += CK_THREADS) {
    if (v->n_task == 0) break;
    const CkRec r = ck_rec(K, S, ph, i);
    const int e = r.x;
    int cat = r.y, b = r.z;
    bool ok = r.w != 0;
    if (!kindB && selectedB(K, e)) {
      // phase B resampled this env: its sums are zero and its category / bin are phase B's draws, recomputed
      // here from phase B's uniforms and cdf (S.p still holds it: phase A's cdf comes after these counts)
      const Rng rng = {K.UB, K.seed, K.stepB, e, e + K.env_id_offset, GO1_VEL_U_PER_ENV};
      const RngD rngd = {K.UDB, K.seed, K.stepB, e, e + K.env_id_offset};
      const int cb = draw_category(rng(GO1_VEL_U_CAT_B));
      if (cb >= 0) {
        cat = cb;
        b = cdf_search(S.p + (size_t)cat * GO1_VEL_MAX_BINS, nb, rngd(GO1_VEL_D_CHOICE_B));
      }
      ok = true;
      for (int k = 0; k < v->n_task; ++k) ok = ok && (0.0f / v->curriculum_ep_len > v->task_threshold[k]);
    }
    if (cat < 0 || cat >= GO1_VEL_N_CATEGORIES) continue;
    if (ok && b >= 0 && b < nb) {
      if (atomicAdd(&S.hist[cat * nb + b], 1) == 0) {
        const int slot = atomicAdd(&S.cnt[2], 1);
        S.list[slot] = cat * nb + b;  // at most GO1_VEL_N_CATEGORIES * nb distinct pairs
      }
    }
  }
  if (kindB && K.extras_time_outs)  // this workgroup's share of the rebinding
    for (int e = blk * CK_THREADS + tid; e < n; e += nblk * CK_THREADS) K.extras_time_outs[e] = K.time_out[e];
  lds_barrier();
  VSTAMP(ph, 1, t0);
  const int n_list = S.cnt[2];
  // weights: cell j of category c gets +0.2 (clipped) once if it was a success bin and once per success
  // env whose bin's neighbourhood holds it -- a sequence of identical clip(w + 0.2, 0, 1) steps, so the
  // count decides the result whatever the order.  Neighbourhoods come from the handle's table
  // (get_local_bins, curriculum.py:123-133, evaluated on the host in the same f64 comparisons).
  if (n_list > 0) {
    ensure_weights(v, K, S);
    for (int i = tid; i < GO1_VEL_N_CATEGORIES * nb; i += CK_THREADS) S.inc[i] = 0;
    lds_barrier();
    for (int l = tid; l < n_list; l += CK_THREADS) {
      const int cb = S.list[l], cat = cb / nb, b = cb % nb, h = S.hist[cb];
      atomicAdd(&S.inc[cb], 1);  // weights[bin_inds[is_success]] += 0.2 (once per distinct bin)
      const int q0 = K.adj_ptr[b], q1 = K.adj_ptr[b + 1];
      for (int q = q0; q < q1; q += 8) {  // eight neighbour indices in flight at a time
        int j[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) j[u] = q + u < q1 ? K.adj_idx[q + u] : -1;
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (j[u] >= 0) atomicAdd(&S.inc[cat * nb + j[u]], h);
      }
    }
    lds_barrier();
    for (int i = tid; i < GO1_VEL_N_CATEGORIES * nb; i += CK_THREADS) {
      const int k = S.inc[i];
      if (k > 0) {
        const int c = i / nb;
        double w = S.w[(size_t)c * GO1_VEL_MAX_BINS + (i - c * nb)];
        for (int t = 0; t < k; ++t) w = fmin(fmax(w + 0.2, 0.0), 1.0);
        S.w[(size_t)c * GO1_VEL_MAX_BINS + (i - c * nb)] = w;
        S.dirty[c] = 1;
        S.wchg = 1;
      }
    }
    lds_barrier();
  }
  VSTAMP(ph, 2, t0);
  // ---- numpy rng.choice(p = w / w.sum()): cdf = cumsum(p) / cdf[-1], wave c for category c, in LDS
  // (S.p), recomputed where the weights changed (or no cdf is cached)
  if (!S.pvalid[0] || !S.pvalid[1] || !S.pvalid[2] || !S.pvalid[3]) ensure_weights(v, K, S);  // uniform
  {
    const int wv = tid >> 6, ln = tid & 63;
    if (wv < GO1_VEL_N_CATEGORIES && (S.dirty[wv] || !S.pvalid[wv])) {
      double* p = S.p + (size_t)wv * GO1_VEL_MAX_BINS;
      const double* w = S.w + (size_t)wv * GO1_VEL_MAX_BINS;
      for (int j = ln; j < nb; j += 64) p[j] = w[j];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      double s = 0.0;
      if (ln == 0) s = np_pairwise_sum<4>(p, nb);
      s = __shfl(s, 0);
      for (int j = ln; j < nb; j += 64) p[j] = p[j] / s;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (ln == 0) {  // numpy's sequential cumsum: the adds are a dependent chain, the LDS reads of a
                      // batch are issued ahead of it (in place, one read-write per element, it would wait
                      // out the LDS latency at every element)
        double acc = 0.0;
        for (int j0 = 0; j0 < nb; j0 += 32) {
          double u[32];
#pragma unroll
          for (int i = 0; i < 32; ++i) u[i] = j0 + i < nb ? p[j0 + i] : 0.0;
#pragma unroll
          for (int i = 0; i < 32; ++i) { acc += u[i]; u[i] = acc; }
#pragma unroll
          for (int i = 0; i < 32; ++i)
            if (j0 + i < nb) p[j0 + i] = u[i];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const double last = p[nb - 1];
      for (int j = ln; j < nb; j += 64) p[j] = p[j] / last;
      if (ln == 0) {
        S.pvalid[wv] = 1;
        S.rec_[wv] = 1;
        S.dirty[wv] = 0;
      }
#ifdef GO1_VEL_STAMPS
      if (ln == 0 && blk == 0) atomicAdd(&g_vstamps[kindB ? 0 : 1][14], 1ull);
#endif
    }
  }
  lds_barrier();
  VSTAMP(ph, 3, t0);
  // ---- new category, cell and command per env (:759-842), this workgroup's envs (list positions
  // blk, blk + nblk, ...; env ids e % nblk == blk beyond the list capacity), 16 lanes per env: lane k < 15
  // draws and finishes command k (the gait rules and binary phases act per command; only the small-command
  // rule pairs commands 0 and 1), lane 15 draws the choice and searches the cdf.  One Philox evaluation per
  // lane instead of ~30 in sequence on one thread; the env's old commands are loaded before the search, so
  // they and the grid cells share one memory round trip.
  {
    const int sub = tid & 15, grp = tid >> 4;
    const int n_own = count > blk ? (count - blk + nblk - 1) / nblk : 0;
    for (int i0 = 0; i0 < n_own; i0 += CK_THREADS / 16) {
      const int i = i0 + grp;
      if (i >= n_own) continue;  // uniform over the env's 16 lanes
      const int e = ck_rec(K, S, ph, blk + i * nblk).x;
      // an env phase A resamples again: phase A writes its state, phase B only its observed commands
      const bool state_out = !(kindB && selectedA(K, e, R));
      const Rng rng = {U, K.seed, step, e, e + K.env_id_offset, GO1_VEL_U_PER_ENV};
      const RngD rngd = {UD, K.seed, step, e, e + K.env_id_offset};
      const int subc = min(sub, GO1_VEL_NUM_COMMANDS - 1);  // clamped: unconditional loads
      // the old command (kept when the category draw fails) is read first and not touched before the draws and
      // the cdf search are done
      const float cmd_old = st.commands[(size_t)e * GO1_VEL_NUM_COMMANDS + subc];
      const double half = v->bin_sizes[subc] / 2.0;
      const int cat = draw_category(rng(ucat));
      float cmd = 0.0f;
      if (cat >= 0) {
        const double u = rngd(sub < GO1_VEL_NUM_COMMANDS ? dch + 1 + sub : dch);
        VSTAMP(ph, 5, t0);
        int idx = 0;
        if (sub == 15) {
          idx = cdf_search(S.p + (size_t)cat * GO1_VEL_MAX_BINS, nb, u);
          if (state_out) {
            st.command_bins[e] = idx;
            st.command_categories[e] = cat;
          }
        }
        idx = __shfl(idx, 15, 16);
        VSTAMP(ph, 6, t0);
        const double cen = K.grid[(size_t)subc * nb + idx];
        if (sub < GO1_VEL_NUM_COMMANDS) {
          const double l = cen + half, h = cen - half;
          cmd = (float)(l + (h - l) * u);
          if (v->gaitwise_curricula && sub >= 5 && sub < 8) {
            if (cat == CAT_PRONK) cmd = remainder1(cmd / 2.0f - 0.25f);
            else if (sub - 5 == cat - 1) cmd = cmd / 2.0f + 0.25f;  // trot: 5, pace: 6, bound: 7
            else cmd = 0.0f;
          }
        }
      } else {
        cmd = sub < GO1_VEL_NUM_COMMANDS ? cmd_old : 0.0f;
      }
      if (v->binary_phases && sub >= 5 && sub < 8) cmd = remainder1(rintf(2.0f * cmd) / 2.0f);
      {
        const float c0 = __shfl(cmd, 0, 16), c1 = __shfl(cmd, 1, 16);
        const float keep = norm2_f(c0, c1) > 0.2f ? 1.0f : 0.0f;
        if (sub < 2) cmd = cmd * keep;
      }
      if (state_out) {
        if (sub < GO1_VEL_NUM_COMMANDS) st.commands[(size_t)e * GO1_VEL_NUM_COMMANDS + sub] = cmd;
        for (int k = sub; k < NC; k += 16) st.command_sums[(size_t)e * NC + k] = 0.0f;
      }
      if (kindB && K.obs && sub < GO1_VEL_NUM_COMMANDS) {  // this step's observation of the resampled commands (:339)
        const float clip = v->clip_obs;
        float val = cmd * v->cmd_scale[sub];
        if (v->add_noise) val = val + (2.0f * rng(GO1_VEL_U_NOISE + 3 + sub) - 1.0f) * v->noise_vec[3 + sub];
        val = clampf(val, -clip, clip);
        K.obs[(size_t)e * GO1_VEL_NUM_OBS + 3 + sub] = val;
        if (K.hist_out) K.hist_out[(size_t)e * K.ld_out + K.hist_w - GO1_VEL_NUM_OBS + 3 + sub] = val;
      }
    }
  }
  VSTAMP(ph, 7, t0);
  // ready for the next phase: success counts and the pair list cleared
  for (int i = tid; i < GO1_VEL_N_CATEGORIES * nb; i += CK_THREADS) S.hist[i] = 0;
  if (tid == 0) S.cnt[2] = 0;
  lds_barrier();
  VSTAMP(ph, 4, t0);
}

// The last curriculum workgroup to finish writes the weights and the recomputed cdfs (every workgroup holds
// the same values; all of them have read the old ones by then).  Release: every workgroup's reads and writes
// precede its ticket; acquire: the last one sees every other workgroup done before it writes.
__device__ void resample_commit(VCfg* v, const CArgs& K, CkShared& S) {
  const int tid = threadIdx.x, nb = K.nb;
  lds_barrier();
  // every workgroup takes the same decisions: with no weight changed and no cdf recomputed there is nothing
  // to commit, and none of them takes a ticket
  if (!S.wchg && !S.rec_[0] && !S.rec_[1] && !S.rec_[2] && !S.rec_[3]) return;
  __syncthreads();  // (a commit: every thread's global accesses precede the ticket's release)
#ifdef GO1_VEL_STAMPS
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const int old = __hip_atomic_fetch_add(K.done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    S.cnt[3] = old == K.nblk - 1;
    if (S.cnt[3]) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  if (!S.cnt[3]) return;
  for (int i = tid; i < GO1_VEL_N_CATEGORIES * nb; i += CK_THREADS) {
    const int c = i / nb, j = i - c * nb;
    if (S.rec_[c]) {  // a category whose weights changed had its cdf recomputed
      K.st.curriculum_weights[i] = S.w[(size_t)c * GO1_VEL_MAX_BINS + j];
      K.cdf[i] = S.p[(size_t)c * GO1_VEL_MAX_BINS + j];
    }
  }
  if (tid < GO1_VEL_N_CATEGORIES && S.rec_[tid]) K.cdf_ok[tid] = 1;
  if (tid == 0) *K.done = 0;  // the next launch's count (stream order)
  VSTAMP(0, 11, t0);
}

// HistoryWrapper.step's shift (history_wrapper.py:22): new[:, :W - 70] = old[:, 70:], by workgroups 1.. of
// the curriculum launch (g0: the thread's index among them, G: their thread count).  A pure HBM stream of
// 2 x 33 MB at 4096 envs x 30 observations.  Measured alternative, not kept: the shift as its own kernel on
// a side stream beside the step kernel -- it overlapped (27 us under the 47 us step kernel), but the two
// cross-stream hand-offs per step left ~11 us of idle GPU between steps: 70.6 against 69.1 us per step.
__device__ void hist_shift(const CArgs& K, size_t g0, size_t G) {
  if (!K.hist_in || !K.hist_out) return;
  const int W = K.hist_w, D = W - GO1_VEL_NUM_OBS;
  const size_t Li = (size_t)K.ld_in, Lo = (size_t)K.ld_out;
  if (K.hist_aligned) {
    // 16-byte chunks: rows are 16-byte aligned (W % 4 == 0), the source starts 70 = 4 x 17 + 2 floats in,
    // so dest chunk i = (z, w) of aligned source chunk 17 + i and (x, y) of chunk 18 + i, which the next
    // lane holds (lane 63 loads it).  Chunks per row padded to a multiple of 64 keep a wave in one row;
    // four chunks per thread are loaded before any is stored (HBM latency x bandwidth needs them in flight).
    // D = W - 70 is 2 mod 4: the last chunk of a row is half (its other half is the new obs row).
    const int Cn = (D + 3) / 4, Cp = (Cn + 63) & ~63;
    const size_t total = (size_t)K.n_envs * Cp;
    const bool last_lane = (threadIdx.x & 63) == 63;
    for (size_t t0 = g0; t0 < total; t0 += 4 * G) {
      float4 own[4];
      size_t ev[4];
      int iv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const size_t t = t0 + u * G;
        ev[u] = t / Cp;
        iv[u] = (int)(t % Cp);
        own[u] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (t < total && iv[u] < Cn) own[u] = reinterpret_cast<const float4*>(K.hist_in + ev[u] * Li)[17 + iv[u]];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const size_t t = t0 + u * G;  // t < total is uniform over the wave (total, G, t0 - lane: multiples of 64)
        if (t >= total) break;
        float nx = __shfl_down(own[u].x, 1), ny = __shfl_down(own[u].y, 1);
        const int i = iv[u];
        if (last_lane && i + 1 < Cn) {
          const float4 o2 = reinterpret_cast<const float4*>(K.hist_in + ev[u] * Li)[18 + i];
          nx = o2.x;
          ny = o2.y;
        }
        if (i < Cn) {
          float* dst = K.hist_out + ev[u] * Lo + 4 * i;
          if (4 * i + 4 <= D) *reinterpret_cast<float4*>(dst) = make_float4(own[u].z, own[u].w, nx, ny);
          else *reinterpret_cast<float2*>(dst) = make_float2(own[u].z, own[u].w);
        }
      }
    }
    return;
  }
  // any other width / alignment: f32 pairs (rows are 8-byte aligned: 70 x 4 B is not a multiple of 16)
  const int W2 = D / 2;
  const size_t total = (size_t)K.n_envs * W2;
  for (size_t i = g0; i < total; i += G) {
    const size_t e = i / W2, k = i % W2;
    const float2 val = *(const float2*)(K.hist_in + e * Li + GO1_VEL_NUM_OBS + 2 * k);
    *(float2*)(K.hist_out + e * Lo + 2 * k) = val;
  }
}

__global__ __launch_bounds__(CK_THREADS) void go1_vel_curriculum_kernel(const go1_vel_config* __restrict__ v_gen,
                                                                        int pn, int pnb,
                                                                        const unsigned long long* pcnt,
                                                                        const CkRec* plist, const double* pcdf,
                                                                        const int32_t* pcdf_ok, CArgs K) {
  VCfg* __restrict__ v = (VCfg*)v_gen;
  if ((int)blockIdx.x >= K.nblk) {
    hist_shift(K, (size_t)(blockIdx.x - K.nblk) * CK_THREADS + threadIdx.x, (size_t)(gridDim.x - K.nblk) * CK_THREADS);
    return;
  }
  __shared__ CkShared S;
  resample_prologue(v, K, S, pn, pnb, pcnt, plist, pcdf, pcdf_ok);
  if (K.maskB) resample_phase(v, K, true, S);
  if (K.doA) resample_phase(v, K, false, S);
  resample_commit(v, K, S);
}

// The selection lists of an explicit resample (go1_vel_resample: reset_idx's mask, or the interval envs) in
// ascending env order, one workgroup: thread t takes a contiguous run of envs, a block-wide scan places the
// runs.  The records carry the state the curriculum's success counts read.
__global__ __launch_bounds__(CK_THREADS) void go1_vel_list_kernel(const go1_vel_config* __restrict__ v_gen, CArgs K,
                                                                  CkRec* list, unsigned long long* cnt) {
  VCfg* __restrict__ v = (VCfg*)v_gen;
  __shared__ int wsum[2][CK_THREADS / 64];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, n = K.n_envs, R = K.R;
  const int NC = v->n_terms + GO1_VEL_SUM_EXTRA;
  const int per = (n + CK_THREADS - 1) / CK_THREADS, eb = tid * per;
  int cb = 0, ca = 0;
  for (int k = 0; k < per; ++k) {
    const int e = eb + k;
    if (e < n) {
      cb += selectedB(K, e) ? 1 : 0;
      ca += selectedA(K, e, R) ? 1 : 0;
    }
  }
  int ib = cb, ia = ca;  // inclusive scans over the wave
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int ub = __shfl_up(ib, o), ua = __shfl_up(ia, o);
    ib += lane >= o ? ub : 0;
    ia += lane >= o ? ua : 0;
  }
  if (lane == 63) { wsum[0][wv] = ib; wsum[1][wv] = ia; }
  __syncthreads();
  int ob = ib - cb, oa = ia - ca, totb = 0, tota = 0;
  for (int w = 0; w < CK_THREADS / 64; ++w) {
    ob += w < wv ? wsum[0][w] : 0;
    oa += w < wv ? wsum[1][w] : 0;
    totb += wsum[0][w];
    tota += wsum[1][w];
  }
  for (int k = 0; k < per; ++k) {
    const int e = eb + k;
    if (e >= n) break;
    const bool sb = selectedB(K, e), sa = selectedA(K, e, R);
    if (!sb && !sa) continue;
    bool ok = true;
    for (int t = 0; t < v->n_task; ++t)
      ok = ok && (K.st.command_sums[(size_t)e * NC + v->task_slot[t]] / v->curriculum_ep_len > v->task_threshold[t]);
    const CkRec r = make_int4(e, K.st.command_categories[e], K.st.command_bins[e], ok ? 1 : 0);
    if (sb) list[ob++] = r;
    if (sa) list[(size_t)n + oa++] = r;
  }
  if (tid == 0) *cnt = (unsigned long long)(uint32_t)totb | ((unsigned long long)(uint32_t)tota << 32);
}

// =====================================================================
//                                C ABI
// =====================================================================
#ifdef GO1_VEL_STAMPS
extern "C" int go1_vel_stamps(void* host, int reset) {
  if (host && hipMemcpyFromSymbol(host, HIP_SYMBOL(g_vstamps), sizeof(g_vstamps), 0, hipMemcpyDeviceToHost) != hipSuccess)
    return 1;
  if (reset) {
    static const unsigned long long z[2][16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_vstamps), z, sizeof(z), 0, hipMemcpyHostToDevice) != hipSuccess) return 1;
  }
  return 0;
}
#endif
struct go1_vel_handle {
  go1_config cfg;
  go1_vel_config vcfg;
  go1_config* d_cfg = nullptr;
  go1_vel_config* d_vcfg = nullptr;
  double* d_grid = nullptr;
  double* d_cdf = nullptr;
  int32_t* d_cdf_ok = nullptr;
  uint8_t* d_mask = nullptr;  // reset_idx's env mask (stream-ordered reuse)
  int32_t* d_adj_ptr = nullptr;  // neighbourhood table of the curriculum update (CSR over the bins)
  int32_t* d_adj_idx = nullptr;
  int32_t* d_done = nullptr;     // completion count of the curriculum workgroups (zero between launches)
  CkRec* d_clist = nullptr;      // selection lists: 3 slots (steps alternate 0 / 1, explicit resamples 2) x (B, A)
  unsigned long long* d_ccnt = nullptr;  // their lengths per slot (B low word, A high word)
  int slot = 0;                  // the next step's slot
  uint32_t ck_delay = 0;         // CArgs.delay (GO1_VEL_CK_DELAY at create; tests only)
  go1_vel_state st;
  const float* env_origins = nullptr;
  bool bound = false;
};

static thread_local std::string g_verr;
static int vfail(int code, const std::string& msg) {
  g_verr = msg;
  return code;
}
#define VHIP_TRY(x)                                                                      \
  do {                                                                                   \
    hipError_t _e = (x);                                                                 \
    if (_e != hipSuccess) return vfail(GO1_E_HIP, std::string(#x ": ") + hipGetErrorString(_e)); \
  } while (0)

// curriculum workgroups: the per-env sampling splits over them (a 4096-env resample: 256 envs each)
static int curriculum_blocks(int n) { return std::max(1, std::min(16, n / 256)); }

static CArgs curriculum_args(go1_vel_handle* h) {
  CArgs K;
  memset(&K, 0, sizeof(K));
  K.st = h->st;
  K.episode_length = h->st.episode_length;
  K.grid = h->d_grid;
  K.adj_ptr = h->d_adj_ptr;
  K.adj_idx = h->d_adj_idx;
  K.cdf = h->d_cdf;
  K.cdf_ok = h->d_cdf_ok;
  K.n_envs = h->cfg.n_envs;
  K.env_id_offset = h->cfg.env_id_offset;
  K.nb = h->vcfg.n_bins;
  K.R = h->vcfg.resample_interval;
  K.nblk = curriculum_blocks(h->cfg.n_envs);
  K.done = h->d_done;
  K.delay = h->ck_delay;
  return K;
}

extern "C" {
int go1_vel_abi_version(void) { return GO1_VEL_ABI_VERSION; }

void go1_vel_abi_sizes(int64_t out[3]) {
  out[0] = sizeof(go1_vel_config);
  out[1] = sizeof(go1_vel_state);
  out[2] = sizeof(go1_vel_step_args);
}

const char* go1_vel_last_error(void) { return g_verr.c_str(); }

int go1_vel_create(const go1_config* cfg, const go1_vel_config* vel, const double* grid, go1_vel_handle** out) {
  if (!cfg || !vel || !grid || !out) return vfail(GO1_E_ARG, "go1_vel_create: null argument");
  if (cfg->n_envs <= 0 || cfg->n_envs % EPB != 0)
    return vfail(GO1_E_ARG, "go1_vel_create: n_envs must be a positive multiple of 16");
  if (vel->n_envs != cfg->n_envs) return vfail(GO1_E_ARG, "go1_vel_create: n_envs differs between the configs");
  if (cfg->terrain_kind != 0) return vfail(GO1_E_ARG, "go1_vel_create: the velocity step runs on the plane");
  if (cfg->n_internal <= 0 || GO1_LAG_STEPS(cfg->decimation) != VLAG)
    return vfail(GO1_E_ARG, "go1_vel_create: decimation must be 4..6 (two stored lag steps)");
  if (vel->n_terms < 0 || vel->n_terms > GO1_VEL_MAX_TERMS) return vfail(GO1_E_ARG, "go1_vel_create: n_terms");
  for (int k = 0; k < vel->n_terms; ++k)
    if (vel->term_ids[k] < 0 || vel->term_ids[k] >= GO1_VT_COUNT) return vfail(GO1_E_ARG, "go1_vel_create: term id");
  if (vel->n_bins <= 0 || vel->n_bins > GO1_VEL_MAX_BINS) return vfail(GO1_E_ARG, "go1_vel_create: n_bins");
  if (vel->resample_interval <= 0 || vel->rand_interval <= 0)
    return vfail(GO1_E_ARG, "go1_vel_create: resample / rand interval");
  if (vel->n_task < 0 || vel->n_task > 4) return vfail(GO1_E_ARG, "go1_vel_create: n_task");
  if (vel->history_len < 1) return vfail(GO1_E_ARG, "go1_vel_create: history_len");
  if (memcmp(cfg->model, GO1_MODEL_F32, sizeof(GO1_MODEL_F32)) != 0)
    return vfail(GO1_E_ARG, "go1_vel_create: model block differs from the compiled Go1 model");
  go1_vel_handle* h = new (std::nothrow) go1_vel_handle();
  if (!h) return vfail(GO1_E_ARG, "go1_vel_create: out of host memory");
  h->cfg = *cfg;
  h->vcfg = *vel;
  if (const char* d = getenv("GO1_VEL_CK_DELAY")) h->ck_delay = (uint32_t)strtoul(d, nullptr, 10);
  const size_t gsz = (size_t)GO1_VEL_N_KEYS * vel->n_bins * sizeof(double);
  const size_t csz = (size_t)GO1_VEL_N_CATEGORIES * vel->n_bins * sizeof(double);
  if (hipMalloc(&h->d_cfg, sizeof(go1_config)) != hipSuccess || hipMalloc(&h->d_vcfg, sizeof(go1_vel_config)) != hipSuccess ||
      hipMalloc(&h->d_grid, gsz) != hipSuccess || hipMalloc(&h->d_cdf, csz) != hipSuccess ||
      hipMalloc(&h->d_cdf_ok, GO1_VEL_N_CATEGORIES * sizeof(int32_t)) != hipSuccess ||
      hipMalloc(&h->d_mask, cfg->n_envs) != hipSuccess || hipMalloc(&h->d_done, sizeof(int32_t)) != hipSuccess ||
      hipMalloc(&h->d_clist, (size_t)6 * cfg->n_envs * sizeof(CkRec)) != hipSuccess ||
      hipMalloc(&h->d_ccnt, 3 * sizeof(unsigned long long)) != hipSuccess) {
    go1_vel_destroy(h);
    return vfail(GO1_E_HIP, "go1_vel_create: hipMalloc failed");
  }

  VHIP_TRY(hipMemcpy(h->d_cfg, cfg, sizeof(go1_config), hipMemcpyHostToDevice));
  VHIP_TRY(hipMemcpy(h->d_vcfg, vel, sizeof(go1_vel_config), hipMemcpyHostToDevice));
  VHIP_TRY(hipMemcpy(h->d_grid, grid, gsz, hipMemcpyHostToDevice));
  {  // get_local_bins (curriculum.py:123-133): cell j is adjacent to bin b when every key is within
     // local_range -- the numpy comparisons grid[:, j] >= grid[:, b] - r and <= grid[:, b] + r in f64
    const int nb = vel->n_bins;
    std::vector<int32_t> ptr(nb + 1, 0), idx;
    for (int b = 0; b < nb; ++b) {
      for (int j = 0; j < nb; ++j) {
        bool adj = true;
        for (int k = 0; k < GO1_VEL_N_KEYS && adj; ++k) {
          const double gb = grid[(size_t)k * nb + b], gj = grid[(size_t)k * nb + j], r = vel->local_range[k];
          adj = gj >= gb - r && gj <= gb + r;
        }
        if (adj) idx.push_back(j);
      }
      ptr[b + 1] = (int32_t)idx.size();
    }
    if (idx.empty()) idx.push_back(0);
    VHIP_TRY(hipMalloc(&h->d_adj_ptr, ptr.size() * sizeof(int32_t)));
    VHIP_TRY(hipMalloc(&h->d_adj_idx, idx.size() * sizeof(int32_t)));
    VHIP_TRY(hipMemcpy(h->d_adj_ptr, ptr.data(), ptr.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    VHIP_TRY(hipMemcpy(h->d_adj_idx, idx.data(), idx.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  }
  VHIP_TRY(hipMemset(h->d_cdf_ok, 0, GO1_VEL_N_CATEGORIES * sizeof(int32_t)));
  VHIP_TRY(hipMemset(h->d_done, 0, sizeof(int32_t)));
  VHIP_TRY(hipMemset(h->d_ccnt, 0, 3 * sizeof(unsigned long long)));
  VHIP_TRY(hipMemset(h->d_clist, 0, (size_t)6 * cfg->n_envs * sizeof(CkRec)));
  *out = h;
  return GO1_OK;
}

int go1_vel_bind(go1_vel_handle* h, const go1_vel_state* s, const go1_plane* planes) {
  if (!h || !s || !planes) return vfail(GO1_E_ARG, "go1_vel_bind: null argument");
  const void* p[] = {s->root, s->dof_pos, s->dof_vel, s->last_actions, s->last_dof_vel, s->lag, s->pos_err_hist,
                     s->vel_hist, s->motor_strength, s->motor_offset, s->friction, s->restitution, s->payload,
                     s->episode_length, s->last_last_actions, s->last_joint_pos_target,
                     s->last_last_joint_pos_target, s->commands, s->gait_indices, s->last_contacts,
                     s->command_sums, s->episode_sums, s->command_bins, s->command_categories,
                     s->curriculum_weights};
  static_assert(sizeof(p) / sizeof(p[0]) == GO1_VEL_STATE_PLANES, "go1_vel_state planes");
  static const char* names[GO1_VEL_STATE_PLANES] = {
      "root", "dof_pos", "dof_vel", "last_actions", "last_dof_vel", "lag", "pos_err_hist", "vel_hist",
      "motor_strength", "motor_offset", "friction", "restitution", "payload", "episode_length",
      "last_last_actions", "last_joint_pos_target", "last_last_joint_pos_target", "commands", "gait_indices",
      "last_contacts", "command_sums", "episode_sums", "command_bins", "command_categories", "curriculum_weights"};
  const int64_t nt = h->vcfg.n_terms, n = h->cfg.n_envs;
  const int64_t width[GO1_VEL_STATE_PLANES] = {13, 12, 12, 12, 12, 12 * VLAG, 24, 24, 12, 12, 1, 1, 1, 1, 12, 12, 12,
                                               GO1_VEL_NUM_COMMANDS, 1, 4, nt + GO1_VEL_SUM_EXTRA, nt + 1, 1, 1,
                                               h->vcfg.n_bins};
  for (int i = 0; i < GO1_VEL_STATE_PLANES; ++i) {
    const go1_plane& d = planes[i];
    const int dt = (i == 13 || i == 22 || i == 23) ? GO1_DTYPE_I32 : (i == 24 ? GO1_DTYPE_F64 : GO1_DTYPE_F32);
    const int64_t rows = i == 24 ? GO1_VEL_N_CATEGORIES : n;
    if (!p[i]) return vfail(GO1_E_ARG, std::string("go1_vel_bind: state plane ") + names[i] + " is null");
    if (d.rows != rows || d.cols != width[i] || d.dtype != dt)
      return vfail(GO1_E_ARG, std::string("go1_vel_bind: state plane ") + names[i] + " must be (" +
                                  std::to_string(rows) + ", " + std::to_string(width[i]) + ") " +
                                  (dt == GO1_DTYPE_I32 ? "int32" : (dt == GO1_DTYPE_F64 ? "float64" : "float32")));
    if (d.col_stride != 1 || (d.rows > 1 && d.row_stride != d.cols))
      return vfail(GO1_E_ARG, std::string("go1_vel_bind: state plane ") + names[i] +
                                  " is not dense row-major: pass a contiguous tensor");
  }
  h->st = *s;
  h->bound = true;
  VHIP_TRY(hipMemset(h->d_cdf_ok, 0, GO1_VEL_N_CATEGORIES * sizeof(int32_t)));  // new weights plane
  return GO1_OK;
}

int go1_vel_set_origins(go1_vel_handle* h, const float* env_origins) {
  if (!h || !env_origins) return vfail(GO1_E_ARG, "go1_vel_set_origins: null argument");
  h->env_origins = env_origins;
  return GO1_OK;
}

int go1_vel_step(go1_vel_handle* h, const go1_vel_step_args* a, void* stream) {
  if (!h || !a) return vfail(GO1_E_ARG, "go1_vel_step: null argument");
  if (!h->bound || !h->env_origins) return vfail(GO1_E_STATE, "go1_vel_step: bind the state and set the origins first");
  if (!a->actions || !a->obs || !a->priv || !a->rew || !a->reset || !a->time_out || !a->extras_time_outs)
    return vfail(GO1_E_ARG, "go1_vel_step: actions and every output buffer are required");
  const bool inj = a->inj_dof != nullptr;
  if (inj && (!a->inj_root || !a->inj_contact || !a->inj_feet))
    return vfail(GO1_E_ARG, "go1_vel_step: partial injected state");
  if ((a->uniforms == nullptr) != (a->uniforms_f64 == nullptr))
    return vfail(GO1_E_ARG, "go1_vel_step: parity mode needs both uniform arrays");
  if (a->resample_next && a->uniforms && (!a->uniforms_next || !a->uniforms_f64_next))
    return vfail(GO1_E_ARG, "go1_vel_step: parity mode resamples ahead with the next step's uniforms");
  const int hist_w = GO1_VEL_NUM_OBS * h->vcfg.history_len;
  const int64_t ld_in = a->obs_history_in_ld ? a->obs_history_in_ld : hist_w;
  const int64_t ld_out = a->obs_history_out_ld ? a->obs_history_out_ld : hist_w;
  if ((a->obs_history_in == nullptr) != (a->obs_history_out == nullptr) ||
      (a->obs_history_in && a->obs_history_in == a->obs_history_out))
    return vfail(GO1_E_ARG, "go1_vel_step: obs_history in and out are two distinct buffers (or both NULL)");
  if (a->obs_history_in && (ld_in < hist_w || ld_out < hist_w || (hist_w & 1) || (ld_in & 1) || (ld_out & 1) ||
                            ((uintptr_t)a->obs_history_in & 7) || ((uintptr_t)a->obs_history_out & 7)))
    return vfail(GO1_E_ARG, "go1_vel_step: obs_history row strides >= 70 x history_len, even, rows 8-byte aligned");
  // out = in + 70 with the same stride: a sliding window, new[:, :W - 70] IS old[:, 70:] (no shift)
  const bool window = a->obs_history_in && ld_in == ld_out && a->obs_history_out == a->obs_history_in + GO1_VEL_NUM_OBS;
  if (a->episode_log_count && (!a->episode_log || a->episode_log_cap < 0))
    return vfail(GO1_E_ARG, "go1_vel_step: a compact episode log needs episode_log and a capacity");
  hipStream_t s = (hipStream_t)stream;
  const int n = h->cfg.n_envs;
  VArgs K;
  K.st = h->st;
  K.a = *a;
  K.env_origins = h->env_origins;
  K.hist_w = hist_w;
  K.hist_ld = ld_out;
  const int slot = h->slot;
  h->slot ^= 1;
  K.clist = h->d_clist + (size_t)slot * 2 * n;
  K.ccnt = h->d_ccnt + slot;
  K.czero = h->d_ccnt + (slot ^ 1);
  K.doA = a->resample_next ? 1 : 0;
  CArgs C = curriculum_args(h);
  C.list = K.clist;
  C.cnt = K.ccnt;
  C.hist_in = window ? nullptr : a->obs_history_in;
  C.hist_out = a->obs_history_out;
  C.ld_in = ld_in;
  C.ld_out = ld_out;
  C.hist_w = K.hist_w;
  C.hist_aligned = C.hist_w % 4 == 0 && ld_in % 4 == 0 && ld_out % 4 == 0 && ((uintptr_t)C.hist_in % 16) == 0 &&
                   ((uintptr_t)C.hist_out % 16) == 0;
  hipEvent_t e0 = (hipEvent_t)a->ev_begin, e1 = (hipEvent_t)a->ev_end;
  auto go = [&](auto kern) {
    if (e0 || e1) hipExtLaunchKernelGGL(kern, dim3(n / SEPB), dim3(TPB), 0, s, e0, e1, 0, h->d_cfg, h->d_vcfg, K);
    else hipLaunchKernelGGL(kern, dim3(n / SEPB), dim3(TPB), 0, s, h->d_cfg, h->d_vcfg, K);
  };
  if (inj) go(go1_vel_step_kernel<true>);
  else go(go1_vel_step_kernel<false>);
  VHIP_TRY(hipGetLastError());
  C.seed = a->rng_seed;
  C.maskB = a->reset;
  C.UB = a->uniforms;
  C.UDB = a->uniforms_f64;
  C.stepB = a->rng_step;
  C.doA = a->resample_next ? 1 : 0;
  C.UA = a->uniforms_next;
  C.UDA = a->uniforms_f64_next;
  C.stepA = a->rng_step + 1;
  C.time_out = a->time_out;
  C.extras_time_outs = a->extras_time_outs;
  C.obs = a->obs;
  // workgroups nblk..: the history shift, one per remaining CU (the launch's LDS allows one workgroup per
  // CU), four 16-byte chunks in flight per lane; fewer for small batches
  const size_t chunks = (size_t)n * (size_t)((K.hist_w - GO1_VEL_NUM_OBS) / 4 + 64);
  const int shift_blocks =
      C.hist_in ? (int)std::min<size_t>(256 - C.nblk, std::max<size_t>(1, (chunks + 4 * CK_THREADS - 1) / (4 * CK_THREADS)))
                : 0;
  hipLaunchKernelGGL(go1_vel_curriculum_kernel, dim3(C.nblk + shift_blocks), dim3(CK_THREADS), 0, s, h->d_vcfg, C.n_envs, C.nb,
                     C.cnt, C.list, C.cdf, C.cdf_ok, C);
  VHIP_TRY(hipGetLastError());
  return GO1_OK;
}

int go1_vel_resample(go1_vel_handle* h, const uint8_t* mask, const float* uniforms, const double* uniforms_f64,
                     uint64_t rng_seed, uint64_t rng_step, void* stream) {
  if (!h) return vfail(GO1_E_ARG, "go1_vel_resample: null handle");
  if (!h->bound) return vfail(GO1_E_STATE, "go1_vel_resample: bind the state first");
  if ((uniforms == nullptr) != (uniforms_f64 == nullptr))
    return vfail(GO1_E_ARG, "go1_vel_resample: parity mode needs both uniform arrays");
  CArgs C = curriculum_args(h);
  C.seed = rng_seed;
  if (mask) {
    C.maskB = mask;
    C.UB = uniforms;
    C.UDB = uniforms_f64;
    C.stepB = rng_step;
  } else {
    C.doA = 1;
    C.UA = uniforms;
    C.UDA = uniforms_f64;
    C.stepA = rng_step;
  }
  // the lists (slot 2) from the mask / the interval condition, then the curriculum on them
  C.list = h->d_clist + (size_t)4 * C.n_envs;
  C.cnt = h->d_ccnt + 2;
  hipLaunchKernelGGL(go1_vel_list_kernel, dim3(1), dim3(CK_THREADS), 0, (hipStream_t)stream, h->d_vcfg, C,
                     const_cast<CkRec*>(C.list), const_cast<unsigned long long*>(C.cnt));
  hipLaunchKernelGGL(go1_vel_curriculum_kernel, dim3(C.nblk), dim3(CK_THREADS), 0, (hipStream_t)stream, h->d_vcfg, C.n_envs, C.nb,
                     C.cnt, C.list, C.cdf, C.cdf_ok, C);
  VHIP_TRY(hipGetLastError());
  return GO1_OK;
}

int go1_vel_reset_idx(go1_vel_handle* h, const int32_t* ids, int32_t n_ids, const float* uniforms,
                      const double* uniforms_f64, uint64_t rng_seed, uint64_t rng_step, float* episode_log,
                      int32_t* episode_log_count, int32_t episode_log_cap, int32_t episode_log_tag, void* stream) {
  if (!h || (!ids && n_ids > 0) || n_ids < 0) return vfail(GO1_E_ARG, "go1_vel_reset_idx: bad argument");
  if (!h->bound || !h->env_origins) return vfail(GO1_E_STATE, "go1_vel_reset_idx: bind the state and origins first");
  if (n_ids == 0) return GO1_OK;  // (:178-179)
  if (episode_log_count && !episode_log) return vfail(GO1_E_ARG, "go1_vel_reset_idx: episode_log missing");
  hipStream_t s = (hipStream_t)stream;
  const int n = h->cfg.n_envs;
  // _resample_commands first (:182): a mask of the ids for the curriculum launch
  uint8_t* mask = h->d_mask;
  VHIP_TRY(hipMemsetAsync(mask, 0, n, s));
  hipLaunchKernelGGL(go1_vel_mask_kernel, dim3((n_ids + 255) / 256), dim3(256), 0, s, ids, n_ids, n, mask);
  int rc = go1_vel_resample(h, mask, uniforms, uniforms_f64, rng_seed, rng_step, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(go1_vel_reset_kernel, dim3((n_ids + EPB - 1) / EPB), dim3(TPB), 0, s, h->d_vcfg, h->st,
                     h->env_origins, ids, n_ids, n, uniforms, rng_seed, rng_step, h->cfg.env_id_offset, episode_log,
                     episode_log_count, episode_log_cap, episode_log_tag);
  VHIP_TRY(hipGetLastError());
  return GO1_OK;
}

int go1_vel_destroy(go1_vel_handle* h) {
  if (!h) return GO1_OK;
  if (h->d_done) (void)hipFree(h->d_done);
  if (h->d_clist) (void)hipFree(h->d_clist);
  if (h->d_ccnt) (void)hipFree(h->d_ccnt);
  if (h->d_cfg) (void)hipFree(h->d_cfg);
  if (h->d_vcfg) (void)hipFree(h->d_vcfg);
  if (h->d_grid) (void)hipFree(h->d_grid);
  if (h->d_cdf) (void)hipFree(h->d_cdf);
  if (h->d_cdf_ok) (void)hipFree(h->d_cdf_ok);
  if (h->d_mask) (void)hipFree(h->d_mask);
  if (h->d_adj_ptr) (void)hipFree(h->d_adj_ptr);
  if (h->d_adj_idx) (void)hipFree(h->d_adj_idx);
  delete h;
  return GO1_OK;
}
}  // extern "C"

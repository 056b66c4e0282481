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
#include "go1_device.h"

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
  __shared__ float s_mlp[MLP_PARK_FLOATS * 64];  // the fragments across the sub-step loop (mlp_park)
  mlp_park(F, s_mlp, lane);
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
  float eo_pre[3] = {K.ter.env_origins[(size_t)e * 3], K.ter.env_origins[(size_t)e * 3 + 1],
                     K.ter.env_origins[(size_t)e * 3 + 2]};
  float cam_pitch = st.base_rotation[(size_t)e * 3 + 1];  // previous step's pitch (:1939)
  // ---- the post-physics state inputs ride with the prologue loads (one wait for all of
  // them); they wait out the sub-step loop in LDS (s_hold, below), so after the physics only
  // the height-scan gathers make a memory round trip
  int ep_in = st.episode_length[e];
  int idx_in = st.curr_pose_index[e];
  int coll_in = st.collision_count[e];
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
  int my_id = sub16 < NT ? c_gen->term_ids[sub16] : GO1_T_NONE;
  float my_scale = A.reward_scales[sub16];
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
  // +8 float2 per env: the four envs' patches start 16 banks apart (unpadded they start on the same bank, and
  // the legs sit at similar cells of their env-centred patches: the corner reads of different envs collided)
  __shared__ float2 s_patch[SEPB][PSZX * PSZY + 8];
  __shared__ float s_phys[(LDS_FLOATS + 63) / 64 * 64];
  __shared__ __attribute__((aligned(16))) float s_self[SEPB][SELF_ENV_FLOATS];  // self-collision scratch
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
  // The post-physics inputs wait out the sub-step loop in LDS, one column per lane: the loop's register
  // peak is at the VGPR + AGPR limit, and these 23 values held across it pushed the kernel into scratch
  // spills (an extra ~1 MB of HBM writes per launch).  hold() re-reads them through an opaque pointer (the
  // compiler would otherwise forward the parked values and keep them in registers after all).
  __shared__ float s_hold[HOLD_N][TPB];
  auto hold = [&](bool park) {
    int hl = lane;
    if (!park) asm volatile("" : "+v"(hl));  // opaque index, not pointer: the reads stay ds_read (not flat)
    float* hp = &s_hold[0][hl];
    auto f = [&](int k, float& v) { if (park) hp[k * TPB] = v; else v = hp[k * TPB]; };
    auto i = [&](int k, int& v) { float x = __int_as_float(v); f(k, x); v = __float_as_int(x); };
#pragma unroll
    for (int k = 0; k < 6; ++k) f(k, traj_in[k]);
#pragma unroll
    for (int k = 0; k < 3; ++k) { f(6 + k, ldv[k]); f(9 + k, la[k]); f(12 + k, eo_pre[k]); }
    f(15, cam_pitch); f(16, my_scale); f(17, my_sum); f(18, my_tot);
    i(19, ep_in); i(20, idx_in); i(21, coll_in); i(22, my_id);
  };
  hold(true);
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
  float cf_raw[CF_RAW] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, cf_leg[9], cf_base[3], cf_hip[3];
  for (int sub = 0; sub < dec; ++sub) {
    MARK(sub_begin);
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
      {
        MlpFrag Fs;
        mlp_unpark(Fs, s_mlp, lane);
        mlp_group3(Fs, b0, b1v, tq);
      }
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
      MARK(phys_call);
#ifndef GO1_ABL_NO_PHYS
      for (int k = 0; k < c->n_internal; ++k) {
        const bool last = (sub == dec - 1) && (k == c->n_internal - 1);
        phys_substep(c, s_phys, P, torque, h, A.sim_gravity, friction, restitution, payload, T, leg, role, last,
                     cf_raw, s_self[el], sub == 0 && k == 0);
      }
#else
      P.qd[0] += 1e-4f * torque[0]; P.qd[1] += 1e-4f * torque[1]; P.qd[2] += 1e-4f * torque[2];
#endif
#pragma unroll
      for (int j = 0; j < 3; ++j) { q[j] = P.q[j]; qd[j] = P.qd[j]; }
      MARK(phys_returned);
    }
    if (A.dbg_torques && owner) {
#pragma unroll
      for (int j = 0; j < 3; ++j) A.dbg_torques[((size_t)sub * n + e) * NDOF + leg * 3 + j] = torque[j];
    }
  }
  cf_sum(cf_raw, role, cf_leg, cf_base, cf_hip);
  hold(false);
  float root[13];
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
    ol[0] = cf_hip[0]; ol[1] = cf_hip[1]; ol[2] = cf_hip[2];
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
  // slots 34 .. 46 = Philox blocks 8 .. 11: lane sub16 < 4 of the env draws block 8 + sub16 and the
  // env's lanes read their slots back from LDS (one evaluation per lane instead of four in a row; one
  // wave per block: its LDS operations complete in order)
  __shared__ float s_u[SEPB][32];
  const bool dr_step = ep % CI(rand_interval) == 0;
  if (dr_step) {
    if (sub16 < 4) {
      float uq[4];
      rng.quad(8 + sub16, uq);
#pragma unroll
      for (int k = 0; k < 4; ++k) s_u[el][4 * sub16 + k] = uq[k];
    }
    const float sv = s_u[el][34 - 32] * CI(strength_range) + CI(strength_lo);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      strength[j] = sv;
      offset[j] = s_u[el][35 + leg * 3 + j - 32] * CI(offset_range) + CI(offset_lo);
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
    for (int i = 0; i < 13; ++i) finite = finite & (fabsf(root[i]) < GO1_DIVERGED);
#pragma unroll
    for (int j = 0; j < 3; ++j) finite = finite & (fabsf(q[j]) < GO1_DIVERGED) & (fabsf(qd[j]) < GO1_DIVERGED);
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
  // noise uniforms rng(47 + i) (:472-473): the env's observed noisy columns use slots 47 .. 49
  // (gravity), 52 .. 63 (dof pos) and 64 .. 75 (dof vel), i.e. Philox blocks 11 .. 18: lane
  // sub16 < 8 draws block 11 + sub16 into LDS (one evaluation per lane; it was two), and role
  // r < 3 reads slots 52 + d and 64 + d, role 3 slots 47, 48, 49
  const int dn = leg * 3 + (role < 3 ? role : 0);
  float un = 0.0f, uv = 0.0f, ug[3] = {0.0f, 0.0f, 0.0f};
  if (CI(add_noise)) {
    if (sub16 < 8) {
      float uq[4];
      rng.quad(11 + sub16, uq);
#pragma unroll
      for (int k = 0; k < 4; ++k) s_u[el][4 * sub16 + k] = uq[k];
    }
    un = s_u[el][52 + dn - 44];
    uv = s_u[el][64 + dn - 44];
#pragma unroll
    for (int i = 0; i < 3; ++i) ug[i] = s_u[el][47 + i - 44];
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
    put(0, pg[0], CI(noise_gravity), ug[0], true);
    put(1, pg[1], CI(noise_gravity), ug[1], true);
    put(2, pg[2], CI(noise_gravity), ug[2], true);
    put(3, cmd[0] * 1.0f, 0.0f, 0.0f, false);
    put(4, cmd[1] * 1.0f, 0.0f, 0.0f, false);
  }
  if (CI(timestep_in_obs) && role == 3 && leg == 1)
    put(41, (float)(reset ? 0 : ep) / CI(max_episode_length), 0.0f, 0.0f, false);
  if (role < 3) {
    const int j = role, d = dn;
    const float qj = sel3(j, q), qdj = sel3(j, qd), aj = sel3(j, act);
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
// zero the stamp buffer (before the launch to be read: a wave records only as many slots as it executes
// markers, so slots of an earlier launch with more markers would otherwise survive behind them)
int go1_debug_stamps_clear(void) {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_go1_stamps)) != hipSuccess) return 1;
  if (hipMemset(p, 0, sizeof(g_go1_stamps)) != hipSuccess) return 1;
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
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
  // the capsules' deepest-point search (go1_device.h seg_deepest) takes at most 3 grid lines per direction and 4 cell
  // diagonals per half link (0.1065 m): cells of at least 0.05 m
  if (cfg->terrain_kind == 1 && !(cfg->horizontal_scale >= 0.0499f))
    return fail(GO1_E_ARG, "go1_create: horizontal_scale < 0.05 m is not supported by the capsule contact search");
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

/*
 * go1_velocity.h -- C ABI of the MI355X-native Go1 velocity-tracking step (BASELINE configs[1]:
 * scripts/train_velocity_tracking.py, 4096 Go1 on a plane, CoRL reward terms, gait commands and the
 * reward-threshold command curriculum).
 *
 * It replaces, for VelocityTrackingEasyEnv (go1_gym/envs/go1/velocity_tracking/__init__.py:11-44) on
 * go1_gym/envs/base/legged_robot_velocity_tracking.py (bare :N below):
 *
 *   go1_vel_step()      <- LeggedRobot.step                           :60-106
 *                          (_compute_torques :925-964 with the actuator net :1256-1271, the Isaac Gym
 *                           simulate / refresh calls :76-82, :113-115 replaced by the native articulated-body
 *                           integrator of go1_mi355x.h, post_physics_step :108-154, _post_physics_step_callback
 *                           :693-727, _step_contact_targets :844-923, check_termination :156-166,
 *                           compute_reward :281-318 over CoRLRewards (go1_gym/envs/rewards/corl_rewards.py),
 *                           reset_idx :168-257, compute_observations :320-509)
 *                          + HistoryWrapper.step's obs_history shift (go1_gym/envs/wrappers/history_wrapper.py:18-24)
 *   go1_vel_reset_idx() <- LeggedRobot.reset_idx(env_ids)               :168-257
 *   go1_vel_resample()  <- _resample_commands(env_ids) (:728-842) with RewardThresholdCurriculum.update
 *                          and Curriculum.sample (go1_gym/envs/base/curriculum.py:67-89, :135-154)
 *
 * Conventions as go1_mi355x.h: caller-owned device buffers (PyTorch tensors), asynchronous on the
 * caller's stream, 0 or a negative GO1_E_* code, go1_vel_last_error(), one host thread per handle.
 *
 * Launches per go1_vel_step: the fused env step (one wave per 4 envs, the integrator of the
 * trajectory step) and one single-workgroup curriculum launch.  The curriculum launch resamples the
 * commands of the envs the step reset (their obs / obs_history command columns are rewritten) and,
 * ahead of time, of the envs whose next step starts a resampling interval (episode_length + 1 ==
 * 0 mod resample_interval), with the next step's draws: the reference runs that resample at the start
 * of the next step's post-physics callback (:702-704), and nothing between the two launches reads or
 * writes what it touches.  Weights of the curricula are f64 as numpy keeps them; the command draw is
 * numpy's rng.choice(p = w / w.sum()) inverse cdf and rng.uniform per cell, from caller uniforms
 * (parity mode) or Philox.
 */
#ifndef GO1_VELOCITY_H
#define GO1_VELOCITY_H

#include <stdint.h>

#include "go1_mi355x.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GO1_VEL_ABI_VERSION 2
#define GO1_VEL_NUM_COMMANDS 15  /* x, y, yaw vel, body height, gait freq, phase, offset, bound, duration,
                                    footswing height, body pitch, body roll, stance width, stance length, aux */
#define GO1_VEL_NUM_OBS 70       /* gravity 3, commands 15, dof pos 12, dof vel 12, actions 12, last actions 12,
                                    clock 4 (:337-356, observe_two_prev_actions, observe_clock_inputs) */
#define GO1_VEL_MAX_TERMS 24
#define GO1_VEL_SUM_EXTRA 5      /* command_sums after the terms: lin_vel_raw, ang_vel_raw, lin_vel_residual,
                                    ang_vel_residual, ep_timesteps (:314-318) */
#define GO1_VEL_N_CATEGORIES 4   /* pronk, trot, pace, bound (gaitwise_curricula) */
#define GO1_VEL_N_KEYS 15        /* curriculum keys (_init_command_distribution :1328-1374) */
#define GO1_VEL_MAX_BINS 1024
#define GO1_VEL_AUX 42           /* base lin vel 3, base ang vel 3, foot positions 12 (world), torques 12,
                                    joint_pos_target 12: the VelocityTrackingEasyEnv.step extras
                                    (velocity_tracking/__init__.py:25-41) the state planes do not hold */
/* Parity-mode f32 uniforms per env (legged_tracking_amd/vel_layout.py) */
#define GO1_VEL_U_CAT_A 0        /* category draw of the periodic resample (:760) */
#define GO1_VEL_U_CAT_B 1        /* category draw of the resample inside reset_idx */
#define GO1_VEL_U_DR 2           /* _randomize_dof_props every rand_interval: strength 1, offsets 12 */
#define GO1_VEL_U_RESET_DR 15    /* _randomize_dof_props in reset_idx (:183) */
#define GO1_VEL_U_RESET_DOF 28   /* _reset_dofs (:974): 12 */
#define GO1_VEL_U_RESET_YAW 40   /* _reset_root_states yaw (:1007-1009) */
#define GO1_VEL_U_RESET_VEL 41   /* base velocities (:1014): 6 */
#define GO1_VEL_U_NOISE 47       /* observation noise (:394): one per obs column */
#define GO1_VEL_U_PER_ENV (GO1_VEL_U_NOISE + GO1_VEL_NUM_OBS)
/* Parity-mode f64 uniforms per env (the curricula's numpy RandomState) */
#define GO1_VEL_D_CHOICE_A 0     /* rng.choice's random_sample, then the 15 rng.uniform cell draws */
#define GO1_VEL_D_CHOICE_B 16
#define GO1_VEL_D_PER_ENV 32

/* CoRLRewards functions the step evaluates (go1_gym/envs/rewards/corl_rewards.py) */
enum go1_vel_term {
  GO1_VT_TRACKING_LIN_VEL = 0,   /* :15-18 */
  GO1_VT_TRACKING_ANG_VEL,       /* :20-23 */
  GO1_VT_LIN_VEL_Z,              /* :25-27 */
  GO1_VT_ANG_VEL_XY,             /* :29-31 */
  GO1_VT_ORIENTATION,            /* :33-35 */
  GO1_VT_TORQUES,                /* :37-39 */
  GO1_VT_DOF_ACC,                /* :41-43 */
  GO1_VT_ACTION_RATE,            /* :45-47 */
  GO1_VT_COLLISION,              /* :49-52, redefined identically :176-179 */
  GO1_VT_DOF_POS_LIMITS,         /* :54-58 */
  GO1_VT_JUMP,                   /* :60-65 */
  GO1_VT_TRACKING_CONTACTS_SHAPED_FORCE, /* :67-75 */
  GO1_VT_TRACKING_CONTACTS_SHAPED_VEL,   /* :77-84 */
  GO1_VT_DOF_POS,                /* :86-88 */
  GO1_VT_DOF_VEL,                /* :90-92 */
  GO1_VT_ACTION_SMOOTHNESS_1,    /* :94-98 */
  GO1_VT_ACTION_SMOOTHNESS_2,    /* :100-105 */
  GO1_VT_FEET_SLIP,              /* :107-113 (updates last_contacts) */
  GO1_VT_FEET_CLEARANCE_CMD_LINEAR, /* :130-135 */
  GO1_VT_ORIENTATION_CONTROL,    /* :181-193 */
  GO1_VT_RAIBERT_HEURISTIC,      /* :195-237 */
  GO1_VT_COUNT
};

typedef struct go1_vel_config {
  int32_t n_envs;              /* must equal the physics config's n_envs */
  int32_t n_terms;             /* reward terms with a nonzero scale, Cfg.reward_scales order */
  int32_t term_ids[GO1_VEL_MAX_TERMS];
  uint32_t nonpos_slots;       /* bit k: slot k's scaled reward is <= 0 for every env (its scale times the
                                  term's fixed sign), i.e. it lands in rew_buf_neg (:293-296) */
  int32_t reward_mode;         /* 0 sum, 1 only_positive_rewards, 2 only_positive_rewards_ji22_style (:302-305) */
  int32_t resample_interval;   /* int(resampling_time / dt) (:702) */
  int32_t rand_interval;       /* int(rand_interval) (:715) */
  int32_t add_noise;           /* (:393-394) */
  int32_t use_terminal_body_height; /* (:163-166) */
  int32_t history_len;         /* HistoryWrapper num_observation_history: obs_history width = 70 x this */
  int32_t n_bins;              /* curriculum grid columns, <= GO1_VEL_MAX_BINS */
  int32_t gaitwise_curricula;  /* (:782-799) */
  int32_t binary_phases;       /* (:832-835) */
  int32_t n_task;              /* task keys with a reward scale (:746-750), <= 4 */
  int32_t task_slot[4];        /* their command_sums slot */
  float task_threshold[4];     /* f32(curriculum_thresholds[k] * reward_scales[k]) */
  float curriculum_ep_len;     /* min(max_episode_length, resample_interval) (:733) */
  float max_episode_length;
  float dt;
  float clip_obs;
  float cmd_scale[GO1_VEL_NUM_COMMANDS];
  float noise_vec[GO1_VEL_NUM_OBS];
  float obs_scale_dof_pos, obs_scale_dof_vel;
  float priv_friction_shift, priv_friction_scale, priv_rest_shift, priv_rest_scale;
  float strength_range, strength_lo, offset_range, offset_lo;
  float reset_dof_range, reset_dof_lo, reset_vel_range, reset_vel_lo, yaw_range, yaw_lo;
  float base_init_state[13];
  float default_dof_pos[12];
  float dof_pos_limits[24];    /* soft limits (lo, hi) per dof (:622-625) */
  float tracking_sigma, tracking_sigma_yaw, gait_force_sigma, gait_vel_sigma, kappa_gait_probs;
  float base_height_target, sigma_rew_neg, terminal_body_height;
  int32_t pad;
  double local_range[GO1_VEL_N_KEYS];  /* update's neighbourhood (:755-757) */
  double bin_sizes[GO1_VEL_N_KEYS];
} go1_vel_config;

/* Per-env state, SoA (n_envs, width) row-major, f32 unless noted.  The first 15 planes are the physics
 * planes of go1_state with the same meaning. */
#define GO1_VEL_STATE_PLANES 25
typedef struct go1_vel_state {
  float* root;              /* 13 */
  float* dof_pos;           /* 12 */
  float* dof_vel;           /* 12 */
  float* last_actions;      /* 12 */
  float* last_dof_vel;      /* 12 */
  float* lag;               /* 12 x GO1_LAG_STEPS(decimation) (go1_state.lag) */
  float* pos_err_hist;      /* 24 */
  float* vel_hist;          /* 24 */
  float* motor_strength;    /* 12 */
  float* motor_offset;      /* 12 */
  float* friction;          /* 1 */
  float* restitution;       /* 1 */
  float* payload;           /* 1 */
  int32_t* episode_length;  /* 1 */
  float* last_last_actions; /* 12 */
  float* last_joint_pos_target;      /* 12 */
  float* last_last_joint_pos_target; /* 12 */
  float* commands;          /* 15 */
  float* gait_indices;      /* 1 */
  float* last_contacts;     /* 4 (feet_slip) */
  float* command_sums;      /* n_terms + GO1_VEL_SUM_EXTRA */
  float* episode_sums;      /* n_terms + 1 (reward_scales order, then total) */
  int32_t* command_bins;    /* 1 */
  int32_t* command_categories; /* 1 */
  double* curriculum_weights;  /* (GO1_VEL_N_CATEGORIES, n_bins) f64 -- not per env */
} go1_vel_state;

typedef struct go1_vel_step_args {
  const float* actions;             /* (n_envs, 12) */
  float gravity_vec[3];             /* self.gravity_vec at the start of post_physics_step (projected gravity) */
  float gravity_vec_after[3];       /* self.gravity_vec after this step's _randomize_gravity (orientation_control) */
  float sim_gravity[3];             /* gravity the integrator applies */
  float reward_scales[GO1_VEL_MAX_TERMS]; /* slot order, x dt */
  uint64_t rng_seed, rng_step;      /* Philox keys; the ahead-of-time resample uses rng_step + 1 */
  const float* uniforms;            /* parity mode: (n_envs, GO1_VEL_U_PER_ENV) of this step, NULL -> Philox */
  const double* uniforms_f64;       /* parity mode: (n_envs, GO1_VEL_D_PER_ENV) of this step */
  const float* uniforms_next;       /* parity mode: the next step's (for its resample, done ahead) or NULL:
                                       no ahead-of-time resample in this call */
  const double* uniforms_f64_next;
  int32_t resample_next;            /* 1: resample the next step's interval envs ahead (go1_vel_step's default
                                       use); 0: leave them (the caller runs go1_vel_resample before the step) */
  int32_t pad;
  /* parity mode: injected physics instead of the native integrator */
  const float* inj_dof;             /* (decimation, n_envs, 12, 2) */
  const float* inj_root;            /* (n_envs, 13) */
  const float* inj_contact;         /* (n_envs, 17, 3) */
  const float* inj_feet;            /* (n_envs, 4, 6): foot positions, foot velocities (rigid_body_state) */
  /* outputs */
  float* obs;                       /* (n_envs, 70) */
  float* priv;                      /* (n_envs, 2) */
  float* rew;                       /* (n_envs) */
  uint8_t* reset;                   /* (n_envs) */
  uint8_t* time_out;                /* (n_envs) */
  uint8_t* extras_time_outs;        /* (n_envs): time_out, rebound only on steps with a reset (:251-252) */
  float* contact_forces;            /* (n_envs, 17, 3) or NULL */
  const float* obs_history_in;      /* (n_envs, 70 x history_len) rows obs_history_in_ld apart, or NULL (no
                                       history output) */
  float* obs_history_out;           /* cat(in[:, 70:], obs) (HistoryWrapper.step), rows obs_history_out_ld apart:
                                       another buffer, or in + 70 with the same row stride (a sliding window
                                       over rows wider than the history: the shift is the identity and skipped,
                                       only the new observation is written) */
  float* aux;                       /* (n_envs, GO1_VEL_AUX) or NULL */
  /* compact episode log, a ring: each env reset this step writes n_terms + 3 floats (n_terms + 1 episode
     sums, tag, env index) at row (uint32) atomicAdd(*episode_log_count, 1) % episode_log_cap; the tag is
     stored as its int32 bits (exact for every tag; read the column as int32), the env index as a float */
  float* episode_log;
  int32_t* episode_log_count;
  int32_t episode_log_cap;
  int32_t episode_log_tag;
  /* optional debug outputs */
  float* dbg_torques;               /* (decimation, n_envs, 12) */
  float* dbg_terms;                 /* (n_envs, GO1_VEL_MAX_TERMS) unscaled, slot order */
  float* dbg_gait;                  /* (n_envs, 12): foot_indices 4, clock_inputs 4, desired_contact_states 4 */
  void* ev_begin;                   /* optional hipEvent_t pair around the step kernel */
  void* ev_end;
  int64_t obs_history_in_ld;        /* row strides of obs_history_in / _out in floats (0: 70 x history_len); */
  int64_t obs_history_out_ld;       /* >= 70 x history_len, the window of a row is contiguous (ABI v2) */
} go1_vel_step_args;

typedef struct go1_vel_handle go1_vel_handle;

int go1_vel_abi_version(void);
/* sizeof go1_vel_config, go1_vel_state, go1_vel_step_args */
void go1_vel_abi_sizes(int64_t out[3]);
const char* go1_vel_last_error(void);
/* phys: the integrator / actuator / action fields of a go1_config (terrain_kind 0: the plane);
 * grid: host (GO1_VEL_N_KEYS, n_bins) f64 bin centroids (Curriculum.grid). */
int go1_vel_create(const go1_config* phys, const go1_vel_config* vel, const double* grid, go1_vel_handle** out);
/* planes: GO1_VEL_STATE_PLANES descriptors (go1_plane), go1_vel_state order; curriculum_weights is
 * (GO1_VEL_N_CATEGORIES, n_bins) f64 (dtype 2). */
#define GO1_DTYPE_F64 2
int go1_vel_bind(go1_vel_handle* h, const go1_vel_state* state, const go1_plane* planes);
/* env_origins (n_envs, 3) f32 device (_get_env_origins :1693-1733) */
int go1_vel_set_origins(go1_vel_handle* h, const float* env_origins);
int go1_vel_step(go1_vel_handle* h, const go1_vel_step_args* args, void* stream);
/* reset_idx(env_ids): _resample_commands, DR, dofs, root, buffers; the reset envs' episode sums are
 * appended to the compact log (NULL: not logged).  uniforms as in go1_vel_step (NULL: Philox(seed, step)). */
int go1_vel_reset_idx(go1_vel_handle* h, const int32_t* ids, int32_t n_ids, const float* uniforms,
                      const double* uniforms_f64, uint64_t rng_seed, uint64_t rng_step, float* episode_log,
                      int32_t* episode_log_count, int32_t episode_log_cap, int32_t episode_log_tag, void* stream);
/* _resample_commands for the envs of mask (uint8 per env) with draws of the B (reset) kind, or, with
 * mask NULL, the interval resample of the envs whose episode_length + 1 == 0 mod resample_interval
 * (the A kind) -- what a step does ahead of time for its successor. */
int go1_vel_resample(go1_vel_handle* h, const uint8_t* mask, const float* uniforms, const double* uniforms_f64,
                     uint64_t rng_seed, uint64_t rng_step, void* stream);
int go1_vel_destroy(go1_vel_handle* h);

#ifdef __cplusplus
}
#endif
#endif /* GO1_VELOCITY_H */
